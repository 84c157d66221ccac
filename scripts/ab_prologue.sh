cd $GRAFT_REPO_ROOT
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-dropin --skip-roofline --pp 0"
for i in 1 2; do
  $B > gpurun_out/a.log 2>&1 && echo "asm $(tail -1 gpurun_out/a.log | cut -c80-100)"
  GGML_MI355X_LIB=$PWD/llama-mi50.cpp_amd/lib_noasm/libggml-mi355x.so $B > gpurun_out/b.log 2>&1 && echo "noasm $(tail -1 gpurun_out/b.log | cut -c80-100)"
done
OUT=gpurun_out/pa bash scripts/prof_decode.sh > /dev/null 2>&1
GGML_MI355X_LIB=$PWD/llama-mi50.cpp_amd/lib_noasm/libggml-mi355x.so OUT=gpurun_out/pb bash scripts/prof_decode.sh > /dev/null 2>&1
for d in pa pb; do echo $d; head -3 gpurun_out/$d/run_kernel_stats.csv | cut -d, -f1,4; done
