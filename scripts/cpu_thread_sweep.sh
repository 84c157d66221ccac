cat /sys/fs/cgroup/cpu.max 2>&1; nproc; python -c "import os; print(os.cpu_count(), len(os.sched_getaffinity(0)))"
G=/tmp/mx_bench_llama3_8b_q4_k_m.gguf
for t in 16 32 64; do timeout -k 5 200 oracle/_ref/ref-llama-bench -m $G -t $t -p 32 -n 16 -r 1 2>/dev/null | tail -1; done
