cd /root/repo
S=scripts/r6.sh
bash $S "tests tests/test_dropin_gpu.py tests/test_ops_gpu.py tests/test_refops_gpu.py tests/test_dropin_shapes_gpu.py -k dropin+or+set_rows+or+flash_attn+or+FLASH+or+SET_ROWS+or+llama3_8b+or+mixtral" ; \
bash $S "tbo perf_mulmat perf -b MI355X0 -o MUL_MAT -p type_a=(q4_0|q8_0|q4_K|q5_K|q6_K),type_b=f32,m=4096,n=(1|2|3|4|5|8),k=14336" && \
bash $S "prof prof_pp512_fa1 -fa 1 -p 512 -n 0 -c 512 -r 2" "prof prof_pp512_fa0 -fa 0 -p 512 -n 0 -c 512 -r 2" && \
bash $S "lb ab_f16_a -fa 1 -p 0 -n 128 -r 5" "lb ab_q8_a -fa 1 -p 0 -n 128 -r 5 -ctk q8_0 -ctv q8_0" "envlb ab_q8nd_a GGML_MI355X_NO_KV_DEFER=1 -- -fa 1 -p 0 -n 128 -r 5 -ctk q8_0 -ctv q8_0" "lb ab_q8kf16v_a -fa 1 -p 0 -n 128 -r 5 -ctk q8_0 -ctv f16" \
  "lb ab_f16_b -fa 1 -p 0 -n 128 -r 5" "lb ab_q8_b -fa 1 -p 0 -n 128 -r 5 -ctk q8_0 -ctv q8_0" "envlb ab_q8nd_b GGML_MI355X_NO_KV_DEFER=1 -- -fa 1 -p 0 -n 128 -r 5 -ctk q8_0 -ctv q8_0" "lb ab_q8kf16v_b -fa 1 -p 0 -n 128 -r 5 -ctk q8_0 -ctv f16"
