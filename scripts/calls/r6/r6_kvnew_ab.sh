#!/bin/bash
# round 6: attribution of the decode attention's new-row cost (GGML_MI355X_KVNEW_DBG, timing only)
cd "$(dirname "$0")/../../.."
for dbg in 0 1 2; do
  GGML_MI355X_KVNEW_DBG=$dbg OUT=gpurun_out/r6 bash scripts/r6.sh "prof prof_kvnew_dbg$dbg -fa 1 -p 0 -n 128 -c 256 -r 1 -ctk 8" > gpurun_out/r6/kvnew_dbg$dbg.txt 2>&1 || exit $?
  echo "dbg=$dbg $(grep -h 'k_fattn_dec2' gpurun_out/r6/prof_kvnew_dbg${dbg}_kernel_stats.csv)"
done
GGML_MI355X_NO_KV_DEFER=1 OUT=gpurun_out/r6 bash scripts/r6.sh "prof prof_kvnew_nodefer -fa 1 -p 0 -n 128 -c 256 -r 1 -ctk 8" > gpurun_out/r6/kvnew_nodefer.txt 2>&1 || exit $?
echo "nodefer $(grep -h 'k_fattn_dec2\|kv_store' gpurun_out/r6/prof_kvnew_nodefer_kernel_stats.csv)"
