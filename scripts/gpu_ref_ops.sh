#!/bin/bash
# Runs the reference parity harness (oracle/_ref/test-backend-ops, built from the
# reference sources) against libggml-mi355x.so, one op family at a time.
# Stops at the first crash/timeout so a faulting kernel never gets re-run.
cd "$(dirname "$0")/.."
export GGML_BACKEND_PATH=$PWD/llama-mi50.cpp_amd/lib/libggml-mi355x.so
OUT=${OUT:-gpurun_out/refops}
mkdir -p $OUT
OPS=${OPS:-"ADD MUL SCALE RMS_NORM ROPE SOFT_MAX SET_ROWS GET_ROWS CPY CONT SWIGLU,GEGLU,REGLU,GEGLU_ERF,GEGLU_QUICK MUL_MAT FLASH_ATTN_EXT MUL_MAT_ID ARGSORT SUM_ROWS"}
for op in $OPS; do
  timeout -k 10 ${TMO:-240} oracle/_ref/test-backend-ops -b MI355X0 -o $op > $OUT/$op.log 2>&1
  rc=$?
  echo "$op rc=$rc $(grep -c 'OK' $OUT/$op.log) ok $(grep -c 'FAIL' $OUT/$op.log) fail $(grep -c 'not supported' $OUT/$op.log) unsupported"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ $rc -ge 128 ]; then
    echo "stopping after $op (rc=$rc)"; exit $rc
  fi
done
exit 0
