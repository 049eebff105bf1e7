#!/usr/bin/env bash
# Llama-3-70B Q4_K_M on one MI355X: quantised kernels only (auto: the f16 copies do not fit the 45 %
# budget) vs f16 copies (NLS_DENSE_WEIGHTS=1) with the hand dense GEMMs / with mode 7.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() {  # tag concurrency env...
  local tag=$1 c=$2; shift 2
  env "$@" timeout -k 10 420 python -u bench.py --no-rtt --serve-load 0 --model llama-3-70b --ftype Q4_K_M \
      --concurrency $c --steps 20 --warmup 3 > gpurun_out/l70_$tag.log 2>&1
  local rc=$?
  echo "$tag rc=$rc $(tail -1 gpurun_out/l70_$tag.log | python3 -c 'import json,sys
try:
    d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["timings_s"])
except Exception as e: print("parse error", e)')"
  [ $rc -eq 0 ] || exit $rc
}
run b128_auto 128 NLS_DENSE_WEIGHTS=auto
run b128_dense_lib 128 NLS_DENSE_WEIGHTS=1 NLS_LIB_GEMM=1
run b128_dense_nolib 128 NLS_DENSE_WEIGHTS=1 NLS_LIB_GEMM=0
run b512_dense_lib 512 NLS_DENSE_WEIGHTS=1 NLS_LIB_GEMM=1
run b512_auto 512 NLS_DENSE_WEIGHTS=auto
