#!/usr/bin/env bash
# Last validation of the round + the 70B batch-256 policy check and the sampled-mix number.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_check.sh all || exit $?
run() {  # tag args...
  local tag=$1; shift
  timeout -k 10 420 python -u bench.py --no-rtt --serve-load 0 --steps 40 --warmup 5 "$@" > gpurun_out/f3_$tag.log 2>&1 \
      || { tail -5 gpurun_out/f3_$tag.log; exit 1; }
  echo "$tag $(tail -1 gpurun_out/f3_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
run sampled50_b512 --sample-frac 0.5
run l70_b256_auto --model llama-3-70b --concurrency 256
export NLS_DENSE_WEIGHTS=0
run l70_b256_quant --model llama-3-70b --concurrency 256
unset NLS_DENSE_WEIGHTS
