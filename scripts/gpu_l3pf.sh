#!/bin/bash
# batch-1 decode: Infinity-Cache prefetch of each layer's FFN weights on a side stream (A/B)
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
run() {
  local label=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 150 --warmup 10 --no-rtt --serve-load 0 $BARGS > gpurun_out/pf3_$label.log 2>&1 || { tail -20 gpurun_out/pf3_$label.log; exit 1; }
  echo "$label $BARGS $(tail -1 gpurun_out/pf3_$label.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
BARGS="--concurrency 1"
for rep in 1 2; do
  run off NLS_L3_PREFETCH=0
  run wg256 NLS_L3_PREFETCH=1 NLS_L3_PREFETCH_WG=256
  run wg512 NLS_L3_PREFETCH=1 NLS_L3_PREFETCH_WG=512
  run wg1024 NLS_L3_PREFETCH=1 NLS_L3_PREFETCH_WG=1024
done
