#!/bin/bash
# attention split policy: GPU tests of the touched kernels, then old (min 64 keys) vs adaptive
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or argmax or lm_head or qgemv or split" > gpurun_out/attnb1_tests.log 2>&1 || { tail -30 gpurun_out/attnb1_tests.log; exit 1; }
tail -1 gpurun_out/attnb1_tests.log
run() {
  local label=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 150 --warmup 10 --no-rtt --serve-load 0 $BARGS > gpurun_out/ab_$label.log 2>&1 || { tail -20 gpurun_out/ab_$label.log; exit 1; }
  echo "$label $BARGS $(tail -1 gpurun_out/ab_$label.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
for rep in 1 2; do
  for pt in "1 128" "1 1024" "1 4096" "16 4096"; do
    set -- $pt
    BARGS="--concurrency $1 --prompt-len $2"
    run c$1_p$2_old NLS_ATTN_MIN_CHUNK=64
    run c$1_p$2_new NLS_ATTN_MIN_CHUNK=0
  done
done
