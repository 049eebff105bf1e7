#!/bin/bash
# MoE down projection split-K: tests, then Mixtral B=256 decode over NLS_MOE_KS_DN
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "moe or mapped or mixtral" > gpurun_out/moeks_tests.log 2>&1 || { tail -30 gpurun_out/moeks_tests.log; exit 1; }
tail -1 gpurun_out/moeks_tests.log
run() {
  local label=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --model mixtral-8x7b --ftype Q5_K_M --steps 30 --warmup 5 --no-rtt --serve-load 0 $BARGS > gpurun_out/moeks_$label.log 2>&1 || { tail -20 gpurun_out/moeks_$label.log; exit 1; }
  echo "$label $BARGS $(tail -1 gpurun_out/moeks_$label.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["timings_s"]["prefill_all"])')"
}
BARGS="--concurrency 256"
for ks in 1 2 4 8; do run ks$ks NLS_MOE_KS_DN=$ks; done
BARGS="--concurrency 128"
for ks in 1 4; do run b128ks$ks NLS_MOE_KS_DN=$ks; done
rm -f /tmp/nls_bench/*.gguf
