#!/bin/bash
# Mixtral decode: grouped-GEMM token threshold (NLS_MOE_GEMM_T) at mid batch sizes, then a B=256 profile
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  local label=$1; shift
  env "$@" timeout -k 10 500 python -u bench.py --model mixtral-8x7b --ftype Q5_K_M --steps 30 --warmup 5 --no-rtt --serve-load 0 $BARGS > gpurun_out/th_$label.log 2>&1 || { tail -20 gpurun_out/th_$label.log; exit 1; }
  echo "$label $BARGS $(tail -1 gpurun_out/th_$label.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["timings_s"]["prefill_all"])')"
}
for B in 16 32 64; do
  BARGS="--concurrency $B"
  run b${B}t64
  run b${B}t8 NLS_MOE_GEMM_T=8
done
BARGS="--concurrency 64"; run b64t8rt2 NLS_MOE_GEMM_T=8 NLS_MOE_RT_GU=2 NLS_MOE_RT_DN=2
TAG=mixna bash scripts/gpu_prof_mix256.sh
