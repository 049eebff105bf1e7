#!/bin/bash
# attention K/V prefetch depth 1 vs 2 at short / medium context, batch 1 and 16
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
K=$PWD/nats_llm_studio_amd
run() {
  local label=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 150 --warmup 10 --no-rtt --serve-load 0 $BARGS > gpurun_out/pf_$label.log 2>&1 || { tail -20 gpurun_out/pf_$label.log; exit 1; }
  echo "$label $BARGS $(tail -1 gpurun_out/pf_$label.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
for rep in 1 2; do
  for pt in "1 128" "1 1024" "16 1024"; do
    set -- $pt
    BARGS="--concurrency $1 --prompt-len $2"
    run c$1_p$2_pf1 NLS_KERNELS_SO=$K/_kernels.so
    run c$1_p$2_pf2 NLS_KERNELS_SO=$K/_kernels_pf2.so
  done
done
