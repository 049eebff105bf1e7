#!/bin/bash
# A/B of the MoE grouped-GEMM m-block size (NLS_MOE_RT_GU / NLS_MOE_RT_DN = 1/2/4 -> 64/128/256 rows)
# on Mixtral-8x7B Q5_K_M at batch B (default 256); one bench per "gu:dn" pair in $PAIRS.
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
B=${B:-256}
for p in ${PAIRS:-2:2 2:1 1:1 4:2}; do
  gu=${p%:*}; dn=${p#*:}
  NLS_MOE_RT_GU=$gu NLS_MOE_RT_DN=$dn timeout -k 10 300 python -u bench.py --no-rtt --model mixtral-8x7b --ftype Q5_K_M \
    --concurrency $B --steps 20 --warmup 3 > gpurun_out/moe_ab_${gu}_${dn}.log 2>&1 || { echo "gu=$gu dn=$dn failed"; tail -5 gpurun_out/moe_ab_${gu}_${dn}.log; exit 1; }
  echo "gu=$gu dn=$dn $(tail -1 gpurun_out/moe_ab_${gu}_${dn}.log | grep -o '"value": [0-9.]*, "unit"[^,]*, "n_gpus": 1, "steps": 20, "warmup": 3, "ms_per_step": [0-9.]*')"
done
