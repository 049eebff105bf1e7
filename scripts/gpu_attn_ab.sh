#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
K=$PWD/nats_llm_studio_amd
for rep in 1 2; do
for lib in _kernels.so _kernels_pf1.so; do
for cap in "32 512" "128 1024"; do
  set -- $cap
  for pt in "1 4096" "16 4096"; do
    read B P <<< "$pt"
    NLS_KERNELS_SO=$K/$lib NLS_ATTN_SPLIT_CAP=$1 NLS_ATTN_SPLIT_WG=$2 timeout -k 10 200 python -u bench.py --concurrency $B --prompt-len $P --steps 50 --warmup 5 --no-rtt --serve-load 0 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    echo "$lib cap=$1 wg=$2 B=$B P=$P $(tail -1 gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
done
done
