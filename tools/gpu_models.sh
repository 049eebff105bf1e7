#!/bin/bash
# Throughput of every north-star family on ONE MI355X (random-init GGUFs generated on the box).
# RUNS="name ..." selects a subset (default: all but l8b_b512 / qwen7b_b1).
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
run() {  # name model ftype concurrency
  timeout -k 10 420 python -u bench.py --no-rtt --serve-load 0 --tp-leg 0 --model $2 --ftype $3 --concurrency $4 --steps 20 --warmup 3 > gpurun_out/models_$1.log 2>&1
  local rc=$?
  echo "$1 rc=$rc $(tail -1 gpurun_out/models_$1.log | cut -c1-330)"
  case $rc in 124|134|137|139) exit $rc ;; esac
}
RUNS=${RUNS:-"qwen7b_b512 mixtral_b256 mixtral_b1 l70b_b128 l70b_b1"}
for r in $RUNS; do
  case $r in
    qwen7b_b512) run $r qwen2.5-7b Q4_K_M 512 ;;
    qwen7b_b1) run $r qwen2.5-7b Q4_K_M 1 ;;
    mixtral_b256) run $r mixtral-8x7b Q5_K_M 256 ;;
    mixtral_b1) run $r mixtral-8x7b Q5_K_M 1 ;;
    l70b_b128) run $r llama-3-70b Q4_K_M 128 ;;
    l70b_b1) run $r llama-3-70b Q4_K_M 1 ;;
    l8b_b512) run $r llama-3-8b Q4_K_M 512 ;;
  esac
done
rm -f /tmp/nls_bench/*.gguf
