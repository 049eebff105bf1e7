#!/bin/bash
# Throughput of every north-star family on ONE MI355X (random-init GGUFs generated on the box).
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
run() {  # name model ftype concurrency
  timeout -k 10 420 python -u bench.py --no-rtt --model $2 --ftype $3 --concurrency $4 --steps 20 --warmup 3 > gpurun_out/models_$1.log 2>&1
  local rc=$?
  echo "$1 rc=$rc $(tail -1 gpurun_out/models_$1.log | cut -c1-330)"
  case $rc in 124|134|137|139) exit $rc ;; esac
}
run qwen7b_b512 qwen2.5-7b Q4_K_M 512
run mixtral_b256 mixtral-8x7b Q5_K_M 256
run mixtral_b1 mixtral-8x7b Q5_K_M 1
run l70b_b128 llama-3-70b Q4_K_M 128
run l70b_b1 llama-3-70b Q4_K_M 1
rm -f /tmp/nls_bench/*.gguf
