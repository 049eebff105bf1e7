#!/usr/bin/env bash
# Mode-7 A/B at the Llama-3-70B projection shapes (single GPU, large batch).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/blaslt_ab.py --model llama-3-70b --M 128,256,512 \
    --shapes qkv,o,gateup,down,lm_head > gpurun_out/blaslt_ab_70b.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/blaslt_ab_70b.txt | tail -16; exit $rc
