#!/usr/bin/env bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/blaslt_ab.py --model qwen2.5-7b --M 256,512,1024,2048 --shapes qkv,o,gateup,down,lm_head \
    > gpurun_out/blaslt_qwen.txt 2>&1 || { tail -5 gpurun_out/blaslt_qwen.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/blaslt_qwen.txt
