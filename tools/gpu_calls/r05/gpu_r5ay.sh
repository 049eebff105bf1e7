#!/bin/bash
# Q4_K nibble dequant via the scaled fp8 conversion (variant build _kernels__q4fp8.so, -DNLS_Q4_FP8CVT=1):
# kernel tests on the variant, A/B vs the default (magic-number) build, batch-1 bench on both
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
V=$PWD/nats_llm_studio_amd/_kernels__q4fp8.so
NLS_KERNELS_SO=$V timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r5ay_kernels.txt 2>&1 &&
L=nats_llm_studio_amd/_kernels.so,$V &&
timeout -k 10 300 python -u tools/gemm_ab.py --libs $L --M 1 --shapes qkv,o,gateup,down > gpurun_out/r5ay_ab.txt 2>&1 &&
timeout -k 10 300 python -u tools/gemm_ab.py --libs $L --M 16 --shapes qkv,gateup >> gpurun_out/r5ay_ab.txt 2>&1 &&
timeout -k 10 300 python -u tools/gemm_ab.py --libs $L --M 512 --shapes qkv,o,gateup >> gpurun_out/r5ay_ab.txt 2>&1 &&
timeout -k 10 400 python -u bench.py --concurrency 1 --steps 100 --warmup 5 --no-rtt --serve-load 0 > gpurun_out/r5ay_b1_base.json 2> gpurun_out/r5ay_b1_base.log &&
NLS_KERNELS_SO=$V timeout -k 10 400 python -u bench.py --concurrency 1 --steps 100 --warmup 5 --no-rtt --serve-load 0 > gpurun_out/r5ay_b1_fp8.json 2> gpurun_out/r5ay_b1_fp8.log
