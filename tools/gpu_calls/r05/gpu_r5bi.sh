#!/bin/bash
# batch-1 XL weight-stream depth after the fp8-conversion dequant: default (2) vs -DNLS_XL_DEPTH=4 (variant build)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
V=$PWD/nats_llm_studio_amd/_kernels__xl4.so
timeout -k 10 300 python -u tools/gemm_ab.py --libs nats_llm_studio_amd/_kernels.so,$V --M 1 --shapes gateup,lm_head > gpurun_out/r5bi_ab.txt 2>&1 &&
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --concurrency 1 --steps 100 --warmup 5 --no-rtt --serve-load 0 > gpurun_out/r5bi_base$i.json 2> gpurun_out/r5bi_base$i.log &&
  NLS_KERNELS_SO=$V timeout -k 10 300 python -u bench.py --concurrency 1 --steps 100 --warmup 5 --no-rtt --serve-load 0 > gpurun_out/r5bi_xl4_$i.json 2> gpurun_out/r5bi_xl4_$i.log || exit 1
done
