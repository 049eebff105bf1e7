#!/bin/bash
# launch cost + Infinity-Cache-resident GEMV chains
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag/launch_cost.py > gpurun_out/launch_cost_mall.txt 2>&1
