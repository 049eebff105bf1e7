#!/bin/bash
# mode-3 PMC + the new GPU tests
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "dma or rope" --timeout 120 --timeout-method thread > gpurun_out/t2.log 2>&1 || { tail -20 gpurun_out/t2.log; exit 1; }
tail -2 gpurun_out/t2.log
CFG=3,4,8,1 tools/gpu_pmc.sh gateup 256
