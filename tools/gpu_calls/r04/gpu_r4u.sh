#!/bin/bash
# r04: EP all-to-all rehearsal on the GPU (2 ranks on cuda:0), the rest of the rehearsal file, the dense GEMM tests
mkdir -p gpurun_out
step() { local n=$1; shift; local t0=$(date +%s); "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "[step] $n rc=$rc $(( $(date +%s) - t0 ))s"; tail -4 gpurun_out/$n.log; return $rc; }
step rehearsal timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tp_rehearsal_gpu.py &&
step dense timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "hgemm_dense"
