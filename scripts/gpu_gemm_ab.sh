#!/bin/bash
# GEMM variant A/B: kernel tests of each variant lib (LDS GEMM paths), then tools/gemm_ab.py interleaved
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
K=nats_llm_studio_amd
LIBS=${LIBS:-$K/_kernels.so,$K/_kernels_prio.so,$K/_kernels_m32.so,$K/_kernels_m32p.so}
for L in ${LIBS//,/ }; do
  NLS_KERNELS_SO=$PWD/$L timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -k "qgemm_lds or lm_head or add_rmsnorm or qkv_rope" > gpurun_out/ab_tests.log 2>&1 || { echo "tests failed for $L"; tail -20 gpurun_out/ab_tests.log; exit 1; }
  echo "$L: $(tail -1 gpurun_out/ab_tests.log)"
done
for M in ${MS:-512 256}; do
  timeout -k 10 600 python -u tools/gemm_ab.py --libs $LIBS --M $M --rounds 7 > gpurun_out/gemm_ab_$M.txt 2>&1 || { tail -5 gpurun_out/gemm_ab_$M.txt; exit 1; }
  cat gpurun_out/gemm_ab_$M.txt
done
