#!/bin/bash
# PMC of the gate/up GEMM at M=512: quantised LDS GEMM (mode 2) vs dense f16 GEMM (mode 4)
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD TMPDIR=/tmp
for arm in "m2 2,8,4,1 " "m4 4,8,4,1 1"; do
  set -- $arm
  rm -rf gpurun_out/pmc
  CFG=$2 DENSE=${3:-} bash tools/gpu_pmc.sh ${SHAPE:-gateup} 512 > gpurun_out/pmc_$1.txt 2>&1 || { tail -20 gpurun_out/pmc_$1.txt; exit 1; }
  mv gpurun_out/pmc gpurun_out/pmc_$1
done
