#!/bin/bash
# PMC passes for one GEMM shape: scripts/gpu_pmc_gemm.sh + a summary
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
scripts/gpu_pmc_gemm.sh ${1:-gateup} ${2:-256} || exit $?
python tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.txt 2>&1; cat gpurun_out/pmc/summary.txt
