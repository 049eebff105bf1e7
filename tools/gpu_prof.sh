#!/bin/bash
# rocprofv3 kernel traces of the bench at B=512 and B=1 + per-step breakdowns
# BS="256" MODEL=mixtral-8x7b FTYPE=Q5_K_M selects other batches / models
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for B in ${BS:-512 1}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b$B -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-rtt --concurrency $B ${MODEL:+--model $MODEL} ${FTYPE:+--ftype $FTYPE} > gpurun_out/prof_b$B.log 2>&1 || { echo "prof B=$B failed"; tail -5 gpurun_out/prof_b$B.log; exit 1; }
  python tools/analyze_trace.py $(find gpurun_out/prof_b$B -name "*kernel_trace.csv" | head -1) > gpurun_out/prof_b${B}_breakdown.txt
  cat gpurun_out/prof_b${B}_breakdown.txt
done
