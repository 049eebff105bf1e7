#!/bin/bash
# kernel tests -> re-tune large-M configs (mode 3 candidates) -> bench at B=256 / 384 / 512
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
scripts/gpu_tune.sh 128,256,384,512 || exit $?
for B in 384 512; do
  timeout -k 10 300 python -u bench.py --no-rtt --concurrency $B > gpurun_out/bench_b$B.log 2>&1 || { echo "bench B=$B rc=$?"; tail -5 gpurun_out/bench_b$B.log; exit 1; }
  tail -1 gpurun_out/bench_b$B.log
done
