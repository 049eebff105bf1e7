#!/bin/bash
# Full validation pass on a GPU box: gpu tests, smoke, headline bench (B=256), B=1 bench, rocprof B=256.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONPATH=$PWD
tools/gpu_check.sh all || exit $?
timeout -k 10 300 python -u bench.py --concurrency 1 --steps 64 --warmup 8 --no-rtt > gpurun_out/bench_b1.log 2>&1 || exit $?
tail -1 gpurun_out/bench_b1.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b256 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-rtt > gpurun_out/prof_b256.log 2>&1 || exit $?
python tools/analyze_trace.py $(find gpurun_out/prof_b256 -name "*kernel_trace.csv" | head -1) > gpurun_out/prof_b256_breakdown.txt
cat gpurun_out/prof_b256_breakdown.txt
