#!/usr/bin/env bash
# Final validation of the round: full GPU suite, smoke, default bench, batch-1 bench, rocprof B=512 breakdown.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_check.sh all || exit $?
timeout -k 10 300 python -u bench.py --concurrency 1 --steps 200 --warmup 10 --no-rtt --serve-load 0 \
    > gpurun_out/bench_b1.log 2>&1 || exit $?
tail -1 gpurun_out/bench_b1.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp && cd "$OLDPWD"
rm -rf gpurun_out/prof_b512
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b512 -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 3 --no-rtt --serve-load 0 > gpurun_out/prof_b512.log 2>&1 || exit $?
python3 tools/analyze_trace.py $(find gpurun_out/prof_b512 -name "*kernel_trace.csv" | head -1) \
    > gpurun_out/prof_b512_breakdown.txt
head -16 gpurun_out/prof_b512_breakdown.txt
