#!/usr/bin/env bash
# Full GPU validation (tests, smoke, default bench) + a rocprofv3 kernel breakdown of the B=512 decode step.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
scripts/gpu_check.sh all || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$OLDPWD"
rm -rf gpurun_out/prof_b512
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b512 -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 3 --no-rtt --serve-load 0 > gpurun_out/prof_b512.log 2>&1 || exit $?
python3 tools/analyze_trace.py $(find gpurun_out/prof_b512 -name "*kernel_trace.csv" | head -1) \
    > gpurun_out/prof_b512_breakdown.txt
head -25 gpurun_out/prof_b512_breakdown.txt
