#!/bin/bash
# Mixtral-8x7B batch-1 decode kernel breakdown
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mix1 -o run -- python3 -u bench.py --model mixtral-8x7b --ftype Q5_K_M --concurrency 1 --steps 30 --warmup 5 --no-rtt --serve-load 0 > gpurun_out/prof_mix1.log 2>&1 || { tail -5 gpurun_out/prof_mix1.log; exit 1; }
python tools/analyze_trace.py gpurun_out/prof_mix1/run_results.db > gpurun_out/mix1_breakdown.txt 2>&1; head -24 gpurun_out/mix1_breakdown.txt
rm -f /tmp/nls_bench/*.gguf
