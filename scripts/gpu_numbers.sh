#!/bin/bash
# Round numbers: B=1 kernel breakdown, context sweep on Llama-3-8B, then the other north-star families
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b1 -o run -- python3 -u bench.py --concurrency 1 --steps 40 --warmup 5 --no-rtt --serve-load 0 > gpurun_out/prof_b1.log 2>&1 || { tail -5 gpurun_out/prof_b1.log; exit 1; }
python tools/analyze_trace.py gpurun_out/prof_b1/run_results.db > gpurun_out/b1_breakdown.txt 2>&1; head -16 gpurun_out/b1_breakdown.txt
bash scripts/gpu_ctx_sweep.sh || exit $?
RUNS=${RUNS:-"mixtral_b1 mixtral_b256 l70b_b1 l70b_b128 qwen7b_b512"} bash tools/gpu_models.sh
