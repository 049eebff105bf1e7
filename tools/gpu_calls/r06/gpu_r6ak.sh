#!/bin/bash
# round 6, call AK: rocprofv3 kernel traces at batch 1 of Mixtral-8x7B and Llama-3-70B (one GPU) at the final head.
source tools/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PB="python3 bench.py --steps 20 --warmup 3 --no-rtt --serve-load 0 --concurrency 1"
step r6ak_prof_mx 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ak_mx -o run --output-format csv -- $PB --model mixtral-8x7b
python3 tools/analyze_trace.py $(find gpurun_out/prof_ak_mx -name "*kernel_trace.csv" | head -1) > gpurun_out/prof_ak_mx_breakdown.txt && cat gpurun_out/prof_ak_mx_breakdown.txt
rm -f /tmp/nls_bench/*.gguf
step r6ak_prof_70b 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ak_70b -o run --output-format csv -- $PB --model llama-3-70b
python3 tools/analyze_trace.py $(find gpurun_out/prof_ak_70b -name "*kernel_trace.csv" | head -1) > gpurun_out/prof_ak_70b_breakdown.txt && cat gpurun_out/prof_ak_70b_breakdown.txt
rm -rf gpurun_out/prof_ak_mx/*/ gpurun_out/prof_ak_70b/*/ 2>/dev/null
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
