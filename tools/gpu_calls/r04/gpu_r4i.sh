#!/bin/bash
# round 4, call I: where a sampled B=512 decode step spends its time (half / all rows with the reference
# payload's temperature 0.7, top_p 0.95, top_k 40), next to the greedy step
source tools/gpu_steps.sh
step bs50 300 python3 -u bench.py --steps 20 --warmup 5 --serve-load 0 --no-rtt --tp-leg 0 --sample-frac 0.5
step bs100 300 python3 -u bench.py --steps 20 --warmup 5 --serve-load 0 --no-rtt --tp-leg 0 --sample-frac 1.0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step prof_s50 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s50 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-rtt --serve-load 0 --tp-leg 0 --sample-frac 0.5
python3 tools/analyze_trace.py $(find gpurun_out/prof_s50 -name "*kernel_trace.csv" | head -1) > gpurun_out/prof_s50_breakdown.txt
head -24 gpurun_out/prof_s50_breakdown.txt
exit $STEPS_RC
