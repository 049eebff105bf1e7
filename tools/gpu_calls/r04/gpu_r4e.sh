#!/bin/bash
# round 4, call E: greedy-only TP rehearsal (vocab-parallel arg-max on every step) with the control-op
# trace and one-shot state dump, the mixed rehearsal's profile window again, then the B=512 decode bench
# (the driver's 20-step form) and a rocprofv3 kernel trace of it with the r04 dense tuning
source tools/gpu_steps.sh
step tp_greedy 300 env NLS_TP_TRACE=1 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --greedy-only --profile-steps 8
step tp_mixed 300 env NLS_TP_TRACE=1 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --no-ref --profile-steps 8
step b512_20 300 python3 -u bench.py --steps 20 --warmup 5 --serve-load 0 --no-rtt --tp-leg 0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step prof_b512 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b512 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-rtt --serve-load 0 --tp-leg 0
python3 tools/analyze_trace.py $(find gpurun_out/prof_b512 -name "*kernel_trace.csv" | head -1) > gpurun_out/prof_b512_breakdown.txt
head -30 gpurun_out/prof_b512_breakdown.txt
exit $STEPS_RC
