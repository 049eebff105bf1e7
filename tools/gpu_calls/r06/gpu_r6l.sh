#!/bin/bash
# round 6, call L: where the engine chat_model RTT goes -- the 21-token prefill forward (2.28 of 2.62 ms in BENCH_r05)
# per kernel under rocprofv3, next to the batch-1 decode step.
source tools/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step r6l_pf21 300 python3 -u tools/diag/prefill_small.py --tokens 21 --reps 20
step r6l_prof_pf21 300 rocprofv3 --kernel-trace -d gpurun_out/prof_pf21 -o run --output-format csv -- python3 tools/diag/prefill_small.py --tokens 21 --reps 20
python3 tools/diag/trace_totals.py $(find gpurun_out/prof_pf21 -name "*kernel_trace.csv" | head -1) 20 > gpurun_out/prof_pf21_totals.txt; cat gpurun_out/prof_pf21_totals.txt
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
