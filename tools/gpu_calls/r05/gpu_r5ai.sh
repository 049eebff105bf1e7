#!/bin/bash
# round 5, call AI: kernel breakdown of an 8K-token prefill (2048-token chunks) -- the service burst's prefill rate.
source tools/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_pf8k
step r5ai_prof 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_pf8k -o run -- python3 -u tools/prefill_probe.py --lens 8192 --reps 3
f=$(find gpurun_out/prof_pf8k -name "*kernel_trace.csv" | head -1)
python3 tools/prefill_probe.py --analyze "$f" --lens 8192 > gpurun_out/prof_pf8k_breakdown.txt 2>&1
cat gpurun_out/prof_pf8k_breakdown.txt
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
