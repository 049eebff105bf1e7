#!/bin/bash
# round 4, call B: TP=2 rehearsal kernel profile (in-process), rocprof of one 32K prefill, prefill chunk A/B,
# KV-pressure to completion, headline bench
source tools/gpu_steps.sh
step tp_prof 300 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --no-ref --profile-steps 8
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step pf_prof 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pf_prof -o run -- python3 tools/prefill_probe.py --lens 32768 --reps 1
python3 tools/prefill_probe.py --analyze "$(find gpurun_out/pf_prof -name '*kernel_trace.csv' | head -1)" --lens 32768 > gpurun_out/pf_breakdown.txt 2>&1; cat gpurun_out/pf_breakdown.txt
rm -rf gpurun_out/pf_prof
step pf_chunk4k 300 python3 -u tools/prefill_probe.py --lens 8192 32768 --reps 1 --chunk 4096
step kv_pressure 360 python3 -u tools/kv_pressure.py --n 512 --max-tokens 1024 --kv-fraction 0.03 --seconds 300
step bench 600 python3 -u bench.py --steps 20 --warmup 5
exit $STEPS_RC
