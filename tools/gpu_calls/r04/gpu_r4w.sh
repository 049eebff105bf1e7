#!/bin/bash
# round 4, call W: long-prompt TTFT at the head (re-tuned dense table) and a fresh 32K kernel breakdown
source tools/gpu_steps.sh
step pf_head 300 python3 -u tools/prefill_probe.py --lens 8192 32768 --reps 2
grep -h '^{' gpurun_out/pf_head.log
step pf_prof 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pf_prof_w -o run -- python3 tools/prefill_probe.py --lens 32768 --reps 1
python3 tools/prefill_probe.py --analyze "$(find gpurun_out/pf_prof_w -name '*kernel_trace.csv' | head -1)" --lens 32768 > gpurun_out/pf_breakdown_w.txt 2>&1; head -12 gpurun_out/pf_breakdown_w.txt
rm -rf gpurun_out/pf_prof_w
exit $STEPS_RC
