#!/bin/bash
# round 4, call R: chat_model service load (512 concurrent, half sampled, 256 tokens) with 1 / 2 / 4 prefill
# chunks per engine step while a prompt backlog is queued
source tools/gpu_steps.sh
for k in 1 2 4; do
  step sl_k$k 300 env NLS_PREFILL_CHUNKS=$k python3 -u bench.py --steps 20 --warmup 5 --tp-leg 0
  grep -h '^{' gpurun_out/sl_k$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); s=d['service_load']; print('k=$k', d['ms_per_step'], s['tok_s'], s['ttft_p50_ms'], s['wall_s'])"
done
exit $STEPS_RC
