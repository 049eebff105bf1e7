#!/bin/bash
# round 4, call M: the greedy TP rehearsal's second prefill (a) with eager calls on RCCL/gloo and the IPC
# one-shot kernels only inside captured graphs, (b) with the IPC receive buffers allocated fine-grained /
# plain / uncached (the default); consumed-granule re-tag on
source tools/gpu_steps.sh
step reh_noeager 150 env NLS_TP_TRACE=1 NLS_ONESHOT_EAGER=0 NLS_AR_RETAG=1 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --greedy-only --profile-steps 8
grep -h -o "timeout_addnorm': \[[0-9, -]*\]" gpurun_out/reh_noeager.log | head -2 || true
step reh_waves_noeager 150 env NLS_TP_TRACE=1 NLS_REHEARSAL_WAVES=1 NLS_ONESHOT_EAGER=0 NLS_AR_RETAG=1 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --greedy-only
grep -h -o "timeout_addnorm': \[[0-9, -]*\]" gpurun_out/reh_waves_noeager.log | head -2 || true
for k in fine coarse uncached; do
  step reh_${k} 150 env NLS_TP_TRACE=1 NLS_AR_ALLOC=$k NLS_AR_RETAG=1 python3 -u -m nats_llm_studio_amd.parallel.rehearsal --greedy-only --profile-steps 8
  grep -h -o "timeout_addnorm': \[[0-9, -]*\]" gpurun_out/reh_${k}.log | head -2 || true
done
step b1_w8 120 python3 -u bench.py --concurrency 1 --steps 100 --warmup 10 --serve-load 0 --no-rtt --tp-leg 0
step b1_w4 120 env NLS_ATTN_MFMA_WAVES=4 python3 -u bench.py --concurrency 1 --steps 100 --warmup 10 --serve-load 0 --no-rtt --tp-leg 0
grep -h '^{' gpurun_out/b1_w8.log gpurun_out/b1_w4.log | cut -c1-160
# quantised large-M (no f16 copies): mode 9 among the candidates, then B=512 without the copies, old vs new table
step tune_q 600 python3 -u tools/tune_gemv.py --model llama-3-8b --ms 256,512 --out gpurun_out/tune_q8b.json --log gpurun_out/tune_q8b.log
python3 - > gpurun_out/tune_q8b_extra.json <<'PY'
import json
t = json.load(open("gpurun_out/tune_q8b.json"))
print(json.dumps({k: v for k, v in t.items() if not k.startswith("d:") and k.split(":")[-1] in ("256", "512")}))
PY
step b512_q_old 300 env NLS_DENSE_WEIGHTS=0 python3 -u bench.py --steps 20 --warmup 5 --serve-load 0 --no-rtt --tp-leg 0
step b512_q_new 300 env NLS_DENSE_WEIGHTS=0 NLS_TUNING_EXTRA="$(cat gpurun_out/tune_q8b_extra.json)" python3 -u bench.py --steps 20 --warmup 5 --serve-load 0 --no-rtt --tp-leg 0
grep -h '^{' gpurun_out/b512_q_old.log gpurun_out/b512_q_new.log | cut -c1-200
exit $STEPS_RC
