#!/bin/bash
# round 5, call B: (1) the eager one-shot timeout with the PUSHER's view of the timed-out slot (through its IPC
# mapping) and the imported-range overlap check; (2) mode 11 (quantised mode-10 schedule) numerics; (3) mode 11
# vs mode 9 on the Llama-3-8B shapes at 256 / 512 rows; (4) B=512 without the f16 copies (heuristic configs).
source tools/gpu_steps.sh
R="python3 -u -m nats_llm_studio_amd.parallel.rehearsal --greedy-only --profile-steps 4 --no-ref"
step r5b_base 200 env NLS_TP_TRACE=1 NLS_REHEARSAL_WAVES=1 NLS_ONESHOT_EAGER=1 $R
grep -h -o "'addnorm_timeout_detail': {[^}]*}[^}]*}\|'pusher_view_of_rank0': {[^}]*}[^}]*}\|'imported_overlaps': \[[^]]*\]\|'imported_ptrs': \[[^]]*\]\|'own_ptrs': \[[^]]*\]" gpurun_out/r5b_base.log | head -12 || true
step r5b_m11 300 python3 -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k "qgemm11 or quant11"
step r5b_tune 500 python3 -u tools/tune_gemv.py --model llama-3-8b --ms 256,512 --modes 9,11 --out gpurun_out/tune11.json --log gpurun_out/tune11.log
step r5b_b512q 300 env NLS_DENSE_WEIGHTS=0 NLS_TUNING_EXTRA="$(python3 -c "import json;t=json.load(open('gpurun_out/tune11.json'));print(json.dumps({k:v for k,v in t.items() if k.split(':')[-1] in ('256','512')}))")" python3 -u bench.py --steps 20 --warmup 5 --serve-load 0 --no-rtt --tp-leg 0
grep -h '^{' gpurun_out/r5b_b512q.log | cut -c1-300
exit $STEPS_RC
