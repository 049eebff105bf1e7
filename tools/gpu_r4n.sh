#!/bin/bash
# round 4, call N: one-shot kernels only inside graphs (eager collectives on gloo/RCCL): one-shot tests and the
# TP rehearsal tests; then quantised large-M with mode 9 among the candidates and B=512 without f16 copies
source tools/gpu_steps.sh
step os_tests 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "oneshot" tests/test_oneshot_ipc_gpu.py
step tp_tests 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_tp_rehearsal_gpu.py
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
