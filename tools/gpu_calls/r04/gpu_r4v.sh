#!/bin/bash
# round 4, call V: quantised large-M tune with the 4-wave mode-9 tile among the candidates, then B=512 without
# the f16 copies on the current table vs the re-tuned one
source tools/gpu_steps.sh
# decode attention: split 0's first block-table window fetched with ctx_len / tok_seq at one-token launches
step attn_tests 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn"
step b1_a 150 python3 -u bench.py --concurrency 1 --steps 100 --warmup 10 --serve-load 0 --no-rtt --tp-leg 0
step b1_b 150 python3 -u bench.py --concurrency 1 --steps 100 --warmup 10 --serve-load 0 --no-rtt --tp-leg 0
grep -h '^{' gpurun_out/b1_a.log gpurun_out/b1_b.log | cut -c1-200
step tune_q 700 python3 -u tools/tune_gemv.py --model llama-3-8b --ms 256,512 --out gpurun_out/tune_q8b_v.json --log gpurun_out/tune_q8b_v.log
python3 - > gpurun_out/tune_q8b_v_extra.json <<'PY'
import json
t = json.load(open("gpurun_out/tune_q8b_v.json"))
print(json.dumps({k: v for k, v in t.items() if not k.startswith("d:") and k.split(":")[-1] in ("256", "512")}))
PY
cat gpurun_out/tune_q8b_v_extra.json
step b512_q_old 300 env NLS_DENSE_WEIGHTS=0 python3 -u bench.py --steps 20 --warmup 5 --serve-load 0 --no-rtt --tp-leg 0
step b512_q_new 300 env NLS_DENSE_WEIGHTS=0 NLS_TUNING_EXTRA="$(cat gpurun_out/tune_q8b_v_extra.json)" python3 -u bench.py --steps 20 --warmup 5 --serve-load 0 --no-rtt --tp-leg 0
grep -h '^{' gpurun_out/b512_q_old.log gpurun_out/b512_q_new.log | cut -c1-200
exit $STEPS_RC
