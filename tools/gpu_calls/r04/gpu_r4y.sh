#!/bin/bash
# round 4, call Y: Llama-3-70B batch-1 GEMV re-tune (the 8B's r04 XL options among the candidates), then 70B
# batch-1 decode on one GPU with the current table vs the re-tuned M=1 entries
source tools/gpu_steps.sh
step tune70 500 python3 -u tools/tune_gemv.py --model llama-3-70b --ms 1 --out gpurun_out/tune70_y.json --log gpurun_out/tune70_y.log
python3 - > gpurun_out/tune70_y_extra.json <<'PY'
import json
t = json.load(open("gpurun_out/tune70_y.json"))
print(json.dumps({k: v for k, v in t.items() if not k.startswith("d:") and k.endswith(":1") and ":8192" in k}))
PY
cat gpurun_out/tune70_y_extra.json
step l70_b1_base 420 python3 -u bench.py --no-rtt --serve-load 0 --tp-leg 0 --model llama-3-70b --ftype Q4_K_M --concurrency 1 --steps 30 --warmup 3
step l70_b1_tuned 420 env NLS_TUNING_EXTRA="$(cat gpurun_out/tune70_y_extra.json)" python3 -u bench.py --no-rtt --serve-load 0 --tp-leg 0 --model llama-3-70b --ftype Q4_K_M --concurrency 1 --steps 30 --warmup 3
grep -h '^{' gpurun_out/l70_b1_base.log gpurun_out/l70_b1_tuned.log | cut -c1-220
rm -f /tmp/nls_bench/*.gguf
# Llama-3-8B B=512 sustained (100 steps, the package power limit engages): f16 weight copies vs quantised tiles
step s100_dense 300 python3 -u bench.py --steps 100 --warmup 5 --serve-load 0 --no-rtt --tp-leg 0
step s100_quant 300 env NLS_DENSE_WEIGHTS=0 python3 -u bench.py --steps 100 --warmup 5 --serve-load 0 --no-rtt --tp-leg 0
grep -h '^{' gpurun_out/s100_dense.log gpurun_out/s100_quant.log | cut -c150-260
exit $STEPS_RC
