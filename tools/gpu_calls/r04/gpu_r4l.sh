#!/bin/bash
# round 4, call Q: Llama-3-8B batch-1 GEMV re-tune (r04 candidates), then Llama-3-8B batch-1 decode with the
# current table vs the re-tuned M=1 entries
source tools/gpu_steps.sh
step tune8b1 400 python3 -u tools/tune_gemv.py --model llama-3-8b --ms 1 --out gpurun_out/tune8b1.json --log gpurun_out/tune8b1.log
python3 - > gpurun_out/tune8b1_extra.json <<'PY'
import json
t = json.load(open("gpurun_out/tune8b1.json"))
print(json.dumps({k: v for k, v in t.items() if not k.startswith("d:") and k.endswith(":1") and (":4096" in k or "4096:" in k)}))
PY
cat gpurun_out/tune8b1_extra.json
step l8_b1_base 300 python3 -u bench.py --no-rtt --serve-load 0 --tp-leg 0 --model llama-3-8b --ftype Q4_K_M --concurrency 1 --steps 100 --warmup 10
step l8_b1_tuned 300 env NLS_TUNING_EXTRA="$(cat gpurun_out/tune8b1_extra.json)" python3 -u bench.py --no-rtt --serve-load 0 --tp-leg 0 --model llama-3-8b --ftype Q4_K_M --concurrency 1 --steps 100 --warmup 10
step l8_b1_base2 300 python3 -u bench.py --no-rtt --serve-load 0 --tp-leg 0 --model llama-3-8b --ftype Q4_K_M --concurrency 1 --steps 100 --warmup 10
grep -h '^{' gpurun_out/l8_b1_base.log gpurun_out/l8_b1_tuned.log gpurun_out/l8_b1_base2.log | cut -c150-240
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
