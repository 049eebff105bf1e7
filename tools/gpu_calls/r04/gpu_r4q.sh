#!/bin/bash
# round 4, call Q: Qwen2.5-7B batch-1 GEMV re-tune (r04 candidates), then Qwen2.5-7B batch-1 decode with the
# current table vs the re-tuned M=1 entries
source tools/gpu_steps.sh
step tuneqw 400 python3 -u tools/tune_gemv.py --model qwen2.5-7b --ms 1 --out gpurun_out/tuneqw.json --log gpurun_out/tuneqw.log
python3 - > gpurun_out/tuneqw_extra.json <<'PY'
import json
t = json.load(open("gpurun_out/tuneqw.json"))
print(json.dumps({k: v for k, v in t.items() if not k.startswith("d:") and k.endswith(":1") and (":3584" in k or "3584:" in k)}))
PY
cat gpurun_out/tuneqw_extra.json
step qw_b1_base 300 python3 -u bench.py --no-rtt --serve-load 0 --tp-leg 0 --model qwen2.5-7b --ftype Q4_K_M --concurrency 1 --steps 60 --warmup 5
step qw_b1_tuned 300 env NLS_TUNING_EXTRA="$(cat gpurun_out/tuneqw_extra.json)" python3 -u bench.py --no-rtt --serve-load 0 --tp-leg 0 --model qwen2.5-7b --ftype Q4_K_M --concurrency 1 --steps 60 --warmup 5
step qw_b1_base2 300 python3 -u bench.py --no-rtt --serve-load 0 --tp-leg 0 --model qwen2.5-7b --ftype Q4_K_M --concurrency 1 --steps 60 --warmup 5
grep -h '^{' gpurun_out/qw_b1_base.log gpurun_out/qw_b1_tuned.log gpurun_out/qw_b1_base2.log | cut -c150-240
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
