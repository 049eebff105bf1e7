#!/bin/bash
# small-batch (M 2..64) re-tune after the Q4_K fp8-conversion dequant, A/B of the changed entries at batch 16 / 64
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
cp nats_llm_studio_amd/ops/gemv_tuning.json gpurun_out/tune_ms.json &&
timeout -k 10 600 python -u tools/tune_gemv.py --ms 2,4,8,16,32,48,64 --out gpurun_out/tune_ms.json --log gpurun_out/tune_ms.log > gpurun_out/tune_ms.out 2>&1 &&
EXTRA=$(python - <<'PY'
import json
a = json.load(open("nats_llm_studio_amd/ops/gemv_tuning.json"))
b = json.load(open("gpurun_out/tune_ms.json"))
print(json.dumps({k: v for k, v in b.items() if a.get(k) != v}))
PY
) &&
echo "$EXTRA" > gpurun_out/tune_ms_changed.json &&
for B in 16 64; do
  timeout -k 10 300 python -u bench.py --concurrency $B --steps 50 --warmup 5 --no-rtt --serve-load 0 > gpurun_out/r5bc_b${B}_base.json 2> gpurun_out/r5bc_b${B}_base.log &&
  NLS_TUNING_EXTRA="$EXTRA" timeout -k 10 300 python -u bench.py --concurrency $B --steps 50 --warmup 5 --no-rtt --serve-load 0 > gpurun_out/r5bc_b${B}_tuned.json 2> gpurun_out/r5bc_b${B}_tuned.log &&
  timeout -k 10 300 python -u bench.py --concurrency $B --steps 50 --warmup 5 --no-rtt --serve-load 0 > gpurun_out/r5bc_b${B}_base2.json 2> gpurun_out/r5bc_b${B}_base2.log &&
  NLS_TUNING_EXTRA="$EXTRA" timeout -k 10 300 python -u bench.py --concurrency $B --steps 50 --warmup 5 --no-rtt --serve-load 0 > gpurun_out/r5bc_b${B}_tuned2.json 2> gpurun_out/r5bc_b${B}_tuned2.log || exit 1
done
