#!/bin/bash
# batch-1 re-tune after the Q4_K fp8-conversion dequant (A/B of the changed M=1 entries in one box), and the 8B
# B=512 bench without the f16 weight copies (quantised GEMMs, which the conversion also speeds up)
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
cp nats_llm_studio_amd/ops/gemv_tuning.json gpurun_out/tune_m1.json &&
timeout -k 10 500 python -u tools/tune_gemv.py --ms 1 --out gpurun_out/tune_m1.json --log gpurun_out/tune_m1.log > gpurun_out/tune_m1.out 2>&1 &&
EXTRA=$(python - <<'PY'
import json
a = json.load(open("nats_llm_studio_amd/ops/gemv_tuning.json"))
b = json.load(open("gpurun_out/tune_m1.json"))
print(json.dumps({k: v for k, v in b.items() if k.endswith(":1") and a.get(k) != v}))
PY
) &&
echo "$EXTRA" > gpurun_out/tune_m1_changed.json &&
timeout -k 10 300 python -u bench.py --concurrency 1 --steps 100 --warmup 5 --no-rtt --serve-load 0 > gpurun_out/r5ba_b1_base.json 2> gpurun_out/r5ba_b1_base.log &&
NLS_TUNING_EXTRA="$EXTRA" timeout -k 10 300 python -u bench.py --concurrency 1 --steps 100 --warmup 5 --no-rtt --serve-load 0 > gpurun_out/r5ba_b1_tuned.json 2> gpurun_out/r5ba_b1_tuned.log &&
timeout -k 10 300 python -u bench.py --concurrency 1 --steps 100 --warmup 5 --no-rtt --serve-load 0 > gpurun_out/r5ba_b1_base2.json 2> gpurun_out/r5ba_b1_base2.log &&
NLS_TUNING_EXTRA="$EXTRA" timeout -k 10 300 python -u bench.py --concurrency 1 --steps 100 --warmup 5 --no-rtt --serve-load 0 > gpurun_out/r5ba_b1_tuned2.json 2> gpurun_out/r5ba_b1_tuned2.log &&
NLS_DENSE_WEIGHTS=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-rtt --serve-load 0 > gpurun_out/r5ba_nocopies.json 2> gpurun_out/r5ba_nocopies.log
