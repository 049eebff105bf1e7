#!/bin/bash
# batch-1 re-tune of Qwen2.5-7B and Llama-3-70B shapes after the Q4_K fp8-conversion dequant; Qwen A/B bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
cp nats_llm_studio_amd/ops/gemv_tuning.json gpurun_out/tune_fam.json &&
timeout -k 10 400 python -u tools/tune_gemv.py --model qwen2.5-7b --ms 1 --out gpurun_out/tune_fam.json --log gpurun_out/tune_qwen.log > gpurun_out/tune_qwen.out 2>&1 &&
timeout -k 10 500 python -u tools/tune_gemv.py --model llama-3-70b --ms 1 --out gpurun_out/tune_fam.json --log gpurun_out/tune_70b.log > gpurun_out/tune_70b.out 2>&1 &&
EXTRA=$(python - <<'PY'
import json
a = json.load(open("nats_llm_studio_amd/ops/gemv_tuning.json"))
b = json.load(open("gpurun_out/tune_fam.json"))
print(json.dumps({k: v for k, v in b.items() if a.get(k) != v}))
PY
) &&
echo "$EXTRA" > gpurun_out/tune_fam_changed.json &&
timeout -k 10 400 python -u bench.py --model qwen2.5-7b --concurrency 1 --steps 100 --warmup 5 --no-rtt --serve-load 0 > gpurun_out/r5be_q_base.json 2> gpurun_out/r5be_q_base.log &&
NLS_TUNING_EXTRA="$EXTRA" timeout -k 10 300 python -u bench.py --model qwen2.5-7b --concurrency 1 --steps 100 --warmup 5 --no-rtt --serve-load 0 > gpurun_out/r5be_q_tuned.json 2> gpurun_out/r5be_q_tuned.log &&
timeout -k 10 300 python -u bench.py --model qwen2.5-7b --concurrency 1 --steps 100 --warmup 5 --no-rtt --serve-load 0 > gpurun_out/r5be_q_base2.json 2> gpurun_out/r5be_q_base2.log &&
NLS_TUNING_EXTRA="$EXTRA" timeout -k 10 300 python -u bench.py --model qwen2.5-7b --concurrency 1 --steps 100 --warmup 5 --no-rtt --serve-load 0 > gpurun_out/r5be_q_tuned2.json 2> gpurun_out/r5be_q_tuned2.log
