#!/bin/bash
# round 6, call V: batch-1 re-tune of Llama-3-70B (one GPU; its M=1..8 entries predate the Q4_K fp8-conversion dequant
# except gate|up) and Qwen2.5-7B, each benched with the current table and with the fresh entries (NLS_TUNING_EXTRA).
source tools/gpu_steps.sh
cp nats_llm_studio_amd/ops/gemv_tuning.json gpurun_out/tune_r6v.json
step r6v_tune70 900 python3 -u tools/tune_gemv.py --model llama-3-70b --ms 1,2,4,8 --out gpurun_out/tune_r6v.json --log gpurun_out/tune_r6v_70b.log
B="python3 -u bench.py --steps 20 --warmup 3 --no-rtt --serve-load 0 --concurrency 1"
step r6v_70b_cur 400 $B --model llama-3-70b
NLS_TUNING_EXTRA="$(python3 tools/diag/tuning_diff.py gpurun_out/tune_r6v.json)" step r6v_70b_new 300 $B --model llama-3-70b
step r6v_70b_cur2 300 $B --model llama-3-70b
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
