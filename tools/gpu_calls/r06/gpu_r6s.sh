#!/bin/bash
# round 6, call S: Granite-3.0-2B with its first tuned entries (quantised M buckets 1-512, dense M = 256 / 512): the LM
# head's dense entry (the r6r run stopped there), then the B=512 / B=1 steps and the kernel breakdown.
source tools/gpu_steps.sh
cp nats_llm_studio_amd/ops/gemv_tuning.json gpurun_out/tune_r6s.json
step r6s_tune_lm 600 python3 -u tools/tune_gemv.py --model granite-3.0-2b --dense --ms 256,512 --only lm_head --out gpurun_out/tune_r6s.json --log gpurun_out/tune_r6s_d.log
B="python3 -u bench.py --model granite-3.0-2b --steps 20 --warmup 3 --no-rtt --serve-load 0"
step r6s_granite_b512 300 $B
step r6s_granite_b1 300 $B --concurrency 1
BS=512 MODEL=granite-3.0-2b step r6s_prof 500 bash tools/gpu_prof.sh
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
