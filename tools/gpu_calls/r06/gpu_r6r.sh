#!/bin/bash
# round 6, call R: Granite-3.0-2B at B=512 takes 12.84 ms/step, more than Llama-3-8B (11.1): its kernel breakdown, then
# the dense and quantised tuners on its shapes (no table entries yet: the heuristics ran).
source tools/gpu_steps.sh
BS=512 MODEL=granite-3.0-2b step r6r_prof 500 bash tools/gpu_prof.sh
cp nats_llm_studio_amd/ops/gemv_tuning.json gpurun_out/tune_r6r.json
step r6r_tune_q 900 python3 -u tools/tune_gemv.py --model granite-3.0-2b --ms 1,8,16,32,64,256,512 --out gpurun_out/tune_r6r.json --log gpurun_out/tune_r6r_q.log
step r6r_tune_d 900 python3 -u tools/tune_gemv.py --model granite-3.0-2b --dense --ms 256,512 --out gpurun_out/tune_r6r.json --log gpurun_out/tune_r6r_d.log
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
