#!/bin/bash
# round 6, call R: Granite-3.0-2B (head dim 64) at B=512 took 12.84 ms/step, more than Llama-3-8B: the decode attention
# for D = 64 ran on the VALU kernel. Now the MFMA decode kernel covers D = 64: its tests, the Granite step with it vs
# the VALU kernel (NLS_ATTN_MFMA=0), the kernel breakdown, then the quantised and dense tuners on Granite's shapes.
source tools/gpu_steps.sh
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
step r6r_attn_tests 300 $T tests/test_kernels_gpu.py -k "attention"
[ $STEPS_RC -ne 0 ] && exit $STEPS_RC
B="python3 -u bench.py --model granite-3.0-2b --steps 20 --warmup 3 --no-rtt --serve-load 0"
step r6r_granite_mfma 300 $B
NLS_ATTN_MFMA=0 step r6r_granite_valu 300 $B
step r6r_granite_mfma2 300 $B
BS=512 MODEL=granite-3.0-2b step r6r_prof 500 bash tools/gpu_prof.sh
cp nats_llm_studio_amd/ops/gemv_tuning.json gpurun_out/tune_r6r.json
step r6r_tune_q 900 python3 -u tools/tune_gemv.py --model granite-3.0-2b --ms 1,8,16,32,64,256,512 --out gpurun_out/tune_r6r.json --log gpurun_out/tune_r6r_q.log
step r6r_tune_d 900 python3 -u tools/tune_gemv.py --model granite-3.0-2b --dense --ms 256,512 --out gpurun_out/tune_r6r.json --log gpurun_out/tune_r6r_d.log
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
