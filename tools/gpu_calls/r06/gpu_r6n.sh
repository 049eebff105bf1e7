#!/bin/bash
# round 6, call N: non-mapped mode-3 tests at the new 64 / 96-row blocks, then the quantised large-M tuner with them
# (modes 2 / 3 / 9 only) on the Llama-3-8B shapes at M = 256 / 512 and the Llama-3-70B shapes at M = 128 -- written to a
# scratch table, compared against the current entries by hand.
source tools/gpu_steps.sh
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
step r6n_dma_tests 300 $T tests/test_kernels_gpu.py -k "qgemm_dma"
[ $STEPS_RC -ne 0 ] && exit $STEPS_RC
cp nats_llm_studio_amd/ops/gemv_tuning.json gpurun_out/tune_r6n.json
step r6n_tune8b 900 python3 -u tools/tune_gemv.py --model llama-3-8b --ms 256,512 --modes 2,3,9 --out gpurun_out/tune_r6n.json --log gpurun_out/tune_r6n_8b.log
step r6n_tune70b 900 python3 -u tools/tune_gemv.py --model llama-3-70b --ms 128 --modes 2,3,9 --out gpurun_out/tune_r6n.json --log gpurun_out/tune_r6n_70b.log
exit $STEPS_RC
