#!/bin/bash
# round 6, call Q: the dense f16 GEMM at 64-row activation blocks (modes 4 / 6, waves 4, rt 1: 2-3 workgroups per CU):
# its kernel tests, then the dense tuner on the Llama-3-8B shapes at M = 256 / 512 with the current entries (mode 10 /
# mode 4) timed alongside, into a scratch table.
source tools/gpu_steps.sh
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
step r6q_dense_tests 300 $T tests/test_kernels_gpu.py -k "hgemm_dense"
[ $STEPS_RC -ne 0 ] && exit $STEPS_RC
cp nats_llm_studio_amd/ops/gemv_tuning.json gpurun_out/tune_r6q.json
step r6q_tune_dense 900 python3 -u tools/tune_gemv.py --model llama-3-8b --dense --ms 256,512 --modes 4,6 --out gpurun_out/tune_r6q.json --log gpurun_out/tune_r6q_dense.log
exit $STEPS_RC
