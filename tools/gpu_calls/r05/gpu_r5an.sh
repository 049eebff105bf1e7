#!/bin/bash
# round 5, call AN: quantised large-M GEMM winners (modes 2 / 9) for the Llama-3-70B shapes, now that auto runs the
# single-GPU 70B without f16 copies.
source tools/gpu_steps.sh
step r5an_tune 900 python3 -u tools/tune_gemv.py --model llama-3-70b --ms 256,512,1024,2048 --modes 2,9 --out gpurun_out/gemv_tuning_70b.json --log gpurun_out/tune70.log
exit $STEPS_RC
