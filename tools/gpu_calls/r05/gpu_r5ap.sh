#!/bin/bash
# round 5, call AP: tuning-table entry tests (incl. the 70B entries); the 8B quantised shapes re-tuned over modes 2 / 9.
source tools/gpu_steps.sh
step r5ap_tests 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_production_gpu.py -k "tuning_table_entries"
step r5ap_tune 900 python3 -u tools/tune_gemv.py --model llama-3-8b --ms 256,512,1024,2048 --modes 2,9 --out gpurun_out/gemv_tuning_8b.json --log gpurun_out/tune8.log
exit $STEPS_RC
