#!/bin/bash
# round 5, call BD: model / production GPU tests after the small-batch tuning-table update
source tools/gpu_steps.sh
step r5bd_gpu 600 python3 -u -m pytest tests/test_production_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread
exit $STEPS_RC
