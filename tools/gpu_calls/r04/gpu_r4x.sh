#!/bin/bash
# round 4, call X: pinned non_blocking upload semantics, the double-buffered prefill staging (engine GPU tests),
# long-prompt TTFT after the change
source tools/gpu_steps.sh
step race 120 python3 -u tools/pinned_race_probe.py
step model_tests 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_model_gpu.py tests/test_production_gpu.py
step pf_x 300 python3 -u tools/prefill_probe.py --lens 8192 32768 --reps 2
grep -h '^{\|^\[' gpurun_out/race.log gpurun_out/pf_x.log
exit $STEPS_RC
