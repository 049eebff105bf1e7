#!/bin/bash
# round 4, final call: the whole GPU suite at the head, the smoke entry point, the driver's 20-step bench form
# and the default sustained bench with the service load
source tools/gpu_steps.sh
step gpu_suite 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke 200 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench20 300 python3 -u bench.py --steps 20 --warmup 5
step bench_default 400 python3 -u bench.py
grep -h '^{' gpurun_out/bench20.log gpurun_out/bench_default.log | cut -c1-300
exit $STEPS_RC
