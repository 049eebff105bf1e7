#!/bin/bash
# round 6, call M: the full GPU suite at the head, smoke(), the driver's bench command (defaults: RTT + service load),
# (GPU suite summary -> profiles/gpu_tests_r06.txt).
source tools/gpu_steps.sh
step r6m_gpu_tests 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step r6m_smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step r6m_bench 600 python3 -u bench.py --steps 20 --warmup 5
exit $STEPS_RC
