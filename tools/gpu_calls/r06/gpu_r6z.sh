#!/bin/bash
# round 6, final call: the full GPU suite at the head, smoke(), and the driver's bench command.
source tools/gpu_steps.sh
step r6z_gpu_tests 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step r6z_smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step r6z_bench 600 python3 -u bench.py --steps 20 --warmup 5
exit $STEPS_RC
