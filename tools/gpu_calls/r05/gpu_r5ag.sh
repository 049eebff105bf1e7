#!/bin/bash
# round 5, call AG: EP prefill through the IPC row exchange (EP2 / EP4), the forced all-to-all path, the EP decode tests.
source tools/gpu_steps.sh
step r5ag_ep 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_tp_rehearsal_gpu.py -k "row_exchange or alltoall or mixtral"
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
