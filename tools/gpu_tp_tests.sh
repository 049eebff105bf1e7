set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_oneshot_ipc_gpu.py tests/test_tp_rehearsal_gpu.py > gpurun_out/tp_tests.log 2>&1
rc=$?
tail -30 gpurun_out/tp_tests.log
exit $rc
