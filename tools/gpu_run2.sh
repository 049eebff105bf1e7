#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
python -m nats_llm_studio_amd.build > gpurun_out/build.log 2>&1 || { tail gpurun_out/build.log; exit 3; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_kern.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_kern.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python tools/tune_gemv.py > gpurun_out/tune.out 2>&1; rc=$?
echo "tune rc=$rc"; cp nats_llm_studio_amd/ops/gemv_tuning.json gpurun_out/ 2>/dev/null
tail -60 gpurun_out/tune.out
exit $rc
