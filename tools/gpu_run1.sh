#!/bin/bash
# first GPU pass: kernel/model tests, then a short bench + single stream
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 500 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python bench.py --steps 20 --warmup 3 --no-rtt --single-stream > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -20 gpurun_out/bench.log
exit $rc
