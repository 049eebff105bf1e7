#!/bin/bash
# build -> kernel tests -> tune -> bench sweep over concurrency
mkdir -p gpurun_out
export PYTHONPATH=$PWD
python -m nats_llm_studio_amd.build > gpurun_out/build.log 2>&1 || { tail gpurun_out/build.log; exit 3; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_kern.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_kern.log
if [ $rc -ne 0 ]; then exit $rc; fi
if [ "${TUNE:-1}" = "1" ]; then
  rm -f nats_llm_studio_amd/ops/gemv_tuning.json
  timeout -k 10 600 python tools/tune_gemv.py > gpurun_out/tune.out 2>&1; rc=$?
  echo "tune rc=$rc"; cp nats_llm_studio_amd/ops/gemv_tuning.json gpurun_out/ 2>/dev/null
  grep -E "M=  1|M= 16|M= 64" gpurun_out/tune.out
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
for B in ${BS:-1 16 64}; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-rtt --concurrency $B > gpurun_out/bench_b$B.log 2>&1; rc=$?
  echo "bench B=$B rc=$rc"; grep metric gpurun_out/bench_b$B.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/bench_b$B.log; exit $rc; fi
done
