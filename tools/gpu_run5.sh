#!/bin/bash
# build -> GPU tests -> (optional) tune -> bench sweep; env: TESTS, TUNE (0/1), TUNE_MS, BS, STEPS
mkdir -p gpurun_out
export PYTHONPATH=$PWD
python -m nats_llm_studio_amd.build > gpurun_out/build.log 2>&1 || { tail gpurun_out/build.log; exit 3; }
timeout -k 10 900 python -m pytest ${TESTS:-tests} -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
if [ "${TUNE:-0}" = "1" ]; then
  timeout -k 10 900 python tools/tune_gemv.py --ms ${TUNE_MS:-1,2,4,8,16,32,48,64,128,256,512,2048} > gpurun_out/tune.out 2>&1; rc=$?
  echo "tune rc=$rc"; cp nats_llm_studio_amd/ops/gemv_tuning.json gpurun_out/ 2>/dev/null
  grep -E "M=  1 |M= 64|M=128|M=256|M=2048" gpurun_out/tune.out
  [ $rc -ne 0 ] && exit $rc
fi
for B in ${BS:-64 128 256}; do
  timeout -k 10 400 python bench.py --steps ${STEPS:-30} --warmup 5 --no-rtt --concurrency $B > gpurun_out/bench_b$B.log 2>&1; rc=$?
  echo "bench B=$B rc=$rc"; grep metric gpurun_out/bench_b$B.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['timings_s'])"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_b$B.log; exit $rc; }
done
exit 0
