#!/bin/bash
# build -> all GPU tests -> graft smoke -> default bench (driver contract, with RTT) -> rocprof stats
mkdir -p gpurun_out
export PYTHONPATH=$PWD
python -m nats_llm_studio_amd.build > gpurun_out/build.log 2>&1 || { tail gpurun_out/build.log; exit 3; }
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1; rc=$?
echo "bench rc=$rc"; grep metric gpurun_out/bench_default.log
[ $rc -ne 0 ] && { tail -5 gpurun_out/bench_default.log; exit $rc; }
if [ "${PROF:-1}" = "1" ]; then
  for B in ${PROF_BS:-1 64}; do
    bash tools/gpu_prof.sh $B || exit $?
  done
fi
exit 0
