#!/bin/bash
# Dense f16 GEMM (modes 4/5): kernel tests, tuning sweep vs the quantised winners, B=512 bench.
set -u
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "hgemm" > gpurun_out/dense_tests.log 2>&1 || { tail -30 gpurun_out/dense_tests.log; exit 1; }
tail -3 gpurun_out/dense_tests.log
cp nats_llm_studio_amd/ops/gemv_tuning.json gpurun_out/gemv_tuning_dense.json
timeout -k 10 900 python -u tools/tune_gemv.py --dense --ms ${MS:-128,256,512,1024,2048} --out gpurun_out/gemv_tuning_dense.json --log gpurun_out/tune_dense.log ${ONLY:+--only $ONLY} || exit 1
cp gpurun_out/gemv_tuning_dense.json nats_llm_studio_amd/ops/gemv_tuning.json
for arm in 1 0; do
  NLS_DENSE_WEIGHTS=$arm timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --no-rtt --serve-load 0 > gpurun_out/bench_dense$arm.log 2>&1 || { tail -20 gpurun_out/bench_dense$arm.log; exit 1; }
  echo "dense=$arm $(tail -1 gpurun_out/bench_dense$arm.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
