set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for B in 1 16 64; do
  timeout -k 10 300 python -u bench.py --concurrency $B --no-rtt --single-stream > gpurun_out/bench_b$B.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_b$B.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b1 -o run -- python -u bench.py --concurrency 1 --no-rtt --steps 20 > gpurun_out/prof_b1.log 2>&1 || exit $?
echo done
