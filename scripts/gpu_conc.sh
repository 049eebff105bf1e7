set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in 768 1024; do
  timeout -k 10 400 python -u bench.py --concurrency $c --steps 100 --warmup 10 --no-rtt > gpurun_out/bench_c$c.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_c$c.log
done
