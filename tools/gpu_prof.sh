#!/bin/bash
# rocprofv3 kernel trace + stats of the bench (B given as $1, default 64)
mkdir -p gpurun_out
export PYTHONPATH=$PWD
B=${1:-64}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
python -m nats_llm_studio_amd.build > gpurun_out/build.log 2>&1 || exit 3
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b$B -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-rtt --concurrency $B > gpurun_out/prof_b$B.log 2>&1; rc=$?
echo "rc=$rc"; tail -3 gpurun_out/prof_b$B.log
find gpurun_out/prof_b$B -name "*stats*"
exit $rc
