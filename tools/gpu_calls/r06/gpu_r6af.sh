#!/bin/bash
# round 6, call AF: split-K slab sums with the split count as a template constant (splitk_add_rmsnorm_kernel<KS>,
# rope_kv_kernel<KV, KS>: all slab loads issued before the first add) vs the runtime-ks kernels (_kernels_slabrt.so,
# NLS_SLAB_RUNTIME=1): kernel tests, rocprof kernel traces of B=512 under both, benches.
source tools/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step r6af_tests 600 python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "rmsnorm or rope or splitk or slabs"
PB="python3 bench.py --steps 20 --warmup 3 --no-rtt --serve-load 0"
step r6af_prof_new 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_af_new -o run --output-format csv -- $PB
python3 tools/analyze_trace.py $(find gpurun_out/prof_af_new -name "*kernel_trace.csv" | head -1) > gpurun_out/prof_af_new_breakdown.txt && cat gpurun_out/prof_af_new_breakdown.txt
NLS_KERNELS_SO=$PWD/nats_llm_studio_amd/_kernels_slabrt.so step r6af_prof_rt 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_af_rt -o run --output-format csv -- $PB
python3 tools/analyze_trace.py $(find gpurun_out/prof_af_rt -name "*kernel_trace.csv" | head -1) > gpurun_out/prof_af_rt_breakdown.txt && cat gpurun_out/prof_af_rt_breakdown.txt
rm -rf gpurun_out/prof_af_new/*/ gpurun_out/prof_af_rt/*/ 2>/dev/null
B="python3 -u bench.py --steps 20 --warmup 3 --no-rtt --serve-load 0"
step r6af_b512_new 300 $B
NLS_KERNELS_SO=$PWD/nats_llm_studio_amd/_kernels_slabrt.so step r6af_b512_rt 300 $B
step r6af_b512_new2 300 $B
step r6af_b256_new 300 $B --concurrency 256
NLS_KERNELS_SO=$PWD/nats_llm_studio_amd/_kernels_slabrt.so step r6af_b256_rt 300 $B --concurrency 256
rm -f /tmp/nls_bench/*.gguf
step r6af_qw_new 300 $B --model qwen2.5-7b
NLS_KERNELS_SO=$PWD/nats_llm_studio_amd/_kernels_slabrt.so step r6af_qw_rt 300 $B --model qwen2.5-7b
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
