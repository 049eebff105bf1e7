#!/bin/bash
# round 6, call AN (final form after the MoE router-row prefetch): the full GPU suite at the head, smoke(), the driver's bench command, batch 1, Granite B=512 and
# Mixtral B=256 with the final table.
source tools/gpu_steps.sh
step r6an_gpu_tests 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step r6an_smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step r6an_bench 600 python3 -u bench.py --steps 20 --warmup 5
step r6an_b1 300 python3 -u bench.py --steps 100 --warmup 5 --concurrency 1 --no-rtt --serve-load 0
rm -f /tmp/nls_bench/*.gguf
B="python3 -u bench.py --steps 20 --warmup 3 --no-rtt --serve-load 0"
step r6an_granite 300 $B --model granite-3.0-2b
rm -f /tmp/nls_bench/*.gguf
step r6an_mixtral 400 $B --model mixtral-8x7b --concurrency 256
rm -f /tmp/nls_bench/*.gguf
step r6an_qwen 400 $B --model qwen2.5-7b
rm -f /tmp/nls_bench/*.gguf
exit $STEPS_RC
