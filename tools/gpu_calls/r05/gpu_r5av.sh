#!/bin/bash
# batch-1 decode attention latency: split count, workgroup size and kernel family at short/long context
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/attn_b1_r05.jsonl
: > $O
P="python -u tools/attn_b1_probe.py --ctx 128,256,512,2048,8192"
timeout -k 10 120 $P >> $O 2>&1 &&
timeout -k 10 120 $P --splits 1 >> $O 2>&1 &&
timeout -k 10 120 $P --splits 4 >> $O 2>&1 &&
timeout -k 10 120 $P --splits 8 >> $O 2>&1 &&
NLS_ATTN_MFMA_WAVES=4 timeout -k 10 120 $P --splits 1 >> $O 2>&1 &&
NLS_ATTN_MFMA_WAVES=4 timeout -k 10 120 $P --splits 8 >> $O 2>&1 &&
NLS_ATTN_MFMA=0 timeout -k 10 120 $P >> $O 2>&1
