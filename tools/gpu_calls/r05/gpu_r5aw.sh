#!/bin/bash
# micro-batch overlap feasibility at B=512 / 256 (two graph branches)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag/mb_overlap.py --B 512 > gpurun_out/mb_overlap.txt 2>&1 &&
timeout -k 10 300 python -u tools/diag/mb_overlap.py --B 256 >> gpurun_out/mb_overlap.txt 2>&1
