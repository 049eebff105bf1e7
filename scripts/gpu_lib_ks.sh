#!/usr/bin/env bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for ks in 2 4; do
  timeout -k 10 300 python -u tools/blaslt_ab.py --M 256,512,1024 --shapes o,down --lib-ks $ks \
      > gpurun_out/blaslt_ab_ks$ks.txt 2>&1 || { tail -5 gpurun_out/blaslt_ab_ks$ks.txt; exit 1; }
  echo "lib-ks $ks"; grep -v amdgpu.ids gpurun_out/blaslt_ab_ks$ks.txt
done
