set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/blaslt_ab.py --M 256,512,1024 --shapes o,down > gpurun_out/blaslt_ab_addnorm.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/blaslt_ab_addnorm.txt | tail -8; exit $rc
