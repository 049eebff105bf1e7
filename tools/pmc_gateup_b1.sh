cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=$PWD
mkdir -p gpurun_out/pmc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC -d gpurun_out/pmc/p1 -o p1 --output-format csv -- python3 tools/l3_warm_probe.py --shape gateup > gpurun_out/pmc/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_INSTS_SALU -d gpurun_out/pmc/p2 -o p2 --output-format csv -- python3 tools/l3_warm_probe.py --shape gateup > gpurun_out/pmc/p2.log 2>&1
echo rc=$?
