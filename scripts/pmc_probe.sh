# SQ counter passes (one rocprofv3 run each) over a short bench run; PMC_ARGS = bench arguments
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
A=${PMC_ARGS:-"--workload c3 --rows 300000000 --steps 3 --warmup 1 --no-cpu --no-e2e"}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc/p1 -o run -- python bench.py $A > gpurun_out/pmc/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc/p2 -o run -- python bench.py $A > gpurun_out/pmc/p2.log 2>&1
echo rc=$?
