# C4 counters: SQ passes (pmc_probe.sh) + FETCH_SIZE / WRITE_SIZE passes, short bench runs
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/pmc
A="--workload c4 --steps 3 --warmup 1 --no-cpu --no-e2e"
PMC_ARGS="$A" bash scripts/pmc_probe.sh || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc/p3 -o run -- python bench.py $A > gpurun_out/pmc/p3.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc/p4 -o run -- python bench.py $A > gpurun_out/pmc/p4.log 2>&1
echo rc=$?
