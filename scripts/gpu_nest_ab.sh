#!/bin/bash
# GPU suite, then the C4 bench with the one-pass nesting write (default) and with the three passes
# (PQH_NEST_PASSES=3), then C4 rocprofv3 trace + FETCH/WRITE passes.  Each step under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
NO_GZIP=1 NO_BENCH=1 NO_SMOKE=1 BENCH_WORKLOADS=c4 bash scripts/gpu_r03_check.sh || exit $?
echo "== bench_c4_3pass"
PQH_NEST_PASSES=3 timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_c4_3pass.log 2>&1 || exit $?
echo "== bench_c4_b"
timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_c4_b.log 2>&1 || exit $?
[ -n "$NO_PROF" ] || WORKLOADS="c4" bash scripts/gpu_profile_all.sh
