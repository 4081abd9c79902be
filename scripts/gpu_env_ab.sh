#!/bin/bash
# GPU suite, then `bench.py --workload $W` twice per setting: default and with $AB_ENV set (A/B on
# one box).  Each step under its own limit; a failing step ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
W=${W:-c4}
[ -n "$NO_TESTS" ] || { NO_GZIP=1 NO_BENCH=1 NO_SMOKE=1 BENCH_WORKLOADS=$W bash scripts/gpu_r03_check.sh || exit $?; }
for i in 1 2; do
  echo "== bench_${W}_ab$i"
  env $AB_ENV timeout -k 10 300 python bench.py --workload $W --steps 20 --warmup 3 --no-cpu --no-e2e > gpurun_out/bench_${W}_ab$i.log 2>&1 || exit $?
  echo "== bench_${W}_def$i"
  timeout -k 10 300 python bench.py --workload $W --steps 20 --warmup 3 --no-cpu --no-e2e > gpurun_out/bench_${W}_def$i.log 2>&1 || exit $?
done
