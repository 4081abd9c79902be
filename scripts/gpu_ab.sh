#!/bin/bash
# A/B: GPU suite (optional), then bench lines per workload with env variants.
#   TESTS=1 WORKLOADS="c4 c5" VARIANTS="PQH_FORK=0 PQH_FORK=1" bash scripts/gpu_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
if [ "${TESTS:-0}" = 1 ]; then
  env ${TEST_ENV:-X=1} timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/ab/gpu_tests.log 2>&1
  rc=$?; echo "gpu_tests rc=$rc"; tail -3 gpurun_out/ab/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for w in ${WORKLOADS:-c4}; do
  for v in ${VARIANTS:-X=1}; do
    log=gpurun_out/ab/bench_${w}_${v//[=,]/_}.log
    env ${v//,/ } timeout -k 10 300 python -u bench.py --workload $w --steps ${STEPS:-10} --warmup 2 --no-cpu --no-e2e ${AB_ARGS} > $log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "bench $w $v rc=$rc"; tail -5 $log; exit $rc; }
    python - "$log" "$w $v" <<'P'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith('{')][-1]; d = json.loads(l)
print(sys.argv[2], 'ms', d['ms_per_step'], 'GB/s', d['value'], d['roofline']['kernel'], d['roofline']['frac'])
print('   ', {k: v['avg_ms'] for k, v in d['kernels'].items() if v['avg_ms'] > 0.01})
P
  done
done
