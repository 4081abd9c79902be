#!/bin/bash
# One GPU session: the whole -m gpu suite (per-test durations), smoke, the default bench line (with
# the mixed_1b sub-record).  Each step under its own limit; stops at the first abort / fault /
# timeout (test failures, rc 1, continue to the next step).
#   SKIP_TESTS=1 SKIP_SMOKE=1 SKIP_BENCH=1 PYTEST_ARGS="-k codec" BENCH_ARGS="--steps 20 --warmup 5"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAIL:-25} "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
if [ -z "$SKIP_TESTS" ]; then
  step gpu_tests ${TEST_TIMEOUT:-1000} python -u -m pytest tests -q -m gpu --maxfail=10 --durations=15 \
    --timeout 300 --timeout-method thread ${PYTEST_ARGS}
fi
if [ -z "$SKIP_SMOKE" ]; then
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ -z "$SKIP_BENCH" ]; then
  step bench ${BENCH_TIMEOUT:-900} python bench.py ${BENCH_ARGS:---steps 20 --warmup 5}
fi
