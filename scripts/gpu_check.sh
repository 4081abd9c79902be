#!/bin/bash
# One GPU session: parity tests -> smoke -> bench.  Stops at the first GPU fault / abort / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name" ; date
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 30 "gpurun_out/$name.log"
  # 0 ok, 1 test failures: continue; anything else (abort/segv/timeout) stops the session
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step gpu_tests 900 python -m pytest tests -q -m gpu -x ${PYTEST_K:+-k "$PYTEST_K"}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:---steps 10 --warmup 2 --rows 20000000 --no-cpu}
