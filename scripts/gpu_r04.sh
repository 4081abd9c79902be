#!/bin/bash
# r04 GPU session: pytest -m gpu (optionally -k) -> smoke -> benches.  Each GPU step has its own
# limit; a crash / abort / timeout / GPU fault ends the session (no retries).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAIL:-4} "gpurun_out/$name.log" | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  if grep -q "illegal memory access\|Memory access fault" "gpurun_out/$name.log"; then exit 3; fi
  return 0
}
[ -n "$NO_TESTS" ] || step gpu_tests 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"}
[ -z "$SMOKE" ] || step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
for w in $BENCH; do
  step bench_$w 500 python bench.py --workload $w ${BENCH_ARGS}
done
exit 0
