#!/bin/bash
# GPU session: parity tests (all, no -x) -> bench lines.  Each GPU step has its own time limit;
# a crash / abort / timeout ends the session (exit codes > 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAIL:-25} "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step gpu_tests 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
[ -n "$NO_SMOKE" ] || step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
for w in ${BENCH_WORKLOADS:-c3 c2}; do
  step bench_$w 400 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu
done
