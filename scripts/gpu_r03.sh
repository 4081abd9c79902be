#!/bin/bash
# r03 GPU session: parity tests (all, no -x) -> smoke -> default bench -> extra steps from $EXTRA.
# Each GPU step has its own time limit; a crash / abort / timeout ends the session (exit codes > 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAIL:-6} "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
[ -n "$NO_TESTS" ] || step gpu_tests 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
[ -n "$NO_SMOKE" ] || step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[ -n "$NO_BENCH" ] || step bench_default 500 python bench.py
for w in $BENCH_WORKLOADS; do
  step bench_$w 400 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu $BENCH_EXTRA
done
[ -z "$GZIP_PROBE" ] || step gzip_probe 300 python scripts/gzip_probe.py
[ -z "$SNAPPY_PROBE" ] || step snappy_probe 300 python scripts/snappy_probe.py
exit 0
