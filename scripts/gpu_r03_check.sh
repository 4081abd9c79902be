#!/bin/bash
# r03 check session: GPU suite (all) -> smoke -> default bench -> C5z (device SNAPPY / GZIP e2e) ->
# rocprofv3 kernel trace of the C5z bench.  Each GPU step has its own limit; a crash / abort /
# timeout ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAIL:-4} "gpurun_out/$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  if grep -q "illegal memory access\|Memory access fault" "gpurun_out/$name.log"; then exit 3; fi
  return 0
}
[ -n "$NO_TESTS" ] || step gpu_tests 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
[ -n "$NO_SMOKE" ] || step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[ -n "$NO_BENCH" ] || step bench_default 500 python bench.py
for w in ${BENCH_WORKLOADS:-c5z}; do
  step bench_$w 400 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu
done
[ -n "$NO_GZIP" ] || step bench_c5z_gzip 400 python bench.py --workload c5z --codec gzip --steps 10 --warmup 2 --no-cpu
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  step prof_$PROF 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$PROF -o run -- python bench.py --workload $PROF --steps 5 --warmup 1 --no-cpu
fi
exit 0
