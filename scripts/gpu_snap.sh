#!/bin/bash
# Device-codec session: codec parity tests -> C5z (device SNAPPY e2e) -> C5z GZIP with the guarded
# debug build.  Each GPU step has its own limit; a crash / abort / timeout ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAIL:-8} "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  if grep -q "illegal memory access\|HIP error\|Memory access fault" "gpurun_out/$name.log"; then exit 3; fi
  return 0
}
step codec_tests 300 python -u -m pytest tests/test_gpu_codec.py -q -x --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
[ -n "$NO_C5Z" ] || step bench_c5z 400 python bench.py --workload c5z --steps 10 --warmup 2 --no-cpu
[ -n "$NO_SNAP_PROBE" ] || step snappy_probe 300 python scripts/snappy_probe.py
[ -z "$GZ_DBG" ] || step bench_c5z_gzip 400 python bench.py --workload c5z --codec gzip --steps 10 --warmup 2 --no-cpu
exit 0
