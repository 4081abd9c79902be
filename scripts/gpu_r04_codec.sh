#!/bin/bash
# r04 device-codec session: codec GPU tests, then C5 / C5z benches (device SNAPPY e2e with 1 and 4
# staged ranges) and the GZIP e2e.  A crash / timeout / GPU fault ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "gpurun_out/$name.log" | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  if grep -q "illegal memory access\|Memory access fault" "gpurun_out/$name.log"; then exit 3; fi
  return 0
}
step codec_tests 600 python -u -m pytest tests/test_gpu_codec.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
for r in 1 4; do
  step bench_c5_r$r 400 python bench.py --workload c5 --steps 10 --warmup 2 --no-cpu --no-c3 --no-next-row --e2e-dev-ranges $r
  step bench_c5z_r$r 400 python bench.py --workload c5z --steps 10 --warmup 2 --no-cpu --no-c3 --no-next-row --e2e-dev-ranges $r
done
step bench_c5z_gzip 400 python bench.py --workload c5z --codec gzip --steps 10 --warmup 2 --no-cpu --no-c3 --no-next-row
exit 0
