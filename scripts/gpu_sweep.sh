#!/bin/bash
# One bench line per BASELINE config (C1, C3, C4, C5) and the supplementary C5z with device SNAPPY /
# GZIP end to end, into gpurun_out/sweep/.  Each step under its own limit; a crash / timeout / GPU
# fault ends the session.   WORKLOADS="c1 c3" bash scripts/gpu_sweep.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep
step() {
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/sweep/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 1 "gpurun_out/sweep/$name.log" | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
  if grep -q "illegal memory access\|Memory access fault" "gpurun_out/sweep/$name.log"; then exit 3; fi
  return 0
}
A="--steps 10 --warmup 2 --no-c3 --no-mixed --no-next-row ${SWEEP_ARGS}"
for w in ${WORKLOADS:-c1 c3 c4 c5 c5z}; do
  step bench_$w 400 python bench.py --workload $w $A
done
if [ -z "$NO_GZIP" ]; then
  step bench_c5z_gzip 400 python bench.py --workload c5z --codec gzip $A --no-cpu
fi
exit 0
