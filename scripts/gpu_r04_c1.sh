#!/bin/bash
# r04 C1 session: k_flat (one launch) against the three kernels (PQH_FLAT=0), then the
# one-launch run's kernel trace + stats and FETCH_SIZE / WRITE_SIZE in separate passes.  Each GPU step has
# its own limit; a crash / abort / timeout / GPU fault ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/r04_c1
mkdir -p "$OUT"
A="--workload c1 --steps 50 --warmup 5 ${C1_ARGS}"
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
  if grep -q "illegal memory access\|Memory access fault" "$OUT/$name.log"; then exit 3; fi
  return 0
}
step bench_flat 400 python bench.py $A
step bench_three 400 env PQH_FLAT=0 python bench.py $A --no-cpu
[ -n "$NO_PROF" ] && exit 0
P="--workload c1 --steps 50 --warmup 5 --no-cpu --no-e2e"
step prof_trace 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/prof_trace" -o run -- python bench.py $P
step prof_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T --output-format csv -d "$OUT/prof_fetch" -o run -- python bench.py $P
step prof_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T --output-format csv -d "$OUT/prof_write" -o run -- python bench.py $P
exit 0
