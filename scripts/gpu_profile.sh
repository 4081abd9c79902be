#!/bin/bash
# rocprofv3 kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in separate passes (gfx950 slots).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out
mkdir -p "$OUT"
ARGS=${PROF_ARGS:---steps 10 --warmup 2 --no-cpu}
run() {  # run <name> <timeout> <rocprof args...>
  local name=$1 to=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$to" rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o run -- python bench.py $ARGS > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 5 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
run prof_trace 600 --kernel-trace --stats -T
run prof_fetch 600 --pmc FETCH_SIZE --kernel-trace -T
run prof_write 600 --pmc WRITE_SIZE --kernel-trace -T
find "$OUT"/prof_* -name "*.csv" | head -20
