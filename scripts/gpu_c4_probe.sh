#!/bin/bash
# C4 overlap probe: the bench step under graph replay (default), direct launches with the side
# streams (PQH_GRAPH=0) and one stream (PQH_FORK=0); a rocprofv3 kernel trace of the graph-replayed
# steps (start / end of every kernel, for scripts/overlap.py); the SQ LDS counters of k_ba_chain.
# Each step under its own limit; the first failure ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/c4probe
mkdir -p "$OUT"
W=${W:-c4}
A="--workload $W --steps 10 --warmup 2 --no-cpu --no-e2e --no-c3 --no-mixed --no-next-row"
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 1 "$OUT/$name.log" | cut -c1-240
  if [ $rc -ne 0 ]; then exit $rc; fi
}
if [ -z "$SKIP_BENCH" ]; then
  step bench_graph 300 python bench.py $A
  PQH_GRAPH=0 step bench_direct 300 python bench.py $A
  PQH_FORK=0 step bench_onestream 300 python bench.py $A
fi
if [ -z "$SKIP_TRACE" ]; then
  step trace 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/trace" -o run -- python bench.py $A
fi
if [ -n "$SQ" ]; then
  step sq1 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace -T --output-format csv -d "$OUT/sq1" -o run -- python bench.py $A
  step sq2 120 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace -T --output-format csv -d "$OUT/sq2" -o run -- python bench.py $A
fi
exit 0
