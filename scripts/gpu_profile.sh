#!/bin/bash
# Profiles of the tree: per workload (WORKLOADS="c2 c4 mixed" by default) a rocprofv3 kernel trace + stats, then FETCH_SIZE
# and WRITE_SIZE in separate passes (gfx950 counter slots), each under its own limit; the first
# failure ends the session.  Summarise with
#   python scripts/pmc_summary.py r05_<w> gpurun_out prof_<w>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out
mkdir -p "$OUT"
run() {  # run <name> <timeout> <bench args> -- <rocprof args...>
  local name=$1 to=$2 args=$3; shift 3
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o run -- python bench.py $args > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
SKIP="--no-cpu --no-e2e --no-c3 --no-mixed --no-next-row"
for w in ${WORKLOADS:-c2 c4 mixed}; do
  case $w in
    c2) A="--steps 10 --warmup 2 $SKIP" ;;
    mixed) A="--workload mixed --steps 5 --warmup 1 $SKIP" ;;
    c5z_gzip) A="--workload c5z --codec gzip --steps 10 --warmup 2 $SKIP" ;;
    *) A="--workload $w --steps 10 --warmup 2 $SKIP" ;;
  esac
  run prof_${w}_trace 600 "$A" --kernel-trace --stats -T
  run prof_${w}_fetch 600 "$A" --pmc FETCH_SIZE --kernel-trace -T
  run prof_${w}_write 600 "$A" --pmc WRITE_SIZE --kernel-trace -T
done
