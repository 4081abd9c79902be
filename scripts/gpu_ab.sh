#!/bin/bash
# A/B on one box: GPU suite (optional), then bench lines per workload with env variants, each
# variant run ROUNDS times interleaved (box-to-box spread is ~5%, so only same-box runs compare);
# optional SQ LDS counters per variant (SQ=1) and a graph-replay kernel trace per variant (TRACE=1).
#   TESTS=1 WORKLOADS="c4 c5" VARIANTS="PQH_HIP_LIB=libpqhip_base.so PQH_HIP_LIB=libpqhip.so" bash scripts/gpu_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/ab
mkdir -p "$OUT"
if [ "${TESTS:-0}" = 1 ]; then
  env ${TEST_ENV:-X=1} timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/gpu_tests.log" 2>&1
  rc=$?; echo "gpu_tests rc=$rc"; tail -3 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
fi
for w in ${WORKLOADS:-c4}; do
  A="--workload $w --steps ${STEPS:-10} --warmup 2 --no-cpu --no-e2e --no-c3 --no-mixed --no-next-row ${AB_ARGS}"
  for r in $(seq 1 ${ROUNDS:-1}); do
    for v in ${VARIANTS:-X=1}; do
      tag=${w}_${v//[=,\/]/_}_r$r
      log=$OUT/bench_$tag.log
      env ${v//,/ } timeout -k 10 300 python -u bench.py $A > "$log" 2>&1
      rc=$?; [ $rc -eq 0 ] || { echo "bench $w $v rc=$rc"; tail -5 "$log"; exit $rc; }
      python - "$log" "$w $v r$r" <<'P'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith('{')][-1]; d = json.loads(l)
print(sys.argv[2], 'ms', d['ms_per_step'], 'GB/s', d['value'], d['roofline']['kernel'], d['roofline']['frac'])
print('   ', {k: v['avg_ms'] for k, v in d['kernels'].items() if v['avg_ms'] > 0.01})
P
    done
  done
  for v in ${VARIANTS:-X=1}; do
    tag=${w}_${v//[=,\/]/_}
    if [ "${TRACE:-0}" = 1 ]; then
      env ${v//,/ } timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/trace_$tag" -o run -- python bench.py $A > "$OUT/trace_$tag.log" 2>&1
      rc=$?; [ $rc -eq 0 ] || { echo "trace $tag rc=$rc"; exit $rc; }
      python scripts/overlap.py "$OUT/trace_$tag/run_kernel_trace.csv" --steps 0:12 | sed "s/^/[$tag graph] /" | head -20
    fi
    if [ "${SQ:-0}" = 1 ]; then
      env ${v//,/ } timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS --kernel-trace -T --output-format csv -d "$OUT/sq_$tag" -o run -- python bench.py $A > "$OUT/sq_$tag.log" 2>&1
      rc=$?; [ $rc -eq 0 ] || { echo "sq $tag rc=$rc"; exit $rc; }
      python - "$OUT/sq_$tag/run_counter_collection.csv" "$tag" <<'P'
import csv, collections, sys
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    k = r['Kernel_Name'].split('(')[0].replace('pqhip::', '')
    agg[k][r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in agg.items():
    if not k.startswith('__'):
        print(sys.argv[2], k, {c: round(sum(x) / len(x)) for c, x in v.items()})
P
    fi
  done
done
