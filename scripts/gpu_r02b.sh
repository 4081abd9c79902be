#!/bin/bash
# Round-2 refresh: C4 / C5 / C5z / C3 / C1 bench lines (kernel times, e2e incl. device SNAPPY).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2b
for w in ${WORKLOADS:-c4 c5z c5 c3 c1}; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 10 --warmup 2 --no-cpu > gpurun_out/r2b/bench_$w.log 2>&1
  rc=$?; echo "bench $w rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python - "$w" <<'P'
import json, sys
l = [x for x in open(f"gpurun_out/r2b/bench_{sys.argv[1]}.log") if x.startswith('{')][-1]; d = json.loads(l)
print(sys.argv[1], d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['frac'])
print({k: v['avg_ms'] for k, v in d['kernels'].items() if v['avg_ms'] > 0.01})
for e in ('e2e', 'e2e_device_snappy'):
    if d.get(e): print(e, d[e]['gbps'], d[e].get('k_snappy'))
P
done
