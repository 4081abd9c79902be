#!/bin/bash
# Round-2 final: GPU suite + smoke, then C4 / C5 / C5z / C3 bench lines (e2e incl. device SNAPPY).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fin
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/fin/gpu_tests.log 2>&1
rc=$?; echo "gpu_tests rc=$rc"; tail -2 gpurun_out/fin/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/fin/smoke.log; [ $rc -eq 0 ] || exit $rc
for w in ${WORKLOADS:-c4 c5z c5 c3}; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 10 --warmup 2 --no-cpu > gpurun_out/fin/bench_$w.log 2>&1
  rc=$?; echo "bench $w rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python - "$w" <<'P'
import json, sys
l = [x for x in open(f"gpurun_out/fin/bench_{sys.argv[1]}.log") if x.startswith('{')][-1]; d = json.loads(l)
print(sys.argv[1], d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['traffic'])
print({k: v['avg_ms'] for k, v in d['kernels'].items() if v['avg_ms'] > 0.01})
for e in ('e2e', 'e2e_device_snappy'):
    if d.get(e): print(e, d[e]['gbps'], d[e]['ms_per_step'], d[e].get('k_snappy'))
P
done
