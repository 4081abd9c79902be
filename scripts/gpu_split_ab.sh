#!/bin/bash
# k_delta_split vs k_delta_fused (PQH_DELTA_SPLIT=0) on one box: C3 whole file + the rank-0 proxy of
# N = 2 / 4 / 8 (c3_strong), the mixed 1B-row file, C5's DELTA_LENGTH lengths.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/split
for v in 1 0; do
  PQH_DELTA_SPLIT=$v timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --no-next-row \
    > gpurun_out/split/bench_c2_split$v.log 2>&1 || { echo "bench split=$v rc=$?"; tail -5 gpurun_out/split/bench_c2_split$v.log; exit 1; }
  PQH_DELTA_SPLIT=$v timeout -k 10 300 python -u bench.py --workload c5 --steps 10 --warmup 2 --no-cpu --no-e2e \
    --no-next-row --no-c3 --no-mixed > gpurun_out/split/bench_c5_split$v.log 2>&1 || { echo "c5 split=$v rc=$?"; exit 1; }
  python - gpurun_out/split/bench_c2_split$v.log gpurun_out/split/bench_c5_split$v.log $v <<'P'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
c3, m = d['c3_strong'], d['mixed_1b']
print('split', sys.argv[3], 'C3 ms', c3['ms_per_step'], 'proxy', [(p['n_gpus'], p['rank0_ms_per_step'], p['predicted_efficiency']) for p in c3['proxy']])
print('   mixed ms', m['ms_per_step'], 'frac', m['step_roofline']['frac'], {k: v['avg_ms'] for k, v in m['kernels'].items() if v['avg_ms'] > 0.05},
      'proxy', [(p['n_gpus'], p['predicted_efficiency']) for p in m['proxy']])
e = json.loads([x for x in open(sys.argv[2]) if x.startswith('{')][-1])
print('   C5 ms', e['ms_per_step'], {k: v['avg_ms'] for k, v in e['kernels'].items() if v['avg_ms'] > 0.01})
P
done
