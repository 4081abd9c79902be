#!/bin/bash
# Ticket atomics vs dispatch order (blockIdx) for k_delta_split and k_ba_chain, one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ticket
A="--steps 10 --warmup 2 --no-cpu --no-e2e --no-next-row --no-mixed"
for v in "PQH_SPLIT_TICKET=1" "PQH_SPLIT_TICKET=0" "PQH_DELTA_SPLIT=0"; do
  env $v timeout -k 10 400 python -u bench.py --workload c3 $A > gpurun_out/ticket/c3_$v.log 2>&1 || { echo "c3 $v failed"; tail -3 gpurun_out/ticket/c3_$v.log; exit 1; }
  python - gpurun_out/ticket/c3_$v.log "$v" <<'P'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
print(sys.argv[2], 'C3 ms', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items() if v['avg_ms'] > 0.02})
P
done
for v in "PQH_CHAIN_TICKET=1" "PQH_CHAIN_TICKET=0" "PQH_CHAIN_TICKET=1" "PQH_CHAIN_TICKET=0"; do
  env $v timeout -k 10 400 python -u bench.py --workload c4 $A --no-c3 > gpurun_out/ticket/c4_$v.log 2>&1 || { echo "c4 $v failed"; tail -3 gpurun_out/ticket/c4_$v.log; exit 1; }
  python - gpurun_out/ticket/c4_$v.log "$v" <<'P'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
print(sys.argv[2], 'C4 ms', d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items() if v['avg_ms'] > 0.02})
P
done
