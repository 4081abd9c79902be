#!/bin/bash
# C5z device-SNAPPY A/B: codec tests and the bench's device-codec record per library variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/snap
for lib in ${LIBS:-libpqhip.so}; do
  PQH_HIP_LIB=$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k snappy > gpurun_out/snap/tests_$lib.log 2>&1 || { echo "tests $lib failed"; tail -5 gpurun_out/snap/tests_$lib.log; exit 1; }
  PQH_HIP_LIB=$lib timeout -k 10 400 python bench.py --workload c5z --steps 10 --warmup 2 --no-cpu --no-c3 --no-next-row > gpurun_out/snap/bench_$lib.log 2>&1 || exit $?
  python - "gpurun_out/snap/bench_$lib.log" "$lib" <<'P'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith('{')][-1]; d = json.loads(l); e = d['e2e_device_snappy']
print(sys.argv[2], 'e2e', d['e2e']['gbps'], 'dev', e['gbps'], {k: v['avg_ms'] for k, v in e['device_codec']['kernels'].items()})
P
done
