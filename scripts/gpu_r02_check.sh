#!/bin/bash
# Round-2 check: the whole GPU suite, smoke, then the default bench line (C2, CPU baseline included).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r2/gpu_tests.log 2>&1
rc=$?; echo "gpu_tests rc=$rc"; tail -4 gpurun_out/r2/gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r2/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r2/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/r2/bench_default.log | cut -c1-400
exit $rc
