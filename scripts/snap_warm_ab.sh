#!/bin/bash
# Same-box A/B of the snappy spec warm-up (PQH_HIP_LIB variants): rocprofv3 kernel stats of the URL
# probe (512 pages) per variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in libpqhip.so ${VARIANTS:-libpqhip_w64.so libpqhip_w96.so}; do
  PQH_HIP_LIB=$v PROBE_MODES=mw PROBE_COPIES=512 PROBE_CASES=url_1MiB,runs_1MiB timeout -k 10 200 \
    rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_$v -o run -- python scripts/snappy_probe.py \
    > gpurun_out/ab_$v.log 2>&1 || exit $?
  echo "== $v"; grep "ok=" gpurun_out/ab_$v.log
  grep -h "k_snap" gpurun_out/ab_$v/run_kernel_stats.csv | cut -d, -f1,4 | sed 's/(.*)"/"/'
done
