#!/bin/bash
# Build experiment variants of libpqhip (lib/<name>.so, loaded with PQH_HIP_LIB=<name>.so):
#   bash scripts/build_variants.sh "seg96:-DPQH_CHAIN_SEG=96" "snapprof:-DPQH_SNAP_PROF"
cd "$(dirname "$0")/.."
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  PQH_HIP_LIB=$name.so PQH_HIPFLAGS="$flags" python parquet-go_amd/build.py --force > /dev/null || exit 1
  echo "built parquet-go_amd/lib/$name.so ($flags)"
done
python parquet-go_amd/build.py > /dev/null
