#!/bin/bash
# Build experiment variants of libpqhip (lib/<name>.so, loaded with PQH_HIP_LIB=<name>.so):
#   bash scripts/build_variants.sh "copy128:-DPQH_COPY_TILE=131072" "big:-DPQH_COPY_TILE=131072 -DPQH_DICT_SPAN_X=4"
cd "$(dirname "$0")/.."
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  PQH_HIP_LIB=$name.so PQH_HIPFLAGS="$flags" python parquet-go_amd/build.py --force > /dev/null || exit 1
  echo "built parquet-go_amd/lib/$name.so ($flags)"
done
python parquet-go_amd/build.py > /dev/null
