#!/bin/bash
# ASan + UBSan run of the CPU suite over the sanitizer builds of the host parsers (libpqhip's
# codec.cpp + file_reader.cpp, libpqgen, the oracle's refdecode.c): the walker, thrift reader and
# codecs parse the mutation fuzzers' and the reference's corrupt files here.  CPU only (no GPU
# sanitizer on this pool).  Log: profiles/r03/sanitizers.log
#   bash scripts/run_sanitized.sh [pytest args]
set -e
cd "$(dirname "$0")/.."
PQH_SANITIZE=1 python parquet-go_amd/build.py --sanitize
make -s -C oracle SAN=1
ASAN_LIB=$(gcc -print-file-name=libasan.so)
UBSAN_LIB=$(gcc -print-file-name=libubsan.so)
mkdir -p profiles/r03
set +e
PQH_LIBDIR=$PWD/parquet-go_amd/lib/san ORC_LIB=$PWD/oracle/build/san/liborcl.so PQH_AUTOBUILD=0 \
LD_PRELOAD="$ASAN_LIB:$UBSAN_LIB" \
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1:allow_user_segv_handler=1 \
UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
python -m pytest tests -m "not gpu" -q -p no:xdist -p no:cacheprovider "$@" 2>&1 | tee profiles/r03/sanitizers.log
rc=${PIPESTATUS[0]}
echo "sanitized CPU suite exit status: $rc" | tee -a profiles/r03/sanitizers.log
exit $rc
