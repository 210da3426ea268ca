#!/bin/bash
# AddressSanitizer + UBSan runs of (1) the native host code (_edvhost: request
# collection, SigningSerializer, base58, arenas, the decode pool, output lists)
# under the CPU test suites that drive it, and (2) the kernels' own math and
# per-signature algorithm compiled for the CPU (libedv_hostcheck: field
# arithmetic, half-size scalars, the R side's [S]B, the walk, the signer,
# SHA-256/512, the async ledger) under the suites that drive that.  Host code
# only (no GPU; the GPU build is not instrumented).  Builds into /tmp, leaves
# the in-tree libraries alone.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
PYINC=$(python3 -c "import sysconfig; print(sysconfig.get_paths()['include'])")
EXT=$(python3 -c "import sysconfig; print(sysconfig.get_config_var('EXT_SUFFIX'))")
OUT=${ASAN_OUT:-/tmp/edv_asan}
mkdir -p $OUT
g++ -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -std=c++17 -fPIC -shared -I$PYINC \
  $R/indy-plenum_amd/csrc/edv_host.cpp -o $OUT/_edvhost$EXT
LIBASAN=$(gcc -print-file-name=libasan.so)
LIBUBSAN=$(gcc -print-file-name=libubsan.so)
cd $R
EDV_HOSTEXT_OVERRIDE=$OUT/_edvhost$EXT ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
  LD_PRELOAD="$LIBASAN $LIBUBSAN" python3 -m pytest -x -q -m "not gpu" -p no:cacheprovider \
  tests/test_host_native.py tests/test_authn_host.py tests/test_pool_cpu.py ${ASAN_TESTS:-}
g++ -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -std=c++17 -fPIC -shared -Wno-unknown-pragmas \
  $R/indy-plenum_amd/csrc/edv_hostcheck.cpp -o $OUT/libedv_hostcheck_asan.so
EDV_HOSTCHECK_OVERRIDE=$OUT/libedv_hostcheck_asan.so ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 \
  UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 LD_PRELOAD="$LIBASAN $LIBUBSAN" \
  python3 -m pytest -x -q -m "not gpu" -p no:cacheprovider tests/test_math_host.py tests/test_signer.py \
  tests/test_cabi.py::test_async_ledger_failures_are_sticky
