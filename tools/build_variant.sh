#!/bin/bash
# Build an A/B variant of the product library with extra -D flags:
#   tools/build_variant.sh NAME "-DSOME_FLAG ..."   (the product build's flags otherwise)
# -> indy-plenum_amd/variants/libedv_NAME.so (load it with EDV_LIB=...).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $R/indy-plenum_amd/variants
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -Wall -Wno-unused-function -Xarch_host -march=x86-64-v3 $2 \
  $R/indy-plenum_amd/csrc/edv_verify.hip $R/indy-plenum_amd/csrc/edv_prep.hip $R/indy-plenum_amd/csrc/edv_runtime.hip -o $R/indy-plenum_amd/variants/libedv_$1.so
echo built variants/libedv_$1.so
