#!/bin/bash
# s11: parity on the new prep sources, then A/B against HEAD's library
set -o pipefail
export TAG=s11
STEP=test bash tools/gpu_r03.sh || exit 1
MODES_STR=";--batch 262144 --steps 6" VARIANTS="variants/libedv_head.so libedv.so variants/libedv_nosqn.so variants/libedv_norcp.so" \
  TAG=s11 REPS=5 bash tools/ab_main.sh || exit 1
