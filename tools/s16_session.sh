#!/bin/bash
# s16: the whole tree as the driver will run it: GPU suite + smoke, default bench line
set -o pipefail
export TAG=s16
STEP=test,bench bash tools/gpu_r03.sh || exit 1
