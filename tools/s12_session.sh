#!/bin/bash
# s12: the committed sources: bench line (C2 + legs), rocprof stats, PMC passes
set -o pipefail
export TAG=s12
STEP=bench,prof,pmc bash tools/gpu_r03.sh || exit 1
