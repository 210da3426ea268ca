#!/bin/bash
# s17: final kernel sources: rocprof stats + PMC passes (pmc_latest.json must match HEAD's sources)
set -o pipefail
export TAG=s17
STEP=prof,pmc bash tools/gpu_r03.sh || exit 1
