set -o pipefail
export TAG=s10
STEP=spawn,c3 bash tools/gpu_r03.sh || exit 1
PMC_NAME=c2 PMC_GROUPS="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVES;TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum;TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum" bash tools/pmc_extra.sh || exit 1
PMC_NAME=b18 PMC_BENCH_ARGS="--batch 262144 --steps 3" PMC_GROUPS="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum;FETCH_SIZE" bash tools/pmc_extra.sh || exit 1
