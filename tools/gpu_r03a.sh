set -o pipefail
export TAG=r03a
bash tools/gpu_round.sh && bash tools/pmc_inner.sh && echo PMCOK
