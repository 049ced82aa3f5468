set -o pipefail
bash tools/profile_round.sh r04p && \
bash tools/pmc_sq.sh r04p_sq --no-secondary && \
bash tools/pmc_sq.sh r04p_sq_ipd --no-secondary --workload ipd
