set -o pipefail
bash tools/profile_round.sh r04k && \
bash tools/pmc_sq.sh r04k_sq --no-secondary && \
bash tools/pmc_sq.sh r04k_sq_ipd --no-secondary --workload ipd
