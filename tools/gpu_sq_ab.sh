set -o pipefail
bash tools/pmc_sq.sh sq_v0 && bash tools/pmc_sq.sh sq_v1 --synth-variant 1
