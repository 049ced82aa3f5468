set -o pipefail
REPS=1 bash tools/gpu_bench_ab.sh r04v 2 3
