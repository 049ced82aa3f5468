set -o pipefail
bash tools/gpu_bench_ab.sh r04h 0 1 && \
REPS=2 BENCH_ARGS="--no-secondary" bash tools/ab_libs.sh r04h libavz.so libavz_refhalf.so
