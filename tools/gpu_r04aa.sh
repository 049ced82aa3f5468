set -o pipefail
out=gpurun_out/r04aa; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests_default.log 2>&1 || { tail -30 $out/tests_default.log; exit 1; }
tail -2 $out/tests_default.log
REPS=2 BENCH_ARGS="--no-secondary" bash tools/ab_libs.sh r04aa libavz.so libavz_prev.so && \
REPS=2 BENCH_ARGS="--no-secondary --n-fft 512" bash tools/ab_libs.sh r04aa_512 libavz.so libavz_prev.so
