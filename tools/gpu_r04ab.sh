set -o pipefail
out=gpurun_out/r04ab; mkdir -p $out
AVZ_LIB=$PWD/real-time-audio-visual-zooming_amd/avz/libavz_fwd.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests_fwd.log 2>&1 || { tail -30 $out/tests_fwd.log; exit 1; }
tail -2 $out/tests_fwd.log
REPS=2 BENCH_ARGS="--no-secondary --n-fft 512" bash tools/ab_libs.sh r04ab libavz_fwd.so libavz.so
