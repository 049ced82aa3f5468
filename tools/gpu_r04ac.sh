set -o pipefail
out=gpurun_out/r04ac; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests_default.log 2>&1 || { tail -30 $out/tests_default.log; exit 1; }
tail -2 $out/tests_default.log
REPS=1 bash tools/ab_libs.sh r04ac libavz.so libavz_prev.so
