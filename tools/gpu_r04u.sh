set -o pipefail
out=gpurun_out/r04u; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests_default.log 2>&1 || { tail -30 $out/tests_default.log; exit 1; }
tail -2 $out/tests_default.log
REPS=2 bash tools/gpu_bench_ab.sh r04u 2 3
