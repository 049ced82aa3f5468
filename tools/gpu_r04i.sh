set -o pipefail
out=gpurun_out/r04i; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests_default.log 2>&1 || { tail -30 $out/tests_default.log; exit 1; }
tail -3 $out/tests_default.log
AVZ_LIB=$PWD/real-time-audio-visual-zooming_amd/avz/libavz_refhalf.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_host.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests_refhalf.log 2>&1 || { tail -30 $out/tests_refhalf.log; exit 1; }
tail -3 $out/tests_refhalf.log
REPS=2 bash tools/gpu_bench_ab.sh r04i 0 1
