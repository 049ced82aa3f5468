set -o pipefail
out=gpurun_out/r04r; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_neural.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests_neural.log 2>&1 || { tail -30 $out/tests_neural.log; exit 1; }
tail -2 $out/tests_neural.log
timeout -k 10 600 python -u bench.py --workload unet --no-cpu --steps 2 --warmup 1 > $out/bench_unet.json 2> $out/bench_unet.err || { tail -20 $out/bench_unet.err; exit 1; }
tail -c 1500 $out/bench_unet.json
