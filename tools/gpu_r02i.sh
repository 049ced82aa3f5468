set -o pipefail
out=gpurun_out/r02i; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_scene.py tests/test_gpu_configs2.py -m gpu -x -v -s --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1 || { tail -40 $out/gpu_tests.log; exit 1; }
grep -E "PASSED|FAILED|max \||generated|ms|shard" $out/gpu_tests.log | tail -30
timeout -k 10 300 python bench.py > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-600
