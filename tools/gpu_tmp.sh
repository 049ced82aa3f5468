set -o pipefail
mkdir -p gpurun_out/r06z
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r06z/pytest.log 2>&1; echo "full rc $?"
tail -5 gpurun_out/r06z/pytest.log
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_hybrid.py tests/test_gpu_ibm_exact.py > gpurun_out/r06z/pytest2.log 2>&1; echo "again rc $?"
tail -3 gpurun_out/r06z/pytest2.log
