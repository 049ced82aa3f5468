set -o pipefail
mkdir -p gpurun_out/r06t
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ibm_exact.py -s > gpurun_out/r06t/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|frames|utterances|N=" gpurun_out/r06t/pytest.log | head -30
[ $rc -eq 0 ] || exit 1
bash tools/gpu_ab_r06.sh r06t 1 "k2|python bench.py --ibm-kappa 2" "k16|python bench.py --ibm-kappa 16" "k64|python bench.py --ibm-kappa 64" "koff|python bench.py --ibm-kappa -1"
