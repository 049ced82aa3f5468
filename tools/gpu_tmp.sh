set -o pipefail
mkdir -p gpurun_out/r06v
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "seams or skipped or multi_round" > gpurun_out/r06v/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert" gpurun_out/r06v/pytest.log | head -20
[ $rc -eq 0 ] || exit 1
bash tools/gpu_ab_r06.sh r06v 2 "base|AVZ_LIB=ab/base/libavz.so python bench.py --ibm-kappa -1" "pk|AVZ_LIB=ab/pk/libavz.so python bench.py --ibm-kappa -1" "basek|AVZ_LIB=ab/base/libavz.so python bench.py" "pkk|AVZ_LIB=ab/pk/libavz.so python bench.py" "old|cd ab/r05 && python bench.py"
