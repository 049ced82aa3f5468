set -o pipefail
mkdir -p gpurun_out/r06s
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r06s/pytest.log 2>&1; rc=$?
tail -5 gpurun_out/r06s/pytest.log
[ $rc -eq 0 ] || exit 1
bash tools/gpu_ab_r06.sh r06s 2 "k16|python bench.py --ibm-kappa 16" "koff|python bench.py --ibm-kappa -1" "nocert|AVZ_LIB=ab/nocert/libavz.so python bench.py"
