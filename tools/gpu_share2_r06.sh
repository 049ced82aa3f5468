#!/bin/bash
# Work-sharing build: IBM exact + parity GPU tests, the trace, a same-box A/B.
set -o pipefail
out=gpurun_out/${TAG:-r06sh2}
mkdir -p $out
D=real-time-audio-visual-zooming_amd/avz
AVZ_LIB=$D/libavz_dev.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_ibm_exact.py tests/test_gpu_parity.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 200 python tools/xtrace.py > $out/xt.txt 2>&1 || { tail -20 $out/xt.txt; exit 1; }
grep -v amdgpu.ids $out/xt.txt | head -14
bash tools/gpu_ab_r06.sh ${TAG:-r06sh2}/ab 2 \
  "base|AVZ_LIB=$D/libavz.so python bench.py --no-cpu --no-secondary --steps 20" \
  "share|AVZ_LIB=$D/libavz_dev.so python bench.py --no-cpu --no-secondary --steps 20"
