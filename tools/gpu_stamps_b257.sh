#!/bin/bash
# Phase stamps of the per-utterance synthesis at B = 256 / 257 / 300 (stamped build
# libavz_st0.so): the piece blocks' rows against the whole-only rows.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/st257
export AVZ_LIB=real-time-audio-visual-zooming_amd/avz/libavz_st0.so
timeout -k 10 200 python -u tools/phase_profile.py --utt --batch 256 > gpurun_out/st257/b256.txt 2>&1 &&
timeout -k 10 200 python -u tools/phase_profile.py --utt --batch 257 --rows 0:8,8:256 > gpurun_out/st257/b257.txt 2>&1 &&
timeout -k 10 200 python -u tools/phase_profile.py --utt --batch 300 --rows 0:176,176:256 > gpurun_out/st257/b300.txt 2>&1
rc=$?
for f in gpurun_out/st257/*.txt; do echo "=== $f"; grep -v amdgpu.ids $f; done
exit $rc
