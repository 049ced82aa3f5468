#!/bin/bash
# Phase stamps of the given stamped builds (libavz_st<W>.so = -DAVZ_STAMPS -DAVZ_STAMP_WAVE=W).
#   gpurun -- 'bash tools/stamps.sh <tag> 1 3'
set -o pipefail
out=gpurun_out/$1; shift
mkdir -p $out
D=real-time-audio-visual-zooming_amd/avz
for w in "$@"; do
  AVZ_LIB=$D/libavz_st$w.so timeout -k 10 200 python tools/phase_profile.py ${STAMP_ARGS} > $out/stamps_wave$w.txt 2>&1 || { tail -20 $out/stamps_wave$w.txt; exit 1; }
  echo "== wave $w"; grep -v amdgpu.ids $out/stamps_wave$w.txt
done
