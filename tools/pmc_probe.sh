#!/bin/bash
# Counter discovery + SQ/TA/TD passes + phase stamps of the bench at HEAD.
#   gpurun -- 'bash tools/pmc_probe.sh <tag>'
set -o pipefail
tag=${1:-probe}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $out/counters_list.txt 2>&1 || true
grep -oE "\b(TA|TD|TCP|TCC|SQ)_[A-Z0-9_]+" $out/counters_list.txt | sort -u > $out/counter_names.txt || true
bash tools/pmc_sq.sh $tag/sq > $out/sq.txt 2>&1 || { tail -20 $out/sq.txt; exit 1; }
P3="TA_TA_BUSY TA_BUFFER_READ_WAVEFRONTS TD_TD_BUSY TD_LOAD_WAVEFRONT"
timeout -k 10 300 rocprofv3 --pmc $P3 --output-format csv -d $out/p3 -o run \
  -- python3 bench.py --no-cpu --steps 5 --warmup 2 --no-kernel-timing > $out/p3.log 2>&1 || tail -5 $out/p3.log
AVZ_LIB=real-time-audio-visual-zooming_amd/avz/libavz_stamps.so timeout -k 10 200 python tools/phase_profile.py > $out/phase.log 2>&1 || tail -5 $out/phase.log
cat $out/sq.txt
grep -v amdgpu.ids $out/phase.log
wc -l $out/counter_names.txt
