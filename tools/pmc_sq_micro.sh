#!/bin/bash
# SQ counters of the FFT micro-benchmark kernels (tools/micro/fftbench.py).
set -o pipefail
out=gpurun_out/${1:-sqm}
mkdir -p $out
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2"
P2="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $out/p$i -o run \
    -- python3 tools/micro/fftbench.py > $out/p$i.log 2>&1 || { tail -20 $out/p$i.log; exit 1; }
done
timeout -k 10 120 python3 tools/micro/fftbench.py
