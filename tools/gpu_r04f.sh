set -o pipefail
mkdir -p gpurun_out/r04f
timeout -k 10 150 python -u tools/ab_synth.py --normalize none --rounds 2 > gpurun_out/r04f/ab_none.log 2>&1 && \
timeout -k 10 150 python -u tools/ab_synth.py --workload ipd --batch 1024 --rounds 2 --calls 10 > gpurun_out/r04f/ab_ipd.log 2>&1
rc=$?
grep -v amdgpu gpurun_out/r04f/ab_none.log gpurun_out/r04f/ab_ipd.log
exit $rc
