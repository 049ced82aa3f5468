set -o pipefail
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04f2_smoke.log 2>&1 || { tail -20 gpurun_out/r04f2_smoke.log; exit 1; }
tail -3 gpurun_out/r04f2_smoke.log
bash tools/profile_round.sh r04f2 && \
bash tools/pmc_sq.sh r04f2_sq --no-secondary
