set -o pipefail
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04z_smoke.log 2>&1 || { tail -20 gpurun_out/r04z_smoke.log; exit 1; }
tail -3 gpurun_out/r04z_smoke.log
bash tools/profile_round.sh r04z && \
bash tools/pmc_sq.sh r04z_sq --no-secondary
