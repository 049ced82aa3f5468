set -o pipefail
# Ablation builds (libavz_expN.so) against the default library, same bench.
mkdir -p gpurun_out/exp
for v in ${VARIANTS:-libavz.so libavz_exp1.so libavz_exp2.so libavz_exp3.so libavz_exp4.so libavz_exp5.so}; do
  AVZ_LIB=$PWD/real-time-audio-visual-zooming_amd/avz/$v timeout -k 10 120 python bench.py --no-cpu --steps 10 > gpurun_out/exp/$v.log 2>&1 || { tail -5 gpurun_out/exp/$v.log; exit 1; }
  echo $v $(tail -1 gpurun_out/exp/$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: round(v*1e3,1) for k, v in d["roofline"]["kernels_ms"].items()})')
done
