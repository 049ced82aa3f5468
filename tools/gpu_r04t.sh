set -o pipefail
out=gpurun_out/r04t; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests_default.log 2>&1 || { tail -30 $out/tests_default.log; exit 1; }
tail -2 $out/tests_default.log
for rep in 1 2; do
for cfg in "libavz.so 2" "libavz_inv.so 2" "libavz.so 0"; do
  set -- $cfg
  AVZ_LIB=$PWD/real-time-audio-visual-zooming_amd/avz/$1 AVZ_SYNTH_VARIANT=$2 timeout -k 10 200 python bench.py --no-cpu --no-secondary --n-fft 512 > $out/b512_${1}_v$2_$rep.json 2>&1 || { tail -5 $out/b512_${1}_v$2_$rep.json; exit 1; }
  tail -1 $out/b512_${1}_v$2_$rep.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], round(d["value"]/1e9,2), "G", round(d["ms_per_step"]*1e3,1), "us", {k: round(v*1e3,1) for k,v in d["roofline"].get("kernels_ms",{}).items()})' "$1 v$2"
done
done
