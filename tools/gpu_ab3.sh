set -o pipefail
out=gpurun_out/${1:-ab}; mkdir -p $out
D=real-time-audio-visual-zooming_amd/avz
run() { # name lib args
  AVZ_LIB=$D/$2 timeout -k 10 120 python bench.py --no-cpu ${@:3} > $out/b_$1.log 2>&1 || { tail -5 $out/b_$1.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('$out/b_$1.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$1', round(d['value']/1e9,2), 'G', {k: round(x*1e3,1) for k,x in r['kernels_ms'].items()})"
}
for rep in 1 2; do
run new_$rep libavz.so
run px0_$rep libavz_px0.so
run old_$rep libavz.so --synth-variant 1
done
