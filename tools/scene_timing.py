"""Time the scene generators for a bench batch (B = 256, 4 s, 2 interferers): host numpy
(avz.synth.make_batch) vs device (make_batch_device: host RNG draws + avz_scene_mix)."""
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."),
                os.path.join(os.path.dirname(__file__), "..", "real-time-audio-visual-zooming_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from avz import synth  # noqa: E402

B, S = 256, 64000
dev = torch.device("cuda:0")
synth.make_batch_device(2, n_samples=S, device=dev)
torch.cuda.synchronize()
t0 = time.perf_counter()
draws = [synth.scene_draws(b, S, 2) for b in range(B)]
t1 = time.perf_counter()
mix, tgt, itf = synth.make_batch_device(B, n_samples=S, device=dev)
torch.cuda.synchronize()
t2 = time.perf_counter()
hm, ht, hi = synth.make_batch(B, n_samples=S)
t3 = time.perf_counter()
err = max(float(np.max(np.abs(mix.cpu().numpy() - hm))), float(np.max(np.abs(tgt.cpu().numpy() - ht))))
print(f"B={B} S={S}: host draws {t1 - t0:.2f} s; device generator (draws + mixing) {t2 - t1:.2f} s; "
      f"host numpy generator {t3 - t2:.2f} s; max |device - host| = {err:.2e}")
