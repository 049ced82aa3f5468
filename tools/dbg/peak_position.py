"""Where the utterance peak falls (synthesis step of 16 frames) for the bench's synthetic
batch: the running-scale rescale covers the steps before the peak's step."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "real-time-audio-visual-zooming_amd"))
import numpy as np
import torch
import avz
from avz import synth

dev = torch.device("cuda:0")
B, S = 256, 64000
for start in (0, 1000):
    dm, dt, di = synth.make_batch_device(B, start=start, n_samples=S, n_interferers=2, device=dev, rng="philox")
    plan = avz.MVDRPlan(n_fft=1024, sigma=1.0, mic_d=0.01, mask="ibm", postfilter="ibm",
                        normalize="none", max_batch=B, max_samples=S)
    out, peak = plan.run(dm, ref_tgt=dt, ref_int=di)
    n = plan.out_len(S)
    a = out[:, :n].abs().argmax(dim=1).cpu().numpy()
    seg = (a // 512)              # segment j
    step = (seg + 1) // 16         # step that wrote it
    h = np.bincount(step, minlength=8)
    print("start", start, "peak step histogram", h.tolist(), "mean fraction rescaled",
          float(np.mean(np.minimum(step * 16 - 1, 124).clip(0) / 124)))
    # input mixture peak positions too
    m = dm[:, 0, :].abs().argmax(dim=1).cpu().numpy() // (512 * 16)
    print("  mixture ch0 peak step histogram", np.bincount(m, minlength=8).tolist())
