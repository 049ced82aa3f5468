"""Debug helper: configs[2]-like shard through MVDRPlan twice; saves both outputs and reports
where they differ (run under AVZ_LIB=<lib> to pick the build)."""
import sys
import numpy as np
import torch
import avz
from avz import synth

B, S, N, K = int(sys.argv[2]) if len(sys.argv) > 2 else 512, 64000, 1024, 3
dev = torch.device("cuda")
dm, dt, di = synth.make_batch_device(B, start=0, n_samples=S, n_interferers=K, device=dev, rng="philox")
plan = avz.MVDRPlan(n_fft=N, sigma=1.0, mic_d=0.01, mask="ibm", postfilter="ibm",
                    normalize="peak", max_batch=B, max_samples=S)
o1, p1 = plan.run(dm, ref_tgt=dt, ref_int=di)
o1 = o1.clone(); p1 = p1.clone()
o2, p2 = plan.run(dm, ref_tgt=dt, ref_int=di)
d = (o1 - o2).abs()
print("max |o1-o2|", float(d.max()), "n diff", int((d > 0).sum()), "peak diff", float((p1 - p2).abs().max()))
if (d > 0).any():
    bad = torch.nonzero(d.amax(dim=1) > 0).flatten().tolist()
    print("utterances differing:", len(bad), bad[:20])
    b = bad[0]
    idx = torch.nonzero(d[b] > 0).flatten()
    print("utt", b, "samples", int(idx.numel()), "first", idx[:10].tolist(), "segments", sorted(set((idx // 512).tolist()))[:40])
np.save(sys.argv[1], o1.cpu().numpy())
