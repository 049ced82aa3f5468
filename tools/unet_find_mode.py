"""U-Net (configs[4]) fp32 forward with MIOpen's find mode (torch.backends.cudnn.benchmark)
against the default heuristic choice: time per 256 chunks and the mask difference."""
import os, sys, time
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "real-time-audio-visual-zooming_amd")]
import torch
from avz import neural as N
dev = torch.device("cuda:0")
torch.manual_seed(0)
model = N.FreqPreservingUNet().eval().to(dev).to(memory_format=torch.channels_last)
x = torch.randn(256, 2, 513, 64, device=dev).contiguous(memory_format=torch.channels_last)
def t(fn, n=3):
    fn(); torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t0) / n * 1e3
with torch.no_grad():
    ref = model(x)
    print("fp32 CL heuristic   %.1f ms / 256 chunks" % t(lambda: model(x)), flush=True)
    torch.backends.cudnn.benchmark = True
    t0 = time.perf_counter(); out = model(x); torch.cuda.synchronize()
    print("find-mode first call %.1f s" % (time.perf_counter() - t0), flush=True)
    print("fp32 CL find mode   %.1f ms / 256 chunks" % t(lambda: model(x)), flush=True)
    print("  max |diff| vs heuristic %.2e" % (model(x) - ref).abs().max().item(), flush=True)
