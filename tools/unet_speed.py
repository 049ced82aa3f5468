"""U-Net (configs[4]) forward speed on the device: fp32 default / channels_last / bf16."""
import os, sys, time
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "real-time-audio-visual-zooming_amd")]
import torch
from avz import neural as N
dev = torch.device("cuda:0")
torch.manual_seed(0)
model = N.FreqPreservingUNet().eval().to(dev)
x = torch.randn(256, 2, 513, 64, device=dev)
def t(fn, n=3):
    fn(); torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t0) / n * 1e3
with torch.no_grad():
    ref = model(x)
    print("fp32 default        %.1f ms / 256 chunks" % t(lambda: model(x)), flush=True)
    mcl = model.to(memory_format=torch.channels_last); xcl = x.to(memory_format=torch.channels_last)
    print("fp32 channels_last  %.1f ms" % t(lambda: mcl(xcl)), flush=True)
    out = mcl(xcl); print("  max diff vs default %.2e" % (out - ref).abs().max().item())
    with torch.autocast("cuda", dtype=torch.bfloat16):
        print("bf16 autocast CL    %.1f ms" % t(lambda: mcl(xcl)), flush=True)
        ob = mcl(xcl).float()
    print("  bf16 max diff %.2e" % (ob - ref).abs().max().item(), flush=True)
