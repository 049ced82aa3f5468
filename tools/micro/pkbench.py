"""Packed vs scalar fp32 register DFTs (tools/micro/pkbench.hip): FFT/us/CU of the arithmetic
alone, and the two transforms' largest difference on one set of inputs.
    hipcc -O3 -std=c++17 --offload-arch=gfx950 -fno-slp-vectorize -shared -fPIC \
        tools/micro/pkbench.hip -o tools/micro/libpkbench.so && python tools/micro/pkbench.py"""
import ctypes as ct
import os
import torch

here = os.path.dirname(os.path.abspath(__file__))
lib = ct.CDLL(os.path.join(here, "libpkbench.so"))
for f in (lib.pk_run,):
    f.argtypes = [ct.c_int, ct.c_void_p, ct.c_void_p, ct.c_int, ct.c_int]
lib.pk_check_run.argtypes = [ct.c_void_p, ct.c_void_p]
dev = torch.device("cuda")
inp = torch.randn(1 << 16, device=dev)
out = torch.empty(512 * 256, device=dev)
assert lib.pk_check_run(inp.data_ptr(), out.data_ptr()) == 0
torch.cuda.synchronize()
a, b = out[:4096], out[4096:8192]
print(f"check: max |scalar - packed| {float((a - b).abs().max()):.3e} (max |X| {float(a.abs().max()):.2f})")
iters, blocks = 400, 512
for packed in (0, 1, 0, 1):
    for _ in range(2):
        lib.pk_run(packed, inp.data_ptr(), out.data_ptr(), blocks, iters)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    assert lib.pk_run(packed, inp.data_ptr(), out.data_ptr(), blocks, iters) == 0
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3
    ffts = blocks * 8 * iters  # 4 waves x 2 lane groups, one 1024-pt FFT's arithmetic each
    print(f"{'packed' if packed else 'scalar':6s}: {us:8.1f} us  {ffts / us / 256:6.2f} FFT/us/CU")
