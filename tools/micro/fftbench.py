"""FFT-phase throughput (FFTs per microsecond per CU) for several FFT shapes / wave
counts. python tools/micro/fftbench.py (needs libfftbench.so next to it)."""
import ctypes as ct
import os
import torch

here = os.path.dirname(os.path.abspath(__file__))
lib = ct.CDLL(os.path.join(here, "libfftbench.so"))
lib.run_bench.argtypes = [ct.c_int, ct.c_void_p, ct.c_void_p, ct.c_int, ct.c_int]
dev = torch.device("cuda")
inp = torch.randn(512 * 131072, device=dev)  # 256 MB: variants 14-16 stream from it
out = torch.empty(1024 * 1024, device=dev)
iters = 200
names = {0: "x2 (32 pts/lane), 8 waves/block", 1: "x1 (16 pts/lane), 16 waves/block",
         2: "x1 (16 pts/lane), 8 waves/block", 3: "x2, 4 waves/block (x2 blocks/CU)",
         4: "x2 FFT only, 4 waves/block", 5: "x2 + bpermute/swap bins, 4 w/b",
         6: "x2 + wave-local LDS spectrum, 4 w/b", 7: "x2 arithmetic + LDS twiddles, no transpose",
         8: "x2 arithmetic only (no LDS at all)", 9: "x2 FFT only, addtid planar transpose",
         10: "pairs: FFT + in-register IBM bins, LDS tw", 11: "current: FFT + LDS bin phase, LDS tw",
         12: "pairs, register twiddles", 13: "current, register twiddles",
         14: "current + next-step loads (512 KB/block)", 15: "current + loads (16 KB/block, cached)",
         16: "current + loads not feeding the FFT", 17: "current + dwordx2 loads (same bytes)",
         18: "current + one channel's loads", 19: "current + 1/8 of the loads",
         20: "LDS tw, one channel's loads, two steps ahead", 21: "LDS tw, one channel's loads, one step ahead",
         22: "pairs + LDS-DMA staged frames (4 streams)",
         23: "p3 FFT only (16 pts/lane, 2 transposes), 4 w/b x4", 24: "p3 + wave-local spectrum round trip",
         25: "x1 FFT only (permlane32), 4 w/b x4",
         26: "x2 FFT only, 8 w/b, waves in phase", 27: "x2 FFT only, 8 w/b, SIMD pairs half an FFT apart",
         28: "x2 FFT only, addtid planar transpose, no drain",
         29: "x2 FFT only, register (DPP) transpose"}
ffts_per_block = {29: 8, 28: 8, 26: 16, 27: 16, 23: 4, 24: 4, 25: 4, 0: 16, 1: 16, 2: 8, 3: 8, 4: 8, 5: 8, 6: 8, 7: 8, 8: 8, 9: 8, 10: 8, 11: 8, 12: 8, 13: 8, 14: 8, 15: 8, 16: 8, 17: 8, 18: 8, 19: 8, 20: 8, 21: 8, 22: 8}
import sys
VARS = [(int(a.split(':')[0]), int(a.split(':')[1])) for a in sys.argv[1:]] or [(4, 512), (23, 1024), (24, 1024), (25, 1024)]
for v, blocks in VARS:
    for _ in range(2):
        lib.run_bench(v, inp.data_ptr(), out.data_ptr(), blocks, iters)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    assert lib.run_bench(v, inp.data_ptr(), out.data_ptr(), blocks, iters) == 0
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3
    ffts = blocks * ffts_per_block[v] * iters
    print(f"{names[v]:40s} blocks={blocks:4d}: {us:8.1f} us  {ffts / us / 256:6.2f} FFT/us/CU  "
          f"({us / iters:.2f} us per phase)")
