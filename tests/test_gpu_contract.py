"""ABI contract of avz_mvdr_batch (include/avz.h): calls with distinct caller workspaces
run concurrently on two streams and equal their serial runs; a device length above the
host max_len is clamped (no write outside the caller's rows or workspace); an undersized
external mask is rejected before any launch."""
import ctypes as ct

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N, S = 1024, 64000


def _ibm_plan(avz, max_batch, max_samples=S):
    return avz.MVDRPlan(n_fft=N, sigma=1.0, mic_d=0.01, mask="ibm", postfilter="ibm",
                        normalize="peak", max_batch=max_batch, max_samples=max_samples)


def test_two_streams_distinct_workspaces(gpu_device):
    import avz
    from avz import synth
    k = 48
    d = lambda a: torch.from_numpy(a).to(gpu_device)  # noqa: E731
    batches = [tuple(d(a) for a in synth.make_batch(k, start=s, n_samples=S, n_interferers=2))
               for s in (0, 1000)]
    plan = _ibm_plan(avz, k)
    ws = [plan.alloc_workspace(k, S, gpu_device) for _ in batches]
    serial = []
    for (m, t, i), w in zip(batches, ws):
        o, p = plan.run(m, ref_tgt=t, ref_int=i, workspace=w)
        serial.append((o.clone(), p.clone()))
    # the plan's own workspace gives the same result as a caller workspace
    o0, p0 = plan.run(*batches[0][:1], ref_tgt=batches[0][1], ref_int=batches[0][2])
    assert torch.equal(o0, serial[0][0]) and torch.equal(p0, serial[0][1])
    streams = [torch.cuda.Stream(gpu_device) for _ in batches]
    outs = [plan.alloc_out(k, S, gpu_device) for _ in batches]
    peaks = [torch.empty(k, dtype=torch.float32, device=gpu_device) for _ in batches]
    torch.cuda.synchronize()
    for rep in range(4):
        for j, ((m, t, i), w, st) in enumerate(zip(batches, ws, streams)):
            plan.run(m, ref_tgt=t, ref_int=i, workspace=w, out=outs[j], peak=peaks[j],
                     stream=st)
        torch.cuda.synchronize()
        for j in range(2):
            assert torch.equal(outs[j], serial[j][0]), (rep, j)
            assert torch.equal(peaks[j], serial[j][1]), (rep, j)


def test_workspace_too_small_rejected(gpu_device):
    import avz
    plan = _ibm_plan(avz, 4)
    x = torch.zeros((4, 2, S), device=gpu_device)
    r = torch.zeros((4, S), device=gpu_device)
    small = torch.empty(plan.workspace_bytes(4, S) - 256, dtype=torch.uint8, device=gpu_device)
    with pytest.raises(avz.AvzError):
        plan.run(x, ref_tgt=r, ref_int=r, workspace=small)


def test_device_length_above_max_len_is_clamped(gpu_device):
    import avz
    rng = np.random.default_rng(3)
    L, B = 16000, 2
    guard = 4096
    plan = _ibm_plan(avz, B)
    x = torch.from_numpy(0.1 * rng.standard_normal((B, 2, L)).astype(np.float32)).to(gpu_device)
    t = torch.from_numpy(0.1 * rng.standard_normal((B, L)).astype(np.float32)).to(gpu_device)
    i = torch.from_numpy(0.1 * rng.standard_normal((B, L)).astype(np.float32)).to(gpu_device)
    n_out = plan.out_len(L)
    sentinel = 12345.0
    out_big = torch.full((B, n_out + guard), sentinel, device=gpu_device)
    out = out_big[:, :n_out]
    wbytes = plan.workspace_bytes(B, L)
    ws_big = torch.full((wbytes + (1 << 20),), 0x5A, dtype=torch.uint8, device=gpu_device)
    good = torch.tensor([L, L], dtype=torch.int32, device=gpu_device)
    ref, ref_peak = plan.run(x, good, max_len=L, ref_tgt=t, ref_int=i)
    ref, ref_peak = ref[:, :n_out].clone(), ref_peak.clone()
    bad = torch.tensor([L, 10 ** 6], dtype=torch.int32, device=gpu_device)
    _, peak = plan.run(x, bad, max_len=L, ref_tgt=t, ref_int=i, out=out,
                       workspace=ws_big[:wbytes])
    torch.cuda.synchronize()
    assert torch.all(out_big[:, n_out:] == sentinel), "write past the output row"
    assert torch.all(ws_big[wbytes:] == 0x5A), "write past the workspace"
    assert torch.equal(out, ref) and torch.equal(peak, ref_peak)


def test_undersized_external_mask_rejected(gpu_device):
    import avz
    from avz import _lib
    plan = avz.MVDRPlan(n_fft=N, sigma=1e-5, mic_d=0.01, mask="external", postfilter="floor",
                        normalize="none", max_batch=2, max_samples=32000)
    x = torch.zeros((2, 2, 32000), device=gpu_device)
    T = plan.frames(32000)
    for shape in ((2, plan.F, T - 1), (2, plan.F - 1, T), (1, plan.F, T)):
        with pytest.raises(ValueError):
            plan.run(x, ext_mask=torch.zeros(shape, device=gpu_device))
    # the ABI itself checks the extents it is given
    m = torch.zeros((2, plan.F, T), device=gpu_device)
    lens = torch.full((2,), 32000, dtype=torch.int32, device=gpu_device)
    out = plan.alloc_out(2, 32000, gpu_device)
    a = _lib.AvzBatchArgs()
    a.batch, a.len, a.max_len = 2, lens.data_ptr(), 32000
    a.mix, a.mix_stride, a.ch_stride = x.data_ptr(), x.stride(0), x.stride(1)
    a.ext_mask = m.data_ptr()
    a.mask_stride_b, a.mask_stride_f, a.mask_stride_t = m.stride()
    a.out, a.out_stride = out.data_ptr(), out.stride(0)
    a.mask_bins, a.mask_frames = plan.F, T - 1
    s = ct.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert _lib.lib.avz_mvdr_batch(plan._h, ct.byref(a), s) == _lib.AVZ_ERR_SHAPE
    a.mask_frames = T
    assert _lib.lib.avz_mvdr_batch(plan._h, ct.byref(a), s) == _lib.AVZ_OK
    torch.cuda.synchronize()
