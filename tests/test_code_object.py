"""Resource usage of the shipped kernels, read from the built libavz.so's gfx950 code object
(AMDGPU metadata note): no kernel may use scratch (a spill path runs far slower than the
register path the kernels were tuned for), and the chain kernels must keep the occupancy
their launch geometry assumes. CPU only: the code object is unbundled with the ROCm LLVM
tools, nothing runs on a GPU."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import code_object  # noqa: E402

LIB = code_object.DEFAULT_LIB

pytestmark = pytest.mark.skipif(
    not (os.path.exists(LIB) and os.path.exists(os.path.join(code_object.LLVM, "llvm-readelf"))),
    reason="libavz.so not built or ROCm LLVM tools absent")


@pytest.fixture(scope="module")
def kernels():
    res = code_object.resources(LIB)
    names = code_object.demangle(list(res))
    return dict(zip(names, res.values()))


def test_every_kernel_is_listed(kernels):
    # the chain, the stage exports and the around-the-chain kernels are all in the library
    for k in ("avz_analysis_kernel", "avz_solve_kernel", "avz_synthesis_kernel",
              "avz_synthesis_utt_kernel", "avz_synthesis_utt512_kernel", "avz_finalize_kernel", "avz_stft_kernel", "avz_metrics_sums_kernel",
              "avz_spectral_rows_kernel", "scene_ar_kernel"):
        assert any(k in n for n in kernels), k


def test_no_kernel_uses_scratch(kernels):
    spill = {n: (r["scratch"], r["vgpr_spill"], r["sgpr_spill"]) for n, r in kernels.items()
             if r["scratch"] != 0 or r["vgpr_spill"] > 0}
    assert not spill, spill


def test_chain_kernels_fit_two_waves_per_simd(kernels):
    # 256-thread blocks at two per CU (N = 1024 analysis / synthesis, N = 512 synthesis) and
    # the one 512-thread per-utterance synthesis block per CU (both sizes) need <= 256 VGPRs; the
    # three-block N = 512 analysis needs <= 168
    for n, r in kernels.items():
        if "avz_analysis_kernel<512" in n:
            assert r["vgpr"] + max(r["agpr"], 0) <= 168, (n, r)
        elif any(k in n for k in ("avz_analysis_kernel", "avz_synthesis_kernel",
                                  "avz_synthesis_utt_kernel", "avz_synthesis_utt512_kernel")):
            assert r["vgpr"] + max(r["agpr"], 0) <= 256, (n, r)
