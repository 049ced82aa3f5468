"""ctypes binding of libavz.so (include/avz.h). Fails loudly when the library is missing.

There is no CPU fallback anywhere in ``avz``: if the HIP library cannot be loaded
the import of this module raises.
"""
from __future__ import annotations

import ctypes as ct
import os

# PyTorch-ROCm ships its own libamdhip64 (SONAME libamdhip64.so.7). Loading torch
# first makes libavz.so's NEEDED libamdhip64.so.7 resolve to that same runtime, so
# torch's device pointers and stream handles are valid for our launches. Loading
# libavz first would map a second HIP runtime (/opt/rocm) into the process.
import torch  # noqa: F401,E402

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("AVZ_LIB", os.path.join(_HERE, "libavz.so"))

AVZ_OK = 0
AVZ_ERR_ARG = -1
AVZ_ERR_SHAPE = -2
AVZ_ERR_HIP = -3
AVZ_ERR_UNSUPPORTED = -4
AVZ_ERR_ALIGN = -5

MASK_IBM, MASK_IPD, MASK_EXTERNAL, MASK_ONES = 0, 1, 2, 3
PF_NONE, PF_IBM_TARGET, PF_EXT_FLOOR, PF_EXT_MUL, PF_IRM = 0, 1, 2, 3, 4
FALLBACK_MIC0, FALLBACK_MEAN, FALLBACK_BATCH = 0, 1, 2
NORM_NONE, NORM_PEAK = 0, 1
BF_MVDR, BF_HYBRID_NULL = 0, 1
FEAT_LOGMAG_IPD, FEAT_TFLITE = 1, 2

EXPORTED = [
    "avz_plan_create", "avz_plan_destroy", "avz_plan_get_config", "avz_num_frames",
    "avz_mvdr_batch", "avz_plan_set_timing", "avz_plan_get_timing", "avz_stft",
    "avz_plan_set_timing_period",
    "avz_chunk_split", "avz_chunk_merge", "avz_mask_features", "avz_srp_scan",
    "avz_projection_metrics", "avz_scene_workspace_bytes", "avz_scene_mix", "avz_strerror",
    "avz_last_hip_error", "avz_version", "avz_mvdr_workspace_bytes",
    "avz_mvdr_covariance", "avz_solve_covariance", "avz_apply_istft", "avz_beamform_spectral",
    "avz_istft", "avz_scene_generate_workspace_bytes", "avz_scene_generate",
    "avz_projection_metrics_scaled", "avz_plan_set_ibm_stats", "avz_plan_set_diagnostics",
    "avz_ibm_window",
]


class AvzConfig(ct.Structure):
    _fields_ = [
        ("fs", ct.c_int), ("n_fft", ct.c_int), ("hop", ct.c_int),
        ("sigma", ct.c_double), ("angle_deg", ct.c_double), ("mic_d", ct.c_double),
        ("c_sound", ct.c_double), ("fmin_hz", ct.c_double),
        ("mask_mode", ct.c_int), ("postfilter", ct.c_int),
        ("pf_floor", ct.c_double), ("weight_eps", ct.c_double),
        ("normalize", ct.c_int), ("norm_eps", ct.c_double),
        ("max_batch", ct.c_int), ("max_samples", ct.c_int),
        ("beamformer", ct.c_int), ("bypass_hz", ct.c_double), ("cond_max", ct.c_double),
        ("singular_fallback", ct.c_int), ("ibm_kappa", ct.c_double),
    ]


class AvzBatchArgs(ct.Structure):
    _fields_ = [
        ("batch", ct.c_int), ("len", ct.c_void_p), ("max_len", ct.c_int),
        ("mix", ct.c_void_p), ("mix_stride", ct.c_longlong), ("ch_stride", ct.c_longlong),
        ("ref_tgt", ct.c_void_p), ("ref_int", ct.c_void_p), ("ref_stride", ct.c_longlong),
        ("ext_mask", ct.c_void_p), ("mask_stride_b", ct.c_longlong),
        ("mask_stride_f", ct.c_longlong), ("mask_stride_t", ct.c_longlong),
        ("out", ct.c_void_p), ("out_stride", ct.c_longlong), ("peak", ct.c_void_p),
        ("cov_out", ct.c_void_p), ("w_out", ct.c_void_p),
        ("mask_bins", ct.c_int), ("mask_frames", ct.c_int),
        ("workspace", ct.c_void_p), ("workspace_bytes", ct.c_longlong),
    ]


class AvzSpectralArgs(ct.Structure):
    _fields_ = [
        ("batch", ct.c_int), ("frames", ct.c_int),
        ("Y", ct.c_void_p), ("y_stride_b", ct.c_longlong), ("y_stride_m", ct.c_longlong),
        ("y_stride_f", ct.c_longlong),
        ("mask", ct.c_void_p), ("mask_stride_b", ct.c_longlong), ("mask_stride_f", ct.c_longlong),
        ("steer", ct.c_void_p),
        ("S", ct.c_void_p), ("s_stride_b", ct.c_longlong), ("s_stride_f", ct.c_longlong),
        ("cov_out", ct.c_void_p), ("w_out", ct.c_void_p), ("fallback", ct.c_void_p),
    ]


class AvzError(RuntimeError):
    pass


ABI_VERSION = 3  # INTEGRATION.md section 4 (3: avz_config.ibm_kappa)


def hip_runtimes_mapped() -> list:
    """Paths of every libamdhip64 mapped into this process."""
    paths = set()
    try:
        with open("/proc/self/maps") as fh:
            for line in fh:
                if "libamdhip64" in line:
                    paths.add(os.path.realpath(line.split()[-1]))
    except OSError:
        pass
    return sorted(paths)


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libavz.so not found at {LIB_PATH}; run __graft_entry__.build() "
                          "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
    lib = ct.CDLL(LIB_PATH)
    rts = hip_runtimes_mapped()
    if len(rts) > 1:
        raise ImportError(f"two HIP runtimes mapped into the process: {rts}")
    P = ct.c_void_p
    lib.avz_plan_create.argtypes = [ct.POINTER(P), ct.POINTER(AvzConfig)]
    lib.avz_plan_destroy.argtypes = [P]
    lib.avz_plan_get_config.argtypes = [P, ct.POINTER(AvzConfig)]
    lib.avz_num_frames.argtypes = [P, ct.c_int]
    lib.avz_mvdr_batch.argtypes = [P, ct.POINTER(AvzBatchArgs), P]
    lib.avz_mvdr_workspace_bytes.argtypes = [P, ct.c_int, ct.c_int]
    lib.avz_mvdr_workspace_bytes.restype = ct.c_longlong
    lib.avz_mvdr_covariance.argtypes = [P, ct.POINTER(AvzBatchArgs), P]
    lib.avz_solve_covariance.argtypes = [P, ct.c_int, P, P, P, P, P]
    lib.avz_apply_istft.argtypes = [P, ct.POINTER(AvzBatchArgs), P, P]
    lib.avz_beamform_spectral.argtypes = [P, ct.POINTER(AvzSpectralArgs), P]
    lib.avz_istft.argtypes = [P, ct.c_int, ct.c_int, P, ct.c_longlong, ct.c_longlong, P,
                              ct.c_longlong, P, P, ct.c_longlong, P]
    for name in ("avz_mvdr_covariance", "avz_solve_covariance", "avz_apply_istft",
                 "avz_beamform_spectral", "avz_istft"):
        getattr(lib, name).restype = ct.c_int
    lib.avz_stft.argtypes = [P, ct.c_int, ct.c_int, P, ct.c_int, P, ct.c_longlong, ct.c_longlong,
                             P, ct.c_longlong, ct.c_longlong, ct.c_longlong, P]
    I, LL = ct.c_int, ct.c_longlong
    lib.avz_plan_set_timing.argtypes = [P, I]
    lib.avz_plan_set_timing_period.argtypes = [P, I]
    lib.avz_plan_get_timing.argtypes = [P, ct.POINTER(ct.c_double), ct.POINTER(I)]
    lib.avz_plan_set_ibm_stats.argtypes = [P, P]
    lib.avz_plan_set_diagnostics.argtypes = [P, I, I]
    lib.avz_ibm_window.argtypes = [I, ct.POINTER(ct.c_float)]
    lib.avz_chunk_split.argtypes = [I, I, I, P, P, P, P, LL, LL, P, LL, LL, P]
    lib.avz_chunk_merge.argtypes = [I, I, I, I, P, P, P, LL, P, LL, P, I, ct.c_double, P]
    lib.avz_mask_features.argtypes = [P, I, I, P, I, P, LL, LL, P, LL, LL, LL, LL, P]
    D = ct.c_double
    lib.avz_srp_scan.argtypes = [P, I, P, I, P, LL, LL, I, D, D, D, D, P, P]
    lib.avz_projection_metrics.argtypes = [I, I, P, P, LL, P, LL, P, LL, P, P, P]
    lib.avz_projection_metrics_scaled.argtypes = [I, I, P, P, LL, P, D, P, LL, P, LL, P, P, P]
    lib.avz_scene_workspace_bytes.argtypes = [I, I, I]
    lib.avz_scene_workspace_bytes.restype = LL
    lib.avz_scene_mix.argtypes = [I, I, I, P, P, P, D, D, D, D, D, P, LL, LL, P, P, LL, P, LL, P]
    lib.avz_scene_generate_workspace_bytes.argtypes = [I, I, I]
    lib.avz_scene_generate_workspace_bytes.restype = LL
    lib.avz_scene_generate.argtypes = [I, LL, I, I, ct.c_uint, D, D, D, D, D, P, LL, LL, P, P, LL,
                                       P, LL, P]
    lib.avz_strerror.argtypes = [ct.c_int]
    lib.avz_strerror.restype = ct.c_char_p
    lib.avz_last_hip_error.restype = ct.c_char_p
    for name in ("avz_plan_create", "avz_plan_destroy", "avz_plan_get_config", "avz_num_frames",
                 "avz_mvdr_batch", "avz_stft", "avz_chunk_split", "avz_chunk_merge",
                 "avz_plan_set_timing", "avz_plan_get_timing", "avz_mask_features",
                 "avz_plan_set_timing_period",
                 "avz_srp_scan", "avz_projection_metrics", "avz_scene_mix",
                 "avz_scene_generate", "avz_projection_metrics_scaled", "avz_version",
                 "avz_plan_set_ibm_stats", "avz_plan_set_diagnostics", "avz_ibm_window"):
        getattr(lib, name).restype = ct.c_int
    if lib.avz_version() != ABI_VERSION:  # the struct layouts above are version 3's
        raise ImportError(f"libavz ABI version {lib.avz_version()} != {ABI_VERSION} "
                          "(AvzBatchArgs / AvzSpectralArgs layouts); rebuild")
    return lib


lib = _load()


def check(rc: int, what: str) -> int:
    if rc < 0:
        msg = lib.avz_strerror(rc).decode()
        if rc == AVZ_ERR_HIP:
            msg += ": " + lib.avz_last_hip_error().decode()
        raise AvzError(f"{what} failed ({rc}): {msg}")
    return rc
