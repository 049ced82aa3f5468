// avz_spectral.hip — spectral-domain beamformers for callers that already hold an STFT
// (gfx950), and the solve-from-covariance stage export.
//
//  * batch_mvdr(Y[M,F,T], mask[F,T], f_bins, d_vectors, sigma) -> S[F,T]
//    (rt_av_zoom/core/tf_lite_version/inference.py:85-179): covariance weighted by
//    sqrt(1 - mask + 1e-10) (so 1 - mask + 1e-10 on R), normalised by sum(1 - mask) + 1e-6,
//    + sigma I, no low-frequency skip, w = R^-1 d / (d^H R^-1 d + 1e-10), S = w^H y; one
//    np.linalg.solve over all bins, so a singular bin sends EVERY bin of the call to the
//    fallback w~ = [1, 0]^T (then normalised) — AVZ_FALLBACK_BATCH.
//  * hybrid_hard_null_bf(Y, mask, f_bins) -> S (Final_pipeline/src/inference.py:28-98):
//    f < 200 Hz passes mic 0; else the hard null of hybrid_weights_d.
//
// Layout: up to 64 frames (the 2-s chunk items) 16 lanes per (item, bin) row, 4 rows per
// wave, frames held in registers between the covariance and the apply
// (avz_spectral_rows_kernel); longer spectra one wave per row, frames across lanes, the row
// re-read (L1/L2 hit) for the apply. The masked 2x2 covariance is accumulated per lane in
// fp64 and reduced across the row's lanes; the fp64 2x2 solve is shared by them.
// Algorithmic bytes: 2 x 8 B (Y) + 4 B (mask) + 8 B (S) = 28 B per TF-bin. An optional post-filter gain from
// the same mask (x max(M, floor) / x M) is fused into the store.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "avz_common.hpp"

namespace avz {

constexpr int kSpecThreads = 256;  // 4 waves = 4 rows per block

__device__ __forceinline__ double wave_sum_d(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int PF>
__device__ __forceinline__ float spec_gain(const ChainArgs& P, float M) {
  if constexpr (PF == PF_EXT_FLOOR) return fmaxf(M, P.pf_floor);
  else if constexpr (PF == PF_EXT_MUL) return M;
  else return 1.0f;
}

// S[t] = gain(M[t]) * (conj(w0) y0[t] + conj(w1) y1[t]) over the row's frames.
template <int PF>
__device__ __forceinline__ void spec_apply_row(const SpecArgs& S, const ChainArgs& P,
                                               const float2* y0, const float2* y1,
                                               const float* m, float2* out,
                                               const double (&w)[4], int lane) {
  for (int t = lane; t < S.frames; t += 64) {
    const float2 a = y0[t], e = y1[t];
    const double sr = w[0] * a.x + w[1] * a.y + w[2] * e.x + w[3] * e.y;
    const double si = w[0] * a.y - w[1] * a.x + w[2] * e.y - w[3] * e.x;
    const float g = spec_gain<PF>(P, m[t]);
    out[t] = make_float2((float)sr * g, (float)si * g);
  }
}

template <int N, bool HYB, int PF>
__global__ void __launch_bounds__(kSpecThreads) avz_spectral_kernel(SpecArgs S, ChainArgs P) {
  constexpr int F = N / 2 + 1;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * (kSpecThreads / 64) + wave;
  if (row >= (long long)S.batch * F) return;
  const int b = (int)(row / F), k = (int)(row % F);
  const float2* y0 = reinterpret_cast<const float2*>(S.Y) + b * S.y_sb + k * S.y_sf;
  const float2* y1 = y0 + S.y_sm;
  const float* m = S.M + b * S.m_sb + k * S.m_sf;
  double c[5] = {0, 0, 0, 0, 0};
  for (int t = lane; t < S.frames; t += 64) {
    const float2 a = y0[t], e = y1[t];
    const float mn = 1.0f - m[t];  // float32, as numpy's 1.0 - (float32 mask)
    const double wg = (double)mn + P.weight_eps;
    const double ar = a.x, ai = a.y, er = e.x, ei = e.y;
    c[0] = fma(wg, ar * ar + ai * ai, c[0]);
    c[1] = fma(wg, er * er + ei * ei, c[1]);
    c[2] = fma(wg, ar * er + ai * ei, c[2]);  // Re y0 conj(y1)
    c[3] = fma(wg, ai * er - ar * ei, c[3]);  // Im y0 conj(y1)
    c[4] += (double)mn;
  }
#pragma unroll
  for (int q = 0; q < 5; ++q) c[q] = wave_sum_d(c[q]);
  const double* d = S.steer + 4 * k;
  double w[4];
  if constexpr (HYB) {
    hybrid_weights_d(c, k, N, P, d[0], d[1], d[2], d[3], w);
  } else {
    bool sing = false;
    mvdr_weights_d(c, k, N, P, d[0], d[1], d[2], d[3], w, &sing);
    if (sing && P.singular_fallback == 2 && lane == 0) atomicOr(S.flag + b, 1);
  }
  if (lane == 0) {
    if (S.cov_out) {
#pragma unroll
      for (int q = 0; q < 5; ++q) S.cov_out[row * 5 + q] = c[q];
    }
    if (S.w_out) {
#pragma unroll
      for (int q = 0; q < 4; ++q) S.w_out[row * 4 + q] = (float)w[q];
    }
  }
  spec_apply_row<PF>(S, P, y0, y1, m, reinterpret_cast<float2*>(S.S) + b * S.s_sb + k * S.s_sf,
                     w, lane);
}

// Spectra of at most 64 frames (the chunk drivers' 2-s items): 16 lanes per (item, bin)
// row, 4 rows per wave, each lane holding its 4 frames in registers from the covariance
// pass to the apply (Y and the mask read from HBM once), the fp64 reduction over the row's
// 16 lanes and the fp64 solve shared by them (4 rows per wave instead of 1).
constexpr int kRowLanes = 16, kRowFpl = 4;  // 16 lanes x 4 frames = 64 frames per row
template <int N, bool HYB, int PF>
__global__ void __launch_bounds__(kSpecThreads) avz_spectral_rows_kernel(SpecArgs S, ChainArgs P) {
  constexpr int F = N / 2 + 1;
  const int sub = threadIdx.x & (kRowLanes - 1);
  const long long row = ((long long)blockIdx.x * kSpecThreads + threadIdx.x) / kRowLanes;
  const bool live = row < (long long)S.batch * F;
  const long long rr = live ? row : 0;  // a dead row group recomputes row 0, stores nothing
  const int b = (int)(rr / F), k = (int)(rr % F);
  const float2* y0 = reinterpret_cast<const float2*>(S.Y) + b * S.y_sb + k * S.y_sf;
  const float2* y1 = y0 + S.y_sm;
  const float* m = S.M + b * S.m_sb + k * S.m_sf;
  float2 a[kRowFpl], e[kRowFpl];
  float mv[kRowFpl];
#pragma unroll
  for (int j = 0; j < kRowFpl; ++j) {
    const int t = sub + kRowLanes * j;
    const bool ok = t < S.frames;
    a[j] = ok ? y0[t] : make_float2(0.f, 0.f);
    e[j] = ok ? y1[t] : make_float2(0.f, 0.f);
    mv[j] = ok ? m[t] : 1.0f;  // absent frame: noise weight 1 - M = 0, |y|^2 = 0
  }
  double c[5] = {0, 0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < kRowFpl; ++j) {
    const float mn = 1.0f - mv[j];  // float32, as numpy's 1.0 - (float32 mask)
    const double wg = (double)mn + P.weight_eps;
    const double ar = a[j].x, ai = a[j].y, er = e[j].x, ei = e[j].y;
    c[0] = fma(wg, ar * ar + ai * ai, c[0]);
    c[1] = fma(wg, er * er + ei * ei, c[1]);
    c[2] = fma(wg, ar * er + ai * ei, c[2]);  // Re y0 conj(y1)
    c[3] = fma(wg, ai * er - ar * ei, c[3]);  // Im y0 conj(y1)
    c[4] += (double)mn;
  }
#pragma unroll
  for (int q = 0; q < 5; ++q)
    for (int o = kRowLanes / 2; o > 0; o >>= 1) c[q] += __shfl_xor(c[q], o, 64);
  const double* d = S.steer + 4 * k;
  double w[4];
  if constexpr (HYB) {
    hybrid_weights_d(c, k, N, P, d[0], d[1], d[2], d[3], w);
  } else {
    bool sing = false;
    mvdr_weights_d(c, k, N, P, d[0], d[1], d[2], d[3], w, &sing);
    if (live && sub == 0 && sing && P.singular_fallback == 2) atomicOr(S.flag + b, 1);
  }
  if (!live) return;
  if (sub == 0) {
    if (S.cov_out) {
#pragma unroll
      for (int q = 0; q < 5; ++q) S.cov_out[row * 5 + q] = c[q];
    }
    if (S.w_out) {
#pragma unroll
      for (int q = 0; q < 4; ++q) S.w_out[row * 4 + q] = (float)w[q];
    }
  }
  float2* out = reinterpret_cast<float2*>(S.S) + b * S.s_sb + k * S.s_sf;
#pragma unroll
  for (int j = 0; j < kRowFpl; ++j) {
    const int t = sub + kRowLanes * j;
    if (t < S.frames) {
      const double sr = w[0] * a[j].x + w[1] * a[j].y + w[2] * e[j].x + w[3] * e[j].y;
      const double si = w[0] * a[j].y - w[1] * a[j].x + w[2] * e[j].y - w[3] * e[j].x;
      const float g = spec_gain<PF>(P, mv[j]);
      out[t] = make_float2((float)sr * g, (float)si * g);
    }
  }
}

// batch_mvdr's fallback for the items whose solve met a singular bin: every bin of the
// item is redone with w~ = [1, 0]^T (normalised). One block per item, a no-op unless the
// item's flag is set (rare), so the launch costs a few microseconds, not a row sweep.
template <int N, int PF>
__global__ void __launch_bounds__(kSpecThreads) avz_spectral_fixup_kernel(SpecArgs S, ChainArgs P) {
  constexpr int F = N / 2 + 1;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int b = blockIdx.x;
  if (b >= S.batch || S.flag[b] == 0) return;
  for (int k = wave; k < F; k += kSpecThreads / 64) {
    const long long row = (long long)b * F + k;
    double w[4];
    batch_fallback_weights_d(S.steer[4 * k], S.steer[4 * k + 1], w);
    if (lane == 0 && S.w_out) {
#pragma unroll
      for (int q = 0; q < 4; ++q) S.w_out[row * 4 + q] = (float)w[q];
    }
    const float2* y0 = reinterpret_cast<const float2*>(S.Y) + b * S.y_sb + k * S.y_sf;
    spec_apply_row<PF>(S, P, y0, y0 + S.y_sm, S.M + b * S.m_sb + k * S.m_sf,
                       reinterpret_cast<float2*>(S.S) + b * S.s_sb + k * S.s_sf, w, lane);
  }
}

// Solve stage export: w_out[b][k] from caller covariance sums cov_in[b][k][5] (the cov_out
// layout: sum m|y0|^2, sum m|y1|^2, Re/Im sum m y0 conj(y1), sum m).
template <int N, bool HYB>
__global__ void __launch_bounds__(256) avz_solve_cov_kernel(SpecArgs S, ChainArgs P) {
  constexpr int F = N / 2 + 1;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)S.batch * F) return;
  const int b = (int)(i / F), k = (int)(i % F);
  double c[5];
#pragma unroll
  for (int q = 0; q < 5; ++q) c[q] = S.cov_in[i * 5 + q];
  const double* d = S.steer + 4 * k;
  double w[4];
  if constexpr (HYB) {
    hybrid_weights_d(c, k, N, P, d[0], d[1], d[2], d[3], w);
  } else {
    bool sing = false;
    mvdr_weights_d(c, k, N, P, d[0], d[1], d[2], d[3], w, &sing);
    if (sing && P.singular_fallback == 2) atomicOr(S.flag + b, 1);
  }
  reinterpret_cast<float4*>(S.w_out)[i] = make_float4((float)w[0], (float)w[1], (float)w[2], (float)w[3]);
}

template <int N>
__global__ void __launch_bounds__(256) avz_solve_cov_fixup_kernel(SpecArgs S) {
  constexpr int F = N / 2 + 1;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)S.batch * F) return;
  const int b = (int)(i / F), k = (int)(i % F);
  if (S.flag[b] == 0) return;
  double w[4];
  batch_fallback_weights_d(S.steer[4 * k], S.steer[4 * k + 1], w);
  reinterpret_cast<float4*>(S.w_out)[i] = make_float4((float)w[0], (float)w[1], (float)w[2], (float)w[3]);
}

}  // namespace avz

using namespace avz;

template <int N, bool HYB, int PF>
static void launch_spec_t(const SpecArgs* s, const ChainArgs* p, hipStream_t st) {
  constexpr int F = N / 2 + 1;
  const long long rows = (long long)s->batch * F;
  if (s->frames <= kRowLanes * kRowFpl) {
    const long long per_block = kSpecThreads / kRowLanes;  // 16 rows
    hipLaunchKernelGGL((avz_spectral_rows_kernel<N, HYB, PF>),
                       dim3((unsigned)((rows + per_block - 1) / per_block)), dim3(kSpecThreads), 0,
                       st, *s, *p);
  } else {
    hipLaunchKernelGGL((avz_spectral_kernel<N, HYB, PF>), dim3((unsigned)((rows + 3) / 4)),
                       dim3(kSpecThreads), 0, st, *s, *p);
  }
  if (!HYB && p->singular_fallback == 2)
    hipLaunchKernelGGL((avz_spectral_fixup_kernel<N, PF>), dim3((unsigned)s->batch),
                       dim3(kSpecThreads), 0, st, *s, *p);
}

template <int N, bool HYB>
static int launch_spec_pf(const SpecArgs* s, const ChainArgs* p, hipStream_t st) {
  switch (p->postfilter) {
    case PF_NONE: launch_spec_t<N, HYB, PF_NONE>(s, p, st); break;
    case PF_EXT_FLOOR: launch_spec_t<N, HYB, PF_EXT_FLOOR>(s, p, st); break;
    case PF_EXT_MUL: launch_spec_t<N, HYB, PF_EXT_MUL>(s, p, st); break;
    default: return -4;
  }
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int avz_launch_spectral(int n_fft, const SpecArgs* s, const ChainArgs* p, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (s->batch <= 0) return 0;
  if (p->singular_fallback == 2 &&
      hipMemsetAsync(s->flag, 0, sizeof(int) * s->batch, st) != hipSuccess)
    return -3;
  const bool hyb = p->beamformer == BF_HYBRID_NULL;
  if (n_fft == 1024) return hyb ? launch_spec_pf<1024, true>(s, p, st) : launch_spec_pf<1024, false>(s, p, st);
  if (n_fft == 512) return hyb ? launch_spec_pf<512, true>(s, p, st) : launch_spec_pf<512, false>(s, p, st);
  return -4;
}

template <int N>
static int launch_solve_cov_t(const SpecArgs* s, const ChainArgs* p, hipStream_t st) {
  constexpr int F = N / 2 + 1;
  const long long n = (long long)s->batch * F;
  const dim3 grid((unsigned)((n + 255) / 256));
  if (p->beamformer == BF_HYBRID_NULL) {
    hipLaunchKernelGGL((avz_solve_cov_kernel<N, true>), grid, dim3(256), 0, st, *s, *p);
  } else {
    hipLaunchKernelGGL((avz_solve_cov_kernel<N, false>), grid, dim3(256), 0, st, *s, *p);
    if (p->singular_fallback == 2)
      hipLaunchKernelGGL(avz_solve_cov_fixup_kernel<N>, grid, dim3(256), 0, st, *s);
  }
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int avz_launch_solve_cov(int n_fft, const SpecArgs* s, const ChainArgs* p, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (s->batch <= 0) return 0;
  if (p->singular_fallback == 2 &&
      hipMemsetAsync(s->flag, 0, sizeof(int) * s->batch, st) != hipSuccess)
    return -3;
  if (n_fft == 1024) return launch_solve_cov_t<1024>(s, p, st);
  if (n_fft == 512) return launch_solve_cov_t<512>(s, p, st);
  return -4;
}
