// avz_common.hpp — device helpers shared by the MVDR kernels (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#include "avz_fft.hpp"
#include "avz_internal.h"

namespace avz {

typedef __amdgpu_buffer_rsrc_t rsrc_t;

__device__ __forceinline__ rsrc_t make_rsrc(const float* p, long long n_floats) {
  long long bytes = (p == nullptr || n_floats <= 0) ? 0 : n_floats * 4;
  if (bytes > 0x7fffffffLL) bytes = 0x7fffffffLL;
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ float bload(rsrc_t r, int elem) {
  // Offsets >= the descriptor's byte length read 0: scipy's zero extension/padding.
  // A negative index becomes the largest dword offset (always out of range) via a
  // select, so no voffset + immediate split can depend on 32-bit wraparound.
  const unsigned off = (elem < 0) ? 0xfffffffcu : (unsigned)elem * 4u;
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
}

// Diagnostic build only (-DAVZ_STAMPS): wave 0 accumulates s_memrealtime (100 MHz)
// deltas per phase into g_stamps[linear block id][16] (phase lists: tools/phase_profile.py).
#ifdef AVZ_STAMPS
#ifndef AVZ_STAMP_WAVE  // the wave whose lane 0 stamps
#define AVZ_STAMP_WAVE 0
#endif
static __device__ unsigned long long* g_stamps;
#define AVZ_STAMP_DECL() unsigned long long stamp_prev = 0
#define AVZ_STAMP_INIT() stamp_prev = __builtin_amdgcn_s_memrealtime()
#define AVZ_STAMP(i)                                                        \
  do {                                                                      \
    if (threadIdx.x == 64 * AVZ_STAMP_WAVE && g_stamps) {                   \
      const unsigned long long now_ = __builtin_amdgcn_s_memrealtime();     \
      atomicAdd(g_stamps + (blockIdx.y * gridDim.x + blockIdx.x) * 16 + (i), now_ - stamp_prev); \
      stamp_prev = now_;                                                    \
    }                                                                       \
  } while (0)
#else
#define AVZ_STAMP_DECL() (void)0
#define AVZ_STAMP_INIT() (void)0
#define AVZ_STAMP(i) (void)0
#endif
// Diagnostic build only (-DAVZ_XTRACE: the g_stamps buffer without the phase stamps): thread 0
// stores absolute s_memrealtime ticks or counts into g_stamps[block][i] (tools/xtrace.py).
#ifdef AVZ_XTRACE
#ifndef AVZ_STAMPS
static __device__ unsigned long long* g_stamps;
#endif
#define AVZ_XT(i, v)                                                                    \
  do {                                                                                  \
    if (threadIdx.x == 0 && g_stamps)                                                   \
      g_stamps[(blockIdx.y * gridDim.x + blockIdx.x) * 16 + (i)] = (unsigned long long)(v); \
  } while (0)
#else
#define AVZ_XT(i, v) (void)0
#endif

// Unchecked-sign form for a wave whose samples are all at index >= 0: the offset is a
// plain multiple of 4 so the per-register constant folds into the instruction's
// immediate offset (one address VGPR for all of a lane's loads).
__device__ __forceinline__ float bload_nn(rsrc_t r, int elem) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, elem * 4, 0, 0));
}

// Hide a value's provenance from the optimiser: per-iteration recomputation of
// lane-constant terms (window weights) then stays in the loop instead of being hoisted
// out and held in (or spilled from) registers for the whole kernel.
__device__ __forceinline__ void opaque(float& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void opaque_i(int& x) { asm volatile("" : "+v"(x)); }

// LDS-only barrier: leaves global loads (the next frame's prefetch) in flight.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

template <int N>
struct KCfg;
template <>
struct KCfg<1024> {
  using Fft = Fft1024x2;
  static constexpr int PPL = Fft::PPL;       // complex points per lane
  static constexpr int FPW = 2;              // FFTs per wave (lane groups of 32)
  static constexpr int GROUP_BYTES = Fft::GROUP_BYTES;
  static constexpr int WAVE_BYTES = 2 * GROUP_BYTES;
  static constexpr int IN_STRIDE = 32;       // sample stride between registers
  static constexpr int OUT_STRIDE = 32;      // bin/time stride between registers
  static constexpr int TW_BYTES = 32 * 32 * 8;  // block-shared W1024^{l k1} table
  static constexpr int BLOCKS_PER_CU = 2;
  static constexpr int SYN_BLOCKS_PER_CU = 2;
  static constexpr int SYN_R = 1;  // synthesis frames per lane group per step
};
template <>
struct KCfg<512> {
  using Fft = Fft512x2;
  static constexpr int PPL = Fft::PPL;
  static constexpr int FPW = 2;
  static constexpr int GROUP_BYTES = 16 * 34 * 8;
  static constexpr int WAVE_BYTES = 2 * GROUP_BYTES;
  static constexpr int IN_STRIDE = 32;
  static constexpr int OUT_STRIDE = 16;
  static constexpr int TW_BYTES = 0;
  // analysis at 3 blocks (12 waves) per CU: 168 VGPRs, 3 x 35 KB LDS; 97.9 -> 81.0 us at
  // B = 256 (profiles/r03/n512_occupancy.txt); 4 spills and runs 85 us, the synthesis
  // gains nothing from 3 (spills at 168 VGPRs)
  static constexpr int BLOCKS_PER_CU = 3;
  static constexpr int SYN_BLOCKS_PER_CU = 2;
  // synthesis frames per lane group per step: 2 -> 16 frames (and 8 packed inverse pairs,
  // two per wave) per step in the same 70 KB of LDS as N = 1024's 8
  static constexpr int SYN_R = 2;
};

template <int N, int NT>
struct Geo {
  using C = KCfg<N>;
  static constexpr int NWAVE = NT / 64;
  static constexpr int H = N / 2;
  static constexpr int NB = N / 2;          // bins per q-row (bin N/2 rides with k = 0)
  static constexpr int F = N / 2 + 1;
  static constexpr int Q = NT / NB;         // frame groups in the per-bin phase
  static constexpr int NSLOT = NWAVE * C::FPW;
  static constexpr int SLOT_LDS = NWAVE * C::WAVE_BYTES;
  // LDS map: [FFT slots][OLA carry 2 x H f32][twiddles][Nyquist sums Q x 5 f64][2 coefs]
  static constexpr int CARRY_OFF = SLOT_LDS;
  static constexpr int TW_OFF = CARRY_OFF + 2 * H * 4;
  static constexpr int NYQ_OFF = TW_OFF + C::TW_BYTES;
  static constexpr int LDS_BYTES = NYQ_OFF + Q * 5 * 8 + 16;
  static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
  static_assert(NB * 5 * 8 * Q <= SLOT_LDS, "covariance reduction must fit the slot area");
};

template <int N>
__device__ __forceinline__ cf* slot_ptr(unsigned char* lds, int s) {
  using C = KCfg<N>;
  return reinterpret_cast<cf*>(lds + (s / C::FPW) * C::WAVE_BYTES + (s % C::FPW) * C::GROUP_BYTES);
}

// Per-lane geometry of the wave FFT (input sample / output index of each register).
template <int N>
struct LaneMap {
  int in0;    // input index of register 0 (lane part)
  int grp;    // lane group (N=512: which of the two FFTs; N=1024: 0)
  int out0;   // output index of register 0
  __device__ __forceinline__ void init(int lane) {
    if constexpr (N == 1024) {
      in0 = lane & 31;
      grp = lane >> 5;
      out0 = lane & 31;
    } else {
      in0 = lane & 31;
      grp = lane >> 5;
      out0 = (lane & 15) + 256 * ((lane >> 4) & 1);
    }
  }
};

// a = (z + conj zp)/2, b = (z - conj zp)/(2i): split of a packed real pair.
// Written so that a self-partnered bin (DC, Nyquist: zp == z) yields exact +0
// imaginary parts, as pocketfft's r2c does (matters for the IPD angle test).
__device__ __forceinline__ void split_pair(cf z, cf zp, cf& a, cf& b) {
  a = {0.5f * (z.x + zp.x), 0.5f * (z.y - zp.y)};
  b = {0.5f * (z.y + zp.y), 0.5f * (zp.x - z.x)};
}
// The same split without the 1/2 factors (2a, 2b): exact, so sums of products of it
// are exactly 4x the sums of the halved values (the solve scales them back by 1/4).
__device__ __forceinline__ void split_pair2(cf z, cf zp, cf& a2, cf& b2) {
  a2 = {z.x + zp.x, z.y - zp.y};
  b2 = {z.y + zp.y, zp.x - z.x};
}
// DC / Nyquist bins: both parts are real; imaginary parts are +0 (pocketfft r2c).
__device__ __forceinline__ void split_self(cf z, cf& a, cf& b) {
  a = {z.x, 0.0f};
  b = {z.y, 0.0f};
}

// Heuristic phase mask (masked_mvdr.py:37-46): 0.01 where angle(Y0) == angle(Y1)
// as float32, else 1.0. A cross-product test settles every bin whose angles differ
// by far more than an fp32 ulp. Real bins (DC / Nyquist: imaginary parts exactly +0
// from split_pair2) have angle +0 or +pi by the sign bit of the real part, exactly as
// atan2f(+0, x); only the rare near-colinear complex bins reach atan2f, so a wave
// skips that code unless one of its lanes needs it.
__device__ __forceinline__ bool ipd_clear(cf a, cf b) {  // angles certainly differ
  const float cr = a.y * b.x - a.x * b.y;
  const float n2 = (a.x * a.x + a.y * a.y) * (b.x * b.x + b.y * b.y);
  return cr * cr > 1e-10f * n2;
}
__device__ __forceinline__ float ipd_weight_exact(cf a, cf b) {
  const unsigned ia = __float_as_uint(a.y), ib = __float_as_uint(b.y);
  if ((ia | ib) == 0u)  // both imaginary parts +0
    return (signbit(a.x) == signbit(b.x)) ? 0.01f : 1.0f;
  const float pa = atan2f(a.y, a.x), pb = atan2f(b.y, b.x);
  return (fabsf(pa - pb) > 0.0f) ? 1.0f : 0.01f;
}
__device__ __forceinline__ float ipd_weight(cf a, cf b) {
  return ipd_clear(a, b) ? 1.0f : ipd_weight_exact(a, b);
}

struct Acc32 {
  float c00, c11, c01r, c01i, cm;
  __device__ __forceinline__ void zero() { c00 = c11 = c01r = c01i = cm = 0.f; }
  __device__ __forceinline__ void add(cf x0, cf x1, float wgt, float m) {
    c00 = fmaf(wgt, x0.x * x0.x + x0.y * x0.y, c00);
    c11 = fmaf(wgt, x1.x * x1.x + x1.y * x1.y, c11);
    c01r = fmaf(wgt, x0.x * x1.x + x0.y * x1.y, c01r);  // Re x0 conj(x1)
    c01i = fmaf(wgt, x0.y * x1.x - x0.x * x1.y, c01i);  // Im x0 conj(x1)
    cm += m;
  }
  // Binary weight (IBM, clear IPD frames): the selected inputs carry the weight (w^2 = w),
  // 4 selects + 8 fma; the weight count goes to cm separately (popcount of the bits).
  __device__ __forceinline__ void add_sel(cf x0, cf x1, bool on) {
    const cf m0 = on ? x0 : cf{0.f, 0.f};
    const cf m1 = on ? x1 : cf{0.f, 0.f};
    c00 = fmaf(m0.x, x0.x, c00);
    c00 = fmaf(m0.y, x0.y, c00);
    c11 = fmaf(m1.x, x1.x, c11);
    c11 = fmaf(m1.y, x1.y, c11);
    c01r = fmaf(m0.x, x1.x, c01r);  // Re x0 conj(x1)
    c01r = fmaf(m0.y, x1.y, c01r);
    c01i = fmaf(m0.y, x1.x, c01i);  // Im x0 conj(x1)
    c01i = fmaf(-m0.x, x1.y, c01i);
  }
};
struct Acc64 {
  double c[5];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < 5; ++i) c[i] = 0.0;
  }
  __device__ __forceinline__ void add(const Acc32& a) {
    c[0] += (double)a.c00;
    c[1] += (double)a.c11;
    c[2] += (double)a.c01r;
    c[3] += (double)a.c01i;
    c[4] += (double)a.cm;
  }
};

// Apply coefficients of weights w: S = conj(w0) y0 + conj(w1) y1 evaluated on the packed
// mic pair Z = y0 + i y1 as S = alpha Z[k] + beta conj(Z[N-k]).
__device__ __forceinline__ void coef_from_w(double w0r, double w0i, double w1r, double w1i,
                                            cf& alpha, cf& beta, float* w_dbg) {
  // alpha = (conj w0 - i conj w1)/2 ; beta = (conj w0 + i conj w1)/2
  alpha = {(float)(0.5 * (w0r - w1i)), (float)(0.5 * (-w0i - w1r))};
  beta = {(float)(0.5 * (w0r + w1i)), (float)(0.5 * (-w0i + w1r))};
  if (w_dbg) {
    w_dbg[0] = (float)w0r;
    w_dbg[1] = (float)w0i;
    w_dbg[2] = (float)w1r;
    w_dbg[3] = (float)w1i;
  }
}

// Per-bin MVDR weights in fp64 (oracle_debug.py:66-79):
//   w~ = (R/(sum m + 1e-6) + sigma I)^{-1} d ; w = w~ / (d^H w~ + 1e-10);
//   singular -> w = [1, 0] (or ones/2, oracle_reverb.py:133-135); f < fmin -> w = 0.
// d = steering vector (masked_mvdr.py:22-35). c = {sum m|y0|^2, sum m|y1|^2,
// Re/Im sum m y0 conj(y1), sum m}. w = {Re w0, Im w0, Re w1, Im w1}. *singular is set
// when the loaded covariance is exactly singular (whatever the fallback policy).
__device__ __forceinline__ void mvdr_weights_d(const double (&c)[5], int k, int n_fft,
                                               const ChainArgs& A, double d0r, double d0i,
                                               double d1r, double d1i, double (&w)[4],
                                               bool* singular) {
  double w0r = 0, w0i = 0, w1r = 0, w1i = 0;
  const double fk = (double)k * A.fs / (double)n_fft;
  if (!(fk < A.fmin_hz)) {
    const double nrm = c[4] + 1e-6;
    const double a = c[0] / nrm + A.sigma, e = c[1] / nrm + A.sigma;
    const double br = c[2] / nrm, bi = c[3] / nrm;
    const double det = a * e - (br * br + bi * bi);
    double t0r, t0i, t1r, t1i;
    bool solved = true;
    if (!isfinite(det)) {
      // NaN / Inf in Y or the mask: LAPACK's gesv (np.linalg.solve / inv) raises only on an
      // exactly zero pivot, so the reference returns NaN weights here in every mode
      w0r = w0i = w1r = w1i = __builtin_nan("");
      solved = false;
    } else if (det == 0.0) {
      if (singular) *singular = true;
      if (A.singular_fallback == 1) {  // oracle_reverb.py:133-135: ones(n)/n, not normalised
        w0r = 0.5;
        w1r = 0.5;
        solved = false;
      } else if (A.singular_fallback == 0) {  // oracle_debug.py:78-79: [1, 0], not normalised
        w0r = 1.0;
        solved = false;
      } else {  // batch_mvdr (tf_lite_version/inference.py:143-157): w~ = [1, 0], normalised
        t0r = 1.0; t0i = 0.0; t1r = 0.0; t1i = 0.0;
      }
    } else {
      // w~0 = (e d0 - b d1)/det ; w~1 = (a d1 - conj(b) d0)/det
      t0r = e * d0r - (br * d1r - bi * d1i);
      t0i = e * d0i - (br * d1i + bi * d1r);
      t1r = a * d1r - (br * d0r + bi * d0i);
      t1i = a * d1i - (br * d0i - bi * d0r);
      t0r /= det; t0i /= det; t1r /= det; t1i /= det;
    }
    if (solved) {
      // den = conj(d0) w~0 + conj(d1) w~1 + 1e-10
      const double dr = d0r * t0r + d0i * t0i + d1r * t1r + d1i * t1i + 1e-10;
      const double di = d0r * t0i - d0i * t0r + d1r * t1i - d1i * t1r;
      const double dd = dr * dr + di * di;
      w0r = (t0r * dr + t0i * di) / dd;
      w0i = (t0i * dr - t0r * di) / dd;
      w1r = (t1r * dr + t1i * di) / dd;
      w1i = (t1i * dr - t1r * di) / dd;
    }
  }
  w[0] = w0r; w[1] = w0i; w[2] = w1r; w[3] = w1i;
}

// batch_mvdr's item-level fallback weights (tf_lite_version/inference.py:149-157): every
// bin w~ = [1, 0]^T, normalised: w = [1 / (conj(d0) + 1e-10), 0].
__device__ __forceinline__ void batch_fallback_weights_d(double d0r, double d0i,
                                                         double (&w)[4]) {
  const double dr = d0r + 1e-10, di = -d0i;  // conj(d0) + 1e-10
  const double dd = dr * dr + di * di;
  w[0] = dr / dd;
  w[1] = -di / dd;
  w[2] = 0.0;
  w[3] = 0.0;
}

__device__ __forceinline__ void mvdr_solve_d(const double (&c)[5], int k, int n_fft,
                                             const ChainArgs& A, double d0r, double d0i,
                                             double d1r, double d1i, cf& alpha, cf& beta,
                                             float* w_dbg) {
  double w[4];
  mvdr_weights_d(c, k, n_fft, A, d0r, d0i, d1r, d1i, w, nullptr);
  coef_from_w(w[0], w[1], w[2], w[3], alpha, beta, w_dbg);
}

// Per-bin hybrid hard-null weights in fp64 (Final_pipeline/src/inference.py:28-98):
//   f < bypass_hz -> w = [1, 0] (mic 0 passes);
//   R = sum m y y^H / (sum m + 1e-6), v_int = principal eigenvector of R with v_int[0]
//   made real: v_int * (|v_int[0]| + 1e-10) / v_int[0];
//   C = [v_tgt, v_int]; cond_2(C) > cond_max (or singular) -> w = v_tgt / 2,
//   else w = (C^H)^-1 [1, 0]^T.
// v_tgt = (vt0, vt1): the plan's phase-normalised steering vector (inference.py:16-26).
// Where the reference's eigenvector has v_int[0] == 0 (R diagonal with R11 >= R00, e.g.
// no noise-weighted frames) it divides by zero and np.linalg.cond then raises; here
// that bin takes the delay-and-sum fallback.
__device__ __forceinline__ void hybrid_weights_d(const double (&c)[5], int k, int n_fft,
                                                 const ChainArgs& A, double t0r, double t0i,
                                                 double t1r, double t1i, double (&w)[4]) {
  const double fk = (double)k * A.fs / (double)n_fft;
  if (fk < A.bypass_hz) {
    w[0] = 1.0; w[1] = 0.0; w[2] = 0.0; w[3] = 0.0;
    return;
  }
  const double nrm = c[4] + 1e-6;
  const double a = c[0] / nrm, e = c[1] / nrm;
  const double br = c[2] / nrm, bi = c[3] / nrm;  // R01 = b, R10 = conj(b)
  const double b2 = br * br + bi * bi;
  const double hd = 0.5 * (a - e);
  const double lam = 0.5 * (a + e) + sqrt(hd * hd + b2);
  // eigenvector of lam: [lam - e, conj b] (a >= e) or [b, lam - a] (a < e)
  double u0r, u0i, u1r, u1i;
  if (a >= e) {
    u0r = lam - e; u0i = 0.0; u1r = br; u1i = -bi;
  } else {
    u0r = br; u0i = bi; u1r = lam - a; u1i = 0.0;
  }
  const double un = sqrt(u0r * u0r + u0i * u0i + u1r * u1r + u1i * u1i);
  u0r /= un; u0i /= un; u1r /= un; u1i /= un;
  // v = u (|u0| + 1e-10) / u0 = u conj(u0) (|u0| + 1e-10) / |u0|^2
  const double m0 = u0r * u0r + u0i * u0i;
  const double a0 = sqrt(m0);
  const double g = (a0 + 1e-10) / m0;
  const double v0r = a0 + 1e-10, v0i = 0.0;
  const double v1r = (u1r * u0r + u1i * u0i) * g;
  const double v1i = (u1i * u0r - u1r * u0i) * g;
  double w0r = 0.5 * t0r, w0i = 0.5 * t0i, w1r = 0.5 * t1r, w1i = 0.5 * t1i;  // delay-and-sum
  if (isfinite(v1r) && isfinite(v1i) && m0 > 0.0) {
    // det C = t0 v1 - v0 t1
    const double dr = (t0r * v1r - t0i * v1i) - (v0r * t1r - v0i * t1i);
    const double di = (t0r * v1i + t0i * v1r) - (v0r * t1i + v0i * t1r);
    const double det2 = dr * dr + di * di;
    // sigma_max^2 of C: eigenvalue of C^H C = [[p, r], [conj r, q]]
    const double p = t0r * t0r + t0i * t0i + t1r * t1r + t1i * t1i;
    const double q = v0r * v0r + v0i * v0i + v1r * v1r + v1i * v1i;
    const double rr = t0r * v0r + t0i * v0i + t1r * v1r + t1i * v1i;  // conj(t) . v
    const double ri = t0r * v0i - t0i * v0r + t1r * v1i - t1i * v1r;
    const double hpq = 0.5 * (p - q);
    const double smax2 = 0.5 * (p + q) + sqrt(hpq * hpq + rr * rr + ri * ri);
    // cond = smax2 / |det C|; keep the solve only when cond <= cond_max
    if (det2 > 0.0 && smax2 <= A.cond_max * sqrt(det2)) {
      // w = [conj(v1), -conj(v0)] / conj(det C)
      const double ir = dr / det2, ii = di / det2;  // 1 / conj(det) = det / |det|^2
      w0r = v1r * ir + v1i * ii;
      w0i = v1r * ii - v1i * ir;
      w1r = -(v0r * ir + v0i * ii);
      w1i = -(v0r * ii - v0i * ir);
    }
  }
  w[0] = w0r; w[1] = w0i; w[2] = w1r; w[3] = w1i;
}

__device__ __forceinline__ void hybrid_solve_d(const double (&c)[5], int k, int n_fft,
                                               const ChainArgs& A, double t0r, double t0i,
                                               double t1r, double t1i, cf& alpha, cf& beta,
                                               float* w_dbg) {
  double w[4];
  hybrid_weights_d(c, k, n_fft, A, t0r, t0i, t1r, t1i, w);
  coef_from_w(w[0], w[1], w[2], w[3], alpha, beta, w_dbg);
}

__device__ __forceinline__ cf apply_bin(cf alpha, cf beta, cf z, cf zp, float g) {
  const cf s = c_add(c_mul(alpha, z), c_mul(beta, c_conj(zp)));
  return {g * s.x, g * s.y};
}


// ---- host side
// Dynamic-LDS attribute of one kernel, set once per device (thread-safe: the first caller
// on a device sets it; concurrent first callers both set the same value).
template <auto Kern>
static bool lds_ready(int lds) {
  static std::atomic<int> state[64];  // 0 unset, 1 set, -1 failed
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return false;
  if (dev < 64) {
    const int st = state[dev].load(std::memory_order_acquire);
    if (st != 0) return st > 0;
  }
  const bool ok = hipFuncSetAttribute((const void*)Kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      lds) == hipSuccess;
  if (dev < 64) state[dev].store(ok ? 1 : -1, std::memory_order_release);
  return ok;
}

}  // namespace avz
