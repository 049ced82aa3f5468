// avz_ibm_exact.hpp — reference-exact IBM decisions for frames the fp32 path cannot settle.
//
// The oracle IBM (rt_av_zoom/core/oracle_debug.py:42-53) decides noise <=> |S_int| > |S_tgt|
// on two SEPARATE scipy STFTs: pocketfft in fp64 on the exact fp64 windowed frame (fp32
// samples x fp32-rounded Hann), scaled by 1/sum(win) (= 2^-9 at N = 1024, 2^-8 at 512: exact),
// rounded to complex64, magnitudes by numpy's complex64 absolute (np.abs). The analysis kernel
// decides the same inequality on ONE fp32 transform of the packed pair z = tgt + i int
// (ibm_noise: |T|^2 - |I|^2 = Re(Z[k] Z[N-k])), whose error scales with the frame's whole
// energy ||z||: fine wherever the decision margin is above that error, random where it is
// not -- near-ties, and frames whose two references both sit below fp32 resolution of the
// louder one (the synthetic generator's digital-silence blocks: every source zeroed at once).
//
// Certificate (per (bin, frame), reference waves): with delta = kappa eps ||z|| bounding the
// error of every output bin, |dD| <= delta (|Zk| + |Zp|) + delta^2 <= (2 sqrt 2 + 1) delta m,
// m = max(|Re Zk|, |Im Zk|, |Re Zp|, |Im Zp|, delta). A frame with any bin whose |D| does not
// clear that bound is deferred: its fp32 decisions are dropped (noise bits 0, no covariance
// terms) and, at the end of the (chunk) item, the block recomputes both reference spectra of
// the frame in fp64 (ref_spectrum_exact), rounds them to complex64, takes numpy's magnitudes
// (np_abs_c64) and adds the frame's exact decisions and covariance terms. Everything else is
// untouched, so a batch without such frames runs the fp32 path only.
#pragma once
#include "avz_common.hpp"

namespace avz {

// numpy 2.x np.abs of complex64 (loops_unary_complex SIMD path, the one that runs on this
// box and on the GPU hosts: AVX2/AVX-512 with FMA): larger * sqrt(fma(r, r, 1)), r =
// smaller / larger, all in fp32 -- not hypotf (which rounds sqrt(x^2 + y^2) from fp64 and
// differs in ~1/3 of random inputs). Pinned against np.abs in tests/test_ibm_exact_host.py.
// The division and the square root are evaluated in fp64 and rounded once to fp32: with a
// 53-bit intermediate (>= 2 x 24 + 2 bits) that double rounding equals the correctly rounded
// fp32 result, whatever the device's fp32 div / sqrt lowering; v_fma_f32 and v_mul_f32 are
// IEEE single roundings.
__device__ __forceinline__ float np_abs_c64(float re, float im) {
  const float a = fabsf(re), b = fabsf(im);
  const float l = fmaxf(a, b), s = fminf(a, b);
  if (l == 0.0f) return 0.0f;
  const float r = (float)((double)s / (double)l);
  const float sq = (float)sqrt((double)fmaf(r, r, 1.0f));
  return l * sq;
}

struct cd {
  double x, y;
};
__device__ __forceinline__ cd cd_add(cd a, cd b) { return {a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ cd cd_sub(cd a, cd b) { return {a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ cd cd_mul(cd a, cd b) {
  return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x};
}
__device__ __forceinline__ cd cd_mi(cd a) { return {a.y, -a.x}; }  // -i a

// forward DFTs of 4 and 8 points (W = exp(-2 pi i / R)), in place, natural order
__device__ __forceinline__ void cd_dft4(cd& a0, cd& a1, cd& a2, cd& a3) {
  const cd s0 = cd_add(a0, a2), d0 = cd_sub(a0, a2);
  const cd s1 = cd_add(a1, a3), d1 = cd_mi(cd_sub(a1, a3));
  a0 = cd_add(s0, s1);
  a2 = cd_sub(s0, s1);
  a1 = cd_add(d0, d1);
  a3 = cd_sub(d0, d1);
}
template <int R>
__device__ __forceinline__ void cd_dft(cd (&v)[R]) {
  if constexpr (R == 4) {
    cd_dft4(v[0], v[1], v[2], v[3]);
  } else {
    static_assert(R == 8, "radix 4 or 8");
    cd e0 = v[0], e1 = v[2], e2 = v[4], e3 = v[6];
    cd o0 = v[1], o1 = v[3], o2 = v[5], o3 = v[7];
    cd_dft4(e0, e1, e2, e3);
    cd_dft4(o0, o1, o2, o3);
    constexpr double h = 0.70710678118654752440;
    const cd w1o = {h * (o1.x + o1.y), h * (o1.y - o1.x)};     // W8^1 o1
    const cd w2o = cd_mi(o2);                                  // W8^2 o2
    const cd w3o = {h * (o3.y - o3.x), -h * (o3.x + o3.y)};    // W8^3 o3
    v[0] = cd_add(e0, o0);
    v[4] = cd_sub(e0, o0);
    v[1] = cd_add(e1, w1o);
    v[5] = cd_sub(e1, w1o);
    v[2] = cd_add(e2, w2o);
    v[6] = cd_sub(e2, w2o);
    v[3] = cd_add(e3, w3o);
    v[7] = cd_sub(e3, w3o);
  }
}

// Exact-path geometry: the real N-point reference transform as an M = N/2 complex transform
// of z[m] = x[2m] + i x[2m + 1], 64 lanes x RX points, Stockham radix-RX passes in LDS.
template <int N>
struct XGeo {
  static constexpr int M = N / 2;
  static constexpr int RX = M / 64;                      // 8 (N = 1024) or 4 (N = 512)
  static constexpr int PASSES = (RX == 8) ? 3 : 4;       // 8^3 = 512, 4^4 = 256
  static constexpr int SCRATCH = M * 16;                 // one wave's transform buffer
  static_assert(RX == 8 || RX == 4, "N = 1024 or 512");
};

// The exact phase's tables in LDS, copied once per block from the plan's: the fp64 twiddles
// twl[j] = W_N^j, j < N/2 (W^(j + N/2) = -W^j; xtw [N][2]) and the fp32 window (xwin [N]).
template <int N>
__device__ __forceinline__ void xtab_fill(const double* xtw, const float* xwin, cd* twl,
                                          float* win, int tid, int nt) {
  const double2* tw = reinterpret_cast<const double2*>(xtw);
  for (int j = tid; j < N / 2; j += nt) {
    const double2 w = tw[j];
    twl[j] = {w.x, w.y};
  }
  for (int j = tid; j < N; j += nt) win[j] = xwin[j];
}
template <int N>
__device__ __forceinline__ cd xtw_at(const cd* twl, int j) {  // W_N^j, 0 <= j < N
  const cd w = twl[j & (N / 2 - 1)];
  return (j & (N / 2)) ? cd{-w.x, -w.y} : w;
}

// The lane's samples of one reference frame (x: the stream's descriptor, zero outside
// [0, L); s0: the frame's first sample, may be negative): xs[2 r + e] = x[s0 + 2 (lane + 64 r)
// + e], r < RX -- the packed points z[lane + 64 r] of the first pass.
template <int N>
__device__ __forceinline__ void ref_frame_load(rsrc_t x, int s0, int lane, float (&xs)[N / 64]) {
#pragma unroll
  for (int r = 0; r < N / 128; ++r) {
    const int n = 2 * (lane + 64 * r);
    xs[2 * r] = bload(x, s0 + n);
    xs[2 * r + 1] = bload(x, s0 + n + 1);
  }
}

// Magnitudes mag[k] (k = 0 .. N/2) of one reference frame, exactly as the oracle forms them:
// fp64 transform of the fp64 windowed frame (fp32 samples x the reference's fp32 window,
// exact products), rounded to complex64, numpy's |.|. One wave (64 lanes); xs, wv: the lane's
// samples (ref_frame_load); twl, win: the LDS tables (xtab_fill); buf: the wave's XGeo::SCRATCH bytes of LDS (16-B aligned); mag: N/2 + 1 floats
// of LDS. The twiddles come from LDS with each pass's data reads: no global-memory latency
// inside the transform (from the plan's table in global memory each pass waited on it).
template <int N>
__device__ __forceinline__ void ref_spectrum_exact(const float (&xs)[N / 64], const cd* twl,
                                                   const float* win, cd* buf, float* mag,
                                                   int lane) {
  using X = XGeo<N>;
  constexpr int M = X::M, RX = X::RX;
  cd v[RX];
#pragma unroll
  for (int r = 0; r < RX; ++r) {
    const float2 w = reinterpret_cast<const float2*>(win)[lane + 64 * r];
    v[r] = {(double)w.x * (double)xs[2 * r], (double)w.y * (double)xs[2 * r + 1]};
  }
  // Stockham autosort: pass with span Ns: inputs j + r M/RX, twiddle W_{Ns RX}^{r k},
  // outputs (j - k) RX + k + r Ns (k = j mod Ns); one wave, in place (a wave's LDS reads are
  // all issued before its writes, and LDS executes a wave's instructions in order)
  int Ns = 1;
#pragma unroll
  for (int p = 0; p < X::PASSES; ++p) {
    const int j = lane;
    const int k = j & (Ns - 1);
    if (p > 0) {
      cd w[RX];
#pragma unroll
      for (int r = 1; r < RX; ++r) w[r] = xtw_at<N>(twl, (r * k * (N / (Ns * RX))) & (N - 1));
#pragma unroll
      for (int r = 0; r < RX; ++r) v[r] = buf[j + r * (M / RX)];
#pragma unroll
      for (int r = 1; r < RX; ++r) v[r] = cd_mul(v[r], w[r]);
    }
    cd_dft<RX>(v);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
    for (int r = 0; r < RX; ++r) buf[(j - k) * RX + k + r * Ns] = v[r];
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    Ns *= RX;
  }
  // real split: X[k] = E[k] + W_N^k O[k], E = (Z[k] + conj Z[M-k]) / 2, O = -i (Z[k] - conj
  // Z[M-k]) / 2; X[0] = Re Z0 + Im Z0, X[M] = Re Z0 - Im Z0
#pragma unroll
  for (int q = 0; q < RX; ++q) {
    const int k = lane + 64 * q;
    const cd zk = buf[k], zm = buf[(M - k) & (M - 1)];
    const cd w = twl[k];
    float re, im;
    if (k == 0) {
      re = (float)(zk.x + zk.y);
      im = 0.0f;
    } else {
      const cd e = {0.5 * (zk.x + zm.x), 0.5 * (zk.y - zm.y)};
      const cd o = {0.5 * (zk.y + zm.y), 0.5 * (zm.x - zk.x)};
      const cd xo = cd_mul(w, o);
      re = (float)(e.x + xo.x);
      im = (float)(e.y + xo.y);
    }
    mag[k] = np_abs_c64(re, im);
    if (k == 0) mag[M] = np_abs_c64((float)(zk.x - zk.y), 0.0f);
  }
}

}  // namespace avz
