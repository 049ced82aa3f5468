// avz_kernels.hip — standalone STFT kernel (stage API, parity tests) for gfx950.
// The beamforming chain itself lives in avz_chunked.hip.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "avz_common.hpp"

namespace avz {

// ---------------------------------------------------------------------------
// Standalone STFT (stage API / parity): Y[b][c][k][t] = scipy.signal.stft(x[b][c])
// One block per (utterance, NSLOT-frame batch); each lane group transforms one
// frame of the packed channel pair, then threads split the pair per bin.
constexpr int kStftThreads = 512;

// Mask-model input features of one (k, t) from the two mic spectra y0, y1:
//  FEAT_LOGMAG_IPD (full_audio_generating_pipeline/inference.py:90-94, NCHW [b][2][F][T]):
//    c=0 log(|y0| + 1e-7), c=1 angle(y0) - angle(y1)
//  FEAT_TFLITE (Final_pipeline/src/inference.py:198-203, 117-128, NHWC [b][F][T][4]):
//    log_mag, sin(ipd), cos(ipd), linspace(0, 1, F)[k]
// float32 throughout, as numpy computes them on scipy's complex64 STFT.
template <int FEAT, int F>
__device__ __forceinline__ void write_features(const StftArgs& A, int b, int k, int t, cf y0,
                                               cf y1) {
  const float lm = logf(sqrtf(y0.x * y0.x + y0.y * y0.y) + 1e-7f);
  const float ipd = atan2f(y0.y, y0.x) - atan2f(y1.y, y1.x);
  float* o = A.F_out + (long long)b * A.f_sb + (long long)k * A.f_sf + (long long)t * A.f_st;
  if constexpr (FEAT == FEAT_LOGMAG_IPD) {
    o[0] = lm;
    o[A.f_sc] = ipd;
  } else {
    // np.linspace(0, 1, F, dtype=float32): k * (1/(F-1)) in fp64, last element exactly 1
    const float fm = (k == F - 1) ? 1.0f : (float)((double)k * (1.0 / (F - 1)));
    float s, c;
    sincosf(ipd, &s, &c);
    o[0] = lm;
    o[A.f_sc] = s;
    o[2 * A.f_sc] = c;
    o[3 * A.f_sc] = fm;
  }
}

template <int N, int FEAT>
__global__ void __launch_bounds__(kStftThreads, 1) avz_stft_kernel(StftArgs A) {
  using C = KCfg<N>;
  using G = Geo<N, kStftThreads>;
  constexpr int H = G::H, F = G::F, NSLOT = G::NSLOT, PPL = C::PPL;
  extern __shared__ __align__(16) unsigned char lds[];
  cf* twid = reinterpret_cast<cf*>(lds + G::TW_OFF);
  C::Fft::fill_twiddles(twid, threadIdx.x, kStftThreads);
  const int b = blockIdx.x;
  const int f0 = blockIdx.y * NSLOT;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int L = min(A.len[b], A.max_len);
  const int T = (L + H - 1) / H + 1;
  if (f0 >= T || L < N) return;
  __syncthreads();

  typename C::Fft fft;
  fft.init(lane);
  LaneMap<N> lm;
  lm.init(lane);
  const int my_slot = wave * C::FPW + lm.grp;
  cf* spec = slot_ptr<N>(lds, my_slot);
  const float* xb = A.x + (long long)b * A.x_stride;
  const rsrc_t re = make_rsrc(xb, L);
  const rsrc_t im = make_rsrc(A.channels > 1 ? xb + A.ch_stride : nullptr, L);
  float wa0, wac, was;
  {
    double s, c;
    sincospi(2.0 * lm.in0 / N, &s, &c);
    const double sc = 2.0 / N;
    wa0 = (float)(0.5 * sc);
    wac = (float)(0.5 * sc * c);
    was = (float)(0.5 * sc * s);
  }
  cf v[PPL];
  const int s0 = (f0 + my_slot) * H - N / 2 + lm.in0;
  static_for<0, PPL>([&](auto r) {
    constexpr int j = (C::IN_STRIDE * 32 / N) * r;
    constexpr float cr = W32::c[j % 32], sr = -W32::s[j % 32];
    const float w = fmaf(was, sr, fmaf(-wac, cr, wa0));
    v[r] = {bload(re, s0 + C::IN_STRIDE * r) * w, bload(im, s0 + C::IN_STRIDE * r) * w};
  });
  fft.forward(v, spec, twid);
  static_for<0, PPL>([&](auto k) { spec[lm.out0 + C::OUT_STRIDE * k] = v[k]; });
  __syncthreads();
  float2* Y = reinterpret_cast<float2*>(A.Y);
  for (int idx = tid; idx < F * NSLOT; idx += kStftThreads) {
    const int k = idx / NSLOT, f = idx % NSLOT;
    const int t = f0 + f;
    if (t >= T) continue;
    const cf* Z = slot_ptr<N>(lds, f);
    cf a, c;
    split_pair(Z[k], Z[(N - k) & (N - 1)], a, c);
    if constexpr (FEAT != FEAT_NONE) {
      write_features<FEAT, F>(A, b, k, t, a, c);
    } else {
      const long long o = (long long)b * A.y_stride_b + (long long)k * A.y_stride_f + t;
      Y[o] = make_float2(a.x, a.y);
      if (A.channels > 1) Y[o + A.y_stride_c] = make_float2(c.x, c.y);
    }
  }
}

}  // namespace avz

using namespace avz;

template <int N, int FEAT>
static int launch_stft_t(const StftArgs* a, hipStream_t st) {
  auto kern = avz_stft_kernel<N, FEAT>;
  const int lds = Geo<N, kStftThreads>::LDS_BYTES;
  if (!lds_ready<avz_stft_kernel<N, FEAT>>(lds)) return -3;
  constexpr int NS = Geo<N, kStftThreads>::NSLOT;
  dim3 grid(a->batch, (a->max_frames + NS - 1) / NS);
  hipLaunchKernelGGL(kern, grid, dim3(kStftThreads), lds, st, *a);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int avz_launch_stft(int n_fft, const StftArgs* a, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (a->batch <= 0) return 0;
  switch (a->feat) {
    case FEAT_NONE:
      if (n_fft == 1024) return launch_stft_t<1024, FEAT_NONE>(a, st);
      if (n_fft == 512) return launch_stft_t<512, FEAT_NONE>(a, st);
      break;
    case FEAT_LOGMAG_IPD:
      if (n_fft == 1024) return launch_stft_t<1024, FEAT_LOGMAG_IPD>(a, st);
      if (n_fft == 512) return launch_stft_t<512, FEAT_LOGMAG_IPD>(a, st);
      break;
    case FEAT_TFLITE:
      if (n_fft == 1024) return launch_stft_t<1024, FEAT_TFLITE>(a, st);
      if (n_fft == 512) return launch_stft_t<512, FEAT_TFLITE>(a, st);
      break;
  }
  return -4;
}
