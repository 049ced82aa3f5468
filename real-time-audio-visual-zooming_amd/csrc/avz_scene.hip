// avz_scene.hip — on-device synthetic scene mixing (gfx950): the reference's anechoic
// far-field generator, full_audio_generating_pipeline/world_building.py:47-59 (per-mic
// fractional delay by an rfft phase shift over the WHOLE signal) with the SIR / AWGN /
// shared-peak conventions of Final_pipeline/src/simulation.py:167-202 (the bench's
// generator, avz/synth.py make_scene). Sources and unit-normal noise come from the host
// RNG (so the device scene is the host scene); everything after them runs here.
//
// Fractional delay. irfft(rfft(y) * exp(-2 pi i f tau), n) is the circular convolution
// of y with the periodic kernel (delta = tau * fs samples, n even; irfft drops the
// imaginary part of the Nyquist bin):
//   h[d] = -(1/n) (-1)^d sin(pi delta) cot(pi (d - delta) / n),   d = 0 .. n-1,
// so image[m] = sum_j y[j] h[(m - j) mod n]. The kernel table is built in fp64 and the
// O(n^2) sum runs on the VALU in fp32 (relative error ~1e-6 against the fp64 FFT path):
// there is no length-n (64000 = 2^9 5^3) FFT on the device, and the generator is outside
// every timed region. A source whose sin(pi delta) vanishes (broadside) is copied.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "avz_internal.h"

namespace avz {

constexpr int kConvThreads = 256;
constexpr int kConvOut = 8;                          // outputs per thread
constexpr int kConvM = kConvThreads * kConvOut;      // 2048 outputs per block
constexpr int kConvJ = 256;                          // inputs per LDS tile
constexpr int kConvH = kConvM + kConvJ;              // kernel values per tile (2304)

// delta of (utterance b, source s, mic c): tau_mic * fs with world_building.py:47-51
// tau_1 = (d/2) cos(theta)/c, tau_2 = (d/2) cos(theta - pi)/c
__device__ __forceinline__ double scene_delta(const SceneArgs& A, int b, int s, int mic) {
  const double th = A.angles_deg[(long long)b * A.n_src + s] * (M_PI / 180.0);
  const double tau = (A.mic_d / 2) * cos(th - (mic ? M_PI : 0.0)) / A.c_sound;
  return tau * A.fs;
}

// h tables: one per (utterance, source, mic) signal, h[d] in fp64 -> fp32
__global__ void __launch_bounds__(256) avz_scene_kernel_fill(SceneArgs A) {
  const long long n = A.n;
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long nsig = (long long)A.batch * A.n_src * 2;
  if (idx >= nsig * n) return;
  const int sig = (int)(idx / n);
  const int d = (int)(idx % n);
  const int mic = sig & 1, s = (sig >> 1) % A.n_src, b = (sig >> 1) / A.n_src;
  const double delta = scene_delta(A, b, s, mic);
  const double x = ((double)d - delta) / (double)n;
  double sn, cs;
  sincospi(x, &sn, &cs);
  const double sd = sinpi(delta);
  const double h = -(1.0 / (double)n) * ((d & 1) ? -1.0 : 1.0) * sd * (cs / sn);
  A.hk[idx] = (float)h;
}

// image[sig][m] = sum_j src[b][s][j] h[sig][(m - j) mod n]; grid (ceil(n/2048), nsig).
// Thread t owns outputs M0 + 8t .. M0 + 8t + 7; per 256-input tile the block stages the
// inputs and the 2304 kernel values they meet, and each thread slides an 8-output window
// over 16 kernel values per 8 inputs (4 ds_read_b128 + 2 broadcast reads per 64 FMAs).
__global__ void __launch_bounds__(kConvThreads) avz_scene_conv_kernel(SceneArgs A) {
  __shared__ __align__(16) float y_t[kConvJ];
  __shared__ __align__(16) float h_t[kConvH];
  const int n = A.n;
  const int sig = blockIdx.y;
  const int mic = sig & 1, s = (sig >> 1) % A.n_src, b = (sig >> 1) / A.n_src;
  const float* y = A.src + ((long long)b * A.n_src + s) * n;
  float* img = A.img + (long long)sig * n;
  const int M0 = blockIdx.x * kConvM;
  const int tid = threadIdx.x;
  // broadside (sin(pi delta) ~ 0): the phase shift is 1 to within fp64 rounding
  if (fabs(sinpi(scene_delta(A, b, s, mic))) < 1e-12) {
    for (int m = M0 + tid; m < min(M0 + kConvM, n); m += kConvThreads) img[m] = y[m];
    return;
  }
  const float* h = A.hk + (long long)sig * n;
  float acc[kConvOut];
#pragma unroll
  for (int r = 0; r < kConvOut; ++r) acc[r] = 0.0f;
  for (int j0 = 0; j0 < n; j0 += kConvJ) {
    __syncthreads();
    y_t[tid] = (j0 + tid < n) ? y[j0 + tid] : 0.0f;
    // h_t[i] = h[(M0 - j0 - 255 + i) mod n]
    int base = (M0 - j0 - (kConvJ - 1)) % n;
    if (base < 0) base += n;
    for (int i = tid; i < kConvH; i += kConvThreads) {
      int d = base + i;
      if (d >= n) d -= n;
      if (d >= n) d -= n;
      h_t[i] = h[d];
    }
    __syncthreads();
#pragma unroll 2
    for (int q0 = 0; q0 < kConvJ; q0 += 8) {
      const int hb = kConvOut * tid - q0 + (kConvJ - 8);  // multiple of 8: 16-B aligned
      float hw[16];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const float4 t4 = *reinterpret_cast<const float4*>(h_t + hb + 4 * v);
        hw[4 * v] = t4.x; hw[4 * v + 1] = t4.y; hw[4 * v + 2] = t4.z; hw[4 * v + 3] = t4.w;
      }
      const float4 ya = *reinterpret_cast<const float4*>(y_t + q0);
      const float4 yb = *reinterpret_cast<const float4*>(y_t + q0 + 4);
      const float yq[8] = {ya.x, ya.y, ya.z, ya.w, yb.x, yb.y, yb.z, yb.w};
#pragma unroll
      for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int r = 0; r < kConvOut; ++r) acc[r] = fmaf(yq[q], hw[r - q + 7], acc[r]);
    }
  }
#pragma unroll
  for (int r = 0; r < kConvOut; ++r) {
    const int m = M0 + kConvOut * tid + r;
    if (m < n) img[m] = acc[r];
  }
}

// One block per utterance: simulation.py:167-202 on the images.
//   tgt_m = image(target), int_m = g * sum_k image(interferer k), g for SIR sir_db on mic 1;
//   noisy = clean + sqrt(mean(clean^2) / 10^(snr/10)) * z  (world.py:93-98 add_awgn);
//   peak = max |noisy| + 1e-9 over both mics; outputs / peak.
constexpr int kMixThreads = 256;
__device__ __forceinline__ double block_sum(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int w = 0; w < kMixThreads / 64; ++w) t += red[w];
  return t;
}
__device__ __forceinline__ float block_max(float v, float* red) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float t = 0.0f;
#pragma unroll
  for (int w = 0; w < kMixThreads / 64; ++w) t = fmaxf(t, red[w]);
  return t;
}

__global__ void __launch_bounds__(kMixThreads) avz_scene_mix_kernel(SceneArgs A) {
  __shared__ double red[kMixThreads / 64];
  __shared__ float redf[kMixThreads / 64];
  const int b = blockIdx.x, tid = threadIdx.x, n = A.n, K = A.n_src - 1;
  const float* im = A.img + (long long)b * A.n_src * 2 * n;  // [src][mic][n]
  auto tgt_img = [&](int mic, int m) -> double { return (double)im[(long long)mic * n + m]; };
  auto int_img = [&](int mic, int m) -> double {
    double v = 0.0;
    for (int k = 1; k <= K; ++k) v += (double)im[((long long)k * 2 + mic) * n + m];
    return v;
  };
  double st = 0.0, si = 0.0;
  for (int m = tid; m < n; m += kMixThreads) {
    const double t = tgt_img(0, m), i = int_img(0, m);
    st += t * t;
    si += i * i;
  }
  const double p_t = block_sum(st, red) / n;
  const double p_i = block_sum(si, red) / n;
  const double g = (K > 0 && p_i > 0) ? sqrt(p_t / (p_i * pow(10.0, A.sir_db / 10.0))) : 1.0;
  double sc[2] = {0.0, 0.0};
  for (int m = tid; m < n; m += kMixThreads) {
#pragma unroll
    for (int mic = 0; mic < 2; ++mic) {
      const double cl = tgt_img(mic, m) + g * int_img(mic, m);
      sc[mic] += cl * cl;
    }
  }
  double sig_n[2];
#pragma unroll
  for (int mic = 0; mic < 2; ++mic) {
    const double p = block_sum(sc[mic], red) / n;
    sig_n[mic] = (p == 0.0) ? 0.0 : sqrt(p / pow(10.0, A.snr_db / 10.0));
  }
  const float* z = A.noise + (long long)b * 2 * n;
  float pk = 0.0f;
  for (int m = tid; m < n; m += kMixThreads) {
#pragma unroll
    for (int mic = 0; mic < 2; ++mic) {
      const double v = tgt_img(mic, m) + g * int_img(mic, m) + sig_n[mic] * (double)z[(long long)mic * n + m];
      pk = fmaxf(pk, (float)fabs(v));
    }
  }
  // the peak in fp64 would need a second reduction type; |v| rounded to fp32 first
  // changes 1/(peak + 1e-9) by < 1 ulp of fp32
  const double peak = (double)block_max(pk, redf) + 1e-9;
  float* mix = A.mix + (long long)b * A.mix_stride;
  for (int m = tid; m < n; m += kMixThreads) {
#pragma unroll
    for (int mic = 0; mic < 2; ++mic) {
      const double v = tgt_img(mic, m) + g * int_img(mic, m) + sig_n[mic] * (double)z[(long long)mic * n + m];
      mix[(long long)mic * A.ch_stride + m] = (float)(v / peak);
    }
    A.tgt[(long long)b * A.ref_stride + m] = (float)(tgt_img(0, m) / peak);
    A.itf[(long long)b * A.ref_stride + m] = (float)(g * int_img(0, m) / peak);
  }
}

}  // namespace avz

using namespace avz;

extern "C" int avz_launch_scene(const SceneArgs* a, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const long long nsig = (long long)a->batch * a->n_src * 2;
  const long long tot = nsig * a->n;
  hipLaunchKernelGGL(avz_scene_kernel_fill, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0,
                     st, *a);
  hipLaunchKernelGGL(avz_scene_conv_kernel, dim3((a->n + kConvM - 1) / kConvM, (unsigned)nsig),
                     dim3(kConvThreads), 0, st, *a);
  hipLaunchKernelGGL(avz_scene_mix_kernel, dim3(a->batch), dim3(kMixThreads), 0, st, *a);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
