// avz_metrics.hip — projection metrics of a batch on the device (gfx950).
//
// Final_pipeline/src/metrics.py:102-123 (calculate_osnr_osir) and
// scripts/run_metrics.py:6-36 (calculate_metrics_manual) are projections of the output
// onto the normalised target / interference references. Both reduce to six fp64 inner
// products per utterance, <o,o>, <t,t>, <i,i>, <o,t>, <o,i>, <t,i>: one streaming pass
// (float4 loads, fp64 accumulation, one atomicAdd per block and sum) and a per-utterance
// epilogue that evaluates the reference's formulas from them.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "avz_internal.h"

namespace avz {

constexpr int kMetThreads = 256;
constexpr int kMetPerThread = 16;  // samples per thread per block (4 x float4)

__device__ __forceinline__ void met_acc(double (&s)[6], float o, float t, float i) {
  const double ov = o, tv = t, iv = i;
  s[0] = fma(ov, ov, s[0]);
  s[1] = fma(tv, tv, s[1]);
  s[2] = fma(iv, iv, s[2]);
  s[3] = fma(ov, tv, s[3]);
  s[4] = fma(ov, iv, s[4]);
  s[5] = fma(tv, iv, s[5]);
}

// grid (ceil(max_len / (256 * 16)), batch). Each block streams one 4096-sample tile of
// the three signals; a wave's loads cover contiguous 1 KB (VEC: float4 per lane, all
// rows 16-byte aligned) or 256 B (scalar) spans per instruction.
template <bool VEC>
__global__ void __launch_bounds__(kMetThreads) avz_metrics_sums_kernel(MetricsArgs A) {
  __shared__ double red[kMetThreads / 64][6];
  const int b = blockIdx.y;
  const int L = min(A.len[b], A.max_len);
  const float* o = A.est + (long long)b * A.est_stride;
  const float* t = A.tgt + (long long)b * A.tgt_stride;
  const float* i = A.itf + (long long)b * A.itf_stride;
  const long long tile = (long long)blockIdx.x * kMetThreads * kMetPerThread;
  double s[6] = {0, 0, 0, 0, 0, 0};
  if constexpr (VEC) {
    float4 ov[kMetPerThread / 4], tv[kMetPerThread / 4], iv[kMetPerThread / 4];
#pragma unroll
    for (int j = 0; j < kMetPerThread / 4; ++j) {
      const long long n = tile + 4 * ((long long)j * kMetThreads + threadIdx.x);
      if (n + 3 < L) {
        ov[j] = *reinterpret_cast<const float4*>(o + n);
        tv[j] = *reinterpret_cast<const float4*>(t + n);
        iv[j] = *reinterpret_cast<const float4*>(i + n);
      } else {
        float a[3][4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool in = n + e < L;
          a[0][e] = in ? o[n + e] : 0.f;
          a[1][e] = in ? t[n + e] : 0.f;
          a[2][e] = in ? i[n + e] : 0.f;
        }
        ov[j] = make_float4(a[0][0], a[0][1], a[0][2], a[0][3]);
        tv[j] = make_float4(a[1][0], a[1][1], a[1][2], a[1][3]);
        iv[j] = make_float4(a[2][0], a[2][1], a[2][2], a[2][3]);
      }
    }
#pragma unroll
    for (int j = 0; j < kMetPerThread / 4; ++j) {
      met_acc(s, ov[j].x, tv[j].x, iv[j].x);
      met_acc(s, ov[j].y, tv[j].y, iv[j].y);
      met_acc(s, ov[j].z, tv[j].z, iv[j].z);
      met_acc(s, ov[j].w, tv[j].w, iv[j].w);
    }
  } else {
#pragma unroll
    for (int j = 0; j < kMetPerThread; ++j) {
      const long long n = tile + (long long)j * kMetThreads + threadIdx.x;
      if (n < L) met_acc(s, o[n], t[n], i[n]);
    }
  }
#pragma unroll
  for (int q = 0; q < 6; ++q)
    for (int off = 32; off > 0; off >>= 1) s[q] += __shfl_xor(s[q], off, 64);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int q = 0; q < 6; ++q) red[w][q] = s[q];
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    double v = 0.0;
#pragma unroll
    for (int ww = 0; ww < kMetThreads / 64; ++ww) v += red[ww][threadIdx.x];
    atomicAdd(A.sums + (long long)b * 6 + threadIdx.x, v);
  }
}

// One thread per utterance: metrics[b] = {OSINR, OSIR, SDR, SIR} in dB.
__global__ void avz_metrics_final_kernel(MetricsArgs A) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= A.batch) return;
  const double* s = A.sums + (long long)b * 6;
  // an un-normalised output scored as the peak-normalised one: o -> c o in the sums
  const double c = A.est_peak ? 1.0 / ((double)A.est_peak[b] + A.est_eps) : 1.0;
  const double oo = s[0] * c * c, tt = s[1], ii = s[2], ot = s[3] * c, oi = s[4] * c, ti = s[5];
  const double eps = 1e-10;
  const double nt = sqrt(tt) + eps, ni = sqrt(ii) + eps, no = sqrt(oo) + eps;
  // metrics.py:102-123: t^ = t/(|t|+eps), i^ = i/(|i|+eps); alpha = <o,t^>, beta = <o,i^>
  {
    const double tn2 = tt / (nt * nt), in2 = ii / (ni * ni), tin = ti / (nt * ni);
    const double al = ot / nt, be = oi / ni;
    const double pt = al * al * tn2, pi = be * be * in2;
    // |o - al t^ - be i^|^2
    const double pn = oo + pt + pi - 2.0 * al * (ot / nt) - 2.0 * be * (oi / ni) +
                      2.0 * al * be * tin;
    A.metrics[(long long)b * 4 + 0] = 10.0 * log10(pt / (pi + fmax(pn, 0.0) + eps));
    A.metrics[(long long)b * 4 + 1] = 10.0 * log10(pt / (pi + eps));
  }
  // run_metrics.py:6-36: the output is normalised too; +1e-10 on both powers
  {
    const double on2 = oo / (no * no), tn2 = tt / (nt * nt), in2 = ii / (ni * ni);
    const double tin = ti / (nt * ni);
    const double al = ot / (no * nt), be = oi / (no * ni);
    const double pt = al * al * tn2;
    const double pi = be * be * in2 + 1e-10;
    const double pa = on2 + al * al * tn2 + be * be * in2 - 2.0 * al * al - 2.0 * be * be +
                      2.0 * al * be * tin;
    const double pn = fmax(pa, 0.0) + 1e-10;
    A.metrics[(long long)b * 4 + 2] = 10.0 * log10(pt / (pi + pn));
    A.metrics[(long long)b * 4 + 3] = 10.0 * log10(pt / pi);
  }
}

}  // namespace avz

using namespace avz;

extern "C" int avz_launch_metrics(const MetricsArgs* a, void* stream) {
  if (a->batch <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(a->sums, 0, sizeof(double) * 6 * a->batch, st) != hipSuccess) return -3;
  const long long per_block = (long long)kMetThreads * kMetPerThread;
  const dim3 grid((unsigned)((a->max_len + per_block - 1) / per_block), a->batch);
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15u) == 0; };
  const bool vec = al16(a->est) && al16(a->tgt) && al16(a->itf) &&
                   (a->batch == 1 || (a->est_stride % 4 == 0 && a->tgt_stride % 4 == 0 &&
                                      a->itf_stride % 4 == 0));
  if (a->max_len > 0) {
    if (vec)
      hipLaunchKernelGGL(avz_metrics_sums_kernel<true>, grid, dim3(kMetThreads), 0, st, *a);
    else
      hipLaunchKernelGGL(avz_metrics_sums_kernel<false>, grid, dim3(kMetThreads), 0, st, *a);
  }
  hipLaunchKernelGGL(avz_metrics_final_kernel, dim3((a->batch + 63) / 64), dim3(64), 0, st, *a);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
