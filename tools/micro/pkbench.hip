// Packed-fp32 register DFTs against the scalar ones (avz_fft.hpp): FFT arithmetic only
// (a twiddle multiply + two dft32 per iteration on 32 registers per lane, no LDS), 4-wave
// blocks at two per CU, as fftbench's "x2 arithmetic only" variant; and a check kernel that
// runs one transform both ways. Timed from tools/micro/pkbench.py.
#include <hip/hip_runtime.h>
#include "pk_fft.hpp"
using namespace avz;

template <bool PK>
__global__ void __launch_bounds__(256, 2) pk_arith(const float* in, float* out, int iters) {
  const int lane = threadIdx.x & 63, l = lane & 31;
  cf v[32];
  static_for<0, 32>([&](auto r) { v[r] = {in[(l + 32 * r) & 1023], in[(l + 32 * r + 7) & 1023]}; });
  for (int it = 0; it < iters; ++it) {
    if constexpr (PK) {
      pk::f2 p[32];
      static_for<0, 32>([&](auto k) { p[k] = pk::f2{v[k].x, v[k].y}; });
      static_for<0, 32>([&](auto k) { p[k] = pk::cmul(p[k], pk::f2{0.70710678f, -0.70710678f}); });
      pk::dft32(p);
      __builtin_amdgcn_sched_barrier(0);
      pk::dft32(p);
      static_for<0, 32>([&](auto k) { v[k] = cf{p[k].x, p[k].y}; });
    } else {
      static_for<0, 32>([&](auto k) { v[k] = c_mul(v[k], cf{0.70710678f, -0.70710678f}); });
      dft32(v);
      __builtin_amdgcn_sched_barrier(0);
      dft32(v);
    }
  }
  float acc = 0;
  static_for<0, 32>([&](auto k) { acc += v[k].x + v[k].y; });
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// one dft32 of 64 lanes' inputs both ways: out[0 .. 4096) scalar, [4096 .. 8192) packed
__global__ void pk_check(const float* in, float* out) {
  const int lane = threadIdx.x;
  cf v[32];
  pk::f2 p[32];
  static_for<0, 32>([&](auto r) {
    v[r] = {in[lane * 64 + 2 * r], in[lane * 64 + 2 * r + 1]};
    p[r] = pk::f2{v[r].x, v[r].y};
  });
  dft32(v);
  pk::dft32(p);
  static_for<0, 32>([&](auto r) {
    out[lane * 64 + 2 * r] = v[r].x;
    out[lane * 64 + 2 * r + 1] = v[r].y;
    out[4096 + lane * 64 + 2 * r] = p[r].x;
    out[4096 + lane * 64 + 2 * r + 1] = p[r].y;
  });
}

extern "C" int pk_run(int packed, const float* in, float* out, int blocks, int iters) {
  if (packed)
    hipLaunchKernelGGL(pk_arith<true>, dim3(blocks), dim3(256), 0, 0, in, out, iters);
  else
    hipLaunchKernelGGL(pk_arith<false>, dim3(blocks), dim3(256), 0, 0, in, out, iters);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
extern "C" int pk_check_run(const float* in, float* out) {
  hipLaunchKernelGGL(pk_check, dim3(1), dim3(64), 0, 0, in, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
