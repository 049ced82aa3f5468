// pk_fft.hpp -- packed-fp32 form of Fft1024x2's register DFTs (micro-benchmark only, not in
// the shipped kernels): a complex value is one float2 vector, so complex adds, subtracts and
// the tangent-form twiddled butterflies issue as v_pk_add_f32 / v_pk_fma_f32 (two fp32
// results per lane per instruction, 64 FLOP/clk/SIMD against 32 for scalar FMA). Same
// algorithm and constants as avz_fft.hpp's dft4 / dft4_tw / bfly_tw / dft16 / dft32, so the
// instruction count and the throughput compare one to one (tools/micro/fftbench.py 30, 31).
#pragma once
#include "../../real-time-audio-visual-zooming_amd/csrc/avz_fft.hpp"

namespace avz {
namespace pk {

typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 rot(f2 b) { return f2{-b.y, b.x}; }  // i b
__device__ __forceinline__ f2 splat(float s) { return f2{s, s}; }

// y0 = a + w b, y1 = a - w b, w = W32^J (compile time), tangent form as bfly_tw
template <int J>
__device__ __forceinline__ void bfly_tw(f2 a, f2 b, f2& y0, f2& y1) {
  constexpr int j = ((J % 32) + 32) % 32;
  if constexpr (j == 0) {
    y0 = a + b;
    y1 = a - b;
  } else if constexpr (j == 8) {  // w = -i: w b = -i b
    y0 = a - rot(b);
    y1 = a + rot(b);
  } else if constexpr (j == 16) {
    y0 = a - b;
    y1 = a + b;
  } else if constexpr (j == 24) {  // w = +i
    y0 = a + rot(b);
    y1 = a - rot(b);
  } else {
    constexpr float c = W32::c[j], s = W32::s[j];
    if constexpr ((c < 0 ? -c : c) >= (s < 0 ? -s : s)) {
      constexpr float t = s / c;  // w b = c (b + t i b)
      const f2 u = fma2(splat(t), rot(b), b);
      y0 = fma2(splat(c), u, a);
      y1 = fma2(splat(-c), u, a);
    } else {
      constexpr float t = c / s;  // w b = s (t b + i b)
      const f2 u = fma2(splat(t), b, rot(b));
      y0 = fma2(splat(s), u, a);
      y1 = fma2(splat(-s), u, a);
    }
  }
}

__device__ __forceinline__ void dft4(f2& a0, f2& a1, f2& a2, f2& a3) {
  const f2 t0 = a0 + a2, t1 = a0 - a2, t2 = a1 + a3, t3 = a1 - a3;
  a0 = t0 + t2;
  a2 = t0 - t2;
  a1 = t1 - rot(t3);  // t1 - i t3
  a3 = t1 + rot(t3);
}

template <int J1>
__device__ __forceinline__ void dft4_tw(f2& a0, f2& a1, f2& a2, f2& a3) {
  f2 t0, t1, sm, df;
  bfly_tw<2 * J1>(a0, a2, t0, t1);
  bfly_tw<2 * J1>(a1, a3, sm, df);
  f2 o0, o1, o2, o3;
  bfly_tw<J1>(t0, sm, o0, o2);
  bfly_tw<J1 + 8>(t1, df, o1, o3);
  a0 = o0;
  a1 = o1;
  a2 = o2;
  a3 = o3;
}

__device__ __forceinline__ void dft16(f2 (&v)[16]) {
  static_for<0, 4>([&](auto n2) { dft4(v[n2], v[n2 + 4], v[n2 + 8], v[n2 + 12]); });
  f2 t[16];
  static_for<0, 4>([&](auto k1) {
    f2 a0 = v[0 + 4 * k1], a1 = v[1 + 4 * k1], a2 = v[2 + 4 * k1], a3 = v[3 + 4 * k1];
    dft4_tw<2 * k1>(a0, a1, a2, a3);
    t[k1 + 0] = a0;
    t[k1 + 4] = a1;
    t[k1 + 8] = a2;
    t[k1 + 12] = a3;
  });
  static_for<0, 16>([&](auto i) { v[i] = t[i]; });
}

__device__ __forceinline__ void dft32(f2 (&v)[32]) {
  f2 e[16], o[16];
  static_for<0, 16>([&](auto i) {
    e[i] = v[2 * i];
    o[i] = v[2 * i + 1];
  });
  dft16(e);
  dft16(o);
  static_for<0, 16>([&](auto k) { bfly_tw<k>(e[k], o[k], v[k], v[k + 16]); });
}

// complex multiply: (a.x w.x - a.y w.y, a.x w.y + a.y w.x) = a.x w + a.y (i w)
__device__ __forceinline__ f2 cmul(f2 a, f2 w) { return fma2(splat(a.y), rot(w), splat(a.x) * w); }

}  // namespace pk
}  // namespace avz
