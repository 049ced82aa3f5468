// reg_transpose.hpp — experiment (round 3): a 32 x 32 transpose in registers (DPP +
// v_permlane16_swap) as a replacement for Fft1024x2's LDS transpose. Measured by
// fftbench.py variant 29 against variant 4: 3.17 vs 4.28 FFT/us/CU -- the 544 VALU
// instructions it compiles to (the DPP moves are not fused into the selects) cost more than
// the LDS round trip, and even the 288-instruction ideal would not pay: the FFT is VALU-bound
// once the transpose moves to the VALU. Not used by the product kernels.
#pragma once
#include "../../real-time-audio-visual-zooming_amd/csrc/avz_common.hpp"
namespace avz {
// ------------------------------------------------------------ register transpose
// 32 x 32 transpose inside each 32-lane group without LDS: lane l register r <- lane r
// register l, as five butterfly exchanges on the lane / register index bits. For bit d the
// register pair (a = reg r, c = reg r | d) becomes (a, partner's a) on lanes with lane bit d
// clear and (partner's c, c) on lanes with it set, partner = lane ^ d: d = 1, 2 by DPP
// quad_perm, 4, 8 by DPP row shifts / rotation (cndmask-selected), 16 by v_permlane16_swap
// (one instruction per register pair). 288 VALU instructions per 32 complex registers,
// no LDS traffic.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), CTRL, 0xF, 0xF, true));
}
template <int D>
__device__ __forceinline__ void xchg_bit(float& a, float& c, bool hi) {
  if constexpr (D == 16) {
    const auto rr = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(c), false, false);
    a = __uint_as_float(rr[0]);
    c = __uint_as_float(rr[1]);
  } else {
    // DPP controls: partner = lane ^ D
    constexpr int UP = D == 1 ? 0xB1 : D == 2 ? 0x4E : D == 4 ? 0x104 : 0x128;  // lane l <- l + D (bit clear)
    constexpr int DN = D == 1 ? 0xB1 : D == 2 ? 0x4E : D == 4 ? 0x114 : 0x128;  // lane l <- l - D (bit set)
    const float pc = dpp_mov<DN>(c);  // partner's c, for lanes with the bit set
    const float pa = dpp_mov<UP>(a);  // partner's a, for lanes with the bit clear
    a = hi ? pc : a;
    c = hi ? c : pa;
  }
}
__device__ __forceinline__ void transpose32_regs(cf (&v)[32], int l) {
  const bool b0 = l & 1, b1 = (l >> 1) & 1, b2 = (l >> 2) & 1, b3 = (l >> 3) & 1;
  static_for<0, 32>([&](auto r) {
    if constexpr ((r & 1) == 0) { xchg_bit<1>(v[r].x, v[r + 1].x, b0); xchg_bit<1>(v[r].y, v[r + 1].y, b0); }
  });
  static_for<0, 32>([&](auto r) {
    if constexpr ((r & 2) == 0) { xchg_bit<2>(v[r].x, v[r + 2].x, b1); xchg_bit<2>(v[r].y, v[r + 2].y, b1); }
  });
  static_for<0, 32>([&](auto r) {
    if constexpr ((r & 4) == 0) { xchg_bit<4>(v[r].x, v[r + 4].x, b2); xchg_bit<4>(v[r].y, v[r + 4].y, b2); }
  });
  static_for<0, 32>([&](auto r) {
    if constexpr ((r & 8) == 0) { xchg_bit<8>(v[r].x, v[r + 8].x, b3); xchg_bit<8>(v[r].y, v[r + 8].y, b3); }
  });
  static_for<0, 32>([&](auto r) {
    if constexpr ((r & 16) == 0) { xchg_bit<16>(v[r].x, v[r + 16].x, false); xchg_bit<16>(v[r].y, v[r + 16].y, false); }
  });
}

}  // namespace avz
