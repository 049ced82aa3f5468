// avz_chunked_k.hpp — kernels of the chunk-parallel form of the mask-driven MVDR chain (gfx950).
//
// An utterance's frames are cut into 32-frame chunks; each (chunk, utterance) pair is
// one 256-thread (4-wave) workgroup, two per CU, so a batch of B utterances of T
// frames launches B * ceil(T / 32) independent blocks instead of B long ones.
//
//   analysis   frames -> window -> FFT (mic pair / reference pair packed) -> LDS;
//              thread-per-bin masks (IBM / IPD / external) and masked 2x2 covariance
//              partials over the chunk (fp32) -> part[b][c][5][F]; IBM bits -> mwords.
//   solve      one thread per (utterance, bin): partials summed in fp64, closed-form
//              2x2 MVDR with the plan's steering table -> coef[b][k] (alpha, beta).
//   synthesis  frames -> FFT again -> apply w^H y +
//              post-filter -> two frames packed per inverse FFT -> windowed OLA of the
//              chunk's 31 interior segments -> out; the chunk's first / last
//              half-frame contributions -> heads/tails;
//              block max |out| -> atomicMax(peak_u[b]).
//   finalize   chunk-boundary segments (tails[c-1] + heads[c]), utterance peak,
//              optional in-place peak normalisation of the chunk's segments.
//
// Reference semantics as avz_kernels.hip: rt_av_zoom/core/oracle_debug.py:27-97,
// rt_av_zoom/core/masked_mvdr.py:50-132,
// rt_av_zoom/core/full_audio_generating_pipeline/inference.py:88-118.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <type_traits>

#include "avz_common.hpp"
#include "avz_ibm_exact.hpp"
#ifndef AVZ_NO_IBM_CERT  // diagnostic build: no certificate in the reference-bit path
#define AVZ_NO_IBM_CERT 0
#endif
#ifndef AVZ_CERT_PARTS  // diagnostic: bit 0 frame energy, bit 1 per-bin test, bit 2 min form
#define AVZ_CERT_PARTS 7
#endif

namespace avz {

// Rejected variants of these kernels (round-chained synthesis, finalize folded into
// synthesis, the half-size real inverse, precomputed synthesis windows, LDS-twiddle
// stage-1 stores, ...) are recorded in DESIGN.md §6 and kept under tools/experiments/;
// this file holds only the shipped paths.

constexpr int kChunk = 32;      // frames per chunk = bits of one mask word
constexpr int kSC1 = 16;        // buffer-op cache policy bit: sc1 (L1-bypassing loads, gfx940+)
typedef int v4i_t __attribute__((ext_vector_type(4)));
constexpr int kCThreads = 256;  // 4 waves

template <int N>
struct CGeo {
  using C = KCfg<N>;
  static constexpr int NT = kCThreads;
  static constexpr int NWAVE = NT / 64;
  static constexpr int H = N / 2;
  static constexpr int F = N / 2 + 1;
  static constexpr int NSLOT = NWAVE * C::FPW;     // 8 frame slots
  static constexpr int BPT = (N / 2) / NT;          // bins k < N/2 per thread
  static constexpr int SLOT_LDS = NWAVE * C::WAVE_BYTES;
  static constexpr int TW_OFF = SLOT_LDS;
  static constexpr int MISC_OFF = TW_OFF + C::TW_BYTES;
  static constexpr int LDS_BYTES = MISC_OFF + 64;
  static_assert(BPT >= 1 && BPT * NT == N / 2, "bin mapping");
  static constexpr int BLOCKS = C::BLOCKS_PER_CU;  // resident blocks per CU (= waves per SIMD)
  static_assert(BLOCKS * LDS_BYTES <= 160 * 1024, "resident blocks per CU");
};

// Synthesis frames per lane group per step: KCfg's SYN_R, except the N = 512 external-mask
// post-filters, whose strided mask reads need the registers of the second frame (at R = 2
// they spilled 44-72 B per lane).
template <int N, int PF>
constexpr int kSynR = (N == 512 && (PF == PF_EXT_FLOOR || PF == PF_EXT_MUL)) ? 1 : KCfg<N>::SYN_R;

// Synthesis geometry: as CGeo with R frames per lane group per step (NSLOT frame slots,
// each a lane group's transform area; slot s is "virtual wave" s / FPW of the slot area).
template <int N, int R_ = KCfg<N>::SYN_R>
struct SGeo {
  using C = KCfg<N>;
  static constexpr int NT = kCThreads;
  static constexpr int NWAVE = NT / 64;
  static constexpr int R = R_;
  static constexpr int H = N / 2;
  static constexpr int F = N / 2 + 1;
  static constexpr int NSLOT = NWAVE * C::FPW * R;
  static constexpr int BPT = (N / 2) / NT;
  static constexpr int SLOT_LDS = NWAVE * C::WAVE_BYTES * R;
  static constexpr int TW_OFF = SLOT_LDS;
  static constexpr int MISC_OFF = TW_OFF + C::TW_BYTES;
  static constexpr int LDS_BYTES = MISC_OFF + 64;
  static constexpr int BLOCKS = C::SYN_BLOCKS_PER_CU;
  static_assert(BLOCKS * LDS_BYTES <= 160 * 1024, "resident synthesis blocks per CU");
};

// Per-lane analysis window * 1/sum(win) and synthesis window * sum(win)/N terms.
template <int N>
struct WinCoef {
  float a0, ac, as, s0, sc, ss;
  __device__ __forceinline__ void init(const LaneMap<N>& lm) {
    double s, c;
    sincospi(2.0 * lm.in0 / N, &s, &c);
    const double sca = 2.0 / N;
    a0 = (float)(0.5 * sca);
    ac = (float)(0.5 * sca * c);
    as = (float)(0.5 * sca * s);
    sincospi(2.0 * lm.out0 / N, &s, &c);
    s0 = 0.25f;
    sc = (float)(0.25 * c);
    ss = (float)(0.25 * s);
  }
};

// 1 / (win[m]^2 + win[m + N/2]^2): the istft window-sum normalisation of one sample.
template <int N>
__device__ __forceinline__ float inv_wsum(int m) {
  const float c1 = cospif(2.0f * (float)m / (float)N);
  const float wa = 0.5f - 0.5f * c1, wb = 0.5f + 0.5f * c1;
  return 1.0f / (wa * wa + wb * wb);
}

// Lane constants of the chain kernels (FFT twiddle registers, lane map, window terms,
// the synthesis OLA normalisation and inverse window terms): computed once per block by
// the persistent kernels, not per item (the fp64 sincospi calls cost 1-2 us per item).
template <int N>
struct LaneConst {
  typename KCfg<N>::Fft fft;
  LaneMap<N> lm;
  WinCoef<N> wc;
  float inv[4];  // synthesis OLA: 1 / window-square sum of samples m0 .. m0 + 3
  __device__ __forceinline__ void init(int tid) {
    const int lane = tid & 63;
    fft.init(lane);
    lm.init(lane);
    wc.init(lm);
    const int m0 = 4 * (tid % (N / 8));  // synthesis OLA role (N/2 / 4 float4 groups)
#pragma unroll
    for (int i = 0; i < 4; ++i) inv[i] = inv_wsum<N>(m0 + i);
  }
};

// Analysis window of a lane's points: register r holds sample n0 + IN_STRIDE r, weight
// w = a0 - ac cos(2 pi IN_STRIDE r / N) + as sin(...) (angle addition on the lane's n0).
// Registers PPL/2 apart are N/2 samples apart, where the periodic Hann window satisfies
// w[n + N/2] = 2 a0 - w[n]: one subtraction instead of two FMAs for the upper half.
template <int N = 1024, int PPL>
__device__ __forceinline__ void window_apply(cf (&v)[PPL], float a0, float ac, float as) {
  using C = KCfg<N>;
  static_assert(C::IN_STRIDE * (PPL / 2) == N / 2, "upper-half registers are N/2 later");
  const float a2 = a0 + a0;
  static_for<0, PPL / 2>([&](auto r) {
    constexpr int j = (C::IN_STRIDE * 32 / N) * r;  // 2 pi (IN_STRIDE r)/N = 2 pi j/32
    constexpr float cr = W32::c[j % 32], sr = -W32::s[j % 32];
    const float w = fmaf(as, sr, fmaf(-ac, cr, a0));
    v[r] = c_scale(v[r], w);
    v[r + PPL / 2] = c_scale(v[r + PPL / 2], a2 - w);
  });
}

// IBM decision |S_int| > |S_tgt| (oracle_debug.py:49-53, strict) from the packed reference
// pair z = tgt + i int: 2T = zr + conj(zrp), 2I = (zr - conj zrp)/i, and
// |2T|^2 - |2I|^2 = 4 Re(zr zrp), so noise <=> Re(zr zrp) < 0 (one product, one fma).
__device__ __forceinline__ bool ibm_noise(cf zr, cf zrp) {
  return fmaf(zr.x, zrp.x, -(zr.y * zrp.y)) < 0.0f;
}

// Sum over the 32 lanes of a lane group (DPP within rows, v_permlane16_swap across them).
__device__ __forceinline__ float group32_sum(float e) {
  e += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(e), 0xB1, 0xF, 0xF, false));
  e += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(e), 0x4E, 0xF, 0xF, false));
  e += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(e), 0x141, 0xF, 0xF, false));
  e += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(e), 0x140, 0xF, 0xF, false));
  float lo, hi;
  xhalf<16>(e, lo, hi);
  return lo + hi;
}
__device__ __forceinline__ float frame_energy(const cf (&v)[32]) {
  float e = 0.0f;
  static_for<0, 32>([&](auto r) {
    e = fmaf(v[r].x, v[r].x, e);
    e = fmaf(v[r].y, v[r].y, e);
  });
  return e;
}
// Window + forward FFT with the lane's twiddles in registers (N = 1024 analysis). Both
// FFT stages store each output pair as it is formed (the transpose scratch, then the
// spectrum); after(k) runs right after spectrum output k is stored (the next step's load
// into register k).
struct NoAfter {
  template <class K>
  __device__ __forceinline__ void operator()(K) const {}
};
// en (non-null: IBM reference waves of the plans without the reference-bit hand-off): the
// group's windowed frame energy, the exact-IBM certificate's scale (ibm_exact_frames).
template <class After = NoAfter>
__device__ __forceinline__ void window_fft_reg(cf (&v)[32], const WinCoef<1024>& wc,
                                               const Fft1024x2& fft, cf* spec,
                                               const cf (&tw_reg)[31], const LaneMap<1024>& lm,
                                               After&& after = After{}, float* en = nullptr) {
  window_apply(v, wc.a0, wc.ac, wc.as);
  if (en) *en = group32_sum(frame_energy(v));
  fft.stage1_reg_st(v, spec, tw_reg);
  fft.transpose_read(v, spec);
  fft.stage2_emit(v, [&](auto k, cf x) {
    spec[lm.out0 + 32 * k] = x;
    after(k);
  });
}

// Reference pair of the IBM mask (N = 1024, register twiddles): the reference spectrum is
// only needed for one bit per bin, noise <=> Re(Zr[k] Zr[N - k]) < 0 (ibm_noise). Lane l
// holds Zr[l + 32 k]. Only the upper-half outputs (k >= 16) are stored, as formed, their
// registers taking their next-step loads during the stage; the lower half stays in
// registers, the lane reads the partners N - (l + 32 k), k < 16, back (all in the stored
// upper half but DC's, which is its own partner), publishes the 16 bits as word l of the
// slot (bytes 0..127) and only then reloads registers 0-15 (analysis 80.7-80.9 -> 79.1-79.5
// us against storing all 32 and reading both operands back, profiles/r04/ab_ref_half.txt).
// The Nyquist bin (lane 0, k = 16) stays readable at spec[N / 2].
//
// Certificate (avz_ibm_exact.hpp): the group's windowed frame energy gives delta = cert
// ||z|| (cert = kappa eps, ChainArgs::ibm_cert), a bound on every output bin's error; a bin
// pair whose |Re(Zr[k] Zr[N - k])| does not clear (2 sqrt 2 + 1) delta max(|components|,
// delta) could be decided either way by that error. A frame with such a bin (DC included)
// publishes no noise bits and returns true: the item's exact path decides it
// (ibm_exact_item). delta goes to dl; the Nyquist bin (lane 0, k = 16, left in spec[N / 2])
// is certified by the bin phase's Nyquist wave with it.
// true when the pair's decision is not certified by the error bound dl (= delta)
__device__ __forceinline__ bool ibm_uncertain(cf zr, cf zrp, float dl) {
  const float d = fmaf(zr.x, zrp.x, -(zr.y * zrp.y));
  const float m = fmaxf(fmaxf(fabsf(zr.x), fabsf(zr.y)), fmaxf(fmaxf(fabsf(zrp.x), fabsf(zrp.y)), dl));
  return fabsf(d) < 3.9f * dl * m;
}
template <class After = NoAfter>
__device__ __forceinline__ uint32_t window_fft_reg_ibm_bits(cf (&v)[32], const WinCoef<1024>& wc,
                                                        const Fft1024x2& fft, cf* spec,
                                                        const cf (&tw_reg)[31],
                                                        const LaneMap<1024>& lm, float eg0,
                                                        float eg1, float cert, float& dl,
                                                        After&& after = After{}) {
  constexpr int N = 1024;
  window_apply(v, wc.a0, wc.ac, wc.as);
  const int l = lm.out0;
  fft.stage1_reg_st(v, spec, tw_reg);
  fft.transpose_read(v, spec);
  fft.stage2_emit(v, [&](auto k, cf x) {
    if constexpr (decltype(k)::value >= 16) {
      spec[l + 32 * k] = x;
      after(k);
    }
  });
  dl = cert * sqrtf(lm.grp ? eg1 : eg0);  // delta >= kappa eps ||z|| (the caller's scale)
  __builtin_amdgcn_wave_barrier();
  // the word is built from bit 15 down (w = 2 w + bit): a select of 1 << k per bin held the
  // 16 constants in VGPRs for the whole kernel
  uint32_t w = 0u;
  bool unc = false;
  float slack = __builtin_inff();  // min over bins of |D| - 3.9 dl m (< 0: uncertain)
  const float dl39 = 3.9f * dl;
  static_for<0, 16>([&](auto kk) {
    constexpr int k = 15 - decltype(kk)::value;
    const int m = l + 32 * k;
    cf zp = spec[(N - m) & (N - 1)];
    if (k == 0 && l == 0) zp = v[0];  // DC: its own partner (index 0 is not stored)
    w = (w << 1) | (ibm_noise(v[k], zp) ? 1u : 0u);
    if (!AVZ_NO_IBM_CERT && (AVZ_CERT_PARTS & 2)) {
      if (AVZ_CERT_PARTS & 4) {
        const float d = fmaf(v[k].x, zp.x, -(v[k].y * zp.y));
        const float mm = fmaxf(fmaxf(fabsf(v[k].x), fabsf(v[k].y)),
                               fmaxf(fmaxf(fabsf(zp.x), fabsf(zp.y)), dl));
        slack = fminf(slack, fmaf(-dl39, mm, fabsf(d)));
      } else {
        unc |= ibm_uncertain(v[k], zp, dl);
      }
    }
  });
  if (AVZ_CERT_PARTS & 4) unc = slack < 0.0f;
  uint32_t um = 0u;  // the lane's uncertain bins (bit k: bin l + 32 k), as its word w
  if (__ballot(unc) != 0ull) {  // rare (wave-uniform): which bins, by the same test
    static_for<0, 16>([&](auto kk) {
      constexpr int k = 15 - decltype(kk)::value;
      const int m = l + 32 * k;
      cf zp = spec[(N - m) & (N - 1)];
      if (k == 0 && l == 0) zp = v[0];
      const float d = fmaf(v[k].x, zp.x, -(v[k].y * zp.y));
      const float mm = fmaxf(fmaxf(fabsf(v[k].x), fabsf(v[k].y)),
                             fmaxf(fmaxf(fabsf(zp.x), fabsf(zp.y)), dl));
      um = (um << 1) | (fmaf(-dl39, mm, fabsf(d)) < 0.0f ? 1u : 0u);
    });
    w &= ~um;  // their decisions are the exact path's
  }
  reinterpret_cast<uint32_t*>(spec)[l] = w;
  static_for<0, 16>([&](auto k) { after(k); });
  return um;
}

// Window + forward FFT of the synthesis kernel and of the N = 512 analysis kernel:
//  N = 1024: factored register twiddles (Fft1024x2::stage1_ab_st), both stages' outputs
//            stored as formed (synthesis 73.7-74.1 -> 72.7-73.1 us, profiles/r03d/ab_more.txt);
//  N = 512, IL512: the interleaved Fft512x2 (the two-block synthesis kernel: 81.0 -> 80.3
//            us; the three-block N = 512 analysis kernel ran slower with it, 81.3 -> 82.5 us).
template <int N, bool IL512 = false, class After = NoAfter>
__device__ __forceinline__ void window_fft(cf (&v)[KCfg<N>::PPL], const WinCoef<N>& wc,
                                           const typename KCfg<N>::Fft& fft, cf* spec,
                                           const LaneMap<N>& lm, After&& after = After{},
                                           float* en = nullptr) {
  using C = KCfg<N>;
  float a0 = wc.a0, ac = wc.ac, as = wc.as;
  opaque(a0);
  opaque(ac);
  opaque(as);
  window_apply<N>(v, a0, ac, as);
  if (en) {  // the lane group's windowed frame energy (exact-IBM certificate scale)
    float e = 0.0f;
    static_for<0, C::PPL>([&](auto r) {
      e = fmaf(v[r].x, v[r].x, e);
      e = fmaf(v[r].y, v[r].y, e);
    });
    *en = group32_sum(e);
  }
  if constexpr (N == 1024) {
    fft.stage1_ab_st(v, spec);
    fft.transpose_read(v, spec);
    fft.stage2_emit(v, [&](auto k, cf x) {
      spec[lm.out0 + C::OUT_STRIDE * k] = x;
      after(k);
    });
  } else if constexpr (IL512) {
    fft.forward_emit(v, spec, [&](auto k, cf x) {
      spec[lm.out0 + C::OUT_STRIDE * k] = x;
      after(k);
    });
  } else {
    fft.forward(v, spec);
    static_for<0, C::PPL>([&](auto k) { spec[lm.out0 + C::OUT_STRIDE * k] = v[k]; });
  }
}

// Shared-half loads of a wave's frame pair (Fft1024x2, N = 1024): frames 2w and 2w + 1
// overlap by N/2 = 16 registers, so the wave loads 1536 samples per stream (24 loads)
// instead of 2 x 1024 (32). Lane group 1 holds its frame rotated by N/2 — register r < 16
// is sample 512 + 32 r + l of the frame, r >= 16 is sample 32 (r - 16) + l, i.e. the
// second half of frame 2w — so both groups take the shared half in the same registers:
//   v[j], j < 16:   group 0 samples sp + 32 j, group 1 sp + 1024 + 32 j (own halves);
//   v[16 + 2 i]:    group 0 sample sp + 512 + 64 i, group 1 the next 32 (shared half),
//                   spread to v[16 + 2 i] / v[17 + 2 i] on every lane by one
//                   v_permlane32_swap per float once the loads have landed (pair_finish).
// sp = the pair's first sample + l. The rotation is a circular shift by N/2 of group 1's
// frame: its window weights swap halves (ac, as negated: window_apply's w <-> 2 a0 - w)
// and its spectrum comes out as (-1)^k X[k], undone by (-1)^k1 folded into the stage-1
// twiddles. Analysis kernel only: in the synthesis kernel (LDS twiddles, the sign folded
// into the odd frames' post-filter gain) it measured 73.1 -> 75.1 us against the analysis
// kernel's 80.3 -> 79.0 (profiles/r02z/ab_experiments.txt).
template <bool NONNEG>
__device__ __forceinline__ void pair_loads(cf (&v)[32], rsrc_t r0, rsrc_t r1, int sp, int g) {
  static_for<0, 16>([&](auto j) {
    const int e = sp + 1024 * g + 32 * j;
    v[j].x = NONNEG ? bload_nn(r0, e) : bload(r0, e);
    v[j].y = NONNEG ? bload_nn(r1, e) : bload(r1, e);
  });
  static_for<0, 8>([&](auto i) {
    const int e = sp + 512 + 32 * (2 * i) + 32 * g;
    v[16 + 2 * i].x = NONNEG ? bload_nn(r0, e) : bload(r0, e);
    v[16 + 2 * i].y = NONNEG ? bload_nn(r1, e) : bload(r1, e);
  });
}
__device__ __forceinline__ void pair_finish(cf (&v)[32]) {
  static_for<0, 8>([&](auto i) {
    const auto rx = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[16 + 2 * i].x),
                                                     __float_as_uint(v[16 + 2 * i].x), false, false);
    const auto ry = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[16 + 2 * i].y),
                                                     __float_as_uint(v[16 + 2 * i].y), false, false);
    v[16 + 2 * i] = cf{__uint_as_float(rx[0]), __uint_as_float(ry[0])};
    v[17 + 2 * i] = cf{__uint_as_float(rx[1]), __uint_as_float(ry[1])};
  });
}

// Samples of utterance b: the device length clamped to the host-validated max_len (so an
// inconsistent len[] never moves an access outside the caller's rows), or max_len for all.
// A piece's seam half: written through to memory (agent-scope stores, sc1), so the last
// piece of the utterance to arrive -- on any XCD -- reads it in the same kernel.
// (row: block-uniform base of n floats; i: the thread's element)
__device__ __forceinline__ void store_through(float* row, int n, int i, float4 v) {
  const v4i_t d = {__float_as_int(v.x), __float_as_int(v.y), __float_as_int(v.z),
                   __float_as_int(v.w)};
  __builtin_amdgcn_raw_buffer_store_b128(d, make_rsrc(row, n), 4 * i, 0, kSC1);
}

// len[] is read-only for the whole chain, so it is read through the constant address space:
// with a wave-uniform b that is one s_load_dword (scalar cache) instead of a vector load
// plus readfirstlane on the item / unit start's dependent latency chain.
template <class CA>
__device__ __forceinline__ int utt_len(CA& A, int b) {
  if (!A.len) return A.max_len;
  const __attribute__((address_space(4))) int* lc =
      (const __attribute__((address_space(4))) int*)(A.len);
  return min(lc[b], A.max_len);
}

// Mask value m and covariance weight of one (bin, frame).
template <int MASK>
__device__ __forceinline__ float bin_mask(const ChainArgs& A, int b, cf x0, cf x1, cf zr,
                                          cf zrp, int k, int t, bool& noise, float& wgt) {
  if constexpr (MASK == MASK_IBM) {
    noise = ibm_noise(zr, zrp);
    wgt = noise ? 1.0f : 0.0f;
    return wgt;
  } else if constexpr (MASK == MASK_IPD) {
    wgt = ipd_weight(x0, x1);
    return wgt;
  } else if constexpr (MASK == MASK_ONES) {  // unmasked covariance (SRP, MPDR)
    wgt = 1.0f;
    return 1.0f;
  } else {
    const float M =
        A.ext_mask[(long long)b * A.mask_sb + (long long)k * A.mask_sf + (long long)t * A.mask_st];
    const float m = 1.0f - M;
    wgt = m + A.weight_eps;
    return m;
  }
}

// IRM post-filter gain of one (bin, frame) from the packed reference pair
// (oracle_reverb.py:143-156): with 2T, 2I the unscaled split, |2T|^2/(|2T|^2+|2I|^2+4e-10)
// equals P_t/(P_t + P_i + 1e-10).
__device__ __forceinline__ float irm_gain(cf zr, cf zrp) {
  const float tr = zr.x + zrp.x, ti = zr.y - zrp.y;
  const float ir = zr.y + zrp.y, ii = zr.x - zrp.x;
  const float pt = tr * tr + ti * ti, pi = ir * ir + ii * ii;
  return sqrtf(pt / (pt + pi + 4e-10f));
}

// ================================ analysis ================================
// The kernel's ChainArgs read afresh from the kernarg segment through an opaque address:
// fields only the exact path uses were otherwise loaded at the kernel's start and held
// through the step loop (12 SGPRs more, spilled into VGPR lanes).
// In the constant address space: its fields are scalar loads (uniform). Through a generic
// pointer they were vector loads the compiler took for divergent: every buffer load of the
// exact path then ran in a descriptor waterfall loop.
using KArgs = const __attribute__((address_space(4))) ChainArgs;
__device__ __forceinline__ KArgs& kernarg_chain_args() {
  uintptr_t u = (uintptr_t)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(u));
  return *(KArgs*)u;
}
struct NoTw {};
using Tw1024 = cf[31];  // the register-twiddle path's twiddles (a type tag here)
// Exact-phase LDS layout (after the persistent loop; nothing of the loop's is live): the
// waves' fp64 transform buffers, then (same bytes, after a barrier) the round's mic spectra in
// frame slots 0-3; the round's reference magnitudes; the fp64 twiddle table. The fp32
// twiddle table (TW_OFF, the mic transforms') is kept.
// The round's frames packed one per byte (0xff: none): frame i, or -1, for a block- or
// lane-varying i by shifts (an int array indexed so went to scratch memory, selects included)
__device__ __forceinline__ int pick(uint32_t packed, int i) {
  return (int)(signed char)(packed >> (8 * i));
}
template <int N>
struct XLds {
  using C = KCfg<N>;
  using X = XGeo<N>;
  static constexpr int FR = 4;                              // frames per round
  static constexpr int MP = N / 2 + 4;                      // magnitude row (16-B aligned)
  static constexpr int MIC_BYTES = FR / C::FPW * C::WAVE_BYTES;
  static constexpr int MAG_OFF = (4 * X::SCRATCH > MIC_BYTES) ? 4 * X::SCRATCH : MIC_BYTES;
  static constexpr int TWL_OFF = MAG_OFF + 2 * FR * MP * 4;
  static constexpr int WIN_OFF = TWL_OFF + (N / 2) * 16;    // fp32 window [N]
  static constexpr int SLOT_OFF = WIN_OFF + N * 4;           // XSlot[FR], the round's frames
  static constexpr int SCAN_OFF = SLOT_OFF + FR * 32;       // int[256]: exact_sparse's items
                                                            // (between pieces: exact_claim's
                                                            // 64 candidates)
  static constexpr int SCAN_INTS = 256;
  static constexpr int WL = 32;                             // frames one block decides
  static constexpr int WL_OFF = SCAN_OFF + 256 * 4;         // int4[WL]: (unit, f, e, -)
  static constexpr int CTL_OFF = WL_OFF + WL * 16;          // int[8]: counts, mode
  static constexpr int END = CTL_OFF + 32;
  static_assert(C::FPW == 2 && END <= CGeo<N>::SLOT_LDS, "exact phase LDS");
};

// One deferred frame of the exact path (block-uniform, in LDS): analysis unit, chunk frame f,
// (e: unused), utterance b and length L, chunk c,
// flags bit 0: the frame deferred whole (reference-bit path), bit 1: its Nyquist bin deferred.
struct XSlot {
  int unit, f, e, b, L, c, flags, pad;
};
// slot g's fields as block-uniform scalars (read from LDS they are VGPRs to the compiler: the
// descriptors built from them put every buffer load in a waterfall loop)
__device__ __forceinline__ XSlot slot_u(const XSlot* sl, int g) {
  const XSlot v = sl[g];
  XSlot s;
  s.unit = __builtin_amdgcn_readfirstlane(v.unit);
  s.f = __builtin_amdgcn_readfirstlane(v.f);
  s.e = 0;
  s.b = __builtin_amdgcn_readfirstlane(v.b);
  s.L = __builtin_amdgcn_readfirstlane(v.L);
  s.c = __builtin_amdgcn_readfirstlane(v.c);
  s.flags = __builtin_amdgcn_readfirstlane(v.flags);
  s.pad = 0;
  return s;
}
// The analysis unit u's item: whole items u < n_items (b = u / gx, c = u % gx), tail pieces
// n_items + q (item n_whole + q / P); its partials (chunk partials / the piece's tail slot).
template <int F, class CA>
__device__ __forceinline__ float* unit_item(CA& A, int u, int gx, int n_items, int n_whole, int P,
                                            int& b, int& c) {
  if (u < n_items) {
    b = u / gx;
    c = u % gx;
    return A.part + ((long long)b * A.nchunk + c) * 5 * F;
  }
  const int q = u - n_items, it = n_whole + q / P;
  b = it / gx;
  c = it % gx;
  return A.tpart + (long long)q * 5 * F;
}

// Reference-exact decisions of up to four deferred frames of one unit (avz_ibm_exact.hpp): wave w forms
// the fp64 spectra (ref_spectrum_exact) of reference w & 1 (target / interference) of slots
// w / 2 and w / 2 + 2 -- sample loads first --, waves 0-1 the slots' mic spectra, then thread
// per bin decides |I| > |T| for the slot's deferred bins (the whole frame below N/2, or the
// bins of xdfr[unit][k]; the Nyquist bin when flagged) and adds the frame's covariance terms
// and noise bit to the caller's running sums, in slot (= frame) order.
// After the loop, not in it: inlined at the item's end the step loop's kernels (248-253 of
// 256 VGPRs) spilled 105+ VGPRs; here nothing of the loop is live.
template <int N, bool PER_BIN>
__device__ __forceinline__ void exact_round(KArgs& A, unsigned char* lds, const XSlot* sl, int ns,
                                            Acc32 (&pacc)[CGeo<N>::BPT + 1],
                                            uint32_t (&pbits)[CGeo<N>::BPT + 1]) {
  using C = KCfg<N>;
  using G = CGeo<N>;
  using X = XGeo<N>;
  using XL = XLds<N>;
  constexpr int NT = G::NT, H = G::H, F = G::F, BPT = G::BPT, PPL = C::PPL, MP = XL::MP;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  float* const mag = reinterpret_cast<float*>(lds + XL::MAG_OFF);  // [2 FR][MP]
  const cd* const twl = reinterpret_cast<const cd*>(lds + XL::TWL_OFF);
  const float* const win = reinterpret_cast<const float*>(lds + XL::WIN_OFF);
  cd* const buf = reinterpret_cast<cd*>(lds + wave * X::SCRATCH);
  AVZ_STAMP_DECL();
  AVZ_STAMP_INIT();
#ifdef AVZ_XTRACE  // diagnostic: phase ticks of the rounds (tools/xtrace.py)
  unsigned long long xr_prev = __builtin_amdgcn_s_memrealtime();
#define AVZ_XR(i)                                                                  \
  do {                                                                             \
    if (threadIdx.x == 0 && g_stamps) {                                            \
      const unsigned long long now_ = __builtin_amdgcn_s_memrealtime();            \
      g_stamps[blockIdx.x * 16 + (i)] += now_ - xr_prev;                           \
      xr_prev = now_;                                                              \
    }                                                                              \
  } while (0)
#else
#define AVZ_XR(i) (void)0
#endif
  // lane-derived addresses formed here (hoisted out of the caller's loop they spilled)
  int lane_o = lane;
  opaque_i(lane_o);
  // the wave's two reference frames and (waves 0-1) the mic frames, loads first
  const int ga = wave >> 1, gb = (wave >> 1) + 2;
  const float* const refp = (wave & 1) ? A.ref_int : A.ref_tgt;
  float xa[N / 64], xb[N / 64];
  if (ga < ns) {
    const XSlot s = slot_u(sl, ga);
    ref_frame_load<N>(make_rsrc(refp + (long long)s.b * A.ref_stride, s.L),
                      (s.c * kChunk + s.f) * H - N / 2, lane_o, xa);
  }
  if (gb < ns) {
    const XSlot s = slot_u(sl, gb);
    ref_frame_load<N>(make_rsrc(refp + (long long)s.b * A.ref_stride, s.L),
                      (s.c * kChunk + s.f) * H - N / 2, lane_o, xb);
  }
  if (ga < ns) ref_spectrum_exact<N>(xa, twl, win, buf, mag + (2 * ga + (wave & 1)) * MP, lane_o);
  AVZ_STAMP(4);
  AVZ_XR(8);
  // waves 0-1: the mic frames' loads (one slot per lane group), in flight through the second
  // transform
  cf v[PPL];
  LaneMap<N> lm;
  lm.init(lane_o);
  const int gm = C::FPW * wave + lm.grp;
  if (wave < XL::FR / C::FPW) {
    // the round's slots are frames of one unit (one utterance): one descriptor pair, the
    // lane group's frame in the offset
    const XSlot s = slot_u(sl, 0);
    const float* mixb = A.mix + (long long)s.b * A.mix_stride;
    const rsrc_t r_m0 = make_rsrc(mixb, s.L), r_m1 = make_rsrc(mixb + A.ch_stride, s.L);
    const bool on = gm < ns;
    const int fm = sl[on ? gm : 0].f;
    const int s0 = (s.c * kChunk + fm) * H - N / 2 + lm.in0;
#pragma unroll
    for (int r = 0; r < PPL; ++r) {
      v[r].x = on ? bload(r_m0, s0 + C::IN_STRIDE * r) : 0.0f;
      v[r].y = on ? bload(r_m1, s0 + C::IN_STRIDE * r) : 0.0f;
    }
  }
  if (gb < ns) {
    int lane_b = lane;
    opaque_i(lane_b);
    ref_spectrum_exact<N>(xb, twl, win, buf, mag + (2 * gb + (wave & 1)) * MP, lane_b);
  }
  AVZ_STAMP(5);
  lds_barrier();  // the transform buffers are the mic spectra's slots
  AVZ_STAMP(6);
  AVZ_XR(9);
  if (wave < XL::FR / C::FPW) {  // the mic spectra (zeros for an absent slot)
    WinCoef<N> wc;
    wc.init(lm);
    cf* const spec = slot_ptr<N>(lds, gm);
    if constexpr (N == 1024) {
      // the unrotated frame on the LDS twiddle table: the step's register twiddles (and the
      // pair loads' rotation) stay out of this phase, whose registers they would hold
      Fft1024x2 f;
      f.l = lm.out0;
      window_apply(v, wc.a0, wc.ac, wc.as);
      f.forward(v, spec, reinterpret_cast<const cf*>(lds + G::TW_OFF));
      static_for<0, 32>([&](auto k) { spec[lm.out0 + 32 * k] = v[k]; });
    } else {
      Fft512x2 f;
      f.init(lane_o);
      window_fft<N>(v, wc, f, spec, lm);
    }
  }
  AVZ_STAMP(7);
  lds_barrier();
  AVZ_STAMP(8);
  AVZ_XR(10);
  // decisions |I| > |T| and the frames' covariance terms, thread per bin as the step's,
  // onto the caller's running sums (one unit's frames, in frame order)
  unsigned long long n_exact = 0;
  for (int g = 0; g < ns; ++g) {  // block-uniform
    const XSlot s = slot_u(sl, g);
    const cf* Zm = slot_ptr<N>(lds, g);
    auto put = [&](int j, int k, const Acc32& a, bool dfr, bool noise) {
      if (dfr) {
        pacc[j].c00 += a.c00;
        pacc[j].c11 += a.c11;
        pacc[j].c01r += a.c01r;
        pacc[j].c01i += a.c01i;
        pacc[j].cm += a.cm;
        pbits[j] |= (noise ? 1u : 0u) << s.f;
      }
    };
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      const int kb = tid + j * NT;
      const int kp = (N - kb) & (N - 1);
      // the reference-bit path: the frame's xunc words (written this launch only for frames
      // flagged by the reference waves, flags bit 0; a frame deferred for its Nyquist bin
      // alone has none)
      const bool dfr =
          PER_BIN ? ((A.xdfr[(long long)s.unit * F + kb] >> s.f) & 1u)
                  : ((s.flags & 1) &&
                     ((A.xunc[((long long)s.unit * kChunk + s.f) * 32 + (kb & 31)] >> (kb >> 5)) & 1u));
      Acc32 a;
      a.zero();
      bool noise = false;
      if (dfr) {
        noise = mag[(2 * g + 1) * MP + kb] > mag[(2 * g) * MP + kb];
        cf x0, x1;
        split_pair2(Zm[kb], Zm[kp], x0, x1);
        a.add_sel(x0, x1, noise);
        a.cm = noise ? 1.0f : 0.0f;
        n_exact += 1;
      }
      put(j, kb, a, dfr, noise);
    }
    if (tid == NT - 1) {  // the Nyquist bin
      const bool dfr = (s.flags >> 1) & 1;
      Acc32 a;
      a.zero();
      bool noise = false;
      if (dfr) {
        noise = mag[(2 * g + 1) * MP + N / 2] > mag[(2 * g) * MP + N / 2];
        cf y0, y1;
        split_pair2(Zm[N / 2], Zm[N / 2], y0, y1);
        const float wn = noise ? 1.0f : 0.0f;
        a.add(y0, y1, wn, wn);
        n_exact += 1;
      }
      put(BPT, N / 2, a, dfr, noise);
    }
  }
  if (A.xstat && n_exact) atomicAdd(A.xstat + 1, n_exact);  // diagnostic: decisions
  AVZ_STAMP(9);
  lds_barrier();
  AVZ_STAMP(10);
  AVZ_XR(11);
#undef AVZ_XR
}


// A deferred frame with at most kSparseMax uncertain bins (the Nyquist bin included) is decided
// bin by bin (exact_sparse); the reference-bit path's analysis items mark frames with
// kSparseMax or more uncertain bins as "round" frames (fp64 transforms, exact_round) and
// publish a unit with any for the whole grid to share (ibm_exact_units).
constexpr int kSparseMax = 12;

// Work sharing of the exact path (reference-bit path). A published unit's pieces: its sparse
// frames (if any), then its rounds of kXRound round frames in up to kXPieces - 1 groups (two
// frames a round: one fp64 transform per wave, the round's latency about halved against four).
// xst[u] = {state, arrivals}: state kXOpen | pieces << 16 | next piece while open; claims add
// 1 (a claim past the last piece, or after the reset, finds no piece: harmless; the word stays
// closed, without kXOpen, and the next publish overwrites it); the piece that completes a unit
// resets it to 0. xhint: one bit per published unit, cleared with the reset.
constexpr uint32_t kXOpen = 0x80000000u;
constexpr int kXRound = 2;
struct XPieces {
  uint32_t sp;           // sparse frames
  int n_sp, nr, npr, n;  // sparse pieces (0 / 1), rounds, round pieces, pieces
};
__device__ __forceinline__ XPieces x_pieces(uint32_t pend, uint32_t big) {
  XPieces q;
  q.sp = pend & ~big;
  q.n_sp = q.sp ? 1 : 0;
  q.nr = (__popc(big) + kXRound - 1) / kXRound;
  q.npr = min(q.nr, kXPieces - q.n_sp);
  q.n = q.n_sp + q.npr;
  return q;
}
__device__ __forceinline__ bool x_has_piece(uint32_t v) {
  return (v & kXOpen) && (v & 0xffffu) < ((v >> 16) & 0xffu);
}

// piece p of P (P = 1: the whole item) runs the chunk's steps [p SA / P, (p + 1) SA / P), SA =
// steps per chunk; slot >= 0: its partials go to tail slot `slot` of tpart and its IBM bits
// into the chunk's mask words atomically (the other pieces own the word's other bits).
// seq: the block's item count (parity of the IBM pending-frame word, see pendw).
template <int N, int MASK, bool IRM, class TW>
__device__ __forceinline__ void analysis_item(const ChainArgs& A, unsigned char* lds, int c,
                                              int b, int p, int P, int slot, const TW& tw_reg,
                                              const LaneConst<N>& K, int seq) {
  using C = KCfg<N>;
  using G = CGeo<N>;
  constexpr int NT = G::NT, H = G::H, F = G::F, NSLOT = G::NSLOT, BPT = G::BPT, PPL = C::PPL;
  constexpr int FB = (MASK == MASK_IBM) ? NSLOT / 2 : NSLOT;  // frames per step
  static_assert(kChunk % FB == 0, "steps tile the chunk");
  // IBM without the IRM gains: the reference waves publish per-bin noise bits
  // (window_fft_reg_ibm_bits) instead of the whole reference spectrum
  constexpr bool REFBITS = N == 1024 && MASK == MASK_IBM && !IRM && !std::is_same<TW, NoTw>::value;
  // shared-half frame-pair loads (pair_loads); needs the twiddle signs of the register path
  // (not IPD: its decisions are pinned bit-exact to the reference's, and the rotated
  // transform's rounding moved one of 1.3e5 on the ipd_test golden)
  constexpr bool SHARE = N == 1024 && MASK != MASK_IPD && !std::is_same<TW, NoTw>::value;
  // IBM without the reference-bit hand-off: the reference waves publish each frame's
  // certificate scale delta (MISC_OFF + 16: four floats) and the bin phase defers the
  // uncertified (bin, frame) decisions one by one (dfr)
  constexpr bool DLT = MASK == MASK_IBM && !REFBITS;

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int L = utt_len(A, b);
  if (L < N) return;  // host validates; finalize reports NaN for a bad device length
  const int T = (L + H - 1) / H + 1;
  const int nch = (T + kChunk - 1) / kChunk;
  if (c >= nch) return;
  if (c == 0 && p == 0 && tid == 0) {
    A.peak_u[b] = 0u;
    if (A.peak && A.normalize != NORM_PEAK) A.peak[b] = 0.0f;  // finalize's atomicMax target
  }
  const int t0 = c * kChunk;
  const int nframes = min(kChunk, T - t0);
  constexpr int SA = kChunk / FB;  // steps of a full chunk
  const int s_lo = p * SA / P;      // this piece's steps [s_lo, nstep)
  const int nstep = min((nframes + FB - 1) / FB, (p + 1) * SA / P);
  // IBM: frames (bit = chunk frame) with decisions deferred to the exact path
  // (ibm_exact_units), OR-ed in LDS by the deciding waves before a step barrier, read after
  // the item's last one. Two triples of words used by alternate items: the next item clears
  // its own before its first barrier, which no thread passes before it has read this item's.
  uint32_t* const pendw = reinterpret_cast<uint32_t*>(lds + G::MISC_OFF + 32 + 12 * (seq & 1));
  if (MASK == MASK_IBM && tid == 0) {
    int z = 0;
    opaque_i(z);  // formed here (a zero pair held across the items spilled)
    pendw[0] = (uint32_t)z;  // frames with a deferred decision
    pendw[1] = (uint32_t)z;  // frames with uncertain bins in xunc (reference-bit path)
    pendw[2] = (uint32_t)z;  // of those, frames with kSparseMax or more (round frames)
  }

  const typename C::Fft fft = K.fft;
  // the lane map formed per item from an opaque lane (held across the items from the kernel
  // start, three of its offsets spilled)
  LaneMap<N> lm;
  {
    int ln = threadIdx.x & 63;
    opaque_i(ln);
    lm.init(ln);
  }
  const float cert_raw = A.ibm_cert * (2.0f / N);  // REFBITS: delta per unit raw norm (2 a0)
  const WinCoef<N> wc = K.wc;  // SHARE: the rotated frames' (group 1) already swapped
  const int my_slot = wave * C::FPW + lm.grp;
  cf* my_spec = slot_ptr<N>(lds, my_slot);
  // IBM: waves 0-1 transform the mic pair, waves 2-3 the reference pair (wave-uniform)
  const bool ref = (MASK == MASK_IBM) && (wave * C::FPW >= FB);
  const int my_frame = ref ? my_slot - FB : my_slot;
  const int wave_frame0 = ref ? wave * C::FPW - FB : wave * C::FPW;

  const float* mixb = A.mix + (long long)b * A.mix_stride;
  rsrc_t r_re = make_rsrc(mixb, L), r_im = make_rsrc(mixb + A.ch_stride, L);
  if constexpr (MASK == MASK_IBM) {
    if (ref) {
      r_re = make_rsrc(A.ref_tgt + (long long)b * A.ref_stride, L);
      r_im = make_rsrc(A.ref_int + (long long)b * A.ref_stride, L);
    }
  }
  cf v[PPL];
  auto issue_loads = [&](int step) {
    if constexpr (SHARE) {
      const int sp = (t0 + step * FB + wave_frame0) * H - N / 2 + lm.in0;
      if (t0 + step * FB + wave_frame0 >= 1)
        pair_loads<true>(v, r_re, r_im, sp, lm.grp);
      else
        pair_loads<false>(v, r_re, r_im, sp, lm.grp);
      return;
    }
    const int s0 = (t0 + step * FB + my_frame) * H - N / 2 + lm.in0;
    if (t0 + step * FB + wave_frame0 >= 1) {  // wave-uniform: no negative sample index
      static_for<0, PPL>([&](auto r) {
        v[r].x = bload_nn(r_re, s0 + C::IN_STRIDE * r);
        v[r].y = bload_nn(r_im, s0 + C::IN_STRIDE * r);
      });
    } else {
      static_for<0, PPL>([&](auto r) {
        v[r].x = bload(r_re, s0 + C::IN_STRIDE * r);
        v[r].y = bload(r_im, s0 + C::IN_STRIDE * r);
      });
    }
  };

  // IL_LOADS (register-twiddle path): the next step's loads are issued from inside the
  // FFT's last stage, register k right after its spectrum output is stored, so their issue
  // overlaps the butterflies; a chunk's last step loads from an empty descriptor (reads 0,
  // no memory traffic). Frames of a next step are >= FB >= 1: no negative sample index.
  constexpr bool IL_LOADS = N == 1024 && !std::is_same<TW, NoTw>::value;
  const rsrc_t r_none = make_rsrc(nullptr, 0);
  rsrc_t rn_re = r_none, rn_im = r_none;
  int sp_next = 0;
  auto load_reg = [&](auto kc) {
    constexpr int k = decltype(kc)::value;
    if constexpr (SHARE) {
      if constexpr (k < 16) {
        const int e = sp_next + 1024 * lm.grp + 32 * k;
        v[k].x = bload_nn(rn_re, e);
        v[k].y = bload_nn(rn_im, e);
      } else if constexpr ((k - 16) % 2 == 0) {
        const int e = sp_next + 512 + 32 * (k - 16) + 32 * lm.grp;
        v[k].x = bload_nn(rn_re, e);
        v[k].y = bload_nn(rn_im, e);
      }
    } else {
      v[k].x = bload_nn(rn_re, sp_next + C::IN_STRIDE * k);
      v[k].y = bload_nn(rn_im, sp_next + C::IN_STRIDE * k);
    }
  };

  Acc32 acc[BPT];
  uint32_t bits[BPT];
  uint32_t dfr[BPT];     // DLT: (bin, frame) decisions deferred to the exact path
  int ipd_clear_n[BPT];  // IPD: frames the cross-product test weighted 1
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    acc[j].zero();
    bits[j] = 0u;
    dfr[j] = 0u;
    ipd_clear_n[j] = 0;
  }
  // IRM post-filter gains of this chunk (PF_IRM plans only)
  static_assert(!IRM || MASK == MASK_IBM, "IRM needs the references");
  float* const gain = IRM ? A.pf_gain + ((long long)b * A.nchunk + c) * kChunk * F : nullptr;
  // Nyquist bin N/2: frame `lane` of each step on the last wave's lanes.
  const bool nyq_wave = (wave == G::NWAVE - 1);
  Acc32 an, adc;  // Nyquist; DC (IPD: weighed on the Nyquist wave, not by lane 0)
  an.zero();
  adc.zero();
  uint32_t nyq_bits = 0u, nyq_dfr = 0u;
  // IPD: covariance weight of the main bin loop, 0 on the DC lane (bin tid + 256 j)
  float wone[BPT];
#pragma unroll
  for (int j = 0; j < BPT; ++j) wone[j] = (MASK == MASK_IPD && j == 0 && tid == 0) ? 0.0f : 1.0f;

  AVZ_STAMP_DECL();
  issue_loads(s_lo);
  lds_barrier();  // twiddle table
  AVZ_STAMP_INIT();
  for (int step = s_lo; step < nstep; ++step) {
    const int f0 = t0 + step * FB;
    const bool live = f0 + wave_frame0 < T;  // wave-uniform: any of its frames exist
#ifdef AVZ_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    AVZ_STAMP(0);
#endif
    if (live) {
      if constexpr (SHARE) pair_finish(v);
      // reference-bit path: the two frames' energies (raw samples; the window's maximum 2 a0
      // scales the bound, cert_raw) as wave-uniform values, so nothing extra stays in VGPRs
      // through the FFT (from the windowed input or the spectrum the kernel spilled 5-125)
      float eg0 = (AVZ_CERT_PARTS & 1) ? 0.0f : 1.0f, eg1 = eg0;
      if constexpr (REFBITS && !AVZ_NO_IBM_CERT && (AVZ_CERT_PARTS & 1)) {
        if (ref) {
          const float eg = group32_sum(frame_energy(v));
          eg0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(eg), 0));
          eg1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(eg), 32));
        }
      }
      if constexpr (MASK == MASK_IPD) {
        // Bitwise-identical channel samples give bitwise-identical pocketfft spectra in the
        // reference, hence equal angles (weight 0.01) in every bin of the frame; the packed
        // FFT's split does not reproduce that equality, so the frame is flagged here.
        bool same = true;
        static_for<0, PPL>([&](auto r) {
          same &= __float_as_uint(v[r].x) == __float_as_uint(v[r].y);
        });
        const unsigned long long nb = __ballot(!same);
        const bool ident = (C::FPW == 1) ? nb == 0ull : ((nb >> (32 * lm.grp)) & 0xffffffffull) == 0ull;
        if ((lane & (64 / C::FPW - 1)) == 0) lds[G::MISC_OFF + my_slot] = ident ? 1 : 0;
      }
      if constexpr (IL_LOADS) {
        const bool more = step + 1 < nstep;
        rn_re = more ? r_re : r_none;
        rn_im = more ? r_im : r_none;
        sp_next = (t0 + (step + 1) * FB + (SHARE ? wave_frame0 : my_frame)) * H - N / 2 + lm.in0;
      }
      float en = 0.0f;
      if constexpr (!IL_LOADS) {
        window_fft<N>(v, wc, fft, my_spec, lm, NoAfter{}, (DLT && ref) ? &en : nullptr);
      } else if constexpr (REFBITS) {
        // block-uniform: a chunk's last step issues no loads (analysis 79.7 -> 77.0-78.3 us,
        // profiles/r04/ab_last_step_loads.txt; the other masks' kernels keep the
        // empty-descriptor loads: a second copy of their FFT spills)
        uint32_t um = 0u;
        if (step + 1 < nstep) {
          if (ref)
            um = window_fft_reg_ibm_bits(v, wc, fft, my_spec, tw_reg, lm, eg0, eg1, cert_raw, en,
                                         load_reg);
          else
            window_fft_reg(v, wc, fft, my_spec, tw_reg, lm, load_reg);
        } else {
          if (ref)
            um = window_fft_reg_ibm_bits(v, wc, fft, my_spec, tw_reg, lm, eg0, eg1, cert_raw, en);
          else
            window_fft_reg(v, wc, fft, my_spec, tw_reg, lm);
        }
        const unsigned long long ua = __ballot(um != 0u);
        if (ua != 0ull) {  // rare (wave-uniform): uncertain bins, the exact path's (xunc)
          if ((ua >> (32 * lm.grp)) & 0xffffffffull) {
            KArgs& Ak = kernarg_chain_args();
            const int gxi = (Ak.max_frames + kChunk - 1) / kChunk;
            const int unit = slot < 0 ? b * gxi + c : gxi * Ak.batch + slot;
            Ak.xunc[((long long)unit * kChunk + step * FB + my_frame) * 32 + (lane & 31)] = um;
            int nu = __popc(um);  // the frame's uncertain bins (its lane group's 32 words)
#pragma unroll
            for (int o = 1; o < 32; o <<= 1) nu += __shfl_xor(nu, o, 64);
            if ((lane & 31) == 0) {  // a frame with a deferral, one with its xunc words written
              atomicOr(pendw, 1u << (step * FB + my_frame));
              atomicOr(pendw + 1, 1u << (step * FB + my_frame));
              if (nu >= kSparseMax) atomicOr(pendw + 2, 1u << (step * FB + my_frame));
            }
          }
        }
      } else {
        window_fft_reg(v, wc, fft, my_spec, tw_reg, lm, load_reg, (DLT && ref) ? &en : nullptr);
      }
      // IBM: the reference waves publish each frame's certificate scale delta (the bin phase's
      // per-bin deferrals, the Nyquist bin's); the reference-bit path returns delta itself
      if (MASK == MASK_IBM && ref && (lane & 31) == 0)
        reinterpret_cast<float*>(lds + G::MISC_OFF + 16)[my_frame] = REFBITS ? en : A.ibm_cert * sqrtf(en);
    }
    AVZ_STAMP(3);
    if (!IL_LOADS && step + 1 < nstep) issue_loads(step + 1);
    AVZ_STAMP(11);
    lds_barrier();
    AVZ_STAMP(1);
    const int nvalid = min(FB, T - f0);
    // Thread-per-bin over the step's frames. A full step runs unguarded so all of its
    // LDS reads can issue back to back; only a chunk's last step may be partial.
    uint32_t ipd_fix[BPT];
#pragma unroll
    for (int j = 0; j < BPT; ++j) ipd_fix[j] = 0u;
    // IPD: frames whose two channels are bitwise identical (bit 8 i: slot i)
    const unsigned long long ident_w =
        (MASK == MASK_IPD) ? *reinterpret_cast<const unsigned long long*>(lds + G::MISC_OFF) : 0ull;
    const bool mask_vec = MASK == MASK_EXTERNAL && A.mask_st == 1 && (A.mask_sf & 3) == 0 &&
                          (A.mask_sb & 3) == 0 &&
                          ((reinterpret_cast<uintptr_t>(A.ext_mask) & 15) == 0) && (f0 & 3) == 0;
    float dlt[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if constexpr (DLT) {  // the step's frames' certificate scales
      const float4 q = *reinterpret_cast<const float4*>(lds + G::MISC_OFF + 16);
      dlt[0] = q.x;
      dlt[1] = q.y;
      dlt[2] = q.z;
      dlt[3] = q.w;
    }
    auto bin_phase = [&](auto full, auto vec) {
      // frames whose LDS reads are batched together
      constexpr int G = FB < 4 ? FB : 4;
#pragma unroll
      for (int j = 0; j < BPT; ++j) {
        const int kb = tid + j * NT;
        const int kp = (N - kb) & (N - 1);
#pragma unroll
        for (int g0 = 0; g0 < FB; g0 += G) {
          // External mask with t-contiguous, 16-B aligned rows: the bin's G mask values
          // of a full step in one 16-B load (as the synthesis post-filter).
          float mv[MASK == MASK_EXTERNAL ? 4 : 1];
          if constexpr (MASK == MASK_EXTERNAL && G == 4 && decltype(vec)::value) {
            const float4 m4 = *reinterpret_cast<const float4*>(
                A.ext_mask + (long long)b * A.mask_sb + (long long)kb * A.mask_sf + f0 + g0);
            mv[0] = m4.x;
            mv[1] = m4.y;
            mv[2] = m4.z;
            mv[3] = m4.w;
          }
          cf zm[G], zmp[G], zr[G], zrp[G];
          uint32_t zw[G];  // REFBITS: the frame's noise word of bin column kb & 31
#pragma unroll
          for (int i = 0; i < G; ++i) {
            if (decltype(full)::value || g0 + i < nvalid) {
              const cf* Zm = slot_ptr<N>(lds, g0 + i);
              zm[i] = Zm[kb];
              zmp[i] = Zm[kp];
              if constexpr (REFBITS) {
                zw[i] = reinterpret_cast<const uint32_t*>(slot_ptr<N>(lds, FB + g0 + i))[kb & 31];
              } else if constexpr (MASK == MASK_IBM) {
                const cf* Zr = slot_ptr<N>(lds, FB + g0 + i);
                zr[i] = Zr[kb];
                zrp[i] = Zr[kp];
              }
            }
          }
#pragma unroll
          for (int i = 0; i < G; ++i) {
            if (decltype(full)::value || g0 + i < nvalid) {
              cf x0, x1;
              split_pair2(zm[i], zmp[i], x0, x1);  // 2 y0, 2 y1
              if constexpr (MASK == MASK_IPD) {
                // the exact angle test of near-colinear bins runs after the loop;
                // ipd_clear on the covariance products themselves: |x0|^2 |x1|^2 and
                // Im x0 conj(x1) are the test's norm and cross product. Every frame's
                // products go in at weight 1 (wone: 0 on the DC lane, weighed by the Nyquist
                // wave); the frames the test leaves open get w - 1 after the loop.
                const float p0 = x0.x * x0.x + x0.y * x0.y;
                const float p1 = x1.x * x1.x + x1.y * x1.y;
                const float re = x0.x * x1.x + x0.y * x1.y;
                const float im = x0.y * x1.x - x0.x * x1.y;
                const bool clear = im * im > 1e-10f * (p0 * p1) &&
                                   !((ident_w >> (8 * (g0 + i))) & 1ull);
                ipd_fix[j] |= (clear ? 0u : 1u) << (g0 + i);
                acc[j].c00 = fmaf(wone[j], p0, acc[j].c00);
                acc[j].c11 = fmaf(wone[j], p1, acc[j].c11);
                acc[j].c01r = fmaf(wone[j], re, acc[j].c01r);
                acc[j].c01i = fmaf(wone[j], im, acc[j].c01i);
                continue;
              }
              if constexpr (MASK == MASK_IBM) {
                bool noise;
                if constexpr (REFBITS) {
                  noise = (zw[i] >> (kb >> 5)) & 1u;
                } else {
                  noise = ibm_noise(zr[i], zrp[i]);
                  if (ibm_uncertain(zr[i], zrp[i], dlt[g0 + i])) {  // rare: the exact path's
                    noise = false;
                    dfr[j] |= 1u << (step * FB + g0 + i);
                    atomicOr(pendw, 1u << (step * FB + g0 + i));
                  }
                }
                bits[j] |= (noise ? 1u : 0u) << (step * FB + g0 + i);
                acc[j].add_sel(x0, x1, noise);  // weight count: popcount of bits at the end
                if constexpr (IRM) gain[(step * FB + g0 + i) * F + kb] = irm_gain(zr[i], zrp[i]);
                continue;
              }
              bool noise = false;
              float wgt;
              float m;
              if constexpr (MASK == MASK_EXTERNAL && G == 4 && decltype(vec)::value) {
                m = 1.0f - mv[i];
                wgt = m + A.weight_eps;
              } else {
                m = bin_mask<MASK>(A, b, x0, x1, zr[i], zrp[i], kb, f0 + g0 + i, noise, wgt);
              }
              bits[j] |= (noise ? 1u : 0u) << (step * FB + g0 + i);
              acc[j].add(x0, x1, wgt, m);
              if constexpr (IRM) gain[(step * FB + g0 + i) * F + kb] = irm_gain(zr[i], zrp[i]);
            }
          }
        }
      }
    };
    if (nvalid == FB) {
      if constexpr (MASK == MASK_EXTERNAL) {
        if (mask_vec)
          bin_phase(std::true_type{}, std::true_type{});
        else
          bin_phase(std::true_type{}, std::false_type{});
      } else {
        bin_phase(std::true_type{}, std::false_type{});
      }
    } else {
      bin_phase(std::false_type{}, std::false_type{});
    }
    if constexpr (MASK == MASK_IPD) {
      // Near-colinear (bin, frame) pairs (rare; DC, always one, is the Nyquist wave's):
      // exact weight from the spectra still in LDS. Waves with no such lane skip this.
#pragma unroll
      for (int j = 0; j < BPT; ++j) {
        const int kb = tid + j * NT;
        const int kp = (N - kb) & (N - 1);
        uint32_t f = ipd_fix[j];
        const bool dc = (j == 0 && tid == 0);
        if (dc) f = 0u;
        ipd_clear_n[j] += dc ? 0 : nvalid - __popc(f);  // weight count: exact integers
        while (f) {
          const int i = __builtin_ctz(f);
          f &= f - 1u;
          const cf* Zm = slot_ptr<N>(lds, i);
          cf x0, x1;
          split_pair2(Zm[kb], Zm[kp], x0, x1);
          const float w = ((ident_w >> (8 * i)) & 1ull) ? 0.01f : ipd_weight_exact(x0, x1);
          acc[j].add(x0, x1, w - 1.0f, w);  // the products went in at weight 1
        }
      }
    }
    if (nyq_wave) {
      bool noise = false, nunc = false;
      if (lane < nvalid) {
        int ln = lane;
        opaque_i(ln);  // its slot addresses formed here (held across the items they spilled)
        const cf* Zm = slot_ptr<N>(lds, ln);
        cf y0, y1, zr{0, 0};
        split_pair2(Zm[N / 2], Zm[N / 2], y0, y1);
        if constexpr (MASK == MASK_IBM) zr = slot_ptr<N>(lds, FB + ln)[N / 2];
        float wn;
        float mn = bin_mask<MASK>(A, b, y0, y1, zr, zr, N / 2, f0 + lane, noise, wn);
        if (MASK == MASK_IPD && ((ident_w >> (8 * lane)) & 1ull)) wn = mn = 0.01f;
        if (MASK == MASK_IBM &&
            ibm_uncertain(zr, zr, reinterpret_cast<const float*>(lds + G::MISC_OFF + 16)[lane])) {
          noise = false;  // rare: the exact path's
          wn = mn = 0.0f;
          nunc = true;
          atomicOr(pendw, 1u << (step * FB + lane));
        }
        an.add(y0, y1, wn, mn);
        if constexpr (MASK == MASK_IPD) {  // DC of frame `lane`
          cf d0, d1;
          const cf z0 = Zm[0];
          split_pair2(z0, z0, d0, d1);
          const float wd = ((ident_w >> (8 * lane)) & 1ull) ? 0.01f : ipd_weight_exact(d0, d1);
          adc.add(d0, d1, wd, wd);
        }
        if constexpr (IRM) gain[(step * FB + lane) * F + N / 2] = irm_gain(zr, zr);
      }
      const unsigned long long bal = __ballot(noise);
      nyq_bits |= ((uint32_t)bal & ((1u << FB) - 1u)) << (step * FB);
      if constexpr (MASK == MASK_IBM)
        nyq_dfr |= ((uint32_t)__ballot(nunc) & ((1u << FB) - 1u)) << (step * FB);
    }
    AVZ_STAMP(12);
    lds_barrier();
    AVZ_STAMP(2);
  }

  // ---- reference-exact decisions of the deferred frames (avz_ibm_exact.hpp)
  if constexpr (MASK == MASK_IBM) {
    // the unit's exact-path record (ibm_exact_units, after the block's loop): frames with a
    // deferral, frames with xunc words (reference-bit path), the Nyquist bin's deferrals; the
    // per-bin deferrals
    const uint32_t pend = pendw[0], full = pendw[1];  // block-uniform (after the last barrier)
    // round frames (published units): the reference-bit path's counted ones; every deferred
    // frame of the per-bin kernels (their exact path is rounds only)
    const uint32_t big = REFBITS ? pendw[2] : pend;
    KArgs& Ak = kernarg_chain_args();  // pointers not held through the loop
    const int gxi = (Ak.max_frames + kChunk - 1) / kChunk;  // analysis_items' units
    const int unit = slot < 0 ? b * gxi + c : gxi * Ak.batch + slot;
    if (nyq_wave && lane == 0) {
      reinterpret_cast<uint4*>(Ak.xpend)[unit] = make_uint4(pend, full, nyq_dfr, big);
      // the block's units with deferrals, by position in its item sequence (bit 31: any
      // past the 31st); ibm_exact_units reads only their records
      if (pend) *reinterpret_cast<uint32_t*>(lds + G::MISC_OFF + 56) |= 1u << min(seq, 31);
    }
    if (DLT && pend != 0u) {
#pragma unroll
      for (int j = 0; j < BPT; ++j) Ak.xdfr[(long long)unit * F + tid + j * NT] = dfr[j];
    }
  }

  // ---- chunk partials (a piece's: its tail slot; its bits merged into the chunk's words)
  float* Pt = slot < 0 ? A.part + ((long long)b * A.nchunk + c) * 5 * F
                       : A.tpart + (long long)slot * 5 * F;
  uint32_t* MW = A.mwords + ((long long)b * A.nchunk + c) * F;
  // the piece's bit range (nominal: bits past the chunk's frames are cleared too)
  const uint32_t rng = (P == 1) ? ~0u : ((1u << (kChunk / P)) - 1u) << (kChunk / P * p);
  auto put_word = [&](int k, uint32_t w) {
    if (slot < 0) {
      MW[k] = w;
    } else {
      atomicAnd(MW + k, ~rng);
      atomicOr(MW + k, w);
    }
  };
  constexpr bool DC_NYQ = MASK == MASK_IPD;  // DC sums come from the Nyquist wave
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    const int kb = tid + j * NT;
    if (DC_NYQ && kb == 0) continue;
    // binary weights were folded into the selects: their count is exact in fp32
    if constexpr (MASK == MASK_IBM) acc[j].cm = (float)__popc(bits[j]);
    if constexpr (MASK == MASK_IPD) acc[j].cm += (float)ipd_clear_n[j];
    Pt[0 * F + kb] = acc[j].c00;
    Pt[1 * F + kb] = acc[j].c11;
    Pt[2 * F + kb] = acc[j].c01r;
    Pt[3 * F + kb] = acc[j].c01i;
    Pt[4 * F + kb] = acc[j].cm;
    if constexpr (MASK == MASK_IBM) put_word(kb, bits[j]);
  }
  if (nyq_wave) {
    for (int o = 1; o < 64; o <<= 1) {
      an.c00 += __shfl_xor(an.c00, o, 64);
      an.c11 += __shfl_xor(an.c11, o, 64);
      an.c01r += __shfl_xor(an.c01r, o, 64);
      an.c01i += __shfl_xor(an.c01i, o, 64);
      an.cm += __shfl_xor(an.cm, o, 64);
      if constexpr (DC_NYQ) {
        adc.c00 += __shfl_xor(adc.c00, o, 64);
        adc.c11 += __shfl_xor(adc.c11, o, 64);
        adc.c01r += __shfl_xor(adc.c01r, o, 64);
        adc.c01i += __shfl_xor(adc.c01i, o, 64);
        adc.cm += __shfl_xor(adc.cm, o, 64);
      }
    }
    if (DC_NYQ && lane == 0) {
      Pt[0 * F] = adc.c00;
      Pt[1 * F] = adc.c11;
      Pt[2 * F] = adc.c01r;
      Pt[3 * F] = adc.c01i;
      Pt[4 * F] = adc.cm;
    }
    if (lane == 0) {
      Pt[0 * F + N / 2] = an.c00;
      Pt[1 * F + N / 2] = an.c11;
      Pt[2 * F + N / 2] = an.c01r;
      Pt[3 * F + N / 2] = an.c01i;
      Pt[4 * F + N / 2] = an.cm;
      if constexpr (MASK == MASK_IBM) put_word(N / 2, nyq_bits);
    }
  }

  // ---- a unit with round frames is published for the grid to share (ibm_exact_units): its
  // record, words (per-bin deferrals), partials and mask words (stored above) released at
  // agent scope first
  if constexpr (MASK == MASK_IBM) {
    const uint32_t big = REFBITS ? pendw[2] : pendw[0];  // block-uniform
    if (big != 0u) {
#ifdef AVZ_XTRACE
      const unsigned long long tp = __builtin_amdgcn_s_memrealtime();
#endif
      __syncthreads();
      if (tid == 0) {
        KArgs& Ak = kernarg_chain_args();
        const int gxi = (Ak.max_frames + kChunk - 1) / kChunk;
        const int unit = slot < 0 ? b * gxi + c : gxi * Ak.batch + slot;
        const XPieces q = x_pieces(pendw[0], big);
        Ak.xst[2 * unit + 1] = 0u;  // arrivals
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __hip_atomic_store(Ak.xst + 2 * unit, kXOpen | ((uint32_t)q.n << 16), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_or(Ak.xhint + (unit >> 5), 1u << (unit & 31), __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT);
#ifdef AVZ_XTRACE
        if (g_stamps) {
          g_stamps[blockIdx.x * 16 + 12] += __builtin_amdgcn_s_memrealtime() - tp;
          g_stamps[blockIdx.x * 16 + 13] += 1 + 256 * q.n;  // units published, their pieces
        }
#endif
      }
    }
  }
}

// The block's work units: whole items i, i + gridDim.x, ... below a_whole (a multiple of the
// grid), then the tail items' pieces on the same stride (tail splitting, ChainArgs).
template <int N, int MASK, bool IRM, bool SPLIT, class TW>
__device__ __forceinline__ void analysis_items(const ChainArgs& A, unsigned char* lds, int gx,
                                               int n_items, const TW& tw_reg,
                                               const LaneConst<N>& K) {
  const int P = SPLIT && A.a_pieces > 1 ? A.a_pieces : 1;
  const int n_whole = P > 1 ? A.a_whole : n_items;
  const int n_end = n_whole + (n_items - n_whole) * P;  // whole items, then the pieces
  // one call site (two inlined copies of the item, whole and piece, spilled)
  int seq = 0;
  for (int u = blockIdx.x; u < n_end; u += gridDim.x) {
    const bool whole = u < n_whole;
    const int q = u - n_whole, it = whole ? u : n_whole + q / P;
    analysis_item<N, MASK, IRM>(A, lds, it % gx, it / gx, whole ? 0 : q % P, whole ? 1 : P,
                                whole ? -1 : q, tw_reg, K, seq++);
  }
}

// Sparse form of the exact path (reference-bit path): frames with few uncertain bins decide
// them one by one -- per item (frame f, bin k) the fp64 DFT of both references at k (rounded
// to complex64, numpy's |.|: ref_spectrum_exact's arithmetic) and of the packed mic pair at k
// and N - k (scaled as the analysis transform, rounded to fp32, split as the step's), one wave
// per item over the frame's 1024 samples, reduced across the wave. items[]: LDS, f << 16 | k,
// in frame order; the results go through LDS (res, 6 floats per item) to the bins' threads,
// which add them to their running sums in item order.
template <int N>
__device__ __forceinline__ void exact_sparse(KArgs& A, unsigned char* lds, int b, int L, int c,
                                             const int* items, int n,
                                             Acc32 (&pacc)[CGeo<N>::BPT + 1],
                                             uint32_t (&pbits)[CGeo<N>::BPT + 1]) {
  using G = CGeo<N>;
  using XL = XLds<N>;
  constexpr int H = N / 2, NT = G::NT, BPT = G::BPT;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const cd* const twl = reinterpret_cast<const cd*>(lds + XL::TWL_OFF);
  const float* const win = reinterpret_cast<const float*>(lds + XL::WIN_OFF);
  float* const res = reinterpret_cast<float*>(lds);  // [n][6] (the mic-spectra slots: free)
  const rsrc_t rt = make_rsrc(A.ref_tgt + (long long)b * A.ref_stride, L);
  const rsrc_t ri = make_rsrc(A.ref_int + (long long)b * A.ref_stride, L);
  const float* mixb = A.mix + (long long)b * A.mix_stride;
  const rsrc_t rm0 = make_rsrc(mixb, L), rm1 = make_rsrc(mixb + A.ch_stride, L);
  for (int it = wave; it < n; it += NT / 64) {  // wave-uniform
    const int item = __builtin_amdgcn_readfirstlane(items[it]);
    const int f = item >> 16, k = item & 0xffff;
    const int s0 = (c * kChunk + f) * H - N / 2;
    // every sample load in flight at once (a round trip per few samples ran ~6 us per item)
    float st[N / 64], si[N / 64], sm0[N / 64], sm1[N / 64];
#pragma unroll
    for (int r = 0; r < N / 64; ++r) {
      const int m = lane + 64 * r;
      st[r] = bload(rt, s0 + m);
      si[r] = bload(ri, s0 + m);
      sm0[r] = bload(rm0, s0 + m);
      sm1[r] = bload(rm1, s0 + m);
    }
    double tr = 0.0, ti = 0.0, ir = 0.0, ii = 0.0, ac = 0.0, bs = 0.0, as = 0.0, bc = 0.0;
#pragma unroll
    for (int r = 0; r < N / 64; ++r) {
      const int m = lane + 64 * r;
      const double w = (double)win[m];
      const double xt = w * (double)st[r], xi = w * (double)si[r];
      const double a = w * (double)sm0[r], bb = w * (double)sm1[r];
      const cd tw = xtw_at<N>(twl, (k * m) & (N - 1));  // exp(-2 pi i k m / N)
      tr = fma(xt, tw.x, tr);
      ti = fma(xt, tw.y, ti);
      ir = fma(xi, tw.x, ir);
      ii = fma(xi, tw.y, ii);
      ac = fma(a, tw.x, ac);
      bs = fma(bb, tw.y, bs);
      as = fma(a, tw.y, as);
      bc = fma(bb, tw.x, bc);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      tr += __shfl_xor(tr, o, 64);
      ti += __shfl_xor(ti, o, 64);
      ir += __shfl_xor(ir, o, 64);
      ii += __shfl_xor(ii, o, 64);
      ac += __shfl_xor(ac, o, 64);
      bs += __shfl_xor(bs, o, 64);
      as += __shfl_xor(as, o, 64);
      bc += __shfl_xor(bc, o, 64);
    }
    if (lane == 0) {
      const bool noise = np_abs_c64((float)ir, (float)ii) > np_abs_c64((float)tr, (float)ti);
      constexpr double sc = 2.0 / N;  // the analysis transform's scale ((2/N) Hann window)
      const cf zk = {(float)(sc * (ac - bs)), (float)(sc * (as + bc))};   // Z[k]
      const cf zp = {(float)(sc * (ac + bs)), (float)(sc * (bc - as))};   // Z[N - k]
      Acc32 t;
      t.zero();
      cf x0, x1;
      split_pair2(zk, zp, x0, x1);
      if (k == N / 2) {
        const float wn = noise ? 1.0f : 0.0f;
        t.add(x0, x1, wn, wn);
      } else {
        t.add_sel(x0, x1, noise);
        t.cm = noise ? 1.0f : 0.0f;
      }
      float* q = res + 6 * it;
      q[0] = noise ? 1.0f : 0.0f;
      q[1] = t.c00;
      q[2] = t.c11;
      q[3] = t.c01r;
      q[4] = t.c01i;
      q[5] = t.cm;
    }
  }
  __syncthreads();
  for (int it = 0; it < n; ++it) {  // block-uniform, item (frame) order
    const int item = items[it];
    const int f = item >> 16, k = item & 0xffff;
    const int j = k == N / 2 ? BPT : k / NT;
    if (k == N / 2 ? tid == NT - 1 : (k % NT) == tid) {
      const float* q = res + 6 * it;
#pragma unroll
      for (int jj = 0; jj <= BPT; ++jj) {  // a constant index (indexed, the array went to scratch)
        if (jj != j) continue;
        pacc[jj].c00 += q[1];
        pacc[jj].c11 += q[2];
        pacc[jj].c01r += q[3];
        pacc[jj].c01i += q[4];
        pacc[jj].cm += q[5];
        pbits[jj] |= (q[0] != 0.0f ? 1u : 0u) << f;
      }
    }
  }
  if (A.xstat && tid == 0) atomicAdd(A.xstat + 1, (unsigned long long)n);  // diagnostic
  __syncthreads();
}

// The slot of frame f of unit u (one thread): the unit's item, its length, the frame's flags.
template <int N, bool PER_BIN, class CA>
__device__ __forceinline__ void exact_set_slot(CA& A, XSlot* sl, int g, int u, int f, int gx,
                                               int n_items, int n_whole, int P) {
  constexpr int F = N / 2 + 1;
  XSlot s;
  s.unit = u;
  s.f = f;
  s.e = -1;
  unit_item<F>(A, u, gx, n_items, n_whole, P, s.b, s.c);
  s.L = utt_len(A, s.b);
  const uint4 r = reinterpret_cast<const uint4*>(A.xpend)[u];
  s.flags = (PER_BIN ? 0 : (int)((r.y >> f) & 1u)) | (int)(((r.z >> f) & 1u) << 1);
  s.pad = 0;
  sl[g] = s;
}

// Reference-exact decisions of analysis unit u's deferred frames (record xpend[u]: frames with
// a deferral, frames with uncertain-bin words xunc[u][f] (reference-bit path), the Nyquist
// bin's deferrals; xdfr[u][k] the per-bin
// deferrals of the kernels without the reference-bit hand-off), rounds of up to four frames
// in frame order (exact_round): the unit's partials of the thread's bins (kb = tid + j NT;
// the Nyquist bin: the last thread) as running sums, + each frame's terms in frame order,
// stored once; the noise bits OR-ed into the chunk's mask words (pieces of the chunk on other
// blocks own the other bits). The block must have the exact phase's LDS tables (xtab_fill)
// and the fp32 twiddle table (TW_OFF).
template <int N, bool PER_BIN>
__device__ __forceinline__ void exact_unit(KArgs& A, unsigned char* lds, int u, int gx, int n_items,
                                           int n_whole, int P) {
  using G = CGeo<N>;
  using XL = XLds<N>;
  constexpr int F = N / 2 + 1, NT = G::NT, BPT = G::BPT, FR = XL::FR;
  const int tid = threadIdx.x;
  XSlot* const sl = reinterpret_cast<XSlot*>(lds + XL::SLOT_OFF);
  const uint4 rec = reinterpret_cast<const uint4*>(A.xpend)[u];  // block-uniform
  const uint32_t pend = rec.x;
  if (pend == 0u || rec.w != 0u) return;  // published: ibm_exact_units' sharing
  int b, c;
  float* const Pt = unit_item<F>(A, u, gx, n_items, n_whole, P, b, c);
  if (A.xstat && tid == 0) atomicAdd(A.xstat, (unsigned long long)__popc(pend));
  Acc32 pacc[BPT + 1];
  uint32_t pbits[BPT + 1];
#pragma unroll
  for (int j = 0; j <= BPT; ++j) {
    const int kk = j < BPT ? tid + j * NT : N / 2;
    pbits[j] = 0u;
    if (j < BPT || tid == NT - 1) {
      pacc[j].c00 = Pt[0 * F + kk];
      pacc[j].c11 = Pt[1 * F + kk];
      pacc[j].c01r = Pt[2 * F + kk];
      pacc[j].c01i = Pt[3 * F + kk];
      pacc[j].cm = Pt[4 * F + kk];
    } else {
      pacc[j].zero();
    }
  }
  uint32_t rest = pend;
  if constexpr (!PER_BIN) {
    // frames with at most kSparseMax uncertain bins (the Nyquist bin included): their items in
    // frame order (wave 0, one frame at a time), decided one by one (exact_sparse)
    int* const items = reinterpret_cast<int*>(lds + XL::SCAN_OFF);  // [32 kSparseMax / 2]
    int* const ctl = reinterpret_cast<int*>(lds + XL::CTL_OFF);
    // the pending frames' words in LDS first (one round trip; per frame it was one each)
    uint32_t* const wsm = reinterpret_cast<uint32_t*>(lds + 16384);  // [32][32] (slots: free)
    const uint32_t has_words = reinterpret_cast<const uint4*>(A.xpend)[u].y;  // see exact_round
#pragma unroll
    for (int i = 0; i < kChunk / (G::NT / 32); ++i) {
      const int f = (tid >> 5) + (G::NT / 32) * i;
      if ((pend >> f) & 1u)
        wsm[f * 32 + (tid & 31)] =
            ((has_words >> f) & 1u) ? A.xunc[((long long)u * kChunk + f) * 32 + (tid & 31)] : 0u;
    }
    __syncthreads();
    if (tid < 64) {
      const uint32_t nyq = reinterpret_cast<const uint4*>(A.xpend)[u].z;
      int base = 0;
      uint32_t sparse = 0u;
      for (uint32_t todo = pend; todo != 0u; todo &= todo - 1u) {  // wave-uniform
        const int f = __builtin_ctz(todo);
        const uint32_t w = tid < 32 ? wsm[f * 32 + tid] : 0u;
        int inc = __popc(w);
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) {
          const int y = __shfl_up(inc, o, 64);
          if ((tid & 63) >= o) inc += y;
        }
        const int tot = __shfl(inc, 31, 64), ny = (nyq >> f) & 1u;
        if (tot + ny <= kSparseMax && base + tot + ny <= XL::SCAN_INTS) {
          int at = base + inc - __popc(w);
          for (uint32_t x = w; x != 0u; x &= x - 1u) items[at++] = (f << 16) | (tid + 32 * __builtin_ctz(x));
          if (ny && tid == 0) items[base + tot] = (f << 16) | (N / 2);
          base += tot + ny;
          sparse |= 1u << f;
        }
      }
      if (tid == 0) {
        ctl[0] = base;
        ctl[1] = (int)sparse;
      }
    }
    __syncthreads();
    const int n_sp = ctl[0];
    rest &= ~(uint32_t)ctl[1];
    if (n_sp > 0) exact_sparse<N>(A, lds, b, utt_len(A, b), c, items, n_sp, pacc, pbits);
  }
  while (rest != 0u) {  // block-uniform
    if (tid < FR) {
      uint32_t x = rest;
      for (int i = 0; i < tid && x; ++i) x &= x - 1u;
      if (x) exact_set_slot<N, PER_BIN>(A, sl, tid, u, __builtin_ctz(x), gx, n_items, n_whole, P);
    }
    const int ns = min(FR, __popc(rest));
    for (int i = 0; i < ns; ++i) rest &= rest - 1u;
    __syncthreads();
    exact_round<N, PER_BIN>(A, lds, sl, ns, pacc, pbits);
  }
  uint32_t* const MW = A.mwords + ((long long)b * A.nchunk + c) * F;
#pragma unroll
  for (int j = 0; j <= BPT; ++j) {
    const int kk = j < BPT ? tid + j * NT : N / 2;
    if (j < BPT || tid == NT - 1) {
      Pt[0 * F + kk] = pacc[j].c00;
      Pt[1 * F + kk] = pacc[j].c11;
      Pt[2 * F + kk] = pacc[j].c01r;
      Pt[3 * F + kk] = pacc[j].c01i;
      Pt[4 * F + kk] = pacc[j].cm;
      if (pbits[j]) atomicOr(MW + kk, pbits[j]);
    }
  }
}

// The given sparse frames of unit u (reference-bit path), in frame order, in batches of at
// most XLds::SCAN_INTS (bin, frame) items (exact_sparse) onto the running sums.
template <int N>
__device__ __forceinline__ void exact_sparse_frames(KArgs& A, unsigned char* lds, int u, int b,
                                                    int c, uint32_t frames,
                                                    Acc32 (&pacc)[CGeo<N>::BPT + 1],
                                                    uint32_t (&pbits)[CGeo<N>::BPT + 1]) {
  using G = CGeo<N>;
  using XL = XLds<N>;
  const int tid = threadIdx.x;
  int* const items = reinterpret_cast<int*>(lds + XL::SCAN_OFF);
  int* const ctl = reinterpret_cast<int*>(lds + XL::CTL_OFF);
  uint32_t* const wsm = reinterpret_cast<uint32_t*>(lds + 16384);  // [32][32] (slots: free)
  const uint4 rec = reinterpret_cast<const uint4*>(A.xpend)[u];
#pragma unroll
  for (int i = 0; i < kChunk / (G::NT / 32); ++i) {
    const int f = (tid >> 5) + (G::NT / 32) * i;
    if ((frames >> f) & 1u)
      wsm[f * 32 + (tid & 31)] =
          ((rec.y >> f) & 1u) ? A.xunc[((long long)u * kChunk + f) * 32 + (tid & 31)] : 0u;
  }
  __syncthreads();
  uint32_t todo = frames;
  while (todo != 0u) {  // block-uniform
    if (tid < 64) {
      int base = 0;
      uint32_t took = 0u;
      for (uint32_t t = todo; t != 0u; t &= t - 1u) {  // wave-uniform
        const int f = __builtin_ctz(t);
        const uint32_t w = tid < 32 ? wsm[f * 32 + tid] : 0u;
        int inc = __popc(w);
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) {
          const int y = __shfl_up(inc, o, 64);
          if ((tid & 63) >= o) inc += y;
        }
        const int tot = __shfl(inc, 31, 64), ny = (rec.z >> f) & 1u;
        if (base + tot + ny > XL::SCAN_INTS) break;
        int at = base + inc - __popc(w);
        for (uint32_t x = w; x != 0u; x &= x - 1u) items[at++] = (f << 16) | (tid + 32 * __builtin_ctz(x));
        if (ny && tid == 0) items[base + tot] = (f << 16) | (N / 2);
        base += tot + ny;
        took |= 1u << f;
      }
      if (tid == 0) {
        ctl[0] = base;
        ctl[1] = (int)took;
      }
    }
    __syncthreads();
    const int n = ctl[0];
    todo &= ~(uint32_t)ctl[1];
    exact_sparse<N>(A, lds, b, utt_len(A, b), c, items, n, pacc, pbits);  // ends on a barrier
  }
}

// Piece p of published unit u (XPieces): its terms summed from zero, the noise bits OR-ed into
// the chunk's mask words; with one piece added to the unit's partials at once, otherwise
// stored (xres[u][p]) and, by the piece that completes the unit (arrivals xst[u].y, agent-scope
// release / acquire), added to the partials in piece order -- the same sums whichever blocks
// ran the pieces. The unit's state is reset to 0 when it is complete.
template <int N, bool PER_BIN>
__device__ __forceinline__ void exact_piece(KArgs& A, unsigned char* lds, int u, int p, int gx,
                                            int n_items, int n_whole, int P) {
  using G = CGeo<N>;
  using XL = XLds<N>;
  constexpr int F = N / 2 + 1, NT = G::NT, BPT = G::BPT, FR = XL::FR;
  const int tid = threadIdx.x;
  XSlot* const sl = reinterpret_cast<XSlot*>(lds + XL::SLOT_OFF);
  int* const ctl = reinterpret_cast<int*>(lds + XL::CTL_OFF);
  const uint4 rec = reinterpret_cast<const uint4*>(A.xpend)[u];  // block-uniform
  const XPieces q = x_pieces(rec.x, rec.w);
  int b, c;
  float* const Pt = unit_item<F>(A, u, gx, n_items, n_whole, P, b, c);
  Acc32 pacc[BPT + 1];
  uint32_t pbits[BPT + 1];
#pragma unroll
  for (int j = 0; j <= BPT; ++j) {
    pacc[j].zero();
    pbits[j] = 0u;
  }
  if (p < q.n_sp) {
    if (A.xstat && tid == 0) atomicAdd(A.xstat, (unsigned long long)__popc(q.sp));  // diagnostic
    if constexpr (!PER_BIN) exact_sparse_frames<N>(A, lds, u, b, c, q.sp, pacc, pbits);
  } else {
    constexpr int R = kXRound;
    static_assert(R <= FR, "round frames");
    const int g = p - q.n_sp, r0 = g * q.nr / q.npr, r1 = (g + 1) * q.nr / q.npr;
    if (A.xstat && tid == 0)  // diagnostic: the piece's frames
      atomicAdd(A.xstat, (unsigned long long)(min(R * r1, __popc(rec.w)) - R * r0));
    const int L = utt_len(A, b);
    uint32_t rest = rec.w;
    for (int i = 0; i < r0 * R; ++i) rest &= rest - 1u;
    for (int r = r0; r < r1; ++r) {  // block-uniform
      if (tid < R) {  // the round's slots from the record (no per-slot global reads)
        uint32_t x = rest;
        for (int i = 0; i < tid && x; ++i) x &= x - 1u;
        if (x) {
          const int f = __builtin_ctz(x);
          XSlot s;
          s.unit = u;
          s.f = f;
          s.e = -1;
          s.b = b;
          s.L = L;
          s.c = c;
          s.flags = (PER_BIN ? 0 : (int)((rec.y >> f) & 1u)) | (int)(((rec.z >> f) & 1u) << 1);
          s.pad = 0;
          sl[tid] = s;
        }
      }
      const int ns = min(R, __popc(rest));
      for (int i = 0; i < ns; ++i) rest &= rest - 1u;
      __syncthreads();
      exact_round<N, PER_BIN>(A, lds, sl, ns, pacc, pbits);
    }
  }
  uint32_t* const MW = A.mwords + ((long long)b * A.nchunk + c) * F;
  float* const R = A.xres + ((long long)u * kXPieces + p) * 5 * F;
#pragma unroll
  for (int j = 0; j <= BPT; ++j) {
    const int kk = j < BPT ? tid + j * NT : N / 2;
    if (j < BPT || tid == NT - 1) {
      if (pbits[j]) atomicOr(MW + kk, pbits[j]);
      if (q.n == 1) {
        Pt[0 * F + kk] = Pt[0 * F + kk] + pacc[j].c00;
        Pt[1 * F + kk] = Pt[1 * F + kk] + pacc[j].c11;
        Pt[2 * F + kk] = Pt[2 * F + kk] + pacc[j].c01r;
        Pt[3 * F + kk] = Pt[3 * F + kk] + pacc[j].c01i;
        Pt[4 * F + kk] = Pt[4 * F + kk] + pacc[j].cm;
      } else {
        R[0 * F + kk] = pacc[j].c00;
        R[1 * F + kk] = pacc[j].c11;
        R[2 * F + kk] = pacc[j].c01r;
        R[3 * F + kk] = pacc[j].c01i;
        R[4 * F + kk] = pacc[j].cm;
      }
    }
  }
#ifdef AVZ_XTRACE
  const unsigned long long tf = __builtin_amdgcn_s_memrealtime();
#endif
  __syncthreads();
  if (tid == 0) {
    bool last = true;
    if (q.n > 1) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      const uint32_t arrived =
          __hip_atomic_fetch_add(A.xst + 2 * u + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
      last = arrived == (uint32_t)q.n;
      if (last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    ctl[4] = last ? 1 : 0;
  }
  __syncthreads();
#ifdef AVZ_XTRACE
  const unsigned long long tm = __builtin_amdgcn_s_memrealtime();
  if (tid == 0 && g_stamps) g_stamps[blockIdx.x * 16 + 6] += tm - tf;
#endif
  if (ctl[4]) {  // block-uniform: the unit is complete
    if (q.n > 1) {
      // Pt + piece 0 + piece 1 + ... per element; each piece's loads issued together
      const float* const R0 = A.xres + (long long)u * kXPieces * 5 * F;
      constexpr int M = (5 * F + NT - 1) / NT;
      float v[M];
#pragma unroll
      for (int m = 0; m < M; ++m) v[m] = tid + m * NT < 5 * F ? Pt[tid + m * NT] : 0.0f;
      for (int pp = 0; pp < q.n; ++pp) {  // block-uniform
        float t[M];
#pragma unroll
        for (int m = 0; m < M; ++m)
          t[m] = tid + m * NT < 5 * F ? R0[(long long)pp * 5 * F + tid + m * NT] : 0.0f;
#pragma unroll
        for (int m = 0; m < M; ++m) v[m] += t[m];
      }
#pragma unroll
      for (int m = 0; m < M; ++m)
        if (tid + m * NT < 5 * F) Pt[tid + m * NT] = v[m];
    }
    if (tid == 0) {
      __hip_atomic_store(A.xst + 2 * u + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(A.xst + 2 * u, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_and(A.xhint + (u >> 5), ~(1u << (u & 31)), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
#ifdef AVZ_XTRACE
  if (tid == 0 && g_stamps) g_stamps[blockIdx.x * 16 + 7] += __builtin_amdgcn_s_memrealtime() - tm;
#endif
}

// One open piece claimed for the block (wave 0; cand: 64 ints of LDS): -1 when no published
// unit has a piece left. Candidates: the units of the hint bits (from a block-dependent word,
// at most 64), their states read at once; the block takes one with a piece left (a
// block-dependent choice among them, so the claimants spread) by adding 1 to its state.
__device__ __forceinline__ int exact_claim(KArgs& A, int n_units, int* cand) {
  const int lane = threadIdx.x & 63;
  const int nw = (n_units + 31) >> 5;
  const int w_start = (int)(((long long)blockIdx.x * nw) / gridDim.x);
  for (;;) {  // wave-uniform; a retry follows another block's claim of a unit's last piece
    int count = 0;
    for (int w0 = 0; w0 < nw && count < 64; w0 += 64) {  // wave-uniform
      const int wi = w0 + lane;
      int wid = w_start + wi;
      if (wid >= nw) wid -= nw;
      const uint32_t bits =
          wi < nw ? __hip_atomic_load(A.xhint + wid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
      const int cnt = __popc(bits);
      int pre = cnt;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(pre, o, 64);
        if (lane >= o) pre += y;
      }
      const int tot = __shfl(pre, 63, 64);
      int pos = count + pre - cnt;
      for (uint32_t x = bits; x != 0u && pos < 64; x &= x - 1u) cand[pos++] = wid * 32 + __builtin_ctz(x);
      count += tot;
    }
    count = min(count, 64);
    if (count == 0) return -1;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // cand: LDS, lanes to lanes
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int uid = lane < count ? cand[lane] : -1;
    const uint32_t v =
        uid >= 0 ? __hip_atomic_load(A.xst + 2 * uid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    const unsigned long long m = __ballot(x_has_piece(v));
    if (m == 0ull) return -1;
    int k = (int)(blockIdx.x % (unsigned)__popcll(m));
    unsigned long long mm = m;
    for (; k > 0; --k) mm &= mm - 1ull;
    const int src = __builtin_ctzll(mm);
    int res = -1;
    if (lane == src) {
      const uint32_t old =
          __hip_atomic_fetch_add(A.xst + 2 * uid, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (x_has_piece(old)) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        res = (uid << 8) | (int)(old & 0xffu);
      }
    }
    res = __shfl(res, src, 64);
    if (res >= 0) return res;
    __builtin_amdgcn_wave_barrier();  // cand is rewritten by the next scan
  }
}

// After the persistent loop: the block's own unpublished units with deferrals (the unit mask,
// in analysis_items' order; sparse frames only), decided here (exact_unit), then pieces of the
// published units claimed from the whole grid (exact_claim, exact_piece) until none is left.
// Blocks end their loops at different times, so the exact work of one overlaps the others'
// loops (a separate launch spreading the units over its grid ran 173 us against 159 us at
// kappa 64, configs[1]; the work sharing took configs[1]'s analysis from 147 to 112 us).
template <int N, int MASK, bool IRM, bool SPLIT, class TW>
__device__ __forceinline__ void ibm_exact_units(unsigned char* lds, int gx, int n_items) {
  KArgs& A = kernarg_chain_args();
  using G = CGeo<N>;
  using XL = XLds<N>;
  constexpr bool SHARE = N == 1024 && !std::is_same<TW, NoTw>::value;
  constexpr bool PER_BIN = !(N == 1024 && !IRM && SHARE);  // not the reference-bit path
  AVZ_XT(1, __builtin_amdgcn_s_memrealtime());
  if (A.ibm_cert <= 0.0f) return;
  const int tid = threadIdx.x;
  const int P = SPLIT && A.a_pieces > 1 ? A.a_pieces : 1;
  const int n_whole = P > 1 ? A.a_whole : n_items;
  __syncthreads();  // the block's records, partials (global stores of other waves), unit mask
  const uint32_t mine = *reinterpret_cast<const uint32_t*>(lds + G::MISC_OFF + 56);
  auto tables = [&]() {
    int t = threadIdx.x;
    opaque_i(t);  // formed here (a thread index held from the kernel start went to scratch)
    xtab_fill<N>(A.xtw, A.xwin, reinterpret_cast<cd*>(lds + XL::TWL_OFF),
                 reinterpret_cast<float*>(lds + XL::WIN_OFF), t, G::NT);
    __syncthreads();
  };
  bool have_tables = false;
  int seq = 0;
  auto one = [&](int u) {  // the block's own unpublished units (published ones are shared)
    const int k = seq++;
    if (!((mine >> min(k, 31)) & 1u)) return;
    const uint4 rec = reinterpret_cast<const uint4*>(A.xpend)[u];  // block-uniform
    if (rec.x == 0u || rec.w != 0u) return;
    if (!have_tables) {
      tables();
      have_tables = true;
    }
    exact_unit<N, PER_BIN>(A, lds, u, gx, n_items, n_whole, P);
  };
  const int n_end = n_whole + (n_items - n_whole) * P;  // analysis_items' sequence
  for (int u = blockIdx.x; u < n_end; u += gridDim.x) one(u < n_whole ? u : n_items + u - n_whole);
  AVZ_XT(2, __builtin_amdgcn_s_memrealtime());
  {
    // the published units' pieces, claimed from the whole grid's (the block's own included)
    // until none is left
    const int n_units = n_items + (n_end - n_whole);
    int* const ctl = reinterpret_cast<int*>(lds + XLds<N>::CTL_OFF);
    for (;;) {  // block-uniform
#ifdef AVZ_XTRACE
      const unsigned long long tc = __builtin_amdgcn_s_memrealtime();
#endif
      if (tid < 64) {
        const int got = exact_claim(A, n_units, reinterpret_cast<int*>(lds + XLds<N>::SCAN_OFF));
        if (tid == 0) ctl[2] = got;
      }
#ifdef AVZ_XTRACE
      if (tid == 0 && g_stamps) g_stamps[blockIdx.x * 16 + 14] += __builtin_amdgcn_s_memrealtime() - tc;
#endif
      __syncthreads();
      const int got = ctl[2];
      __syncthreads();
      if (got < 0) break;
      if (!have_tables) {
#ifdef AVZ_XTRACE
        const unsigned long long tt = __builtin_amdgcn_s_memrealtime();
#endif
        tables();
        have_tables = true;
#ifdef AVZ_XTRACE
        if (tid == 0 && g_stamps) g_stamps[blockIdx.x * 16 + 15] += __builtin_amdgcn_s_memrealtime() - tt;
#endif
      }
#ifdef AVZ_XTRACE
      const unsigned long long t0x = __builtin_amdgcn_s_memrealtime();
#endif
      exact_piece<N, PER_BIN>(A, lds, got >> 8, got & 0xff, gx, n_items, n_whole, P);
#ifdef AVZ_XTRACE
      if (tid == 0 && g_stamps) {
        unsigned long long* st = g_stamps + blockIdx.x * 16;
        st[4] += 1;
        st[5] += __builtin_amdgcn_s_memrealtime() - t0x;
      }
#endif
    }
  }
  AVZ_XT(3, __builtin_amdgcn_s_memrealtime());
}

// Persistent grid (about two blocks per CU): block i takes the (chunk, utterance) items
// i, i + gridDim.x, ... so the twiddle table is built once per block and the batch is
// spread evenly over the resident blocks (no second, partly idle round of short blocks);
// a partial last round is split into step-range pieces (analysis_items; the SPLIT instance,
// launched only when the tail splitting is on, so the whole-rounds instance carries none of
// its code).
template <int N, int MASK, bool IRM, bool SPLIT = false>
__global__ void __launch_bounds__(kCThreads, KCfg<N>::BLOCKS_PER_CU) avz_analysis_kernel(ChainArgs A) {
  using G = CGeo<N>;
  extern __shared__ __align__(16) unsigned char lds[];
  AVZ_XT(0, __builtin_amdgcn_s_memrealtime());
  if (MASK == MASK_IBM && threadIdx.x == 0)  // ibm_exact_units' unit mask (after a barrier)
    *reinterpret_cast<uint32_t*>(lds + G::MISC_OFF + 56) = 0u;
  // the per-utterance synthesis' piece finalize state, reset here (the next launch reads it)
  if (A.pstate)
    for (int b = blockIdx.x * kCThreads + threadIdx.x; b < A.batch; b += gridDim.x * kCThreads)
      A.pstate[b] = PieceState{};
  KCfg<N>::Fft::fill_twiddles(reinterpret_cast<cf*>(lds + G::TW_OFF), threadIdx.x, G::NT);
  const int gx = (A.max_frames + kChunk - 1) / kChunk;
  const int n_items = gx * A.batch;
  if constexpr (N == 1024) {
    __syncthreads();
    cf tw_reg[31];
    Fft1024x2 f;
    f.init(threadIdx.x & 63);
    f.load_twiddles(tw_reg, reinterpret_cast<const cf*>(lds + G::TW_OFF));
    if (MASK != MASK_IPD && (threadIdx.x & 32)) {  // rotated frames: (-1)^k1 (pair_loads)
      static_for<0, 16>([&](auto i) { tw_reg[2 * i] = cf{-tw_reg[2 * i].x, -tw_reg[2 * i].y}; });
    }
    LaneConst<N> K;
    K.init(threadIdx.x);
    if (MASK != MASK_IPD && (threadIdx.x & 32)) {  // rotated frames (pair_loads): window
      K.wc.ac = -K.wc.ac;                          // halves swapped, once per kernel (per item
      K.wc.as = -K.wc.as;                          // both signs stayed live and one spilled)
    }
    analysis_items<N, MASK, IRM, SPLIT>(A, lds, gx, n_items, tw_reg, K);
    if constexpr (MASK == MASK_IBM) ibm_exact_units<N, MASK, IRM, SPLIT, Tw1024>(lds, gx, n_items);
  } else {
    LaneConst<N> K;
    K.init(threadIdx.x);
    analysis_items<N, MASK, IRM, SPLIT>(A, lds, gx, n_items, NoTw{}, K);
    if constexpr (MASK == MASK_IBM) ibm_exact_units<N, MASK, IRM, SPLIT, NoTw>(lds, gx, n_items);
  }
}

// ================================ solve ================================
// One thread per (utterance, bin): sum the chunk partials in fp64, closed-form MVDR or
// hybrid hard-null weights with the plan's steering table -> coef[b][k] (+ optional
// cov/w debug outputs).
constexpr int kSolveThreads = 256;

// Covariance sums of bin k of utterance b: fp64 sum of its nch chunk partials, scaled back
// by 1/4 (the analysis accumulates (2 y)(2 y)^H).
// V: split-chunk partial vectors per round trip (the per-utterance kernels' fallback takes
// few: its prefetched samples are live there).
template <int N, int V = 8, bool SPLIT = true>
__device__ __forceinline__ void bin_cov_sums(const ChainArgs& A, int b, int k, int nch,
                                             double (&R)[5]) {
  constexpr int F = N / 2 + 1;
  const float* P = A.part + (long long)b * A.nchunk * 5 * F + k;
#pragma unroll
  for (int q = 0; q < 5; ++q) R[q] = 0.0;
  // chunks of a split tail item (analysis_items) sum their pieces' partials
  const long long it0 = (long long)b * ((A.max_frames + kChunk - 1) / kChunk);
  const int cw =
      SPLIT && A.a_pieces > 1 ? (int)max(0LL, min((long long)nch, A.a_whole - it0)) : nch;
  for (int cc = 0; cc < cw; ++cc) {
#pragma unroll
    for (int q = 0; q < 5; ++q) R[q] += (double)P[((long long)cc * 5 + q) * F];
  }
  if (SPLIT && cw < nch) {
    // the split chunks' pieces: (nch - cw) a_pieces consecutive partial vectors of tpart,
    // V per round trip through a descriptor covering exactly them (absent ones read +0,
    // which leaves the sums unchanged); summed in chunk and piece order
    const int nv = (nch - cw) * A.a_pieces;
    const rsrc_t rt =
        make_rsrc(A.tpart + (it0 + cw - A.a_whole) * A.a_pieces * 5 * F, (long long)nv * 5 * F);
    for (int v0 = 0; v0 < nv; v0 += V) {
      float p[V][5];
#pragma unroll
      for (int i = 0; i < V; ++i)
#pragma unroll
        for (int q = 0; q < 5; ++q) p[i][q] = bload_nn(rt, ((v0 + i) * 5 + q) * F + k);
#pragma unroll
      for (int i = 0; i < V; ++i)
#pragma unroll
        for (int q = 0; q < 5; ++q) R[q] += (double)p[i][q];
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) R[q] *= 0.25;
}
// The same for a block-uniform utterance b (the per-utterance synthesis kernel): the
// partials of up to four chunks per round trip through a buffer descriptor covering
// exactly the utterance's nch chunks, so the loads of absent chunks read +0 without
// branches and the sums (chunk order kept, + 0 changes nothing) are bitwise those above.
template <int N, bool SPLIT = true, int VF = 4>
__device__ __forceinline__ void bin_cov_sums_utt(const ChainArgs& A, int b, int k, int nch,
                                                 double (&R)[5]) {
  constexpr int F = N / 2 + 1;
  if (SPLIT && A.a_pieces > 1 &&
      (long long)b * ((A.max_frames + kChunk - 1) / kChunk) + nch > A.a_whole) {
    bin_cov_sums<N, VF>(A, b, k, nch, R);  // some of its chunks were split (block-uniform)
    return;
  }
  const rsrc_t rp = make_rsrc(A.part + (long long)b * A.nchunk * 5 * F, (long long)nch * 5 * F);
#pragma unroll
  for (int q = 0; q < 5; ++q) R[q] = 0.0;
  for (int c0 = 0; c0 < nch; c0 += 4) {
    float p[4][5];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int q = 0; q < 5; ++q) p[i][q] = bload_nn(rp, ((c0 + i) * 5 + q) * F + k);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int q = 0; q < 5; ++q) R[q] += (double)p[i][q];
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) R[q] *= 0.25;
}
// The solve of bin k of utterance b from its covariance sums: closed-form MVDR or hybrid
// hard-null weights with the plan's steering table -> coef[b][k] (+ the cov / w debug
// outputs, the cov-only stage export, the item-level fallback flag).
template <int N>
__device__ __forceinline__ void solve_bin_out(const ChainArgs& A, int b, int k,
                                              const double (&R)[5]) {
  constexpr int F = N / 2 + 1;
  if (A.cov_only) {  // covariance stage export
#pragma unroll
    for (int q = 0; q < 5; ++q) A.cov_out[((long long)b * F + k) * 5 + q] = R[q];
    return;
  }
  const double* d = A.steer + 4 * k;
  cf al, be;
  float* wdbg = A.w_out ? A.w_out + ((long long)b * F + k) * 4 : nullptr;
  if (A.beamformer == BF_HYBRID_NULL) {
    hybrid_solve_d(R, k, N, A, d[0], d[1], d[2], d[3], al, be, wdbg);
  } else {
    double w[4];
    bool sing = false;
    mvdr_weights_d(R, k, N, A, d[0], d[1], d[2], d[3], w, &sing);
    if (sing && A.singular_fallback == 2) atomicOr(A.flag + b, 1);  // item-level fallback
    coef_from_w(w[0], w[1], w[2], w[3], al, be, wdbg);
  }
  reinterpret_cast<float4*>(A.coef)[(long long)b * F + k] = make_float4(al.x, al.y, be.x, be.y);
  if (A.cov_out) {
#pragma unroll
    for (int q = 0; q < 5; ++q) A.cov_out[((long long)b * F + k) * 5 + q] = R[q];
  }
}

template <int N, bool SPLIT = false>
__global__ void __launch_bounds__(kSolveThreads) avz_solve_kernel(ChainArgs A) {
  constexpr int H = N / 2, F = N / 2 + 1;
  const long long idx = (long long)blockIdx.x * kSolveThreads + threadIdx.x;
  if (idx >= (long long)(A.batch - A.b_lo) * F) return;
  const int b = A.b_lo + (int)(idx / F), k = (int)(idx % F);  // b_lo: first utterance solved
  const int L = utt_len(A, b);
  if (L < N) return;
  const int T = (L + H - 1) / H + 1;
  const int nch = (T + kChunk - 1) / kChunk;
  double R[5];
  bin_cov_sums<N, 8, SPLIT>(A, b, k, nch, R);
  solve_bin_out<N>(A, b, k, R);
}

// The solve of a small split batch (few bins, many partial vectors each: B = 1's 8.23-s
// triple at 512/256 has 17 chunks x 8 pieces): kSolveLanes lanes per bin, each summing a
// contiguous run of the bin's partial vectors (the whole chunks', then the split chunks'
// pieces, bin_cov_sums' order) in fp64, combined by a fixed xor tree -- deterministic, and
// the association differs from the sequential sum only by fp64 rounding. One round trip of
// 20 vectors per lane (160 per bin) where the sequential thread took 17 of 8.
constexpr int kSolveLanes = 8;
template <int N>
__global__ void __launch_bounds__(kSolveThreads) avz_solve_lanes_kernel(ChainArgs A) {
  constexpr int H = N / 2, F = N / 2 + 1, V = 20;
  const int sub = threadIdx.x % kSolveLanes;
  const long long idx = (long long)blockIdx.x * (kSolveThreads / kSolveLanes) +
                        threadIdx.x / kSolveLanes;
  // no early exit: a bin's lanes all take part in the tree (a group is 8 aligned lanes)
  const bool live = idx < (long long)(A.batch - A.b_lo) * F;
  const int b = A.b_lo + (live ? (int)(idx / F) : 0), k = live ? (int)(idx % F) : 0;
  const int L = utt_len(A, b);
  const bool ok = live && L >= N;
  const int T = (max(L, N) + H - 1) / H + 1;
  const int nch = (T + kChunk - 1) / kChunk;
  const long long it0 = (long long)b * ((A.max_frames + kChunk - 1) / kChunk);
  const int cw = A.a_pieces > 1 ? (int)max(0LL, min((long long)nch, A.a_whole - it0)) : nch;
  const int nvec = cw + (nch - cw) * (A.a_pieces > 1 ? A.a_pieces : 0);
  const rsrc_t rp = make_rsrc(A.part + (long long)b * A.nchunk * 5 * F, (long long)cw * 5 * F);
  const rsrc_t rt = cw < nch ? make_rsrc(A.tpart + (it0 + cw - A.a_whole) * A.a_pieces * 5 * F,
                                         (long long)(nvec - cw) * 5 * F)
                             : make_rsrc(nullptr, 0);
  const int per = (nvec + kSolveLanes - 1) / kSolveLanes;
  const int v_lo = sub * per, v_hi = min(nvec, v_lo + per);
  double R[5];
#pragma unroll
  for (int q = 0; q < 5; ++q) R[q] = 0.0;
  for (int v0 = v_lo; v0 < v_hi; v0 += V) {
    float pv[V][5];
#pragma unroll
    for (int i = 0; i < V; ++i) {
      const int v = v0 + i;  // past v_hi: read, not summed
#pragma unroll
      for (int q = 0; q < 5; ++q)
        pv[i][q] = v < cw ? bload(rp, (v * 5 + q) * F + k) : bload(rt, ((v - cw) * 5 + q) * F + k);
    }
#pragma unroll
    for (int i = 0; i < V; ++i)
      if (v0 + i < v_hi)
#pragma unroll
        for (int q = 0; q < 5; ++q) R[q] += (double)pv[i][q];
  }
#pragma unroll
  for (int o = 1; o < kSolveLanes; o <<= 1)
#pragma unroll
    for (int q = 0; q < 5; ++q) R[q] += __shfl_xor(R[q], o, kSolveLanes);
#pragma unroll
  for (int q = 0; q < 4; ++q) R[q] *= 0.25;
  if (ok && sub == 0) solve_bin_out<N>(A, b, k, R);
}

// batch_mvdr's item-level fallback (AVZ_FALLBACK_BATCH): the items whose solve met a
// singular bin get w = [1 / (conj(d0) + 1e-10), 0] on every bin. No-op otherwise.
template <int N>
__global__ void __launch_bounds__(kSolveThreads) avz_solve_fixup_kernel(ChainArgs A) {
  constexpr int F = N / 2 + 1;
  const long long idx = (long long)blockIdx.x * kSolveThreads + threadIdx.x;
  if (idx >= (long long)A.batch * F) return;
  const int b = (int)(idx / F), k = (int)(idx % F);
  if (A.flag[b] == 0) return;
  double w[4];
  batch_fallback_weights_d(A.steer[4 * k], A.steer[4 * k + 1], w);
  cf al, be;
  coef_from_w(w[0], w[1], w[2], w[3], al, be, A.w_out ? A.w_out + idx * 4 : nullptr);
  reinterpret_cast<float4*>(A.coef)[idx] = make_float4(al.x, al.y, be.x, be.y);
}

// ================================ SRP scan ================================
// scripts/debug_srp.py:46-62: P(theta) = sum_{f_lo <= f_k <= f_hi} sum_t |d^H y|^2
//   = sum_k R00 + R11 + 2 Re(conj(d0) d1 R01), conj(d0) d1 = exp(i w_k (tau1 - tau2)),
// from the unmasked covariance partials of the analysis kernel (MASK_ONES); one block
// per utterance: partials -> fp64 R in LDS, one thread per angle, dB relative to the max.
constexpr int kSrpThreads = 256;

template <int N>
__global__ void __launch_bounds__(kSrpThreads) avz_srp_kernel(ChainArgs A, SrpArgs S) {
  constexpr int H = N / 2, F = N / 2 + 1;
  __shared__ double R[F][4];
  __shared__ double red[kSrpThreads / 64];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int L = utt_len(A, b);
  double* out = S.power_db + (long long)b * S.n_angles;
  if (L < N) {
    for (int i = tid; i < S.n_angles; i += kSrpThreads) out[i] = __builtin_nan("");
    return;
  }
  const int T = (L + H - 1) / H + 1;
  const int nch = (T + kChunk - 1) / kChunk;
  const float* P = A.part + (long long)b * A.nchunk * 5 * F;
  for (int k = tid; k < F; k += kSrpThreads) {
    double r[4] = {0, 0, 0, 0};
    for (int cc = 0; cc < nch; ++cc) {
#pragma unroll
      for (int q = 0; q < 4; ++q) r[q] += (double)P[((long long)cc * 5 + q) * F + k];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) R[k][q] = 0.25 * r[q];  // analysis sums (2 y)(2 y)^H
  }
  __syncthreads();
  // f_k = rfftfreq(N, 1/fs)[k]; the scanned bins
  const double df = 1.0 / (N * (1.0 / A.fs));
  const double step = (S.n_angles > 1) ? (S.angle_hi - S.angle_lo) / (S.n_angles - 1) : 0.0;
  double best = -1e300;
  for (int i = tid; i < S.n_angles; i += kSrpThreads) {
    const double ang = (i == S.n_angles - 1 && S.n_angles > 1) ? S.angle_hi : S.angle_lo + i * step;
    const double th = ang * (M_PI / 180.0);
    // tau1 - tau2 = (d/2) cos(th)/c - (d/2) cos(th - pi)/c  (debug_srp.py:17-23)
    const double t1 = (A.mic_d / 2) * cos(0.0) * cos(th - 0) / A.c_sound;
    const double t2 = (A.mic_d / 2) * cos(0.0) * cos(th - M_PI) / A.c_sound;
    double p = 0.0;
    for (int k = 0; k < F; ++k) {
      const double f = k * df;
      if (f < S.f_lo || f > S.f_hi) continue;
      double sn, cs;
      sincos(2.0 * M_PI * f * (t1 - t2), &sn, &cs);
      p += R[k][0] + R[k][1] + 2.0 * (cs * R[k][2] - sn * R[k][3]);
    }
    const double db = 10.0 * log10(p);
    out[i] = db;
    best = fmax(best, db);
  }
  for (int o = 32; o > 0; o >>= 1) best = fmax(best, __shfl_xor(best, o, 64));
  if ((tid & 63) == 0) red[tid >> 6] = best;
  __syncthreads();
  double mx = red[0];
#pragma unroll
  for (int w = 1; w < kSrpThreads / 64; ++w) mx = fmax(mx, red[w]);
  for (int i = tid; i < S.n_angles; i += kSrpThreads) out[i] -= mx;
}

// ================================ synthesis ================================
// SPEC: the frames' spectra come from A.spec (avz_istft: scipy.signal.istft of a given
// S[b][k][t]) instead of the forward FFT of the mixture and the apply step.
template <int N, int PF, bool SPEC>
__device__ __forceinline__ void synthesis_item(const ChainArgs& A, unsigned char* lds, int c,
                                               int b, const LaneConst<N>& K) {
  static_assert(!SPEC || PF == PF_NONE, "spectrum input carries its own post-filter");
  using C = KCfg<N>;
  using G = SGeo<N, kSynR<N, PF>>;
  constexpr int NT = G::NT, H = G::H, F = G::F, NSLOT = G::NSLOT, BPT = G::BPT, PPL = C::PPL;
  constexpr int FB = NSLOT;           // frames per step
  constexpr int NPAIR = FB / 2;       // packed inverse FFTs per step
  constexpr int M4 = H / 4;           // float4 groups per half frame
  constexpr int NSG = NT / M4;        // segment groups
  constexpr int SPT = FB / NSG;       // segments per thread per step
  static_assert(SPT * NSG == FB, "OLA mapping");

  float* red = reinterpret_cast<float*>(lds + G::MISC_OFF);
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int L = utt_len(A, b);
  if (L < N) return;  // host validates; a bad device length reports NaN (finalize)
  const int T = (L + H - 1) / H + 1;
  const int nch = (T + kChunk - 1) / kChunk;
  if (c >= nch) return;
  const int t0 = c * kChunk;
  const int nstep = (min(kChunk, T - t0) + FB - 1) / FB;

  const typename C::Fft fft = K.fft;
  const LaneMap<N> lm = K.lm;
  const WinCoef<N> wc = K.wc;
  const int my_slot = wave * C::FPW + lm.grp;
  cf* my_spec = slot_ptr<N>(lds, my_slot);
  // SGeo::R > 1: the lane group also transforms frames my_slot + NWAVE FPW q, q < R
  constexpr int RSTRIDE = G::NWAVE * C::FPW;

  const float* mixb = A.mix + (long long)b * A.mix_stride;
  const rsrc_t r_m0 = make_rsrc(mixb, L), r_m1 = make_rsrc(mixb + A.ch_stride, L);
  cf v[PPL];
  cf vq[G::R > 1 ? G::R - 1 : 1][G::R > 1 ? PPL : 1];  // frames q >= 1 of the step
  auto load_frame = [&](cf (&x)[PPL], int frame, int wave_frame) {
    const int s0 = frame * H - N / 2 + lm.in0;
    if (wave_frame >= 1) {  // wave-uniform: no negative sample index
      static_for<0, PPL>([&](auto r) {
        x[r].x = bload_nn(r_m0, s0 + C::IN_STRIDE * r);
        x[r].y = bload_nn(r_m1, s0 + C::IN_STRIDE * r);
      });
    } else {
      static_for<0, PPL>([&](auto r) {
        x[r].x = bload(r_m0, s0 + C::IN_STRIDE * r);
        x[r].y = bload(r_m1, s0 + C::IN_STRIDE * r);
      });
    }
  };
  auto issue_loads = [&](int step) {
    const int fb = t0 + step * FB;
    load_frame(v, fb + my_slot, fb + wave * C::FPW);
    if constexpr (G::R > 1) {
#pragma unroll
      for (int q = 1; q < G::R; ++q)
        load_frame(vq[q - 1], fb + my_slot + q * RSTRIDE, fb + wave * C::FPW + q * RSTRIDE);
    }
  };
  AVZ_STAMP_DECL();
  AVZ_STAMP_INIT();
  if constexpr (!SPEC) issue_loads(0);

  // ---- apply coefficients and post-filter bits of this thread's bins tid + 256 j
  const float4* coef = reinterpret_cast<const float4*>(A.coef) + (long long)b * F;
  const uint32_t* MW = A.mwords + ((long long)b * A.nchunk + c) * F;
  cf alpha[BPT], beta[BPT];
  uint32_t bits[BPT];
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    const float4 cw = SPEC ? make_float4(0.f, 0.f, 0.f, 0.f) : coef[tid + j * NT];
    alpha[j] = cf{cw.x, cw.y};
    beta[j] = cf{cw.z, cw.w};
    bits[j] = (PF == PF_IBM_TARGET) ? MW[tid + j * NT] : 0u;
  }
  const bool nyq_wave = (wave == G::NWAVE - 1);
  cf alpha_n{0, 0}, beta_n{0, 0};  // the Nyquist bin N/2 (outside the pairs)
  uint32_t bits_n = 0u;
  // spectrum input: S[b][k][t] rows (t contiguous); frames past spec_frames read as zero
  const float2* Sb = SPEC ? reinterpret_cast<const float2*>(A.spec) + (long long)b * A.spec_sb
                          : nullptr;
  const int TS = SPEC ? min(T, A.spec_frames) : T;
  const bool svec = SPEC && ((A.spec_sb | A.spec_sf) & 1) == 0 &&
                    ((reinterpret_cast<uintptr_t>(A.spec) & 15) == 0);
  if (nyq_wave && !SPEC) {
    const float4 cw = coef[N / 2];
    alpha_n = cf{cw.x, cw.y};
    beta_n = cf{cw.z, cw.w};
    if (PF == PF_IBM_TARGET) bits_n = MW[N / 2];
  }
  const float* irm = (PF == PF_IRM) ? A.pf_gain + ((long long)b * A.nchunk + c) * kChunk * F
                                    : nullptr;
  const bool mask_vec = (PF == PF_EXT_FLOOR || PF == PF_EXT_MUL) && A.mask_st == 1 &&
                        (A.mask_sf & 3) == 0 && (A.mask_sb & 3) == 0 &&
                        ((reinterpret_cast<uintptr_t>(A.ext_mask) & 15) == 0);
  auto gain = [&](uint32_t bb, int i, int t, int k) -> float {  // i: frame bit in chunk
    if (t >= T) return 0.0f;
    if constexpr (PF == PF_IBM_TARGET) {
      return ((bb >> i) & 1u) ? 0.0f : 1.0f;
    } else if constexpr (PF == PF_IRM) {
      return irm[i * F + k];
    } else if constexpr (PF == PF_EXT_FLOOR || PF == PF_EXT_MUL) {
      const float M =
          A.ext_mask[(long long)b * A.mask_sb + (long long)k * A.mask_sf + (long long)t * A.mask_st];
      return PF == PF_EXT_FLOOR ? fmaxf(M, A.pf_floor) : M;
    } else {
      return 1.0f;
    }
  };

  // OLA role: 4 consecutive samples m0.. of segments sgrp + NSG si
  const int m0 = 4 * (tid % M4);
  const int sgrp = tid / M4;
  float inv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) inv[i] = K.inv[i];
  static_assert(M4 == N / 8, "LaneConst's OLA role");
  float4 carry = make_float4(0.f, 0.f, 0.f, 0.f);  // previous frame's second half (sgrp 0)
  float* outb = A.out + (long long)b * A.out_stride;
  float peak = 0.0f;
  const bool ifft_wave = wave < NPAIR / C::FPW;  // waves holding a packed pair

  lds_barrier();  // the previous item's readers
  AVZ_STAMP(4);
  for (int step = 0; step < nstep; ++step) {
    const int f0 = t0 + step * FB;
    const bool more = step + 1 < nstep;
#ifdef AVZ_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    AVZ_STAMP(5);
#endif
    if constexpr (!SPEC) {
      window_fft<N, true>(v, wc, fft, my_spec, lm);
      if constexpr (G::R > 1) {
#pragma unroll
        for (int q = 1; q < G::R; ++q)
          window_fft<N, true>(vq[q - 1], wc, fft, slot_ptr<N>(lds, my_slot + q * RSTRIDE), lm);
      }
      // N = 512: the next step's loads fly through apply, inverse FFT and OLA (the N = 1024
      // inverse runs in the sample registers, so its loads wait until it is done)
      if (N != 1024 && more) issue_loads(step + 1);
    }
    lds_barrier();
    AVZ_STAMP(6);

    // ---- apply w^H y and the post-filter; pack frames (2p, 2p+1) into slot 2p
    auto apply_phase = [&](auto vec) {
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      const int kb = tid + j * NT;
      const int kp = (N - kb) & (N - 1);
      // Branch-free: frames past T were transformed from zeros and get gain 0, and the
      // OLA never writes the segments they touch, so every pair is processed.
      cf za[NPAIR], zap[NPAIR], zb[NPAIR], zbp[NPAIR];
#pragma unroll
      for (int p = 0; p < NPAIR; ++p) {
        const cf* Za = slot_ptr<N>(lds, 2 * p);
        const cf* Zb = slot_ptr<N>(lds, 2 * p + 1);
        za[p] = lds_read(Za + kb);
        zap[p] = lds_read(Za + kp);
        zb[p] = lds_read(Zb + kb);
        zbp[p] = lds_read(Zb + kp);
      }
      // External mask with t-contiguous, 16-B aligned rows (the U-Net / TFLite outputs):
      // the bin's FB gains of this step in FB/4 16-B loads instead of FB scattered ones,
      // each loaded for the two pairs that use it (all FB at once held 16 more VGPRs at
      // N = 512 and spilled 44-72 B)
      constexpr bool VEC = decltype(vec)::value;
      const float4* mp = VEC ? reinterpret_cast<const float4*>(
                                   A.ext_mask + (long long)b * A.mask_sb + (long long)kb * A.mask_sf + f0)
                             : nullptr;
      float4 g4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int p = 0; p < NPAIR; ++p) {
        const int ta = f0 + 2 * p;
        cf* Za = slot_ptr<N>(lds, 2 * p);
        const int ia = step * FB + 2 * p;
        float ga, gb;
        if constexpr (VEC) {
          if (p % 2 == 0) g4 = mp[p / 2];
          ga = (p % 2 == 0) ? g4.x : g4.z;
          gb = (p % 2 == 0) ? g4.y : g4.w;
          if constexpr (PF == PF_EXT_FLOOR) {
            ga = fmaxf(ga, A.pf_floor);
            gb = fmaxf(gb, A.pf_floor);
          }
        } else {
          ga = gain(bits[j], ia, ta, kb);
          gb = gain(bits[j], ia + 1, ta + 1, kb);
        }
        const cf sa = apply_bin(alpha[j], beta[j], za[p], zap[p], ga);
        const cf sb = apply_bin(alpha[j], beta[j], zb[p], zbp[p], gb);
        Za[kp] = {sa.x + sb.y, sb.x - sa.y};  // conj(Sa) + i conj(Sb) at N - k
        // Sa + i Sb at k; at DC irfft keeps only the real parts (written last: kp == kb)
        Za[kb] = (kb == 0) ? cf{sa.x, sb.x} : cf{sa.x - sb.y, sa.y + sb.x};
      }
    }
    };
    // spectrum input: the step's frames of the thread's bins straight from S, packed as
    // above (16-B row segments when the rows are aligned and the step is complete)
    auto spec_phase = [&](auto vec) {
#pragma unroll
      for (int j = 0; j < BPT; ++j) {
        const int kb = tid + j * NT;
        const int kp = (N - kb) & (N - 1);
        const float2* row = Sb + (long long)kb * A.spec_sf + f0;
        cf sv[FB];
        if constexpr (decltype(vec)::value) {
#pragma unroll
          for (int q = 0; q < FB / 2; ++q) {
            const float4 x = reinterpret_cast<const float4*>(row)[q];
            sv[2 * q] = cf{x.x, x.y};
            sv[2 * q + 1] = cf{x.z, x.w};
          }
        } else {
#pragma unroll
          for (int i = 0; i < FB; ++i) {
            const float2 x = (f0 + i < TS) ? row[i] : make_float2(0.f, 0.f);
            sv[i] = cf{x.x, x.y};
          }
        }
#pragma unroll
        for (int p = 0; p < NPAIR; ++p) {
          cf* Za = slot_ptr<N>(lds, 2 * p);
          const cf sa = sv[2 * p], sb = sv[2 * p + 1];
          Za[kp] = {sa.x + sb.y, sb.x - sa.y};
          Za[kb] = (kb == 0) ? cf{sa.x, sb.x} : cf{sa.x - sb.y, sa.y + sb.x};
        }
      }
    };
    if constexpr (SPEC) {
      if (svec && f0 + FB <= TS)  // block-uniform
        spec_phase(std::true_type{});
      else
        spec_phase(std::false_type{});
    } else if constexpr (PF == PF_EXT_FLOOR || PF == PF_EXT_MUL) {
      if (mask_vec && f0 + FB <= T)  // wave-uniform
        apply_phase(std::true_type{});
      else
        apply_phase(std::false_type{});
    } else {
      apply_phase(std::false_type{});
    }
    if (SPEC && nyq_wave && lane < NPAIR) {  // Nyquist bin from S: real parts (irfft)
      const int ta = f0 + 2 * lane;
      if (ta < T) {
        const float2* row = Sb + (long long)(N / 2) * A.spec_sf;
        const float xa = ta < TS ? row[ta].x : 0.f, xb = ta + 1 < TS ? row[ta + 1].x : 0.f;
        slot_ptr<N>(lds, 2 * lane)[N / 2] = {xa, xb};
      }
    }
    if (!SPEC && nyq_wave && lane < NPAIR) {  // Nyquist bin: frame pair `lane`
      const int ta = f0 + 2 * lane;
      if (ta < T) {
        const int ia = step * FB + 2 * lane;
        cf* Za = slot_ptr<N>(lds, 2 * lane);
        const cf* Zb = slot_ptr<N>(lds, 2 * lane + 1);
        const float ga = gain(bits_n, ia, ta, N / 2), gb = gain(bits_n, ia + 1, ta + 1, N / 2);
        const cf za = Za[N / 2], zb = Zb[N / 2];
        Za[N / 2] = {apply_bin(alpha_n, beta_n, za, za, ga).x,
                     apply_bin(alpha_n, beta_n, zb, zb, gb).x};
      }
    }
    lds_barrier();
    AVZ_STAMP(7);

    // ---- inverse FFT of the packed pairs -> windowed frame contributions in slot 2p+1:
    // one packed pair per lane group, two transforms per wave on the waves holding pairs.
    // The N = 1024 transform runs in the sample registers v (the round-1 x1 form with four
    // waves and the loads in flight ran 77.5 vs 73.6 us), so the next step's loads are
    // issued after it (issuing them on the pairless waves first, inside the inverse, or
    // after the overlap-add measured 1-3 us slower).
    if (ifft_wave) {
      const int p = wave * C::FPW + lm.grp;
      cf* Zi = slot_ptr<N>(lds, 2 * p);
      auto inverse = [&](cf (&u)[PPL]) {
        static_for<0, PPL>([&](auto r) { u[r] = c_conj(Zi[lm.in0 + C::IN_STRIDE * r]); });
        float* Cp = reinterpret_cast<float*>(slot_ptr<N>(lds, 2 * p + 1));
        auto emit = [&](auto k, cf x) {
          constexpr float ck = W32::c[k], sk = -W32::s[k];  // cos, sin of 2 pi k / 32
          const float w = fmaf(wc.ss, sk, fmaf(-wc.sc, ck, wc.s0));
          const int n = lm.out0 + C::OUT_STRIDE * k;
          Cp[n] = x.x * w;       // frame 2p   (real part of the inverse)
          Cp[N + n] = -x.y * w;  // frame 2p+1 (imaginary part; conjugation trick)
        };
        if constexpr (N == 1024) {
          fft.stage1_ab_st(u, Zi);
          fft.transpose_read(u, Zi);
          fft.stage2_emit(u, emit);
        } else {
          fft.forward_emit(u, Zi, emit);
        }
      };
      if constexpr (N == 1024) {
        inverse(v);
      } else {
        cf u[PPL];
        inverse(u);
      }
    }
    if (N == 1024 && !SPEC && more) issue_loads(step + 1);
    lds_barrier();
    AVZ_STAMP(8);

    // ---- overlap-add: segment j = f0 - 1 + s = frame s-1 (2nd half) + frame s (1st half)
    auto cframe = [&](int f) -> const float* {
      return reinterpret_cast<const float*>(slot_ptr<N>(lds, 2 * (f >> 1) + 1)) + (f & 1) * N;
    };
#pragma unroll
    for (int si = 0; si < SPT; ++si) {
      const int s = sgrp + si * NSG;
      const float4 vb = *reinterpret_cast<const float4*>(cframe(s) + m0);
      if (s == 0 && step == 0) {  // chunk's first frame: finalize adds the previous tail
        *reinterpret_cast<float4*>(A.heads + ((long long)b * A.nchunk + c) * H + m0) = vb;
        continue;
      }
      const int j = f0 - 1 + s;
      if (j <= T - 2) {
        // unconditional read + value select: the conditional read compiled to four
        // bank-conflicting ds_read_b32 (as in the per-utterance kernel)
        const float4 vp = *reinterpret_cast<const float4*>(cframe(s == 0 ? 0 : s - 1) + H + m0);
        const float4 va = (s == 0) ? carry : vp;
        float4 o;
        o.x = (va.x + vb.x) * inv[0];
        o.y = (va.y + vb.y) * inv[1];
        o.z = (va.z + vb.z) * inv[2];
        o.w = (va.w + vb.w) * inv[3];
        *reinterpret_cast<float4*>(outb + (long long)j * H + m0) = o;
        peak = fmaxf(peak, fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(o.w))));
      }
    }
    if (sgrp == 0) carry = *reinterpret_cast<const float4*>(cframe(FB - 1) + H + m0);
    lds_barrier();
    AVZ_STAMP(9);
  }
  if (sgrp == 0 && nstep * FB == kChunk)  // full chunk: its last frame's tail
    *reinterpret_cast<float4*>(A.tails + ((long long)b * A.nchunk + c) * H + m0) = carry;

  // ---- block max |out| -> utterance running max (non-negative floats order as uints)
  for (int o = 32; o > 0; o >>= 1) peak = fmaxf(peak, __shfl_xor(peak, o, 64));
  if (lane == 0) red[wave] = peak;
  __syncthreads();
  if (tid == 0) {
    float pk = red[0];
#pragma unroll
    for (int w = 1; w < G::NWAVE; ++w) pk = fmaxf(pk, red[w]);
    atomicMax(A.peak_u + b, __float_as_uint(pk));
  }
  AVZ_STAMP(10);
}

// Persistent grid over (chunk, utterance) items, as avz_analysis_kernel.
template <int N, int PF, bool SPEC = false>
__global__ void __launch_bounds__(kCThreads, KCfg<N>::SYN_BLOCKS_PER_CU) avz_synthesis_kernel(ChainArgs A) {
  extern __shared__ __align__(16) unsigned char lds[];
  const int gx = (A.max_frames + kChunk - 1) / kChunk;
  LaneConst<N> K;
  K.init(threadIdx.x);
  const int nsyn = gx * A.batch;
  for (int it = blockIdx.x; it < nsyn; it += gridDim.x)
    synthesis_item<N, PF, SPEC>(A, lds, it % gx, it / gx, K);
}

// ============================ per-utterance synthesis (N = 1024) ============================
// One 8-wave block per CU synthesises WHOLE utterances (b = blockIdx.x, + gridDim.x, ...),
// 16 frames per step, and peak-normalises each one itself at its end: no chunk seams, no
// heads / tails, no finalize launch, and the rescale re-reads the block's own output from
// L2 / Infinity Cache instead of a second HBM pass over the batch. Every wave runs its own
// two frames end to end -- window + forward Fft1024x2 (the next step's loads issued from
// inside its last stage), apply w^H y + post-filter, each frame's real inverse as an
// N/2-point complex Fft512x2 -- with no block barrier in between (the apply reads only the
// wave's own spectra); the block meets twice per step, around the overlap-add of the 16
// segments, which reads neighbouring waves' frames. Reference semantics as the two-block
// kernel + avz_finalize_kernel (oracle_debug.py:80-94, scipy istft's OLA and N/2 trim).
constexpr int kUttThreads = 512;
#ifndef AVZ_PRESOLVE_V
#define AVZ_PRESOLVE_V 16
#endif
#ifndef AVZ_UTT_SHARE
#define AVZ_UTT_SHARE 1
#endif
#ifndef AVZ_UTT_NL0
#define AVZ_UTT_NL0 32
#endif
struct UttGeo {
  static constexpr int N = 1024, H = 512, F = 513, FB = 16;  // frames per step: 8 waves x 2
  static constexpr int SLOT = KCfg<1024>::GROUP_BYTES;       // one frame (transpose rows of 34)
  static constexpr int TW_OFF = FB * SLOT;                   // W1024 table (Fft512x2 inverse)
  static constexpr int COEF_OFF = TW_OFF + KCfg<1024>::TW_BYTES;  // the utterance's alpha, beta
  static constexpr int RED_OFF = COEF_OFF + F * 16;
  static constexpr int LDS_BYTES = RED_OFF + 64;
  static_assert(LDS_BYTES <= 160 * 1024, "one block per CU");
  static_assert(kChunk % FB == 0, "a step stays inside one 32-frame mask chunk");
};
__device__ __forceinline__ cf* utt_frame(unsigned char* lds, int f) {
  return reinterpret_cast<cf*>(lds + f * UttGeo::SLOT);
}

// SOLVE: the block solves its utterance's 513 bins itself (the MVDR solve of
// avz_solve_kernel, one bin per thread, straight into the LDS coefficient table) instead of
// reading the solve kernel's coef[] -- no solve launch (plain MVDR plans without the
// item-level fallback or debug outputs). PIECES: the instance for a split batch (whole
// utterances, then step pieces; synth_split) -- the whole-rounds instance compiles the
// piece logic out (with it the step loop ran 92.7 -> 98.5 us at B = 256).
template <int PF, bool SOLVE, bool PIECES>
__global__ void __launch_bounds__(kUttThreads, 2) avz_synthesis_utt_kernel(ChainArgs A) {
  constexpr int N = UttGeo::N, H = UttGeo::H, F = UttGeo::F, FB = UttGeo::FB;
  extern __shared__ __align__(16) unsigned char lds[];
  cf* twid = reinterpret_cast<cf*>(lds + UttGeo::TW_OFF);
  float* red = reinterpret_cast<float*>(lds + UttGeo::RED_OFF);
  Fft1024x2::fill_twiddles(twid, threadIdx.x, kUttThreads);
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // 0..7
  const int lane = tid & 63;
  // SHARE: a wave's two frames (2 wave, 2 wave + 1) overlap by N/2 and are loaded as in the
  // analysis kernel (pair_loads: 24 sample pairs per lane instead of 32, lane group 1's frame
  // rotated by N/2): its window halves swapped (ac, as negated) and its spectrum's (-1)^k
  // undone by (-1)^k1 on the stage-1 twiddles (the odd j factors twa[j - 1] of k1 = 8 m + j)
  constexpr bool SHARE = AVZ_UTT_SHARE;
  Fft1024x2 fft;
  fft.init(lane);
  LaneMap<N> lm;
  lm.init(lane);
  if (SHARE && lm.grp) {
    static_for<0, 4>([&](auto i) { fft.twa[2 * i] = cf{-fft.twa[2 * i].x, -fft.twa[2 * i].y}; });
  }
  const WinCoef<N> wc0 = [&] {
    WinCoef<N> w;
    w.init(lm);
    if (SHARE && lm.grp) {
      w.ac = -w.ac;
      w.as = -w.as;
    }
    return w;
  }();
  const int my = 2 * wave + lm.grp;  // frame of the step = slot
  // apply bins: m_j = lane + 64 j (j < 4) pairs bin kA = m with kB = N/2 - m; bin N/4 (its
  // own partner) on lanes 0 (frame 2 wave) and 1 (frame 2 wave + 1)
  cf om[4];  // e^{+2 pi i m_j / N}
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double sn, cs;
    sincospi(2.0 * (lane + 64 * j) / N, &sn, &cs);
    om[j] = cf{(float)cs, (float)sn};
  }
  // inverse output: x[k] = conj(z[m]), m = mh + 16 k -> samples 2m, 2m + 1 (0.5 hann)
  float wh_c[2], wh_s[2];
  const int mh = (lane & 15) + 256 * ((lane >> 4) & 1);
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    double sn, cs;
    sincospi(2.0 * (2 * mh + e) / N, &sn, &cs);
    wh_c[e] = (float)(0.25 * cs);
    wh_s[e] = (float)(0.25 * sn);
  }
  // overlap-add role: 4 consecutive samples m0.. of segments sgrp + 4 si
  float inv[4];  // (filled after a first piece's pre-solve: live across it, they spilled)
  __syncthreads();  // twiddle table
  AVZ_STAMP_DECL();
  AVZ_STAMP_INIT();

  // The block's work units g = blockIdx.x, + gridDim.x, ...: the whole utterances g <
  // s_whole, then the pieces q = g - s_whole of the utterances [s_whole, batch) (ChainArgs
  // s_pieces, s_steps): utterance s_whole + q / s_pieces, its steps [p s_steps, (p + 1) s_steps),
  // p = q % s_pieces (the host splits only a partial last round or a batch below the CU
  // count). With the in-kernel piece finalize (s_ipf: the batch has whole rounds, and its
  // rem * s_pieces piece units fit one round) the pieces come FIRST: unit index g < G is
  // piece q = g (none for g >= rem * s_pieces), g >= G whole utterance g - G, so every block
  // runs at most one piece and then its whole utterances, during which the piece's interior
  // is rescaled once its utterance's last piece has published 1/peak. A whole utterance with
  // a bad device length (host validates) reports NaN, as finalize does; such an utterance's
  // pieces, and pieces past an utterance's last step, are skipped (its first piece, or the
  // piece finalize kernel, reports the NaN).
  const int pieces = PIECES && A.s_pieces > 0 ? A.s_pieces : 0;
  const int s_whole = pieces > 0 ? A.s_whole : A.batch;
  const bool ipf = PIECES && pieces > 0 && A.s_ipf;
  const int G = gridDim.x;
  const int n_pu = (A.batch - s_whole) * pieces;  // piece units
  const int n_units = ipf ? G + s_whole : s_whole + n_pu;
  struct Unit {
    int g, b, s_lo, s_hi, slot;  // slot: the piece's seam slot, -1 for a whole utterance
  };
  auto unit_at = [&](int g) -> Unit {
    for (; g < n_units; g += gridDim.x) {
      // lengths read back as block-uniform values: a loop exit decided on a vector load
      // made the next unit's buffer descriptors divergent (a waterfall loop per load)
      const bool is_whole = ipf ? g >= G : g < s_whole;
      if (is_whole) {
        const int gw = ipf ? g - G : g;
        const int Lg = __builtin_amdgcn_readfirstlane(utt_len(A, gw));
        if (Lg >= N) return Unit{g, gw, 0, ((Lg + H - 1) / H + 1 + FB - 1) / FB, -1};
        if (tid == 0 && A.peak) A.peak[gw] = __builtin_nanf("");
        continue;
      }
      const int pc = pieces > 0 ? pieces : 1;  // (0 only in the whole-rounds instance)
      const int q = ipf ? g : g - s_whole;
      if (q >= n_pu) continue;
      const int bq = s_whole + q / pc, lo = (q % pc) * A.s_steps;
      const int Lq = __builtin_amdgcn_readfirstlane(utt_len(A, bq));
      const int ns = ((Lq + H - 1) / H + 1 + FB - 1) / FB;
      if (Lq >= N && lo < ns) return Unit{g, bq, lo, min(ns, lo + A.s_steps), q};
      if (ipf && Lq < N && lo == 0 && tid == 0 && A.peak) A.peak[bq] = __builtin_nanf("");
    }
    return Unit{n_units, A.batch, 0, 0, -1};
  };
  auto rsrcs = [&](int bb, rsrc_t& a0, rsrc_t& a1) {
    bb = __builtin_amdgcn_readfirstlane(bb);
    const float* mixb = A.mix + (long long)bb * A.mix_stride;
    const int len = __builtin_amdgcn_readfirstlane(utt_len(A, bb));
    a0 = make_rsrc(mixb, len);
    a1 = make_rsrc(mixb + A.ch_stride, len);
  };
  cf v[32];
  // a unit's first step (frames f0 ..): at f0 = 0 wave 0's first frame starts N/2 before
  // sample 0 (range-checked offsets); every other frame starts at sample >= 0
  auto first_loads = [&](rsrc_t a0, rsrc_t a1, int f0) {
    if constexpr (SHARE) {
      const int sp = (f0 + 2 * wave) * H - N / 2 + lm.in0;
      if (wave >= 1 || f0 > 0)
        pair_loads<true>(v, a0, a1, sp, lm.grp);
      else
        pair_loads<false>(v, a0, a1, sp, lm.grp);
      return;
    }
    const int s0 = (f0 + my) * H - N / 2 + lm.in0;
    if (wave >= 1 || f0 > 0) {
      static_for<0, 32>([&](auto r) {
        v[r].x = bload_nn(a0, s0 + 32 * r);
        v[r].y = bload_nn(a1, s0 + 32 * r);
      });
    } else {
      static_for<0, 32>([&](auto r) {
        v[r].x = bload(a0, s0 + 32 * r);
        v[r].y = bload(a1, s0 + 32 * r);
      });
    }
  };
  // the utterance's bins solved into the LDS coefficient table (SOLVE)
  auto solve_coefs = [&](int bb, int TT, auto vf) {
    constexpr int VF = decltype(vf)::value;
    float4* ct = reinterpret_cast<float4*>(lds + UttGeo::COEF_OFF);
    const int nch = (TT + kChunk - 1) / kChunk;
    for (int k = tid; k < F; k += kUttThreads) {
      double R[5], w[4];
      bin_cov_sums_utt<N, PIECES, VF>(A, bb, k, nch, R);
      const double* d = A.steer + 4 * k;
      mvdr_weights_d(R, k, N, A, d[0], d[1], d[2], d[3], w, nullptr);
      cf al, be;
      coef_from_w(w[0], w[1], w[2], w[3], al, be, nullptr);
      ct[k] = make_float4(al.x, al.y, be.x, be.y);
    }
  };
  Unit cu = unit_at(blockIdx.x);
  // A piece (the block's first unit) solves before any sample is loaded: its utterance's
  // chunks may have been split by the analysis tail (up to 8 partial vectors per chunk),
  // summed 16 vectors per round trip with the registers the samples would hold (with the
  // samples in flight, 8 per round trip spilled)
  bool coefs_ready = false;
  if (PIECES && SOLVE && cu.slot >= 0) {
    const int Lp = __builtin_amdgcn_readfirstlane(utt_len(A, cu.b));
    solve_coefs(cu.b, (Lp + H - 1) / H + 1, std::integral_constant<int, AVZ_PRESOLVE_V>{});
    coefs_ready = true;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) inv[i] = inv_wsum<N>(4 * (tid & 127) + i);
  if (cu.b < A.batch) {
    rsrc_t a0, a1;
    rsrcs(cu.b, a0, a1);
    first_loads(a0, a1, PIECES ? cu.s_lo * FB : 0);
  }
  // NORM_PEAK: an utterance's rescale (its own output, L1-bypassing loads) runs spread over
  // the NEXT utterance's steps, one slice per overlap-add phase, so its memory traffic hides
  // under that utterance's FFTs; a block's last utterance rescales at once.
  float* rs_out = nullptr;  // pending rescale: output row, scale, float4 groups, done
  float rs_scale = 0.0f;
  int rs_n4 = 0, rs_done = 0;
  constexpr int RS_U = 4;   // float4 groups per thread per slice (8 slices cover 4 s)
  constexpr int RS_UP = 8;   // the same during a piece's steps (4 slices cover 4 s)
  constexpr int RS_BULK = 32;  // after the loop: a 4-s utterance in one round trip of loads
  // s_ipf: a piece's own interior waits for its utterance's 1/peak (pstate[rs_lazy].fin, piece
  // rs_lp): each slice loads it beside the output and stores only once it is published
  int rs_lazy = -1, rs_lp = 0;
  uint32_t* redu = reinterpret_cast<uint32_t*>(red);  // red[8 ..]: block-uniform hand-offs
  auto rescale_slice = [&](auto uc, int lo, int hi, auto issue_more) -> bool {
    constexpr int U = decltype(uc)::value;
    const rsrc_t ro = make_rsrc(rs_out, 4LL * rs_n4);
    int tq = tid;
    if constexpr (PIECES) opaque_i(tq);  // offsets recomputed per slice (hoisted, they spilled)
    float4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const v4i_t d = __builtin_amdgcn_raw_buffer_load_b128(ro, 16 * (lo + u * kUttThreads + tq), 0,
                                                            kSC1);
      x[u] = make_float4(__int_as_float(d.x), __int_as_float(d.y), __int_as_float(d.z),
                         __int_as_float(d.w));
    }
    uint32_t fb = 0;
    if (PIECES && rs_lazy >= 0)
      fb = __hip_atomic_load(&A.pstate[rs_lazy].fin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    issue_more();  // work that overlaps the loads
    if (PIECES && rs_lazy >= 0) {
      fb = __builtin_amdgcn_readfirstlane(fb);
      if (fb == 0u || A.dbg_ipf == 2) return false;  // not yet published: again next step
      rs_scale = __uint_as_float(fb);
      rs_lazy = -1;
    }
    float4* o4 = reinterpret_cast<float4*>(rs_out);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = lo + u * kUttThreads + tq;
      if (i < hi) {
        x[u].x *= rs_scale; x[u].y *= rs_scale; x[u].z *= rs_scale; x[u].w *= rs_scale;
        o4[i] = x[u];
      }
    }
    return true;
  };
  // the pending rescale's remaining part, U float4 loads per thread in flight (a lazy one
  // resolved first, rs_resolve)
  auto rescale_rest = [&](auto uc) {
    constexpr int U = decltype(uc)::value;
    for (; rs_done < rs_n4; rs_done += U * kUttThreads)
      rescale_slice(uc, rs_done, min(rs_n4, rs_done + U * kUttThreads), [] {});
    rs_out = nullptr;
  };
  // A piece's interior still waiting at its block's next utterance end: take 1/peak if it is
  // published, else hand the piece back to the last arriver (.st bit p) -- unless that one
  // has passed it already (bit 32 + p), in which case 1/peak is published by now. Called by
  // every thread after tid 0's redu[12] / redu[10..11] and a barrier (end-of-unit code).
  auto rs_resolve = [&]() {
    const uint32_t fb = redu[12];
    const unsigned long long st = *reinterpret_cast<const unsigned long long*>(redu + 10);
    if (fb != 0u) {
      rs_scale = __uint_as_float(fb);
    } else if ((st >> (32 + rs_lp)) & 1ull) {
      rs_scale = __uint_as_float(__builtin_amdgcn_readfirstlane(
          __hip_atomic_load(&A.pstate[rs_lazy].fin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
    } else {
      rs_out = nullptr;  // handed back
    }
    rs_lazy = -1;
  };
  // A hand-back passes the interior (written by this block's plain stores, complete since
  // the piece's end) to another block on any XCD: released (L2 write-back) before the bit.
  auto hand_back = [&](int bb, int p) -> unsigned long long {  // tid 0
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    return atomicOr(&A.pstate[bb].st, 1ull << p);
  };
  auto rs_resolve_issue = [&]() {  // tid 0, before that barrier
    const uint32_t fb =
        __hip_atomic_load(&A.pstate[rs_lazy].fin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    redu[12] = fb;
    if (fb == 0u) *reinterpret_cast<unsigned long long*>(redu + 10) = hand_back(rs_lazy, rs_lp);
  };
  // the float4 groups of piece p's interior segments [p seg, (p + 1) seg - 2] (<= T - 2)
  auto piece_lo4 = [&](int p, int sg) { return p * sg * H / 4; };
  auto piece_hi4 = [&](int p, int sg, int T) { return min((p + 1) * sg - 1, T - 1) * H / 4; };
  // s_ipf: the last piece of utterance b to arrive forms its np - 1 seams (pieces' halves
  // written through to memory, read the same way) x 1 / sum w^2 -- the OLA's arithmetic --,
  // takes the utterance peak over them and the pieces' interior maxima, writes the seams
  // scaled and peak[b], publishes 1/peak and rescales the interiors handed back to it.
  auto piece_finalize = [&](int b, int T, int np, int sg, float* outb) {
    // thread-derived offsets recomputed here from an opaque tid (hoisted to the kernel start
    // they were held through the steps and spilled)
    int t = tid;
    opaque_i(t);
    const long long slot0 = (long long)(b - s_whole) * pieces;
    const float iw = inv_wsum<N>(t);  // H = kUttThreads: thread t owns sample m = t
    // seam p = tail of piece p - 1 + head of piece p, 8 seams per round trip through
    // descriptors covering the np slots; raw values to the frame slots (free at a unit's end)
    // for the scaled write. Only seams p < np enter the peak: for p = np the tail load still
    // falls inside the descriptor (slot np - 1's tail: no seam, possibly an earlier call's)
    const rsrc_t rt = make_rsrc(A.ptails + slot0 * H, (long long)np * H);
    const rsrc_t rh = make_rsrc(A.pheads + slot0 * H, (long long)np * H);
    float* stash = reinterpret_cast<float*>(lds) + t;
    // the pieces' interior maxima (RMW: after every piece's atomicMax), with the seam loads
    uint32_t pku = 0u;
    if (t == 0) pku = atomicMax(A.peak_u + b, 0u);
    float mx = 0.0f;
    for (int p0 = 1; p0 < np; p0 += 8) {
      float sv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int p = p0 + u;
        sv[u] = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(rt, 4 * ((p - 1) * H + t), 0, kSC1)) +
                __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(rh, 4 * (p * H + t), 0, kSC1));
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (p0 + u < np) {
          sv[u] *= iw;
          mx = fmaxf(mx, fabsf(sv[u]));
          stash[(p0 + u - 1) * H] = sv[u];
        }
      }
    }
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    __syncthreads();  // red[] free
    if (lane == 0) red[wave] = mx;
    if (t == 0) redu[9] = pku;
    __syncthreads();
    float pk = __uint_as_float(redu[9]);
#pragma unroll
    for (int w = 0; w < kUttThreads / 64; ++w) pk = fmaxf(pk, red[w]);
    const float scale = 1.0f / (pk + A.norm_eps);
    float* ot = outb + t;
    for (int p = 1; p < np; ++p) ot[(long long)(p * sg - 1) * H] = stash[(p - 1) * H] * scale;
    if (t == 0) {
      if (A.peak) A.peak[b] = pk;
      __hip_atomic_store(&A.pstate[b].fin, __float_as_uint(scale), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // published before the pass
      uint32_t hi;
      asm volatile("v_mov_b32 %0, -1" : "=v"(hi));  // materialised here (hoisted, it spilled)
      const unsigned long long old = atomicOr(&A.pstate[b].st, (unsigned long long)hi << 32);
      *reinterpret_cast<unsigned long long*>(redu + 10) = old;
      // interiors handed back: their owners' writes, released before their bits, acquired
      if ((uint32_t)old != 0u) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    const unsigned long long hb = *reinterpret_cast<const unsigned long long*>(redu + 10);
    for (int p = 0; p < np; ++p)
      if ((hb >> p) & 1ull) {
        rs_out = outb;
        rs_scale = scale;
        rs_done = piece_lo4(p, sg);
        rs_n4 = piece_hi4(p, sg, T);
        rescale_rest(std::integral_constant<int, 2 * RS_U>{});
      }
  };
  // Across a unit's steps only b and its last step are held (more spilled): a piece is
  // recognised by b >= s_whole, its seam slot and unit index follow from b and the frame.
  const int seg = FB * (A.s_steps > 0 ? A.s_steps : 1);  // frames per piece
  while (cu.b < A.batch) {
    const int b = cu.b;
    const int L = __builtin_amdgcn_readfirstlane(utt_len(A, b));
    const int T = (L + H - 1) / H + 1;
    rsrc_t r0, r1;
    rsrcs(b, r0, r1);
    // the next unit's first step is loaded during this unit's last step (waves >= 1 from
    // inside the FFT, wave 0 right after it) and lands during the rescale (the next unit is
    // looked up again after the loop: held across the steps it spilled)
    int nb = 0, nlen = 0, nf0 = 0;  // the next unit's utterance, length (0: none), 1st frame
    {
      const Unit t = unit_at(cu.g + gridDim.x);
      if (t.b < A.batch) {
        nb = __builtin_amdgcn_readfirstlane(t.b);
        nlen = __builtin_amdgcn_readfirstlane(utt_len(A, t.b));
        nf0 = PIECES ? __builtin_amdgcn_readfirstlane(t.s_lo * FB) : 0;
      }
    }
    // the utterance's apply coefficients into LDS (read per step, so they hold no registers
    // through the FFTs); the previous unit's readers finished at its last barrier. Every
    // piece of an utterance solves its bins too (no solve launch before the kernel).
    {
      float4* ct = reinterpret_cast<float4*>(lds + UttGeo::COEF_OFF);
      if (SOLVE) {
        if (!PIECES || !coefs_ready) solve_coefs(b, T, std::integral_constant<int, 4>{});
        coefs_ready = false;
      } else {
        const float4* coef = reinterpret_cast<const float4*>(A.coef) + (long long)b * F;
        int k0 = tid;
        opaque_i(k0);  // its address computed here (hoisted to the kernel start, it spilled)
        for (int k = k0; k < F; k += kUttThreads) ct[k] = coef[k];
      }
    }
    __syncthreads();
    AVZ_STAMP(15);
    uint32_t bits[9];
    float4 carry = make_float4(0.f, 0.f, 0.f, 0.f);
    float peak = 0.0f;
    float* outb = A.out + (long long)b * A.out_stride;
    const int s_hi = cu.s_hi, s_lo = PIECES ? cu.s_lo : 0;
    int step = s_lo;
    for (; step < s_hi; ++step) {
#ifdef AVZ_STAMPS
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      AVZ_STAMP(13);
#endif
      const int f0 = step * FB, c = f0 / kChunk;
      // lane-derived LDS / global offsets recomputed per step (held across the loop they
      // cost ~100 VGPRs and spilled)
      int ln = lane, tq = tid;
      opaque_i(ln);
      opaque_i(tq);
      if ((f0 % kChunk == 0 || (PIECES && step == s_lo)) && PF == PF_IBM_TARGET) {  // bits
        const uint32_t* MW = A.mwords + ((long long)b * A.nchunk + c) * F;
#pragma unroll
        for (int q = 0; q < 9; ++q)
          bits[q] = MW[q < 4 ? ln + 64 * q : (q < 8 ? H - ln - 64 * (q - 4) : N / 4)];
      }
      // ---- window + forward FFT of frames f0 + 2 wave + g into slot my; the next step's
      // loads go out from inside its last stage (frames >= FB: no negative sample index)
      const bool more = step + 1 < s_hi;
      const bool il = more || wave >= 1 || nf0 > 0;
      // the descriptors of the next step's loads, built from block-uniform scalars (a
      // select between two descriptors went to VGPRs: a waterfall loop around every load)
      rsrc_t q0, q1;
      {
        const int qb = __builtin_amdgcn_readfirstlane(more ? b : nb);
        const int ql = __builtin_amdgcn_readfirstlane(more ? L : nlen);
        const float* qm = A.mix + (long long)qb * A.mix_stride;
        q0 = make_rsrc(qm, ql);
        q1 = make_rsrc(qm + A.ch_stride, ql);
      }
      const int sn = ((more ? f0 + FB : nf0) + (SHARE ? 2 * wave : my)) * H - N / 2 + lm.in0;
      // the next step's loads go out after the apply (issued from inside the forward FFT's
      // last stage, after the FFT or after the inverse measured slower)
      // (registers k < NL0 after the apply, the rest between the inverse's two DFT stages,
      // under its transpose's LDS round trip: with 32 loads per lane 28 + 4 measured best
      // (profiles/r05/ab_next_loads_split.txt), with the 24 of SHARE all after the apply,
      // profiles/r05/ab_share_loads.txt)
      constexpr int NL0 = AVZ_UTT_NL0;
      auto load_k = [&](auto kc) {  // register k's next sample pair (SHARE: as pair_loads)
        constexpr int k = decltype(kc)::value;
        if constexpr (!SHARE) {
          v[k].x = bload_nn(q0, sn + 32 * k);
          v[k].y = bload_nn(q1, sn + 32 * k);
        } else if constexpr (k < 16) {
          const int e = sn + 1024 * lm.grp + 32 * k;
          v[k].x = bload_nn(q0, e);
          v[k].y = bload_nn(q1, e);
        } else if constexpr ((k - 16) % 2 == 0) {
          const int e = sn + 512 + 32 * (k - 16) + 32 * lm.grp;
          v[k].x = bload_nn(q0, e);
          v[k].y = bload_nn(q1, e);
        }
      };
      auto next_loads = [&]() {
        if (il)
          static_for<0, NL0>(load_k);
        else
          first_loads(q0, q1, 0);  // wave 0, last step: the next utterance (or empty)
      };
      auto next_loads_mid = [&]() {
        if (il) static_for<NL0, 32>(load_k);
      };
      if constexpr (SHARE) pair_finish(v);
      window_fft<N>(v, wc0, fft, utt_frame(lds, my), lm);
      AVZ_STAMP(4);
      __builtin_amdgcn_wave_barrier();
      const float* irm = (PF == PF_IRM) ? A.pf_gain + ((long long)b * A.nchunk + c) * kChunk * F
                                        : nullptr;
      auto gain = [&](uint32_t bb, int i, int t, int k) -> float {  // i: frame bit in chunk
        if (t >= T) return 0.0f;
        if constexpr (PF == PF_IBM_TARGET) {
          return ((bb >> i) & 1u) ? 0.0f : 1.0f;
        } else if constexpr (PF == PF_IRM) {
          return irm[i * F + k];
        } else if constexpr (PF == PF_EXT_FLOOR || PF == PF_EXT_MUL) {
          const float M = A.ext_mask[(long long)b * A.mask_sb + (long long)k * A.mask_sf +
                                     (long long)t * A.mask_st];
          return PF == PF_EXT_FLOOR ? fmaxf(M, A.pf_floor) : M;
        } else {
          return 1.0f;
        }
      };
      // ---- apply w^H y + post-filter of the wave's frames, folded into each frame's
      // N/2-point inverse input (written in place over the bins just read):
      //   Zh[m] = A + i B, Zh[N/2 - m] = conj(A) + i conj(B),
      //   A = S[m] + conj(S[N/2 - m]),  B = e^{2 pi i m / N} (S[m] - conj(S[N/2 - m]))
      cf al[9], be[9];
      {
        const float4* ct = reinterpret_cast<const float4*>(lds + UttGeo::COEF_OFF);
#pragma unroll
        for (int q = 0; q < 9; ++q) {
          const float4 w = ct[q < 4 ? ln + 64 * q : (q < 8 ? H - ln - 64 * (q - 4) : N / 4)];
          al[q] = cf{w.x, w.y};
          be[q] = cf{w.z, w.w};
        }
      }
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const int f = 2 * wave + g, t = f0 + f, ib = f0 % kChunk + f;
        cf* Z = utt_frame(lds, f);
        cf za[4], zap[4], zb[4], zbp[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int kA = ln + 64 * j, kB = H - kA;
          za[j] = lds_read(Z + kA);
          zap[j] = lds_read(Z + ((N - kA) & (N - 1)));
          zb[j] = lds_read(Z + kB);
          zbp[j] = lds_read(Z + (N - kB));
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int kA = ln + 64 * j, kB = H - kA;
          cf sa = apply_bin(al[j], be[j], za[j], zap[j], gain(bits[j], ib, t, kA));
          cf sb = apply_bin(al[4 + j], be[4 + j], zb[j], zbp[j], gain(bits[4 + j], ib, t, kB));
          if (j == 0 && ln == 0) {  // DC and Nyquist: irfft keeps the real parts
            sa.y = 0.0f;
            sb.y = 0.0f;
          }
          const cf a = {sa.x + sb.x, sa.y - sb.y};
          const cf d = {sa.x - sb.x, sa.y + sb.y};
          const cf bb = c_mul(om[j], d);
          Z[kA] = {a.x - bb.y, a.y + bb.x};
          Z[kB] = {a.x + bb.y, bb.x - a.y};
        }
        if (ln == g) {  // bin N/4: Zh = 2 conj(S)
          const cf s = apply_bin(al[8], be[8], Z[N / 4], Z[3 * N / 4], gain(bits[8], ib, t, N / 4));
          Z[N / 4] = {2.0f * s.x, -2.0f * s.y};
        }
      }
      AVZ_STAMP(5);
      next_loads();
      AVZ_STAMP(6);
      __builtin_amdgcn_wave_barrier();
      // ---- inverse: lane group g transforms frame 2 wave + g; windowed contributions
      // (samples 2m, 2m + 1 as one float2) over the frame's first 4 KB, the transpose in its
      // second half
      {
        cf* Zi = utt_frame(lds, my);
        cf u[16];
        static_for<0, 16>([&](auto r) { u[r] = c_conj(lds_read(Zi + (ln & 31) + 32 * r)); });
        float2* Cp = reinterpret_cast<float2*>(Zi);
        const int mhs = (ln & 15) + 256 * ((ln >> 4) & 1);
        Fft512x2::forward_tw1024_emit(u, Zi + H, twid, ln, [&](auto k, cf x) {
          constexpr float ck = W32::c[k], sk = -W32::s[k];  // cos, sin of 2 pi (32 k) / N
          const float we = fmaf(wh_s[0], sk, fmaf(-wh_c[0], ck, 0.25f));
          const float wo = fmaf(wh_s[1], sk, fmaf(-wh_c[1], ck, 0.25f));
          Cp[mhs + 16 * k] = make_float2(x.x * we, -x.y * wo);
        }, next_loads_mid);
      }
      AVZ_STAMP(7);
      lds_barrier();
      AVZ_STAMP(8);
      // ---- overlap-add: segment j = f0 - 1 + s = frame s-1 (2nd half) + frame s (1st half);
      // segment -1 (frame 0's first half) is scipy's trimmed N/2
      auto cframe = [&](int f) -> const float* {
        return reinterpret_cast<const float*>(utt_frame(lds, f));
      };
      const int m0 = 4 * (tq & 127), sgrp = __builtin_amdgcn_readfirstlane(tq >> 7);
      // a piece's first step (its first segment is a seam) and the piece's seam slot
      const bool pstart = PIECES && b >= s_whole && f0 % seg == 0;
      const long long pslot = (long long)(b - s_whole) * pieces + f0 / seg;
      auto ola = [&]() {
#pragma unroll
      for (int si = 0; si < 4; ++si) {
        const int s = sgrp + 4 * si;
        const int j = f0 - 1 + s;
        if (j >= 0 && j <= T - 2) {
          const float4 vb = *reinterpret_cast<const float4*>(cframe(s) + m0);
          if (s == 0 && pstart) {  // a piece's first segment is a seam: its half for the
            store_through(A.pheads + pslot * H, H, m0, vb);  // piece finalize
            continue;
          }
          // the previous frame's half read unconditionally (frame 0's when s = 0) and the
          // carry selected by value: a conditional read was split into four ds_read_b32
          // (4-way bank conflicts, 15 % of the kernel's LDS cycles), a pointer select with
          // &carry put carry on the stack
          const float4 vp = *reinterpret_cast<const float4*>(cframe(s == 0 ? 0 : s - 1) + H + m0);
          const float4 va = (s != 0) ? vp : carry;
          float4 o;
          o.x = (va.x + vb.x) * inv[0];
          o.y = (va.y + vb.y) * inv[1];
          o.z = (va.z + vb.z) * inv[2];
          o.w = (va.w + vb.w) * inv[3];
          *reinterpret_cast<float4*>(outb + (long long)j * H + m0) = o;
          peak = fmaxf(peak, fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(o.w))));
        }
      }
      };
      if (rs_out != nullptr && rs_done < rs_n4) {  // a slice of the previous utterance's rescale
        if (PIECES && b >= s_whole) {  // a piece's few steps: larger slices
          const int lo = rs_done, hi = min(rs_n4, rs_done + RS_UP * kUttThreads);
          if (rescale_slice(std::integral_constant<int, RS_UP>{}, lo, hi, ola)) rs_done = hi;
        } else {
          const int lo = rs_done, hi = min(rs_n4, rs_done + RS_U * kUttThreads);
          if (rescale_slice(std::integral_constant<int, RS_U>{}, lo, hi, ola)) rs_done = hi;
        }
      } else {
        ola();
      }
      if (sgrp == 0) carry = *reinterpret_cast<const float4*>(cframe(FB - 1) + H + m0);
      // a piece's last half-frame (seam half): a whole utterance's last step never has a
      // segment f0 + FB - 1 <= T - 2 (its last frame is T - 1 <= f0 + FB - 1)
      if (PIECES && sgrp == 0 && !more && f0 + FB - 1 <= T - 2)
        store_through(A.ptails + pslot * H, H, m0, carry);
      AVZ_STAMP(9);
      lds_barrier();
      AVZ_STAMP(10);
    }
    // ---- utterance peak; NORM_PEAK rescales the block's own output (its stores drained
    // first; L1-bypassing loads), as avz_finalize_kernel did in a second pass over HBM
    for (int o = 32; o > 0; o >>= 1) peak = fmaxf(peak, __shfl_xor(peak, o, 64));
    if (lane == 0) red[wave] = peak;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const bool whole = !PIECES || b < s_whole;
    // s_ipf: a piece interior of this block still waiting for its 1/peak (rs_resolve)
    const bool resolve = PIECES && ipf && whole && rs_lazy >= 0;
    if (resolve && tid == 0) rs_resolve_issue();
    __syncthreads();
    float pk = red[0];
#pragma unroll
    for (int w = 1; w < kUttThreads / 64; ++w) pk = fmaxf(pk, red[w]);
    if (resolve) rs_resolve();
    if (!whole) {  // a piece: its interior's max (non-negative floats order as uints)
      if (ipf) {
        // arrival: the seam halves were written through (sc1) and drained above, the
        // atomicMax completes before the count
        if (tid == 0) {
          atomicMax(A.peak_u + b, __float_as_uint(pk));
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          redu[9] = atomicAdd(&A.pstate[b].cnt, 1u);
        }
        __syncthreads();
        const int p = (step - 1) / A.s_steps;
        const int np = min(pieces, ((T + FB - 1) / FB + A.s_steps - 1) / A.s_steps);
        const bool fin_here = __builtin_amdgcn_readfirstlane(redu[9]) == (uint32_t)(np - 1);
        if (fin_here) piece_finalize(b, T, np, seg, outb);
        // its own interior: rescaled in slices once 1/peak is published
        rs_out = outb;
        rs_lazy = b;
        rs_lp = p;
        rs_done = piece_lo4(p, seg);
        rs_n4 = piece_hi4(p, seg, T);
        if (A.dbg_ipf == 1 && !fin_here) {  // diagnostic: hand back at once (rs_resolve)
          if (tid == 0) {
            redu[12] = 0u;
            *reinterpret_cast<unsigned long long*>(redu + 10) = hand_back(b, p);
          }
          __syncthreads();
          rs_resolve();
        }
      } else if (tid == 0) {
        atomicMax(A.peak_u + b, __float_as_uint(pk));
      }
    } else if (tid == 0 && A.peak) {
      A.peak[b] = pk;
    }
    if (whole && A.normalize == NORM_PEAK) {
      // the previous one's slices left over (an utterance of < 8 steps)
      if (rs_out != nullptr) rescale_rest(std::integral_constant<int, 2 * RS_U>{});
      rs_out = outb;
      rs_scale = 1.0f / (pk + A.norm_eps);
      rs_n4 = (T - 1) * H / 4;
      rs_done = 0;
    }
    __syncthreads();  // red[] of the next unit
    AVZ_STAMP(14);
    // this unit's index (unit_at): from b (whole) or the piece's q, (step - 1) / s_steps its
    // piece
    cu = unit_at((whole ? (ipf ? b + G : b)
                        : (ipf ? 0 : s_whole) + (b - s_whole) * pieces + (step - 1) / A.s_steps) +
                 gridDim.x);
  }
  // a piece interior still lazy: every later unit of the block was skipped (device length
  // < N), so no whole utterance's end resolved it -- take 1/peak or hand it back now
  // (rescale_rest's slices assume a published scale)
  if (PIECES && ipf && rs_lazy >= 0) {
    if (tid == 0) rs_resolve_issue();
    __syncthreads();
    rs_resolve();
  }
  // the block's last utterance, after the loop where the sample registers are dead: every
  // load of a 4-s utterance in flight at once (the single-utterance blocks of B <= #CU
  // rescale here; a latency-bound loop with 8 loads in flight per thread ran ~13 us)
  if (rs_out != nullptr) rescale_rest(std::integral_constant<int, RS_BULK>{});
  AVZ_STAMP(14);
}

// ======================= per-utterance synthesis (N = 512) =======================
// The N = 512 form of avz_synthesis_utt_kernel: one 8-wave block per CU owns whole
// utterances and normalises them itself, but keeps the chunk kernel's step (synthesis_item
// at N = 512): every lane group transforms two frames (R = 2), so a step is 32 frames -- one
// IBM mask chunk -- in 32 slots of 4.3 KB (139 KB), and the 16 packed inverse pairs
// (Sa + i Sb, one complex Fft512x2 per lane group) keep all eight waves busy through the
// inverse (at N = 1024 the same packing would leave half the waves idle, hence that
// kernel's per-frame half-size inverse). Apply: thread t serves bin t & 255 for the frame
// pairs 8 (t >> 8) .. + 8. Seam carried in registers across the chunks, peak and rescale
// in-block (progressive over the next utterance's overlap-add phases), solve in-block
// (SOLVE), as the N = 1024 kernel. Reference semantics as the chunk kernel + finalize.
constexpr int kUtt512Threads = 512;
struct Utt512Geo {
  static constexpr int N = 512, H = 256, F = 257, NWAVE = 8, FPW = 2, R = 2;
  static constexpr int RSTRIDE = NWAVE * FPW;       // 16: a lane group's second frame
  static constexpr int FB = RSTRIDE * R;            // 32 frames per step
  static constexpr int NPAIR = FB / 2;              // 16 packed inverse pairs
  static constexpr int SLOT_LDS = FB * KCfg<512>::GROUP_BYTES;
  static constexpr int COEF_OFF = SLOT_LDS;         // the utterance's alpha, beta
  static constexpr int RED_OFF = COEF_OFF + F * 16;
  static constexpr int LDS_BYTES = RED_OFF + 64;
  static_assert(FB == kChunk, "a step is one mask chunk");
  static_assert(LDS_BYTES <= 160 * 1024, "one block per CU");
  static_assert(KCfg<512>::WAVE_BYTES == FPW * KCfg<512>::GROUP_BYTES, "slot_ptr layout");
};

template <int PF, bool SOLVE>
__global__ void __launch_bounds__(kUtt512Threads, 2) avz_synthesis_utt512_kernel(ChainArgs A) {
  using G = Utt512Geo;
  using C = KCfg<512>;
  constexpr int N = G::N, H = G::H, F = G::F, FB = G::FB, NPAIR = G::NPAIR, RSTRIDE = G::RSTRIDE;
  constexpr int PPL = C::PPL;
  constexpr int M4 = H / 4;                    // float4 groups per half frame
  constexpr int NSG = kUtt512Threads / M4;     // 8 segment groups (one per wave)
  constexpr int SPT = FB / NSG;                // 4 segments per thread per step
  constexpr int PPT = NPAIR / 2;               // 8 frame pairs per apply thread
  extern __shared__ __align__(16) unsigned char lds[];
  float* red = reinterpret_cast<float*>(lds + G::RED_OFF);
  float4* ct = reinterpret_cast<float4*>(lds + G::COEF_OFF);
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  Fft512x2 fft;
  fft.init(lane);
  LaneMap<N> lm;
  lm.init(lane);
  const WinCoef<N> wc = [&] { WinCoef<N> w; w.init(lm); return w; }();
  const int my_slot = wave * G::FPW + lm.grp;  // frames my_slot, my_slot + 16 of the step
  const int p0 = PPT * (wave >> 2);  // apply: pairs p0 .. p0 + 7 (wave-uniform)
  const bool nyq_wave = (wave == G::NWAVE - 1);
  const int sgrp = wave;             // overlap-add: segments wave + 8 si
  static_assert(M4 == 64, "one segment group per wave");
  float inv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) inv[i] = inv_wsum<N>(4 * lane + i);
  const rsrc_t r_none = make_rsrc(nullptr, 0);
  AVZ_STAMP_DECL();
  AVZ_STAMP_INIT();

  auto next_valid = [&](int bb) {
    for (; bb < A.batch; bb += gridDim.x) {
      if (utt_len(A, bb) >= N) break;
      if (tid == 0 && A.peak) A.peak[bb] = __builtin_nanf("");
    }
    return bb;
  };
  auto rsrcs = [&](int bb, rsrc_t& a0, rsrc_t& a1) {
    bb = __builtin_amdgcn_readfirstlane(bb);
    const float* mixb = A.mix + (long long)bb * A.mix_stride;
    const int len = __builtin_amdgcn_readfirstlane(utt_len(A, bb));
    a0 = make_rsrc(mixb, len);
    a1 = make_rsrc(mixb + A.ch_stride, len);
  };
  cf v[PPL], vq[PPL];
  // frames fb + my_slot (v) and fb + my_slot + 16 (vq); a step's first wave starts N/2 before
  // sample 0 only at fb = 0 on wave 0 (range-checked offsets there)
  auto load_step = [&](rsrc_t a0, rsrc_t a1, int fb) {
    const int s0 = (fb + my_slot) * H - N / 2 + lm.in0, s1 = s0 + RSTRIDE * H;
    if (fb + wave * G::FPW >= 1) {
      static_for<0, PPL>([&](auto r) {
        v[r].x = bload_nn(a0, s0 + C::IN_STRIDE * r);
        v[r].y = bload_nn(a1, s0 + C::IN_STRIDE * r);
      });
    } else {
      static_for<0, PPL>([&](auto r) {
        v[r].x = bload(a0, s0 + C::IN_STRIDE * r);
        v[r].y = bload(a1, s0 + C::IN_STRIDE * r);
      });
    }
    static_for<0, PPL>([&](auto r) {
      vq[r].x = bload_nn(a0, s1 + C::IN_STRIDE * r);
      vq[r].y = bload_nn(a1, s1 + C::IN_STRIDE * r);
    });
  };
  int b = next_valid(blockIdx.x);
  if (b < A.batch) {
    rsrc_t a0, a1;
    rsrcs(b, a0, a1);
    load_step(a0, a1, 0);
  }
  // NORM_PEAK rescale of the block's previous utterance, one slice per overlap-add phase
  float* rs_out = nullptr;
  float rs_scale = 0.0f;
  int rs_n4 = 0, rs_done = 0;
  constexpr int RS_U = 4, RS_BULK = 32;
  auto rescale_slice = [&](auto uc, int lo, int hi, auto issue_more) {
    constexpr int U = decltype(uc)::value;
    const rsrc_t ro = make_rsrc(rs_out, 4LL * rs_n4);
    float4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const v4i_t d = __builtin_amdgcn_raw_buffer_load_b128(ro, 16 * (lo + u * kUtt512Threads + tid),
                                                            0, kSC1);
      x[u] = make_float4(__int_as_float(d.x), __int_as_float(d.y), __int_as_float(d.z),
                         __int_as_float(d.w));
    }
    issue_more();
    float4* o4 = reinterpret_cast<float4*>(rs_out);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = lo + u * kUtt512Threads + tid;
      if (i < hi) {
        x[u].x *= rs_scale; x[u].y *= rs_scale; x[u].z *= rs_scale; x[u].w *= rs_scale;
        o4[i] = x[u];
      }
    }
  };
  auto rescale_rest = [&](auto uc) {
    constexpr int U = decltype(uc)::value;
    for (; rs_done < rs_n4; rs_done += U * kUtt512Threads)
      rescale_slice(uc, rs_done, min(rs_n4, rs_done + U * kUtt512Threads), [] {});
    rs_out = nullptr;
  };

  while (b < A.batch) {
    const int L = utt_len(A, b);
    const int T = (L + H - 1) / H + 1;
    const int nstep = (T + FB - 1) / FB;
    rsrc_t r0, r1;
    rsrcs(b, r0, r1);
    const int nb = next_valid(b + gridDim.x);
    rsrc_t n0 = r_none, n1 = r_none;
    if (nb < A.batch) rsrcs(nb, n0, n1);
    if constexpr (SOLVE) {
      const int nch = (T + kChunk - 1) / kChunk;
      for (int k = tid; k < F; k += kUtt512Threads) {
        double R[5], w[4];
        bin_cov_sums_utt<N>(A, b, k, nch, R);
        const double* d = A.steer + 4 * k;
        mvdr_weights_d(R, k, N, A, d[0], d[1], d[2], d[3], w, nullptr);
        cf al, be;
        coef_from_w(w[0], w[1], w[2], w[3], al, be, nullptr);
        ct[k] = make_float4(al.x, al.y, be.x, be.y);
      }
    } else {
      const float4* coef = reinterpret_cast<const float4*>(A.coef) + (long long)b * F;
      for (int k = tid; k < F; k += kUtt512Threads) ct[k] = coef[k];
    }
    __syncthreads();
    AVZ_STAMP(15);
    cf alpha, beta, alpha_n{0, 0}, beta_n{0, 0};
    {
      const float4 w = ct[tid & 255];
      alpha = cf{w.x, w.y};
      beta = cf{w.z, w.w};
      if (nyq_wave) {
        const float4 wn = ct[N / 2];
        alpha_n = cf{wn.x, wn.y};
        beta_n = cf{wn.z, wn.w};
      }
    }
    float4 carry = make_float4(0.f, 0.f, 0.f, 0.f);
    float peak = 0.0f;
    float* outb = A.out + (long long)b * A.out_stride;
    for (int step = 0; step < nstep; ++step) {
      const int f0 = step * FB;
      // lane-derived offsets recomputed per step (hoisted out of the loop they are held in
      // VGPRs through the FFTs and spill)
      int tq = tid, ln = lane;
      opaque_i(tq);
      opaque_i(ln);
      const int kb = tq & 255, kp = (N - kb) & (N - 1), m0 = 4 * ln;
#ifdef AVZ_STAMPS
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      AVZ_STAMP(13);
#endif
      const uint32_t* MW = A.mwords + ((long long)b * A.nchunk + step) * F;
      const uint32_t bits = (PF == PF_IBM_TARGET) ? MW[kb] : 0u;
      const uint32_t bits_n = (PF == PF_IBM_TARGET && nyq_wave) ? MW[N / 2] : 0u;
      window_fft<N, true>(v, wc, fft, slot_ptr<N>(lds, my_slot), lm);
      window_fft<N, true>(vq, wc, fft, slot_ptr<N>(lds, my_slot + RSTRIDE), lm);
      AVZ_STAMP(4);
      lds_barrier();
      AVZ_STAMP(8);
      auto gain = [&](uint32_t bb, int i, int t) -> float {  // i: frame bit in the chunk
        if (t >= T) return 0.0f;
        if constexpr (PF == PF_IBM_TARGET) return ((bb >> i) & 1u) ? 0.0f : 1.0f;
        return 1.0f;
      };
      // ---- apply w^H y + post-filter; frames (2p, 2p + 1) packed as Sa + i Sb into slot 2p
      {
        cf za[PPT], zap[PPT], zb[PPT], zbp[PPT];
#pragma unroll
        for (int q = 0; q < PPT; ++q) {
          const cf* Za = slot_ptr<N>(lds, 2 * (p0 + q));
          const cf* Zb = slot_ptr<N>(lds, 2 * (p0 + q) + 1);
          za[q] = lds_read(Za + kb);
          zap[q] = lds_read(Za + kp);
          zb[q] = lds_read(Zb + kb);
          zbp[q] = lds_read(Zb + kp);
        }
#pragma unroll
        for (int q = 0; q < PPT; ++q) {
          const int p = p0 + q, ta = f0 + 2 * p;
          cf* Za = slot_ptr<N>(lds, 2 * p);
          const cf sa = apply_bin(alpha, beta, za[q], zap[q], gain(bits, 2 * p, ta));
          const cf sb = apply_bin(alpha, beta, zb[q], zbp[q], gain(bits, 2 * p + 1, ta + 1));
          Za[kp] = {sa.x + sb.y, sb.x - sa.y};  // conj(Sa) + i conj(Sb) at N - k
          Za[kb] = (kb == 0) ? cf{sa.x, sb.x} : cf{sa.x - sb.y, sa.y + sb.x};
        }
      }
      if (nyq_wave && lane < NPAIR) {  // Nyquist bin: frame pair `lane`
        const int ta = f0 + 2 * lane;
        if (ta < T) {
          cf* Za = slot_ptr<N>(lds, 2 * lane);
          const cf* Zb = slot_ptr<N>(lds, 2 * lane + 1);
          const float ga = gain(bits_n, 2 * lane, ta), gb = gain(bits_n, 2 * lane + 1, ta + 1);
          const cf za = Za[N / 2], zb = Zb[N / 2];
          Za[N / 2] = {apply_bin(alpha_n, beta_n, za, za, ga).x,
                       apply_bin(alpha_n, beta_n, zb, zb, gb).x};
        }
      }
      AVZ_STAMP(5);
      lds_barrier();
      AVZ_STAMP(10);
      // ---- inverse of pair p = my_slot (every lane group): windowed contributions of
      // frames 2p (real part) and 2p + 1 (imaginary part) into slot 2p + 1
      {
        const int p = my_slot;
        cf* Zi = slot_ptr<N>(lds, 2 * p);
        cf u[PPL];
        static_for<0, PPL>([&](auto r) { u[r] = c_conj(Zi[lm.in0 + C::IN_STRIDE * r]); });
        float* Cp = reinterpret_cast<float*>(slot_ptr<N>(lds, 2 * p + 1));
        fft.forward_emit(u, Zi, [&](auto k, cf x) {
          constexpr float ck = W32::c[k], sk = -W32::s[k];  // cos, sin of 2 pi k / 32
          const float w = fmaf(wc.ss, sk, fmaf(-wc.sc, ck, wc.s0));
          const int n = lm.out0 + C::OUT_STRIDE * k;
          Cp[n] = x.x * w;
          Cp[N + n] = -x.y * w;
        });
      }
      AVZ_STAMP(7);
      // the next step's (or utterance's) loads fly through the overlap-add (issued before
      // the apply they held 64 more VGPRs through it and spilled 80-96 B; after the apply,
      // through the inverse, 0.5-0.8 us slower, profiles/r04/ab_synth_utt512.txt)
      if (step + 1 < nstep) {
        load_step(r0, r1, f0 + FB);
      } else {
        load_step(n0, n1, 0);  // empty descriptors when this is the block's last utterance
      }
      lds_barrier();
      AVZ_STAMP(9);
      // ---- overlap-add: segment j = f0 - 1 + s = frame s-1 (2nd half) + frame s (1st half)
      auto cframe = [&](int f) -> const float* {
        return reinterpret_cast<const float*>(slot_ptr<N>(lds, 2 * (f >> 1) + 1)) + (f & 1) * N;
      };
      auto ola = [&]() {
#pragma unroll
        for (int si = 0; si < SPT; ++si) {
          const int s = sgrp + si * NSG;
          const int j = f0 - 1 + s;
          if (j >= 0 && j <= T - 2) {
            const float4 vb = *reinterpret_cast<const float4*>(cframe(s) + m0);
            const float4 vp = *reinterpret_cast<const float4*>(cframe(s == 0 ? 0 : s - 1) + H + m0);
            const float4 va = (s != 0) ? vp : carry;
            float4 o;
            o.x = (va.x + vb.x) * inv[0];
            o.y = (va.y + vb.y) * inv[1];
            o.z = (va.z + vb.z) * inv[2];
            o.w = (va.w + vb.w) * inv[3];
            *reinterpret_cast<float4*>(outb + (long long)j * H + m0) = o;
            peak = fmaxf(peak, fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(o.w))));
          }
        }
      };
      if (rs_out != nullptr && rs_done < rs_n4) {
        const int lo = rs_done, hi = min(rs_n4, rs_done + RS_U * kUtt512Threads);
        rescale_slice(std::integral_constant<int, RS_U>{}, lo, hi, ola);
        rs_done = hi;
      } else {
        ola();
      }
      if (sgrp == 0) carry = *reinterpret_cast<const float4*>(cframe(FB - 1) + H + m0);
      lds_barrier();
      AVZ_STAMP(11);
    }
    // ---- utterance peak; its rescale (own output, drained, L1-bypassing loads)
    for (int o = 32; o > 0; o >>= 1) peak = fmaxf(peak, __shfl_xor(peak, o, 64));
    if (lane == 0) red[wave] = peak;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    float pk = red[0];
#pragma unroll
    for (int w = 1; w < G::NWAVE; ++w) pk = fmaxf(pk, red[w]);
    if (tid == 0 && A.peak) A.peak[b] = pk;
    if (A.normalize == NORM_PEAK) {
      if (rs_out != nullptr) rescale_rest(std::integral_constant<int, 2 * RS_U>{});
      rs_out = outb;
      rs_scale = 1.0f / (pk + A.norm_eps);
      rs_n4 = (T - 1) * H / 4;
      rs_done = 0;
    }
    __syncthreads();  // red[] and the coefficient table of the next utterance
    AVZ_STAMP(14);
    b = nb;
  }
  if (rs_out != nullptr) rescale_rest(std::integral_constant<int, RS_BULK>{});
  AVZ_STAMP(14);
}

// ================================ finalize ================================
// Finalize blocks handle FCH consecutive chunks (N = 512: two, so a block rescales the same
// 64 KB as N = 1024's one chunk instead of twice as many blocks moving 31 KB each).
template <int N>
constexpr int kFinChunks = N >= 1024 ? 1 : 1024 / N;

// One finalize item: chunks FCH q .. FCH q + FCH - 1 of utterance b, the standalone
// finalize kernel's block (red: NWAVE floats of LDS).
template <int N>
__device__ __forceinline__ void finalize_item(const ChainArgs& A, int q, int b, float* red) {
  constexpr int NT = kCThreads, H = N / 2, NWAVE = NT / 64, FCH = kFinChunks<N>;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int c0 = FCH * q;
  const int L = utt_len(A, b);
  if (L < N) {
    if (c0 == 0 && tid == 0 && A.peak) A.peak[b] = __builtin_nanf("");
    return;
  }
  const int T = (L + H - 1) / H + 1;
  const int nch = (T + kChunk - 1) / kChunk;
  if (c0 >= nch) return;
  const int cend = min(c0 + FCH, nch);  // chunks c0 .. cend - 1
  const float* heads = A.heads + (long long)b * A.nchunk * H;
  const float* tails = A.tails + (long long)b * A.nchunk * H;
  // boundary segment 32 cc - 1 = tail(cc - 1) + head(cc), cc = 1 .. nch - 1
  auto boundary = [&](int cc, int m) -> float {
    return (tails[(long long)(cc - 1) * H + m] + heads[(long long)cc * H + m]) * inv_wsum<N>(m);
  };
  float* outb = A.out + (long long)b * A.out_stride;
  if (A.normalize != NORM_PEAK) {
    // un-normalised output (the batch driver's deferred normalisation): each block writes
    // its chunks' seams and folds their max (chunk 0: the interiors' max) into peak[b],
    // zeroed by the analysis kernel, with an atomicMax on the float's bits (non-negative
    // floats order as unsigned ints) — no redundant reads of the other seams
    float pm = 0.0f;
    for (int c = max(c0, 1); c < cend; ++c) {
      const long long j = (long long)kChunk * c - 1;
      for (int m = tid; m < H; m += NT) {
        const float x = boundary(c, m);
        outb[j * H + m] = x;
        pm = fmaxf(pm, fabsf(x));
      }
    }
    for (int o = 32; o > 0; o >>= 1) pm = fmaxf(pm, __shfl_xor(pm, o, 64));
    if (lane == 0) red[wave] = pm;
    __syncthreads();
    if (tid == 0 && A.peak) {
      float qm = (c0 == 0) ? __uint_as_float(A.peak_u[b]) : 0.0f;
#pragma unroll
      for (int w = 0; w < NWAVE; ++w) qm = fmaxf(qm, red[w]);
      atomicMax(reinterpret_cast<unsigned int*>(A.peak + b), __float_as_uint(qm));
    }
    return;
  }
  // The chunks' interior segments 32c .. 32c+30 are read into registers first: their loads
  // do not depend on the utterance peak, so they stream while the seam maxima below are
  // fetched (all blocks are resident at once; reading them after the peak left every
  // block waiting on its seam loads before any bulk traffic started).
  constexpr int U = ((kChunk - 1) * H / 4 + NT - 1) / NT;
  float4 xin[FCH][U];
#pragma unroll
  for (int g = 0; g < FCH; ++g) {
    const int c = c0 + g;
    const int j0 = kChunk * c, j1 = min(kChunk * c + kChunk - 1, T - 1);
    const float4* o4 = reinterpret_cast<const float4*>(outb + (long long)j0 * H);
    const int n4 = c < cend ? (j1 - j0) * H / 4 : 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = tid + u * NT;
      if (i < n4) xin[g][u] = o4[i];
    }
  }
  float pk = 0.0f;
#pragma unroll 4
  for (int idx = tid; idx < (nch - 1) * H; idx += NT)
    pk = fmaxf(pk, fabsf(boundary(idx / H + 1, idx % H)));
  for (int o = 32; o > 0; o >>= 1) pk = fmaxf(pk, __shfl_xor(pk, o, 64));
  if (lane == 0) red[wave] = pk;
  __syncthreads();
  pk = __uint_as_float(A.peak_u[b]);
#pragma unroll
  for (int w = 0; w < NWAVE; ++w) pk = fmaxf(pk, red[w]);
  if (c0 == 0 && tid == 0 && A.peak) A.peak[b] = pk;
  const float scale = 1.0f / (pk + A.norm_eps);
  for (int c = max(c0, 1); c < cend; ++c) {
    const long long j = (long long)kChunk * c - 1;
    for (int m = tid; m < H; m += NT) outb[j * H + m] = boundary(c, m) * scale;
  }
#pragma unroll
  for (int g = 0; g < FCH; ++g) {
    const int c = c0 + g;
    const int j0 = kChunk * c, j1 = min(kChunk * c + kChunk - 1, T - 1);
    float4* o4 = reinterpret_cast<float4*>(outb + (long long)j0 * H);
    const int n4 = c < cend ? (j1 - j0) * H / 4 : 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = tid + u * NT;
      if (i < n4) {
        float4 x = xin[g][u];
        x.x *= scale; x.y *= scale; x.z *= scale; x.w *= scale;
        o4[i] = x;
      }
    }
  }
}

template <int N>
__global__ void __launch_bounds__(kCThreads) avz_finalize_kernel(ChainArgs A) {
  __shared__ float red[kCThreads / 64];
  finalize_item<N>(A, blockIdx.x, blockIdx.y, red);
}

// Finalize of the per-utterance synthesis kernel's piece utterances b = s_whole + blockIdx.y
// (peak normalisation): the seam segments between its pieces (piece p - 1's last half-frame
// + piece p's first, x 1 / sum w^2), the utterance peak (the pieces' interior maxima in
// peak_u[b] and the seams), peak[b], and the in-place rescale of segments [0, T - 2], block x
// taking kFinPieceU float4 groups per thread of them (every block reduces the few seams
// itself: no cross-block hand-off).
constexpr int kFinPieceU = 4;
constexpr int kMaxPieces = 32;  // pieces per utterance (synth_split; avz_capi.cpp seam_slots)
template <int N>
__global__ void __launch_bounds__(kCThreads) avz_finalize_pieces_kernel(ChainArgs A) {
  constexpr int H = N / 2, NWAVE = kCThreads / 64, FBS = UttGeo::FB;
  __shared__ float red[NWAVE];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int b = A.s_whole + blockIdx.y;
  const int L = utt_len(A, b);
  if (L < N) {
    if (blockIdx.x == 0 && tid == 0 && A.peak) A.peak[b] = __builtin_nanf("");
    return;
  }
  const int T = (L + H - 1) / H + 1;
  const int seg = FBS * A.s_steps;               // frames per piece
  const int n4 = (T - 1) * H / 4;                // float4 groups of segments 0 .. T - 2
  const int g0 = blockIdx.x * kFinPieceU * kCThreads;
  if (g0 >= n4) return;
  const long long slot0 = (long long)(b - A.s_whole) * A.s_pieces;
  // seam segment j = p seg - 1 (p >= 1, j <= T - 2): tail of piece p - 1 + head of piece p
  auto seam = [&](int p, int m) -> float {
    return (A.ptails[(slot0 + p - 1) * H + m] + A.pheads[(slot0 + p) * H + m]) * inv_wsum<N>(m);
  };
  const int n_seam = (T - 2 + 1) / seg;          // p = 1 .. n_seam
  const uint32_t pk_int = A.peak_u[b];  // the pieces' interior maxima (loaded with the rest)
  float4 x[kFinPieceU];
  float* outb = A.out + (long long)b * A.out_stride;
  const float4* o4 = reinterpret_cast<const float4*>(outb);
#pragma unroll
  for (int u = 0; u < kFinPieceU; ++u) {
    const int i = g0 + u * kCThreads + tid;
    if (i < n4) x[u] = o4[i];                    // interior values stream while the seams reduce
  }
  // the seams' max: up to 7 seams x H values with all of a thread's loads in flight (more
  // registers for the 31 seams of 32 pieces ran 10.5 -> 17 us at B = 257: 7 seams)
  constexpr int SU = 7 * H / kCThreads;
  float sv[SU];
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    const int idx = tid + u * kCThreads;
    sv[u] = idx < n_seam * H ? seam(idx / H + 1, idx % H) : 0.0f;
  }
  float pk = 0.0f;
#pragma unroll
  for (int u = 0; u < SU; ++u) pk = fmaxf(pk, fabsf(sv[u]));
  for (int idx = tid + SU * kCThreads; idx < n_seam * H; idx += kCThreads)  // more (not split
    pk = fmaxf(pk, fabsf(seam(idx / H + 1, idx % H)));                      // so finely)
  for (int o = 32; o > 0; o >>= 1) pk = fmaxf(pk, __shfl_xor(pk, o, 64));
  if (lane == 0) red[wave] = pk;
  __syncthreads();
  pk = __uint_as_float(pk_int);
#pragma unroll
  for (int w = 0; w < NWAVE; ++w) pk = fmaxf(pk, red[w]);
  if (blockIdx.x == 0 && tid == 0 && A.peak) A.peak[b] = pk;
  const float scale = 1.0f / (pk + A.norm_eps);
  float4* w4 = reinterpret_cast<float4*>(outb);
#pragma unroll
  for (int u = 0; u < kFinPieceU; ++u) {
    const int i = g0 + u * kCThreads + tid;
    if (i >= n4) continue;
    const int j = 4 * i / H, m = 4 * i % H;
    float4 y = x[u];
    if ((j + 1) % seg == 0) {                    // a seam (j = p seg - 1 <= T - 2)
      const int p = (j + 1) / seg;
      y = make_float4(seam(p, m), seam(p, m + 1), seam(p, m + 2), seam(p, m + 3));
    }
    y.x *= scale; y.y *= scale; y.z *= scale; y.w *= scale;
    w4[i] = y;
  }
}

// Grid x of the finalize kernel: FCH-chunk groups of the longest utterance.
template <int N>
static inline int fin_groups(int nch) { return (nch + kFinChunks<N> - 1) / kFinChunks<N>; }

}  // namespace avz
