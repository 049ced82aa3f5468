// avz_synth_wave.hpp — EXPERIMENT, not built (round 3): a wave-autonomous synthesis kernel
// for N = 1024. It passed the full GPU suite (111/111) when wired in as
// avz_synthesis_kernel's replacement, but measured 83-85 us against the block-synchronous
// kernel's 73-74 us at configs[1] (profiles/r03/synth_wave_ab.txt): VALU instructions +16 %
// (DPP partner fetches, selects, swaps), LDS-array cycles -12 %, and SQ_WAIT_ANY unchanged --
// the barrier waits it removed came back as load / LDS latency waits at two waves per SIMD.
// Kept as a record of the design (residue-permuted second FFT stage so that bin pairs
// (k, N - k) meet on DPP row_mirror partners; register overlap-add).
// Was included by avz_chunked.hip (uses its utt_len / window_apply helpers).
//
// Same result as avz_synthesis_kernel<1024, PF> (rt_av_zoom/core/oracle_debug.py:80-93:
// S = w^H Y, post-filter, scipy istft), restructured so that the four waves of a chunk
// never wait for each other inside the chunk:
//
//   * a 512-thread block (8 waves, one per CU) takes two consecutive chunks of one
//     utterance; wave w owns the 8 consecutive frames 32 c + 8 (w & 3) ... of chunk
//     c = 2 c2 + (w >> 2) and runs them as two macro-steps of four frames a, b, c, d:
//       forward FFT (a, b) -> apply -> packed P_ab = Q_a + i Q_b   (registers)
//       forward FFT (c, d) -> apply -> packed P_cd                 (registers)
//       inverse FFT (P_ab, P_cd) as one Fft1024x2-shaped transform -> 4 windowed frames
//       -> overlap-add in registers (one v_permlane32_swap per sample pair) -> out.
//   * The bin pairs (k, N - k) the apply needs meet in neighbouring lanes, not in LDS:
//     the forward FFT's second stage reads transpose row rho(l) instead of row l, so lane
//     l ends up holding the residue class rho(l) of the bins, and rho puts the classes
//     r and 32 - r on mirror lanes (l, 15 - l) of each 16-lane row. The partner of
//     register k is then register 31 - k of the mirror lane: one DPP row_mirror move per
//     float (lanes 0 and 15 hold the self-paired classes 0 and 16 and use their own
//     registers). No spectrum store, no bin-phase LDS round trip, no block barrier.
//   * Only the transposes use LDS (stride 33, unpaired ds_read_b64: conflict-free for any
//     row permutation), plus the block's twiddle table, the utterance's apply
//     coefficients (one float4 per bin, stored in a lane-group-permuted order so the
//     b128 reads are conflict-free) and six half-frame seam slots.
//   * Seams between waves of a chunk: a wave's first-frame head goes to an LDS slot and
//     the previous wave adds its last tail after the one block barrier per item; chunk
//     seams keep the heads / tails + finalize protocol of the block-synchronous kernel.
#pragma once

#ifndef AVZ_SW_PREF_X
#define AVZ_SW_PREF_X 1
#endif
#ifndef AVZ_SW_PREF_Y
#define AVZ_SW_PREF_Y 1
#endif
namespace avz {
namespace sw {

constexpr int N = 1024, H = 512, F = 513;
constexpr int NT = 512, NW = NT / 64;           // 8 waves
constexpr int FPWV = 8;                         // frames per wave per chunk
constexpr int TSW = 33;                         // transpose row stride (complex elements)
constexpr int GROUP_CF = 32 * TSW;              // one lane group's transpose area
constexpr int WAVE_BYTES = 2 * GROUP_CF * 8;    // 16896
constexpr int TW_OFF = NW * WAVE_BYTES;         // 135168
constexpr int TW_BYTES = 31 * 32 * 8;           // W1024^{q k1}, rows k1 = 1..31
constexpr int COEF_OFF = TW_OFF + TW_BYTES;
constexpr int COEF_BYTES = F * 16;
constexpr int SEAM_OFF = COEF_OFF + COEF_BYTES;
constexpr int NSEAM = 6;                        // waves with (w & 3) >= 1
constexpr int SEAM_BYTES = NSEAM * H * 4;
constexpr int LDS_BYTES = SEAM_OFF + SEAM_BYTES;
static_assert(LDS_BYTES <= 160 * 1024, "one block per CU");

// Residue class held by lane l (0..31) after the forward FFT: rows 0..15 -> {0..7, 25..31,
// 16}, rows 16..31 -> {8..15, 17..24}; classes r and 32 - r sit on mirror lanes l, 15 - l
// of the same 16-lane row ({0, 16} on lanes 0 and 15).
__device__ __forceinline__ int rho(int l) {
  if (l < 8) return l;
  if (l < 15) return l + 17;
  if (l == 15) return 16;
  if (l < 24) return l - 8;
  return l - 7;
}
__device__ __forceinline__ int rho_inv(int r) {
  if (r < 8) return r;
  if (r < 16) return r + 8;
  if (r == 16) return 15;
  if (r < 25) return r + 7;
  return r - 17;
}
// Position of lane l inside its ds_read_b128 lane group ({0-3,12-15,20-27} -> 0..15,
// {4-11,16-19,28-31} -> 16..31): the coefficient of bin m is stored at
// (m & ~31) | perm_l(rho_inv(m & 31)), so the 16 lanes of a group hit 16 distinct bank quads.
__device__ __forceinline__ int perm_l(int l) {
  if (l < 4) return l;
  if (l < 12) return l + 12;
  if (l < 16) return l - 8;
  if (l < 20) return l + 8;
  if (l < 28) return l - 12;
  return l;
}
__device__ __forceinline__ int coef_slot(int m) {
  return m >= 512 ? 512 : ((m & ~31) | perm_l(rho_inv(m & 31)));
}

// Empty asm statements that pin the program order of the code around them (see sw_apply).
__device__ __forceinline__ void pin(cf& x) { asm volatile("" : "+v"(x.x), "+v"(x.y)); }
__device__ __forceinline__ void pin_mem(cf& x, cf& y) {
  asm volatile("" : "+v"(x.x), "+v"(x.y), "+v"(y.x), "+v"(y.y)::"memory");
}
__device__ __forceinline__ float mirror16(float x) {  // DPP row_mirror: lane i <- lane 15 - i
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x140, 0xF, 0xF, false));
}
__device__ __forceinline__ void swap32(float& a, float& b) {  // a.hi <-> b.lo
  const auto rr = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  a = __uint_as_float(rr[0]);
  b = __uint_as_float(rr[1]);
}

// Stage 1 of the 32 x 32 FFT: DFT32 over the registers, twiddle W1024^{q k1} (q = the
// lane's input residue) read from the block table in groups of 8 issued ahead.
__device__ __forceinline__ void stage1(cf (&v)[32], const cf* tw, int q) {
  cf t[8];
  static_for<0, 8>([&](auto j) { t[j] = tw[j * 32 + q]; });
  __builtin_amdgcn_sched_barrier(0);
  dft32(v);
  static_for<0, 4>([&](auto gg) {
    static_for<0, 8>([&](auto j) {
      constexpr int k = 8 * gg + j + 1;
      if constexpr (k < 32) v[k] = c_mul(v[k], t[j]);
    });
    if constexpr (gg < 3) {
      static_for<0, 8>([&](auto j) {
        constexpr int k = 8 * (gg + 1) + j + 1;
        if constexpr (k < 32) t[j] = tw[(k - 1) * 32 + q];
      });
      __builtin_amdgcn_sched_barrier(0);
    }
  });
}
// Transpose through this lane group's area: column `col` in, row `row` out.
__device__ __forceinline__ void transpose(cf (&v)[32], cf* scr, int col, int row) {
  static_for<0, 32>([&](auto k) { scr[k * TSW + col] = v[k]; });
  __builtin_amdgcn_wave_barrier();
  const cf* rp = scr + row * TSW;
  static_for<0, 32>([&](auto j) { v[j] = lds_read(rp + j); });
  __builtin_amdgcn_wave_barrier();
}

// Forward FFT input residues: lane l loads the sample pairs (2l + 64 r', 2l + 1 + 64 r') with
// one 8-byte load per channel and r'; one v_permlane16_swap per register pair then leaves
// lane l < 16 holding residue class q = 2 l and lane l + 16 holding q = 2 l + 1 (all 32 r).
// The stage-1 outputs are stored in the transpose at column l (the lane), so the stage-2
// reader takes input residue j from column sigma(j) = j / 2 (even j), 16 + j / 2 (odd j).
__device__ __forceinline__ int q_of(int l) { return l < 16 ? 2 * l : 2 * (l - 16) + 1; }
template <int J>
struct Sigma {
  static constexpr int v = (J & 1) ? 16 + J / 2 : J / 2;
};
__device__ __forceinline__ void transpose_fwd(cf (&v)[32], cf* scr, int col, int row) {
  static_for<0, 32>([&](auto k) { scr[k * TSW + col] = v[k]; });
  __builtin_amdgcn_wave_barrier();
  const cf* rp = scr + row * TSW;
  static_for<0, 32>([&](auto j) { v[j] = lds_read(rp + Sigma<j>::v); });
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ void swap16(float& a, float& b) {  // rows 1 / 0 of a / b exchanged
  const auto rr = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  a = __uint_as_float(rr[0]);
  b = __uint_as_float(rr[1]);
}
__device__ __forceinline__ float quad_swap1(float x) {  // DPP quad_perm [1,0,3,2]: lane i <- i ^ 1
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xF, 0xF, false));
}

struct Lane {
  int l, g, r, pl;       // natural lane, lane group (frame of the pair), residue, coef slot
  int q;                 // forward input residue (q_of(l))
  bool sp0, sp15;        // self-paired residue classes 0 / 16
};
// Window terms from the twiddle table's first row, tw[q] = W1024^q = (cos, -sin)(2 pi q / N),
// read where they are used instead of being held in registers through the kernel:
// analysis a0 - ac cos + as sin (window_apply), synthesis 0.25 - sc cos + ss sin.
__device__ __forceinline__ void win_terms(const cf* tw, int q, float scale, float& c, float& s) {
  const cf w = tw[q];
  c = w.x * scale;
  s = -w.y * scale;
}

// Post-filter gains of the lane's 16 bins (+ Nyquist on lane 0) for frame t of chunk c.
template <int PF>
struct Gains {
  uint32_t pk[4];        // IBM: 8 frame bits of the wave per bin, 4 bins per word
  uint32_t nyq;          // IBM: the Nyquist bin's 8 bits (lane 0)
  float gv[16], gn;      // IRM / external: gains of the current frame
};

}  // namespace sw

template <int PF>
__device__ __forceinline__ void sw_load_gains(const ChainArgs& A, sw::Gains<PF>& G, const sw::Lane& ln,
                                              int b, int c, int t, int T) {
  using namespace sw;
  if constexpr (PF == PF_IRM) {
    const float* ip = A.pf_gain + (((long long)b * A.nchunk + c) * 32 + (t - 32 * c)) * F;
    const bool ok = t < T;
    static_for<0, 16>([&](auto k) { G.gv[k] = ok ? ip[ln.r + 32 * k] : 0.0f; });
    G.gn = (ok && ln.sp0) ? ip[N / 2] : 0.0f;
  } else if constexpr (PF == PF_EXT_FLOOR || PF == PF_EXT_MUL) {
    const float* mp = A.ext_mask + (long long)b * A.mask_sb + (long long)t * A.mask_st;
    const bool ok = t < T;
    static_for<0, 16>([&](auto k) {
      const float M = ok ? mp[(long long)(ln.r + 32 * k) * A.mask_sf] : 0.0f;
      G.gv[k] = PF == PF_EXT_FLOOR ? (ok ? fmaxf(M, A.pf_floor) : 0.0f) : M;
    });
    const float Mn = (ok && ln.sp0) ? mp[(long long)(N / 2) * A.mask_sf] : 0.0f;
    G.gn = PF == PF_EXT_FLOOR ? (ok ? fmaxf(Mn, A.pf_floor) : 0.0f) : Mn;
  }
}

// Forward FFT of the pair's frames (lane group g <-> frame f + g): window, stage 1 with
// the natural residue l, transpose reading row rho(l), stage 2 -> v[k] = Z[rho(l) + 32 k].
__device__ __forceinline__ void sw_forward(cf (&v)[32], const sw::Lane& ln, const cf* tw, cf* scr) {
  // opaque: recompute the lane's window weights here rather than hoisting 32 of them out of
  // the loops into registers (as window_fft)
  float a0 = 1.0f / sw::N, ac, as;
  sw::win_terms(tw, ln.q, 1.0f / sw::N, ac, as);
  opaque(a0);
  opaque(ac);
  opaque(as);
  // the pair loads' regroup: v[2 r'] / v[2 r' + 1] hold (2l + 64 r', 2l + 1 + 64 r') -> residue q
  static_for<0, 16>([&](auto r) {
    sw::swap16(v[2 * r].x, v[2 * r + 1].x);
    sw::swap16(v[2 * r].y, v[2 * r + 1].y);
  });
  window_apply<1024>(v, a0, ac, as);
  sw::stage1(v, tw, ln.q);
  sw::transpose_fwd(v, scr, ln.l, ln.r);
  dft32(v);
}

// Apply w^H y and the post-filter on the spectrum of the lane group's frame (fi = the
// frame's index among the wave's 8), then pack the pair: P[k] (k < 16) = P_pair[r + 32 (k +
// 16 g)] with P_pair = Q_a + i Q_b, Q = S on bins <= N/2 and conj(S[N - m]) above.
template <int PF>
__device__ __forceinline__ void sw_apply(cf (&v)[32], cf (&P)[16], const sw::Lane& ln,
                                         const float4* coefL, const sw::Gains<PF>& G, int fi) {
  using namespace sw;
  auto gain_zero = [&](int k) -> bool {  // IBM: the (bin, frame) is noise
    return ((G.pk[k >> 2] >> (8 * (k & 3) + fi)) & 1u) != 0u;
  };
  // The coefficients are the same for every pair of the item: an opaque slot index keeps
  // the compiler from hoisting all 16 float4 reads out of the loops (64 VGPRs held).
  int pl = ln.pl;
  asm volatile("" : "+v"(pl));
  const float4* cq = coefL + pl;
  // In batches of 4 bins. The empty asm statements pin the order: a batch's coefficient
  // reads and partner moves may not be hoisted above the previous batch (memory clobber,
  // inputs re-defined) and its results must be computed before the next batch (outputs
  // defined) -- left alone, the scheduler issues all 17 coefficient reads and 32 partner
  // moves first and computes every S at its use, and the kernel spills.
  static_for<0, 4>([&](auto bq) {
    static_for<0, 4>([&](auto i) {
      constexpr int k = 4 * bq + i;
      pin_mem(v[31 - k], v[k]);
    });
    static_for<0, 4>([&](auto i) {
      constexpr int k = 4 * bq + i;
      const cf zo = v[31 - k];
      cf zp = {mirror16(zo.x), mirror16(zo.y)};
      if (ln.sp15) zp = zo;
      if (ln.sp0) zp = v[(32 - k) & 31];
      const float4 cw = cq[32 * k];  // alpha (x, y), beta (z, w)
      const cf z = v[k];
      cf s = {fmaf(cw.x, z.x, fmaf(-cw.y, z.y, fmaf(cw.z, zp.x, cw.w * zp.y))),
              fmaf(cw.x, z.y, fmaf(cw.y, z.x, fmaf(cw.w, zp.x, -cw.z * zp.y)))};
      if constexpr (PF == PF_IBM_TARGET) {
        if (gain_zero(k)) s = cf{0.f, 0.f};
      } else if constexpr (PF != PF_NONE) {
        s = c_scale(s, G.gv[k]);
      }
      v[k] = s;
    });
    static_for<0, 4>([&](auto i) {
      constexpr int k = 4 * bq + i;
      pin(v[k]);
    });
  });
  if (ln.sp0) {  // DC (register 0) and Nyquist (register 16): real parts only, as irfft
    v[0].y = 0.0f;
    const float4 cw = coefL[N / 2];
    const cf z = v[16];
    float sx = fmaf(cw.x, z.x, fmaf(-cw.y, z.y, fmaf(cw.z, z.x, cw.w * z.y)));
    if constexpr (PF == PF_IBM_TARGET) {
      if ((G.nyq >> fi) & 1u) sx = 0.0f;
    } else if constexpr (PF != PF_NONE) {
      sx *= G.gn;
    }
    v[16] = cf{sx, 0.0f};
  }
  // Q on the upper registers, swap to the pair layout and pack, 4 registers at a time
  static_for<0, 4>([&](auto bq) {
    static_for<0, 4>([&](auto i) {
      constexpr int k = 16 + 4 * bq + i;
      pin(v[31 - k]);
    });
    static_for<0, 4>([&](auto i) {
      constexpr int k = 16 + 4 * bq + i;
      const cf so = v[31 - k];
      cf q = {mirror16(so.x), mirror16(so.y)};
      if (ln.sp15) q = so;
      if (ln.sp0) q = v[(32 - k) & 31];
      v[k] = cf{q.x, -q.y};
    });
    static_for<0, 4>([&](auto i) {
      constexpr int k = 16 + 4 * bq + i;
      pin(v[k]);
    });
  });
  static_for<0, 16>([&](auto k) {
    swap32(v[k].x, v[k + 16].x);
    swap32(v[k].y, v[k + 16].y);
    P[k] = cf{v[k].x - v[k + 16].y, v[k].y + v[k + 16].x};
  });
}

// Samples (2l + 64 r', 2l + 1 + 64 r') of both channels -> v[2 r'], v[2 r' + 1] (s0 = the
// frame's first sample + 2 l, even). PAIR: one 8-byte load per channel and r' (8-byte aligned
// rows, even length: the two samples are in or out of range together); else 4-byte loads.
template <bool NONNEG, bool PAIR>
__device__ __forceinline__ void sw_issue_loads(cf (&v)[32], rsrc_t r0, rsrc_t r1, int s0) {
  static_for<0, 16>([&](auto j) {
    const int e = s0 + 64 * j;
    if constexpr (PAIR) {
      const unsigned off = (!NONNEG && e < 0) ? 0xfffffff8u : (unsigned)e * 4u;
      const auto a = __builtin_amdgcn_raw_buffer_load_b64(r0, (int)off, 0, 0);
      const auto b = __builtin_amdgcn_raw_buffer_load_b64(r1, (int)off, 0, 0);
      v[2 * j] = cf{__uint_as_float(a[0]), __uint_as_float(b[0])};
      v[2 * j + 1] = cf{__uint_as_float(a[1]), __uint_as_float(b[1])};
    } else {
      v[2 * j].x = NONNEG ? bload_nn(r0, e) : bload(r0, e);
      v[2 * j].y = NONNEG ? bload_nn(r1, e) : bload(r1, e);
      v[2 * j + 1].x = NONNEG ? bload_nn(r0, e + 1) : bload(r0, e + 1);
      v[2 * j + 1].y = NONNEG ? bload_nn(r1, e + 1) : bload(r1, e + 1);
    }
  });
}

template <int PF>
__device__ __forceinline__ void sw_item(const ChainArgs& A, unsigned char* lds, const sw::Lane& ln,
                                        int c2, int b) {
  using namespace sw;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const cf* tw = reinterpret_cast<const cf*>(lds + TW_OFF);
  cf* scr = reinterpret_cast<cf*>(lds + wave * WAVE_BYTES) + ln.g * GROUP_CF;
  float4* coefL = reinterpret_cast<float4*>(lds + COEF_OFF);
  float* seam = reinterpret_cast<float*>(lds + SEAM_OFF);

  const int L = utt_len(A, b);
  if (L < N) return;  // block-uniform
  const int T = (L + H - 1) / H + 1;
  const int nch = (T + 31) / 32;
  const int c0 = 2 * c2;
  if (c0 >= nch) return;  // block-uniform
  const int c = c0 + (wave >> 2), wc = wave & 3;
  const int fb = 32 * c + FPWV * wc;                                   // wave's first frame
  const int nf = c < nch ? max(0, min(FPWV, T - fb)) : 0;              // wave-uniform
  const int ns = (nf + 3) / 4;                                         // macro-steps

  // the utterance's apply coefficients -> LDS (permuted slots), loaded before anything else
  // so the store waits for them alone (vmcnt counts in issue order)
  {
    const float4* cg = reinterpret_cast<const float4*>(A.coef) + (long long)b * F;
    const float4 cv = cg[tid];
    const float4 cn = cg[N / 2];
    coefL[coef_slot(tid)] = cv;
    if (tid == 0) coefL[N / 2] = cn;
  }
  const float* mixb = A.mix + (long long)b * A.mix_stride;
  const rsrc_t r_m0 = make_rsrc(mixb, L), r_m1 = make_rsrc(mixb + A.ch_stride, L);
  cf X[32], Y[32];
  const bool pair = ((L & 1) == 0) &&
                    (((reinterpret_cast<uintptr_t>(mixb) | reinterpret_cast<uintptr_t>(mixb + A.ch_stride)) & 7) == 0);
  auto loads = [&](cf (&v)[32], int f) {  // frame f + g on lane group g
    const int s0 = (f + ln.g) * H - N / 2 + 2 * ln.l;
    if (pair) {
      if (f >= 1)
        sw_issue_loads<true, true>(v, r_m0, r_m1, s0);
      else
        sw_issue_loads<false, true>(v, r_m0, r_m1, s0);
    } else {
      if (f >= 1)
        sw_issue_loads<true, false>(v, r_m0, r_m1, s0);
      else
        sw_issue_loads<false, false>(v, r_m0, r_m1, s0);
    }
  };
  if (nf > 0) loads(X, fb);

  Gains<PF> G;
  if constexpr (PF == PF_IBM_TARGET) {
    if (nf > 0) {
      const uint32_t* MW = A.mwords + ((long long)b * A.nchunk + c) * F;
      const int sh = 8 * wc;
      static_for<0, 4>([&](auto q) {
        uint32_t w = 0u;
        static_for<0, 4>([&](auto i) {
          w |= ((MW[ln.r + 32 * (4 * q + i)] >> sh) & 0xffu) << (8 * i);
        });
        G.pk[q] = w;
      });
      G.nyq = ln.sp0 ? ((MW[N / 2] >> sh) & 0xffu) : 0u;
    }
  }
  lds_barrier();  // coefficients in LDS (the sample loads stay in flight)

  float* outb = A.out + (long long)b * A.out_stride;
  float carry[16];  // raw windowed second half of the last frame (lane group 1)
#pragma unroll
  for (int k = 0; k < 16; ++k) carry[k] = 0.0f;
  float pk = 0.0f;
  for (int s = 0; s < ns; ++s) {
    const int fa = fb + 4 * s;
    cf Pab[16], Pcd[16];
    // ---- pair (a, b)
    if constexpr (PF != PF_IBM_TARGET && PF != PF_NONE) sw_load_gains<PF>(A, G, ln, b, c, fa + ln.g, T);
    sw_forward(X, ln, tw, scr);
#if AVZ_SW_PREF_Y
    loads(Y, fa + 2);
#endif
    sw_apply<PF>(X, Pab, ln, coefL, G, 4 * s + ln.g);
#if !AVZ_SW_PREF_Y
    loads(Y, fa + 2);
#endif
    // ---- pair (c, d)
    if constexpr (PF != PF_IBM_TARGET && PF != PF_NONE) sw_load_gains<PF>(A, G, ln, b, c, fa + 2 + ln.g, T);
    sw_forward(Y, ln, tw, scr);
    sw_apply<PF>(Y, Pcd, ln, coefL, G, 4 * s + 2 + ln.g);
#if AVZ_SW_PREF_X
    if (s + 1 < ns) loads(X, fa + 4);  // in flight through the inverse and the overlap-add
#endif
    // ---- inverse of (P_ab, P_cd): lane group 0 <- P_ab, group 1 <- P_cd
    cf u[32];
    static_for<0, 16>([&](auto k) {
      swap32(Pab[k].x, Pcd[k].x);
      swap32(Pab[k].y, Pcd[k].y);
      u[k] = c_conj(Pab[k]);
      u[k + 16] = c_conj(Pcd[k]);
    });
    stage1(u, tw, ln.r);
    transpose(u, scr, ln.r, ln.l);
    dft32(u);
    static_for<0, 32>([&](auto k) { pin(u[k]); });  // the transform completes before the OLA
    // u[k] -> x_{2g} = Re, x_{2g+1} = -Im at sample l + 32 k of frames (a, b) / (c, d)
    // ---- overlap-add: group 0 -> segments fa - 1 (a), fa (b); group 1 -> fa + 1 (c), fa + 2 (d)
    const int sA = fa - 1 + 2 * ln.g, sB = fa + 2 * ln.g;
    const bool headA = (s == 0) && ln.g == 0;  // segment fa - 1: the wave's head
    const bool wA = !headA && sA <= T - 2, wB = sB <= T - 2;
    float* head = (wc == 0) ? A.heads + ((long long)b * A.nchunk + c) * H
                            : seam + ((wave >> 2) * 3 + wc - 1) * H;
    float ss, sc;
    win_terms(tw, ln.l, 0.25f, sc, ss);
    opaque(ss);
    opaque(sc);
    // segments in place: u[k].x <- segment A sample l + 32 k, u[k].y <- segment B (k < 16)
    static_for<0, 16>([&](auto k) {
      constexpr float ck = W32::c[k], sk = -W32::s[k];  // cos, sin of 2 pi k / 32
      const float w1 = fmaf(ss, sk, fmaf(-sc, ck, 0.25f));  // 0.5 hann(j) . (scaling)
      const float w2 = 0.5f - w1;                                 // 0.5 hann(j + H)
      const float inv = 0.25f * __builtin_amdgcn_rcpf(fmaf(2.0f * w1, w1, 0.25f - w1));
      const float segB = fmaf(u[k + 16].x, w2, -u[k].y * w1);
      const float send = ln.g ? carry[k] : -u[k + 16].y * w2;
      float lo, hi;
      xhalf<32>(send, lo, hi);
      const float segA = fmaf(u[k].x, w1, ln.g ? lo : hi);
      carry[k] = -u[k + 16].y * w2;
      if (headA) head[ln.l + 32 * k] = segA;  // raw (no window-sum normalisation)
      u[k] = cf{segA * inv, segB * inv};
    });
    // 8-byte stores: lanes 2m / 2m + 1 trade registers k / k + 1 so each holds two
    // consecutive samples (even lane: samples 2m, 2m+1 of row k; odd: of row k + 1)
    const bool odd = ln.l & 1;
    float* pA = outb + (long long)sA * H + (ln.l & ~1) + (odd ? 32 : 0);
    float* pB = outb + (long long)sB * H + (ln.l & ~1) + (odd ? 32 : 0);
    static_for<0, 8>([&](auto kk) {
      constexpr int k = 2 * kk;
      const float a0 = u[k].x, a1 = u[k + 1].x, b0 = u[k].y, b1 = u[k + 1].y;
      const float sa0 = quad_swap1(a0), sa1 = quad_swap1(a1), sb0 = quad_swap1(b0), sb1 = quad_swap1(b1);
      const float2 oa = odd ? make_float2(sa1, a1) : make_float2(a0, sa0);
      const float2 ob = odd ? make_float2(sb1, b1) : make_float2(b0, sb0);
      if (wA) {
        *reinterpret_cast<float2*>(pA + 32 * k) = oa;
        pk = fmaxf(pk, fmaxf(fabsf(oa.x), fabsf(oa.y)));
      }
      if (wB) {
        *reinterpret_cast<float2*>(pB + 32 * k) = ob;
        pk = fmaxf(pk, fmaxf(fabsf(ob.x), fabsf(ob.y)));
      }
    });
#if !AVZ_SW_PREF_X
    if (s + 1 < ns) loads(X, fa + 4);
#endif
  }
  lds_barrier();  // seam slots written
  if (nf == FPWV && ln.g == 1) {
    if (wc < 3) {
      // segment fb + 7: this wave's last tail + the next wave's head (if it has frames)
      const int j0 = fb + FPWV - 1;
      if (j0 <= T - 2) {
        const float* nh = seam + ((wave >> 2) * 3 + wc) * H;
        float ss, sc;
        win_terms(tw, ln.l, 0.25f, sc, ss);
        opaque(ss);
        opaque(sc);
        static_for<0, 16>([&](auto k) {
          constexpr float ck = W32::c[k], sk = -W32::s[k];
          const float w1 = fmaf(ss, sk, fmaf(-sc, ck, 0.25f));
          const float inv = 0.25f * __builtin_amdgcn_rcpf(fmaf(2.0f * w1, w1, 0.25f - w1));
          const int j = ln.l + 32 * k;
          const float o = (carry[k] + nh[j]) * inv;
          outb[(long long)j0 * H + j] = o;
          pk = fmaxf(pk, fabsf(o));
        });
      }
    } else {
      // full chunk: its last frame's tail for finalize
      float* tl = A.tails + ((long long)b * A.nchunk + c) * H;
      static_for<0, 16>([&](auto k) { tl[ln.l + 32 * k] = carry[k]; });
    }
  }
  for (int o = 32; o > 0; o >>= 1) pk = fmaxf(pk, __shfl_xor(pk, o, 64));
  if ((tid & 63) == 0 && nf > 0) atomicMax(A.peak_u + b, __float_as_uint(pk));
  lds_barrier();  // LDS (coefficients, seams) reused by the next item
}

template <int PF>
__global__ void __launch_bounds__(sw::NT, 2) avz_synth_wave_kernel(ChainArgs A) {
  using namespace sw;
  extern __shared__ __align__(16) unsigned char lds[];
  cf* tw = reinterpret_cast<cf*>(lds + TW_OFF);
  for (int i = threadIdx.x; i < 31 * 32; i += NT) {
    const int k1 = (i >> 5) + 1, q = i & 31;
    tw[i] = unit_root((double)(q * k1) / N);
  }
  Lane ln;
  const int lane = threadIdx.x & 63;
  ln.l = lane & 31;
  ln.g = lane >> 5;
  ln.r = rho(ln.l);
  ln.pl = perm_l(ln.l);
  ln.sp0 = ln.l == 0;
  ln.sp15 = ln.l == 15;
  ln.q = q_of(ln.l);
  const int gx = (A.max_frames + 31) / 32;
  const int gx2 = (gx + 1) / 2;
  const int n_items = gx2 * A.batch;
  __syncthreads();  // twiddle table
  for (int it = blockIdx.x; it < n_items; it += gridDim.x) sw_item<PF>(A, lds, ln, it % gx2, it / gx2);
}

}  // namespace avz
