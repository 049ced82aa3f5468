// avz_kernels.hip — hand-written CDNA4 (gfx950) kernels for the mask-driven MVDR chain.
//
// avz_fused_kernel<N, MASK>: one 1024-thread workgroup owns one utterance and runs
//   pass 1  frames -> window -> FFT (packed mic pair / packed ref pair) -> LDS
//           thread-per-bin: separate channels, oracle IBM / IPD / external mask,
//           masked 2x2 covariance partials (fp32 per batch, fp64 running sums)
//   solve   per-bin fp64 closed-form 2x2 Hermitian MVDR weights (+ steering vector)
//   pass 2  frames -> FFT again (recompute beats spilling Y to HBM) -> LDS
//           thread-per-bin: w^H y, post-filter gain, pack two frames into one
//           complex spectrum -> inverse FFT -> windowed overlap-add -> out
//   peak    block max |out|, optional in-place peak normalisation.
// Reference semantics: rt_av_zoom/core/oracle_debug.py:27-97 (IBM path),
// rt_av_zoom/core/masked_mvdr.py:50-132 (IPD path),
// rt_av_zoom/core/full_audio_generating_pipeline/inference.py:88-118 (external mask),
// scipy.signal.stft/istft framing (see oracle/avz_oracle.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "avz_common.hpp"

namespace avz {

template <int N, int MASK, int NT>
__global__ void __launch_bounds__(NT, 1) avz_fused_kernel(FusedArgs A) {
  using C = KCfg<N>;
  using G = Geo<N, NT>;
  constexpr int NWAVE = G::NWAVE;
  constexpr int H = G::H, NB = G::NB, F = G::F, Q = G::Q, NSLOT = G::NSLOT;
  constexpr int FB1 = (MASK == MASK_IBM) ? NSLOT / 2 : NSLOT;  // frames per pass-1 batch
  constexpr int FPT1 = FB1 / Q;                                  // frames per thread, pass 1
  constexpr int FB2 = NSLOT;
  constexpr int FPT2 = FB2 / Q;
  constexpr int PPL = C::PPL;
  static_assert(FPT1 % 4 == 0 && FPT2 % 4 == 0, "mask nibbles hold 4 frames");
  static_assert(FPT2 % 2 == 0 && FPT2 <= 32, "pass-2 frame pairs");

  extern __shared__ __align__(16) unsigned char lds[];
  float* carry = reinterpret_cast<float*>(lds + G::CARRY_OFF);  // [2][H]
  cf* twid = reinterpret_cast<cf*>(lds + G::TW_OFF);
  C::Fft::fill_twiddles(twid, threadIdx.x, NT);

  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably wave-uniform
  const int lane = tid & 63;
  const int L = A.len[b];
  if (L < N) {  // host validates; a bad device length must not fault
    if (tid == 0 && A.peak) A.peak[b] = __builtin_nanf("");
    return;
  }
  const int T = (L + H - 1) / H + 1;  // scipy: ceil(L/H) + 1 frames
  const int NB1 = (T + FB1 - 1) / FB1, NB2 = (T + FB2 - 1) / FB2;
  const int NSTEP = NB1 + NB2;

  // ---------------- per-lane FFT state
  typename C::Fft fft;
  fft.init(lane);
  LaneMap<N> lm;
  lm.init(lane);
  const int my_slot = wave * C::FPW + lm.grp;
  cf* my_spec = slot_ptr<N>(lds, my_slot);

  // analysis window * (1 / sum(win)): win[n] = 0.5 - 0.5 cos(2 pi n / N), n = in0 + IN_STRIDE r
  float wa0, wac, was;
  {
    double s, c;
    sincospi(2.0 * lm.in0 / N, &s, &c);
    const double sc = 2.0 / N;
    wa0 = (float)(0.5 * sc);
    wac = (float)(0.5 * sc * c);
    was = (float)(0.5 * sc * s);
  }
  // synthesis window * sum(win)/N for IFFT output n = out0 + OUT_STRIDE k'
  float ws0, wsc, wss;
  {
    double s, c;
    sincospi(2.0 * lm.out0 / N, &s, &c);
    ws0 = 0.25f;
    wsc = (float)(0.25 * c);
    wss = (float)(0.25 * s);
  }

  // ---------------- buffer descriptors (wave-uniform)
  const float* mixb = A.mix + (long long)b * A.mix_stride;
  const rsrc_t r_m0 = make_rsrc(mixb, L);
  const rsrc_t r_m1 = make_rsrc(mixb + A.ch_stride, L);
  rsrc_t r_t = r_m0, r_i = r_m1;
  if constexpr (MASK == MASK_IBM) {
    r_t = make_rsrc(A.ref_tgt + (long long)b * A.ref_stride, L);
    r_i = make_rsrc(A.ref_int + (long long)b * A.ref_stride, L);
  }

  cf v[PPL];
  AVZ_STAMP_DECL();
  auto issue_loads = [&](int step) {
    bool ref = false;
    int frame;
    if (step < NB1) {
      if constexpr (MASK == MASK_IBM) {
        ref = wave * C::FPW >= FB1;  // uniform: the whole wave transforms references
        frame = step * FB1 + (ref ? my_slot - FB1 : my_slot);
      } else {
        frame = step * FB1 + my_slot;
      }
    } else {
      frame = (step - NB1) * FB2 + my_slot;
    }
    const rsrc_t re = ref ? r_t : r_m0;
    const rsrc_t im = ref ? r_i : r_m1;
    const int s0 = frame * H - N / 2 + lm.in0;
    static_for<0, PPL>([&](auto r) {
      v[r].x = bload(re, s0 + C::IN_STRIDE * r);
      v[r].y = bload(im, s0 + C::IN_STRIDE * r);
    });
  };
  auto window_and_fft = [&]() {
#ifdef AVZ_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    AVZ_STAMP(8);
#endif
    static_for<0, PPL>([&](auto r) {
      constexpr int j = (C::IN_STRIDE * 32 / N) * r;  // 2 pi (IN_STRIDE r)/N = 2 pi j/32
      constexpr float cr = W32::c[j % 32], sr = -W32::s[j % 32];
      const float w = fmaf(was, sr, fmaf(-wac, cr, wa0));
      v[r] = c_scale(v[r], w);
    });
#if defined(AVZ_STAMPS)
    if constexpr (N == 1024) {
      fft.stage1(v, twid);
      AVZ_STAMP(9);
      fft.transpose(v, my_spec);
      AVZ_STAMP(10);
      fft.stage2(v);
    } else {
      fft.forward(v, my_spec, twid);
    }
#else
    fft.forward(v, my_spec, twid);
#endif
    // natural-order spectrum into this lane group's slot
    static_for<0, PPL>([&](auto k) { my_spec[lm.out0 + C::OUT_STRIDE * k] = v[k]; });
#ifdef AVZ_STAMPS
    AVZ_STAMP(11);
#endif
  };

  // ---------------- per-bin thread role
  // Thread (kb, q) owns bin kb for the frames of row q. Bin 0 is self-partnered
  // (kp = 0) and needs no special case. The Nyquist bin N/2 is spread over lanes of
  // the last wave (one frame, or frame pair, per lane) so no wave carries it alone;
  // its running sums live in LDS.
  const int kb = tid % NB;
  const int q = tid / NB;
  const bool nyq = (kb == 0);
  const int kp = (N - kb) & (N - 1);
  const bool nyq_wave = (wave == NWAVE - 1);
  uint8_t* mb = A.maskbits + (long long)b * A.mb_stride;
  double* nyq_acc = reinterpret_cast<double*>(lds + G::NYQ_OFF);  // [5]
  cf* nyq_ab = reinterpret_cast<cf*>(nyq_acc + Q * 5);            // alpha_n, beta_n
  cf alpha{0, 0}, beta{0, 0};

  auto bin_weight = [&](cf x0, cf x1, const cf* Zr, int k, int kk, int t, bool& noise,
                        float& wgt) -> float {
    float m;
    if constexpr (MASK == MASK_IBM) {
      const cf zr = Zr[k], zrp = Zr[kk];
      // 2T = zr + conj(zrp), 2I = (zr - conj zrp)/i ; |2I|^2 > |2T|^2 <=> |I| > |T|
      const float tr = zr.x + zrp.x, ti = zr.y - zrp.y;
      const float ir = zr.y + zrp.y, ii = zr.x - zrp.x;
      noise = ir * ir + ii * ii > tr * tr + ti * ti;
      m = noise ? 1.0f : 0.0f;
      wgt = m;
    } else if constexpr (MASK == MASK_IPD) {
      m = ipd_weight(x0, x1);
      wgt = m;
    } else {
      const float M = A.ext_mask[(long long)b * A.mask_sb + (long long)k * A.mask_sf +
                                 (long long)t * A.mask_st];
      m = 1.0f - M;
      wgt = m + A.weight_eps;
    }
    return m;
  };

  // ======================= pass 1: masks + covariance =======================
  if (tid < 5) nyq_acc[tid] = 0.0;
  issue_loads(0);
  lds_barrier();  // twiddle table + Nyquist sums initialised
  AVZ_STAMP_INIT();
  {
    Acc64 acc;
    acc.zero();
    for (int step = 0; step < NB1; ++step) {
      window_and_fft();
      issue_loads(step + 1);  // step NB1 is pass 2's first batch
      lds_barrier();
      AVZ_STAMP(0);
      const int f0 = step * FB1;
      const int tq = f0 + q * FPT1;
      Acc32 a32;
      a32.zero();
      unsigned nib = 0;
      const int nvalid = T - tq;  // frames of this row that exist (may be <= 0)
#pragma unroll 4
      for (int i = 0; i < FPT1; ++i) {
        if (i < nvalid) {
          const int f = q * FPT1 + i;
          const cf* Zm = slot_ptr<N>(lds, f);
          cf x0, x1;
          split_pair(Zm[kb], Zm[kp], x0, x1);
          bool noise = false;
          float wgt;
          const float m =
              bin_weight(x0, x1, slot_ptr<N>(lds, FB1 + f), kb, kp, tq + i, noise, wgt);
          nib |= (noise ? 1u : 0u) << i;
          a32.add(x0, x1, wgt, m);
        }
      }
      acc.add(a32);
      if (nyq_wave) {  // Nyquist bin: frame `lane` of the batch on lane `lane`
        Acc32 an;
        an.zero();
        bool noise = false;
        if (lane < FB1 && f0 + lane < T) {
          const cf* Zm = slot_ptr<N>(lds, lane);
          cf y0, y1;
          split_pair(Zm[N / 2], Zm[N / 2], y0, y1);
          float wn;
          const float mn = bin_weight(y0, y1, slot_ptr<N>(lds, FB1 + lane), N / 2, N / 2,
                                      f0 + lane, noise, wn);
          an.add(y0, y1, wn, mn);
        }
        for (int o = 1; o < FB1; o <<= 1) {
          an.c00 += __shfl_xor(an.c00, o, 64);
          an.c11 += __shfl_xor(an.c11, o, 64);
          an.c01r += __shfl_xor(an.c01r, o, 64);
          an.c01i += __shfl_xor(an.c01i, o, 64);
          an.cm += __shfl_xor(an.cm, o, 64);
        }
        const unsigned long long bal = __ballot(noise);
        if (lane == 0) {
          nyq_acc[0] += (double)an.c00;
          nyq_acc[1] += (double)an.c11;
          nyq_acc[2] += (double)an.c01r;
          nyq_acc[3] += (double)an.c01i;
          nyq_acc[4] += (double)an.cm;
          if constexpr (MASK == MASK_IBM) {
            for (int j = 0; j < FB1 / 4; ++j)
              if (f0 + 4 * j < T)
                mb[(long long)((f0 >> 2) + j) * F + N / 2] = (uint8_t)((bal >> (4 * j)) & 15u);
          }
        }
      }
      if constexpr (MASK == MASK_IBM) {
#pragma unroll
        for (int j = 0; j < FPT1 / 4; ++j)
          if (tq + 4 * j < T) mb[(long long)((tq >> 2) + j) * F + kb] = (uint8_t)(nib >> (4 * j));
      }
      lds_barrier();
      AVZ_STAMP(1);
    }

    // ============ solve: reduce the Q partial rows, fp64 MVDR ============
    double* part = reinterpret_cast<double*>(lds);
#pragma unroll
    for (int c = 0; c < 5; ++c) part[(q * NB + kb) * 5 + c] = acc.c[c];
    __syncthreads();  // also publishes the global mask nibbles to pass 2
    double R[5] = {0, 0, 0, 0, 0};
    for (int qq = 0; qq < Q; ++qq) {
#pragma unroll
      for (int c = 0; c < 5; ++c) R[c] += part[(qq * NB + kb) * 5 + c];
    }
    const bool dbg = (q == 0);
    float* wdbg = (A.w_out && dbg) ? A.w_out + ((long long)b * F + kb) * 4 : nullptr;
    mvdr_solve(R, kb, N, A, alpha, beta, wdbg);
    if (A.cov_out && dbg) {
#pragma unroll
      for (int c = 0; c < 5; ++c) A.cov_out[((long long)b * F + kb) * 5 + c] = R[c];
    }
    if (tid == 0) {
      double Rn[5];
#pragma unroll
      for (int c = 0; c < 5; ++c) Rn[c] = nyq_acc[c];
      float* wdbgn = A.w_out ? A.w_out + ((long long)b * F + N / 2) * 4 : nullptr;
      mvdr_solve(Rn, N / 2, N, A, nyq_ab[0], nyq_ab[1], wdbgn);
      if (A.cov_out) {
#pragma unroll
        for (int c = 0; c < 5; ++c) A.cov_out[((long long)b * F + N / 2) * 5 + c] = Rn[c];
      }
    }
    lds_barrier();
    AVZ_STAMP(2);
  }

  // ============ pass 2: apply + post-filter + iSTFT overlap-add ============
  // OLA role: 4 consecutive samples m of segments {sgrp + i NSG}
  constexpr int M4 = N / 8;  // float4 groups per half frame
  constexpr int NSG = NT / M4;
  constexpr int SPT = FB2 / NSG;  // segments per thread
  static_assert(SPT * NSG == FB2, "OLA mapping");
  const int m0 = 4 * (tid % M4);
  const int sgrp = tid / M4;
  float peak = 0.0f;
  constexpr int NPAIR = FB2 / 2;
  const bool ifft_wave = wave < NPAIR / C::FPW;
  for (int st2 = 0; st2 < NB2; ++st2) {
    const int step = NB1 + st2;
    const bool more = step + 1 < NSTEP;
    window_and_fft();
    if (!ifft_wave && more) issue_loads(step + 1);  // idle during the inverse FFT: prefetch now
    lds_barrier();
    AVZ_STAMP(3);

    const int f0 = st2 * FB2;
    const int tq = f0 + q * FPT2;
    {
      auto gain = [&](int i, int t, uint32_t bb, int kk) -> float {
        if (t >= T) return 0.0f;
        switch (A.postfilter) {
          case PF_IBM_TARGET: return ((bb >> i) & 1u) ? 0.0f : 1.0f;
          case PF_EXT_FLOOR:
          case PF_EXT_MUL: {
            const float M = A.ext_mask[(long long)b * A.mask_sb + (long long)kk * A.mask_sf +
                                       (long long)t * A.mask_st];
            return A.postfilter == PF_EXT_FLOOR ? fmaxf(M, A.pf_floor) : M;
          }
          default: return 1.0f;
        }
      };
      auto load_bits = [&](int kk) -> uint32_t {  // bit i: frame tq + i is noise (IBM)
        uint32_t bb = 0;
        if (A.postfilter == PF_IBM_TARGET) {
          const uint8_t* row = mb + (long long)(tq >> 2) * F;
#pragma unroll
          for (int j = 0; j < FPT2 / 4; ++j)
            if (tq + 4 * j < T) bb |= (uint32_t)row[j * F + kk] << (4 * j);
        }
        return bb;
      };
      const uint32_t bits = load_bits(kb);
#pragma unroll 2
      for (int pi = 0; pi < FPT2 / 2; ++pi) {
        const int fa = q * FPT2 + 2 * pi;
        const int ta = tq + 2 * pi;
        if (ta < T) {
          cf* Za = slot_ptr<N>(lds, fa);
          const cf* Zb = slot_ptr<N>(lds, fa + 1);
          const float ga = gain(2 * pi, ta, bits, kb), gb = gain(2 * pi + 1, ta + 1, bits, kb);
          const cf za = Za[kb], zap = Za[kp], zb = Zb[kb], zbp = Zb[kp];
          const cf sa = apply_bin(alpha, beta, za, zap, ga);
          const cf sb = apply_bin(alpha, beta, zb, zbp, gb);
          Za[kp] = {sa.x + sb.y, sb.x - sa.y};  // conj(Sa) + i conj(Sb) at N - k
          // Sa + i Sb at k; at DC irfft keeps only the real parts (written last: kp == kb)
          Za[kb] = nyq ? cf{sa.x, sb.x} : cf{sa.x - sb.y, sa.y + sb.x};
        }
      }
      if (nyq_wave && lane < FB2 / 2) {  // Nyquist bin: frame pair `lane` on lane `lane`
        const int fa = 2 * lane;
        const int ta = f0 + fa;
        if (ta < T) {
          uint32_t bn = 0;
          if (A.postfilter == PF_IBM_TARGET)
            bn = (uint32_t)mb[(long long)(ta >> 2) * F + N / 2] >> (ta & 3);
          const cf an = nyq_ab[0], bnn = nyq_ab[1];
          cf* Za = slot_ptr<N>(lds, fa);
          const cf* Zb = slot_ptr<N>(lds, fa + 1);
          const float ga = gain(0, ta, bn, N / 2), gb = gain(1, ta + 1, bn, N / 2);
          const cf za = Za[N / 2], zb = Zb[N / 2];
          Za[N / 2] = {apply_bin(an, bnn, za, za, ga).x, apply_bin(an, bnn, zb, zb, gb).x};
        }
      }
    }
    lds_barrier();
    AVZ_STAMP(4);

    // ---- inverse FFT of packed pairs -> windowed frame contributions (waves < NPAIR/FPW)
    if (ifft_wave) {
      const int p = wave * C::FPW + lm.grp;
      cf* Zi = slot_ptr<N>(lds, 2 * p);
      static_for<0, PPL>([&](auto r) { v[r] = c_conj(Zi[lm.in0 + C::IN_STRIDE * r]); });
      fft.forward(v, Zi, twid);
      float* Cp = reinterpret_cast<float*>(slot_ptr<N>(lds, 2 * p + 1));
      static_for<0, PPL>([&](auto k) {
        constexpr float ck = W32::c[k], sk = -W32::s[k];  // cos, sin of 2 pi k / 32
        const float w = fmaf(wss, sk, fmaf(-wsc, ck, ws0));
        const int n = lm.out0 + C::OUT_STRIDE * k;
        Cp[n] = v[k].x * w;       // frame 2p   (real part of the inverse)
        Cp[N + n] = -v[k].y * w;  // frame 2p+1 (imag part; conj trick)
      });
      if (more) issue_loads(step + 1);
    }
    lds_barrier();
    AVZ_STAMP(5);

    // ---- overlap-add: segment j = frame j (2nd half) + frame j+1 (1st half)
    {
      const int bsel = st2 & 1;
      const float* cin = carry + bsel * H;
      float* cout = carry + (bsel ^ 1) * H;
      float* outb = A.out + (long long)b * A.out_stride;
      auto cframe = [&](int f) -> const float* {
        return reinterpret_cast<const float*>(slot_ptr<N>(lds, 2 * (f >> 1) + 1)) + (f & 1) * N;
      };
#pragma unroll
      for (int si = 0; si < SPT; ++si) {
        const int s = sgrp + si * NSG;
        const int j = f0 - 1 + s;
        if (j >= 0 && j <= T - 2) {
          const float* pa = (s == 0) ? cin + m0 : cframe(s - 1) + H + m0;
          const float* pb = cframe(s) + m0;
          const float4 va = *reinterpret_cast<const float4*>(pa);
          const float4 vb = *reinterpret_cast<const float4*>(pb);
          float in[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {  // 1 / (win[m]^2 + win[m + N/2]^2)
            const float c1 = cospif(2.0f * (float)(m0 + i) / (float)N);
            const float wa = 0.5f - 0.5f * c1, wb = 0.5f + 0.5f * c1;
            in[i] = 1.0f / (wa * wa + wb * wb);
          }
          float4 o;
          o.x = (va.x + vb.x) * in[0];
          o.y = (va.y + vb.y) * in[1];
          o.z = (va.z + vb.z) * in[2];
          o.w = (va.w + vb.w) * in[3];
          *reinterpret_cast<float4*>(outb + (long long)j * H + m0) = o;
          peak = fmaxf(peak, fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(o.w))));
        }
      }
      if (sgrp == 0) {
        *reinterpret_cast<float4*>(cout + m0) =
            *reinterpret_cast<const float4*>(cframe(FB2 - 1) + H + m0);
      }
    }
    lds_barrier();
    AVZ_STAMP(6);
  }

  // ---------------- block max |out|, optional in-place normalisation
  for (int o = 32; o > 0; o >>= 1) peak = fmaxf(peak, __shfl_xor(peak, o, 64));
  float* red = reinterpret_cast<float*>(lds);
  if (lane == 0) red[wave] = peak;
  __syncthreads();
  float pk = red[0];
#pragma unroll
  for (int w = 1; w < NWAVE; ++w) pk = fmaxf(pk, red[w]);
  if (tid == 0 && A.peak) A.peak[b] = pk;
  if (A.normalize == NORM_PEAK) {
    const float scale = 1.0f / (pk + A.norm_eps);
    float* outb = A.out + (long long)b * A.out_stride;
    const int n4 = (T - 1) * H / 4;
    float4* o4 = reinterpret_cast<float4*>(outb);
    for (int i = tid; i < n4; i += NT) {
      float4 x = o4[i];
      x.x *= scale; x.y *= scale; x.z *= scale; x.w *= scale;
      o4[i] = x;
    }
  }
  AVZ_STAMP(7);
}

// ---------------------------------------------------------------------------
// Standalone STFT (stage API / parity): Y[b][c][k][t] = scipy.signal.stft(x[b][c])
// One block per (utterance, NSLOT-frame batch); each lane group transforms one
// frame of the packed channel pair, then threads split the pair per bin.
constexpr int kStftThreads = 512;

template <int N>
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
  const int L = A.len[b];
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
    const long long o = (long long)b * A.y_stride_b + (long long)k * A.y_stride_f + t;
    Y[o] = make_float2(a.x, a.y);
    if (A.channels > 1) Y[o + A.y_stride_c] = make_float2(c.x, c.y);
  }
}

}  // namespace avz

using namespace avz;

#ifndef AVZ_FUSED_THREADS
#define AVZ_FUSED_THREADS 512
#endif
constexpr int kFusedThreads = AVZ_FUSED_THREADS;

#ifdef AVZ_STAMPS
extern "C" int avz_debug_set_stamps(void* dev_ptr) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &dev_ptr, sizeof(dev_ptr)) == hipSuccess ? 0 : -3;
}
#endif

extern "C" int avz_fused_lds_bytes(int n_fft) {
  return n_fft == 1024 ? Geo<1024, kFusedThreads>::LDS_BYTES
         : n_fft == 512 ? Geo<512, kFusedThreads>::LDS_BYTES : -1;
}

template <int N, int MASK>
static int launch_fused_t(const FusedArgs* a, hipStream_t st) {
  auto kern = avz_fused_kernel<N, MASK, kFusedThreads>;
  const int lds = Geo<N, kFusedThreads>::LDS_BYTES;
  static bool attr_done = false;
  if (!attr_done) {
    if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds) !=
        hipSuccess)
      return -3;
    attr_done = true;
  }
  hipLaunchKernelGGL(kern, dim3(a->batch), dim3(kFusedThreads), lds, st, *a);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int avz_launch_fused(int n_fft, int mask_mode, const FusedArgs* a, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (a->batch <= 0) return 0;
  if (n_fft == 1024) {
    switch (mask_mode) {
      case MASK_IBM: return launch_fused_t<1024, MASK_IBM>(a, st);
      case MASK_IPD: return launch_fused_t<1024, MASK_IPD>(a, st);
      case MASK_EXTERNAL: return launch_fused_t<1024, MASK_EXTERNAL>(a, st);
    }
  } else if (n_fft == 512) {
    switch (mask_mode) {
      case MASK_IBM: return launch_fused_t<512, MASK_IBM>(a, st);
      case MASK_IPD: return launch_fused_t<512, MASK_IPD>(a, st);
      case MASK_EXTERNAL: return launch_fused_t<512, MASK_EXTERNAL>(a, st);
    }
  }
  return -4;
}

template <int N>
static int launch_stft_t(const StftArgs* a, hipStream_t st) {
  auto kern = avz_stft_kernel<N>;
  const int lds = Geo<N, kStftThreads>::LDS_BYTES;
  static bool attr_done = false;
  if (!attr_done) {
    if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds) !=
        hipSuccess)
      return -3;
    attr_done = true;
  }
  constexpr int NS = Geo<N, kStftThreads>::NSLOT;
  dim3 grid(a->batch, (a->max_frames + NS - 1) / NS);
  hipLaunchKernelGGL(kern, grid, dim3(kStftThreads), lds, st, *a);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int avz_launch_stft(int n_fft, const StftArgs* a, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (a->batch <= 0) return 0;
  if (n_fft == 1024) return launch_stft_t<1024>(a, st);
  if (n_fft == 512) return launch_stft_t<512>(a, st);
  return -4;
}
