// avz_synth_rolesplit.hip — round-4 experiment, NOT built: the role-split synthesis kernel
// (4 producer waves: forward FFT of step e; 4 consumer waves: apply + per-frame N/2-point
// inverse + overlap-add of step e - 1; double-buffered spectra, one block barrier per step,
// an LDS arrival counter among the consumers). Correct (126/126 GPU tests with it as the
// default, output within 4.2e-7 of the two-block kernel) but synthesis 78.1-79.1 vs
// 70.2-70.3 us (profiles/r04/ab_synth_rolesplit.txt): the producer's forward Fft1024x2
// takes 3.9 us per step and the consumer's apply + Fft512x2 3.9 us (phase stamps,
// profiles/r04/stamps_rolesplit_*.txt) -- the per-SIMD VALU + LDS work per frame is the
// same as the two-block kernel's, so splitting it by role does not shorten it.
// It was spliced into avz_chunked.hip before the finalize section, launched with
// kRsThreads = 512 threads, RsGeo::LDS_BYTES of dynamic LDS, one block per CU.
// ======================= role-split synthesis (N = 1024, time-domain input) =======================
// One 8-wave block per CU, two waves per SIMD of different roles (waves w and w + 4 share a
// SIMD): waves 0-3 PRODUCE step e (load, window, forward Fft1024x2 of frames 2w, 2w + 1 into
// spectrum buffer e & 1), waves 4-7 CONSUME step e - 1 from the other buffer (apply + post-filter,
// each frame's real inverse as an N/2-point complex Fft512x2 on its own frames, windowed
// contributions in place, overlap-add of the step's 8 segments). One block barrier per step
// swaps the buffers; the consumers' overlap-add, which reads neighbouring waves' frames, waits
// on an LDS arrival counter of the four consumer waves only. The (chunk, utterance) items of the
// persistent grid form one stream of steps, so the pipeline runs across item boundaries.
// Replaces the two-block synthesis kernel, whose inverse ran on two of four waves while the
// other two waited at the block barrier (SQ_WAIT_ANY 36 %, profiles/r03o/sq_counters.txt).
constexpr int kRsThreads = 512;
struct RsGeo {
  static constexpr int N = 1024, H = 512, F = 513, FB = 8;
  static constexpr int SLOT = KCfg<1024>::GROUP_BYTES;  // one frame (transpose rows of 34)
  static constexpr int BUF = FB * SLOT;
  static constexpr int CNT_OFF = 2 * BUF;               // consumer arrival counter
  static constexpr int LDS_BYTES = CNT_OFF + 64;
  static_assert(LDS_BYTES <= 160 * 1024, "one block per CU");
};
__device__ __forceinline__ cf* rs_frame(unsigned char* lds, int buf, int f) {
  return reinterpret_cast<cf*>(lds + buf * RsGeo::BUF + f * RsGeo::SLOT);
}

// The block's stream of (item, step): items blockIdx.x, + gridDim.x, ... (item = (chunk c,
// utterance b)), each with nstep steps of FB frames; items without frames are skipped.
// All fields are wave-uniform.
struct RsCursor {
  int it, b, c, L, T, nstep, step;
  __device__ __forceinline__ void seek(const ChainArgs& A, int gx, int n_items) {
    constexpr int N = RsGeo::N, H = RsGeo::H, FB = RsGeo::FB;
    step = 0;
    for (; it < n_items; it += gridDim.x) {
      b = it / gx;
      c = it % gx;
      L = utt_len(A, b);
      if (L < N) continue;
      T = (L + H - 1) / H + 1;
      if (c * kChunk >= T) continue;
      nstep = (min(kChunk, T - c * kChunk) + FB - 1) / FB;
      return;
    }
  }
  __device__ __forceinline__ void start(const ChainArgs& A, int gx, int n_items) {
    it = blockIdx.x;
    seek(A, gx, n_items);
  }
  __device__ __forceinline__ void advance(const ChainArgs& A, int gx, int n_items) {
    if (++step == nstep) {
      it += gridDim.x;
      seek(A, gx, n_items);
    }
  }
  __device__ __forceinline__ int f0() const { return c * kChunk + step * RsGeo::FB; }
};

template <int PF>
__device__ __forceinline__ void rs_producer(const ChainArgs& A, unsigned char* lds, int gx,
                                            int n_items, int n_epochs) {
  constexpr int N = RsGeo::N, H = RsGeo::H;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // 0..3
  const int lane = tid & 63;
  Fft1024x2 fft;
  fft.init(lane);
  LaneMap<N> lm;
  lm.init(lane);
  WinCoef<N> wc;
  wc.init(lm);
  const int my = 2 * wave + lm.grp;  // frame of the step = slot
  const rsrc_t r_none = make_rsrc(nullptr, 0);
  auto rsrcs = [&](const RsCursor& k, rsrc_t& r0, rsrc_t& r1) {
    const float* mixb = A.mix + (long long)k.b * A.mix_stride;
    r0 = make_rsrc(mixb, k.L);
    r1 = make_rsrc(mixb + A.ch_stride, k.L);
  };
  cf v[32];
  // loads of step k into v: unchecked offsets where no sample index of the wave is negative
  auto load_step = [&](const RsCursor& k, rsrc_t r0, rsrc_t r1) {
    const int s0 = (k.f0() + my) * H - N / 2 + lm.in0;
    if (k.f0() + 2 * wave >= 1) {
      static_for<0, 32>([&](auto r) {
        v[r].x = bload_nn(r0, s0 + 32 * r);
        v[r].y = bload_nn(r1, s0 + 32 * r);
      });
    } else {
      static_for<0, 32>([&](auto r) {
        v[r].x = bload(r0, s0 + 32 * r);
        v[r].y = bload(r1, s0 + 32 * r);
      });
    }
  };
  AVZ_STAMP_DECL();
  AVZ_STAMP_INIT();
  RsCursor cur;
  cur.start(A, gx, n_items);
  rsrc_t r0 = r_none, r1 = r_none;
  if (cur.it < n_items) {
    rsrcs(cur, r0, r1);
    load_step(cur, r0, r1);
  }
  AVZ_STAMP(4);
  for (int e = 0; e < n_epochs; ++e) {
    if (e < n_epochs - 1) {
      RsCursor nx = cur;
      nx.advance(A, gx, n_items);
      const bool nv = nx.it < n_items;
      rsrc_t n0 = r0, n1 = r1;
      if (nv && nx.b != cur.b) rsrcs(nx, n0, n1);
      // the next step's loads from inside the FFT's last stage (register k right after its
      // output is stored); a wave whose next frames start before sample 0 (an item's first
      // step at c = 0) loads after the FFT with range-checked offsets
      const bool il = nv && nx.f0() + 2 * wave >= 1;
      const rsrc_t q0 = il ? n0 : r_none, q1 = il ? n1 : r_none;
      const int sn = (nx.f0() + my) * H - N / 2 + lm.in0;
      window_fft<N>(v, wc, fft, rs_frame(lds, e & 1, my), lm, [&](auto kc) {
        constexpr int k = decltype(kc)::value;
        v[k].x = bload_nn(q0, sn + 32 * k);
        v[k].y = bload_nn(q1, sn + 32 * k);
      });
      AVZ_STAMP(5);
      if (nv && !il) load_step(nx, n0, n1);
      cur = nx;
      r0 = n0;
      r1 = n1;
      AVZ_STAMP(6);
    }
    lds_barrier();
    AVZ_STAMP(7);
  }
}

template <int PF>
__device__ __forceinline__ void rs_consumer(const ChainArgs& A, unsigned char* lds, int gx,
                                            int n_items, int n_epochs) {
  constexpr int N = RsGeo::N, H = RsGeo::H, F = RsGeo::F, FB = RsGeo::FB;
  const int ct = threadIdx.x - 256;                             // 0..255
  const int cw = __builtin_amdgcn_readfirstlane(ct >> 6);       // consumer wave 0..3
  const int lane = ct & 63;
  Fft512x2 f5;
  f5.init(lane);
  // apply bins: m_j = lane + 64 j (j < 4) pairs bin kA = m with kB = N/2 - m; bin N/4 (its
  // own partner) on lanes 0 (frame 2 cw) and 1 (frame 2 cw + 1)
  cf om[4];  // e^{+2 pi i m_j / N}
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double sn, cs;
    sincospi(2.0 * (lane + 64 * j) / N, &sn, &cs);
    om[j] = cf{(float)cs, (float)sn};
  }
  // inverse output: u[k] = conj(z[m]), m = mh + 16 k -> samples 2m, 2m + 1 (0.5 hann)
  float wh_c[2], wh_s[2];
  const int mh = (lane & 15) + 256 * ((lane >> 4) & 1);
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    double sn, cs;
    sincospi(2.0 * (2 * mh + e) / N, &sn, &cs);
    wh_c[e] = (float)(0.25 * cs);
    wh_s[e] = (float)(0.25 * sn);
  }
  // overlap-add role: 4 consecutive samples m0.. of segments sgrp + 2 si
  const int m0 = 4 * (ct & 127), sgrp = ct >> 7;
  float inv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) inv[i] = inv_wsum<N>(m0 + i);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(lds + RsGeo::CNT_OFF);
  uint32_t n_arrive = 0;

  // apply coefficients of kA_j (j < 4), kB_j (4 + j), N/4 (8) and the chunk's post-filter
  // bits; the next item's are loaded one epoch ahead (its first step's epoch would otherwise
  // wait on them: 7.8 us of 105 in the phase stamps, profiles/r04c)
  float4 cf4[9], ncf4[9];
  uint32_t bits[9], nbits[9];
  auto fetch = [&](const RsCursor& k, float4 (&w)[9], uint32_t (&bb)[9]) {
    const float4* coef = reinterpret_cast<const float4*>(A.coef) + (long long)k.b * F;
    const uint32_t* MW = A.mwords + ((long long)k.b * A.nchunk + k.c) * F;
#pragma unroll
    for (int q = 0; q < 9; ++q) {
      const int kk = q < 4 ? lane + 64 * q : (q < 8 ? H - lane - 64 * (q - 4) : N / 4);
      w[q] = coef[kk];
      bb[q] = (PF == PF_IBM_TARGET) ? MW[kk] : 0u;
    }
  };
  float4 carry = make_float4(0.f, 0.f, 0.f, 0.f);
  float peak = 0.0f;
  AVZ_STAMP_DECL();
  AVZ_STAMP_INIT();
  RsCursor cur;
  cur.start(A, gx, n_items);
  if (cur.it < n_items) fetch(cur, ncf4, nbits);  // epoch 0: the consumers have no step yet
  for (int e = 0; e < n_epochs; ++e) {
    if (e >= 1) {
      const int b = cur.b, c = cur.c, T = cur.T, step = cur.step;
      const int f0 = cur.f0();
      if (step == 0) {  // the item's prefetched coefficients and post-filter bits
#pragma unroll
        for (int q = 0; q < 9; ++q) {
          cf4[q] = ncf4[q];
          bits[q] = nbits[q];
        }
        carry = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      if (step == cur.nstep - 1) {  // prefetch the next item's
        RsCursor nx = cur;
        nx.advance(A, gx, n_items);
        if (nx.it < n_items) fetch(nx, ncf4, nbits);
      }
      cf al[9], be[9];
#pragma unroll
      for (int q = 0; q < 9; ++q) {
        al[q] = cf{cf4[q].x, cf4[q].y};
        be[q] = cf{cf4[q].z, cf4[q].w};
      }
      AVZ_STAMP(15);
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
      const int buf = (e - 1) & 1;
      // ---- apply w^H y + post-filter of this wave's frames 2 cw, 2 cw + 1, folded into each
      // frame's N/2-point inverse input (written in place over the bins just read):
      //   Zh[m] = A + i B, Zh[N/2 - m] = conj(A) + i conj(B),
      //   A = S[m] + conj(S[N/2 - m]),  B = e^{2 pi i m / N} (S[m] - conj(S[N/2 - m]))
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const int f = 2 * cw + g, t = f0 + f, ib = step * FB + f;
        cf* Z = rs_frame(lds, buf, f);
        cf za[4], zap[4], zb[4], zbp[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int kA = lane + 64 * j, kB = H - kA;
          za[j] = lds_read(Z + kA);
          zap[j] = lds_read(Z + ((N - kA) & (N - 1)));
          zb[j] = lds_read(Z + kB);
          zbp[j] = lds_read(Z + (N - kB));
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int kA = lane + 64 * j, kB = H - kA;
          cf sa = apply_bin(al[j], be[j], za[j], zap[j], gain(bits[j], ib, t, kA));
          cf sb = apply_bin(al[4 + j], be[4 + j], zb[j], zbp[j], gain(bits[4 + j], ib, t, kB));
          if (j == 0 && lane == 0) {  // DC and Nyquist: irfft keeps the real parts
            sa.y = 0.0f;
            sb.y = 0.0f;
          }
          const cf a = {sa.x + sb.x, sa.y - sb.y};
          const cf d = {sa.x - sb.x, sa.y + sb.y};
          const cf bb = c_mul(om[j], d);
          Z[kA] = {a.x - bb.y, a.y + bb.x};
          Z[kB] = {a.x + bb.y, bb.x - a.y};
        }
        if (lane == g) {  // bin N/4: Zh = 2 conj(S)
          const cf s = apply_bin(al[8], be[8], Z[N / 4], Z[3 * N / 4], gain(bits[8], ib, t, N / 4));
          Z[N / 4] = {2.0f * s.x, -2.0f * s.y};
        }
      }
      AVZ_STAMP(8);
      __builtin_amdgcn_wave_barrier();
      // ---- inverse: lane group g transforms frame 2 cw + g; windowed contributions (samples
      // 2m, 2m + 1 as one float2) over the frame's first 4 KB, the transpose in its second half
      {
        cf* Zi = rs_frame(lds, buf, 2 * cw + (lane >> 5));
        cf u[16];
        static_for<0, 16>([&](auto r) { u[r] = c_conj(lds_read(Zi + (lane & 31) + 32 * r)); });
        float2* Cp = reinterpret_cast<float2*>(Zi);
        f5.forward_emit(u, Zi + H, [&](auto k, cf x) {
          constexpr float ck = W32::c[k], sk = -W32::s[k];  // cos, sin of 2 pi (32 k) / N
          const float we = fmaf(wh_s[0], sk, fmaf(-wh_c[0], ck, 0.25f));
          const float wo = fmaf(wh_s[1], sk, fmaf(-wh_c[1], ck, 0.25f));
          Cp[mh + 16 * k] = make_float2(x.x * we, -x.y * wo);
        });
      }
      AVZ_STAMP(9);
      // ---- the four consumer waves' frames are in LDS: arrival counter (LDS-only sync)
      n_arrive += 4;
      if (lane == 0)
        __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      while (__builtin_amdgcn_readfirstlane(
                 __hip_atomic_load(cnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) < n_arrive)
        __builtin_amdgcn_s_sleep(1);
      AVZ_STAMP(10);
      // ---- overlap-add: segment j = f0 - 1 + s = frame s-1 (2nd half) + frame s (1st half)
      float* outb = A.out + (long long)b * A.out_stride;
      auto cframe = [&](int f) -> const float* {
        return reinterpret_cast<const float*>(rs_frame(lds, buf, f));
      };
#pragma unroll
      for (int si = 0; si < 4; ++si) {
        const int s = sgrp + 2 * si;
        const float4 vb = *reinterpret_cast<const float4*>(cframe(s) + m0);
        if (s == 0 && step == 0) {  // chunk's first frame: finalize adds the previous tail
          *reinterpret_cast<float4*>(A.heads + ((long long)b * A.nchunk + c) * H + m0) = vb;
          continue;
        }
        const int j = f0 - 1 + s;
        if (j <= T - 2) {
          const float4 va =
              (s == 0) ? carry : *reinterpret_cast<const float4*>(cframe(s - 1) + H + m0);
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
      if (step == cur.nstep - 1) {  // the item's last step: its tail and its peak
        if (sgrp == 0 && cur.nstep * FB == kChunk)
          *reinterpret_cast<float4*>(A.tails + ((long long)b * A.nchunk + c) * H + m0) = carry;
        for (int o = 32; o > 0; o >>= 1) peak = fmaxf(peak, __shfl_xor(peak, o, 64));
        if (lane == 0) atomicMax(A.peak_u + b, __float_as_uint(peak));
        peak = 0.0f;
      }
      cur.advance(A, gx, n_items);
      AVZ_STAMP(13);
    }
    lds_barrier();
    AVZ_STAMP(14);
  }
}

template <int PF>
__global__ void __launch_bounds__(kRsThreads, 2) avz_synthesis_rs_kernel(ChainArgs A) {
  extern __shared__ __align__(16) unsigned char lds[];
  const int gx = (A.max_frames + kChunk - 1) / kChunk;
  const int n_items = gx * A.batch;
  if (threadIdx.x == 0) *reinterpret_cast<uint32_t*>(lds + RsGeo::CNT_OFF) = 0u;
  // epochs = the block's steps + 1 (producers run epochs 0 .. n - 1, consumers 1 .. n)
  int n_steps = 0;
  {
    RsCursor k;
    k.start(A, gx, n_items);
    while (k.it < n_items) {
      n_steps += k.nstep;
      k.it += gridDim.x;
      k.seek(A, gx, n_items);
    }
  }
  __syncthreads();
  if (n_steps == 0) return;
  if (threadIdx.x < 256)
    rs_producer<PF>(A, lds, gx, n_items, n_steps + 1);
  else
    rs_consumer<PF>(A, lds, gx, n_items, n_steps + 1);
}

