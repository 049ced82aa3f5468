// avz_chunked.hip — launchers of the chunk-parallel chain and the per-utterance synthesis
// kernels (kernels: avz_chunked_k.hpp; the analysis and chunk-synthesis instantiations are
// compiled in their own units, avz_chunked_inst.hpp).
#include "avz_chunked_k.hpp"
#include "avz_chunked_inst.hpp"

namespace avz {
#ifdef AVZ_ONE_TU  // the shipped build: every chain kernel compiled in this unit (Makefile)
#define AVZ_INST template
#else
#define AVZ_INST extern template
#endif
AVZ_ANALYSIS_INST(1024)
AVZ_ANALYSIS_INST(512)
AVZ_SYN_INST(1024)
AVZ_SYN_INST(512)
#undef AVZ_INST
// the per-utterance synthesis kernels: with the launchers in either build
#define AVZ_INST template
AVZ_UTT_INST
#undef AVZ_INST
}  // namespace avz

using namespace avz;

extern "C" int avz_chunk_frames(void) { return kChunk; }

static int resident_cus();

// The per-utterance kernel covers the IBM-target and unfiltered post-filters (the headline
// and the IPD configuration); the IRM and external-mask gains, read per (bin, frame) from
// memory, need registers it does not have (48-56 B of scratch), so those plans keep the
// chunk grid + finalize. It pays for peak normalisation only (the rescale folded in, no
// finalize launch); without it the chunk grid's synthesis + seam pass is the faster pair
// (B = 256: 70.7 + 4.2 vs 79.9 us, profiles/r04/ab_synth_utt.txt).
// At N = 512 (no piece split there) only whole rounds take it: a partial round, or a batch
// below the CU count, runs the chunk grid + finalize (at B = 1 the 8.23-s test triple's 17
// per-utterance steps on one CU took 154 us of synthesis).
template <int N, int PF, bool SPEC>
static bool synth_per_utterance(const ChainArgs* a) {
  return (N == 1024 || (N == 512 && a->batch % resident_cus() == 0)) && !SPEC &&
         (PF == PF_IBM_TARGET || PF == PF_NONE) && a->normalize == NORM_PEAK &&
         a->synth_variant >= 1;
}
// ... and solves the utterance's bins itself (variant 2) when the chain's solve is the plain
// MVDR one: no item-level fallback flags, no covariance / weight debug outputs.
template <int N, int PF>
static bool solve_fused(const ChainArgs* a) {
  return synth_per_utterance<N, PF, false>(a) && a->synth_variant == 2 &&
         a->beamformer == BF_MVDR && a->singular_fallback != 2 && !a->cov_out && !a->w_out &&
         !a->cov_only;
}

// Work split of the N = 1024 per-utterance synthesis (ChainArgs s_whole / s_pieces /
// s_steps / s_ipf): with R resident blocks (one per CU), whole utterances for the full rounds
// floor(B / R) R, and the partial last round's rem utterances -- or a whole batch below R --
// in pieces of s_steps steps (16 frames each) spread over the grid, when that is cheaper than
// one more round of whole utterances. Every piece solves its utterance's bins in-block. With
// full rounds (ipf) the pieces run first and finalize in-kernel (the last arriver forms the
// seams and the peak, each piece rescales its interior during its block's whole utterance);
// a batch below R keeps the piece-finalize launch. Cost model in steps of the kernel (~9.5
// us at two waves per SIMD): a whole round S steps + 2 (the in-block solve and the exposed
// rescale of its last utterance); pieces ceil(rem pu / R) s_steps + 1 (their solve) + 1 + 2
// rem / R without ipf (the finalize launch, ~10 us with its kernel boundary, and its rescale
// traffic).
struct SynthSplit {
  int whole, pieces, steps, grid;
  bool ipf;
};
static SynthSplit synth_split(const ChainArgs* a) {
  constexpr int FB = UttGeo::FB;
  const int R = resident_cus(), B = a->batch;
  const int S = (a->max_frames + FB - 1) / FB;  // steps of the longest utterance
  const SynthSplit all_whole{B, 0, S, std::min(B, R), false};
  if (!a->pheads || !a->ptails || B <= 0) return all_whole;
  const int full = B / R, rem = B - full * R;
  if (rem == 0) return all_whole;
  int pu = std::min(kMaxPieces, std::min(S, std::max(1, R / rem)));
  pu = std::min(pu, a->pseam_slots / rem);
  if (pu < 1) return all_whole;
  const int sp = (S + pu - 1) / pu;
  pu = (S + sp - 1) / sp;
  const long long units = (long long)rem * pu;
  const long long rounds = (units + R - 1) / R;
  const bool ipf = full > 0 && units <= R && a->pstate != nullptr;
  const double c_whole = S + 2.0,
               c_piece = (double)rounds * sp + 1.0 + (ipf ? 0.0 : 1.0 + 2.0 * rem / R);
  if (c_piece >= c_whole) return all_whole;
  return SynthSplit{full * R, pu, sp, full > 0 ? R : (int)std::min<long long>(units, R), ipf};
}

// A split batch whose solve has few threads (<= 64 blocks of one bin per thread): its many
// partial vectors per bin go to kSolveLanes lanes per bin (avz_solve_lanes_kernel).
template <int N>
static bool few_solve_threads(const ChainArgs* a) {
  return (long long)a->batch * (N / 2 + 1) <= 64LL * kSolveThreads;
}
template <int N>
static int solve_blocks(const ChainArgs* a, bool lanes) {
  const long long per = lanes ? kSolveThreads / kSolveLanes : kSolveThreads;
  return (int)(((long long)a->batch * (N / 2 + 1) + per - 1) / per);
}

// Synthesis + output normalisation of the chain and of the stage exports: the per-utterance
// kernel (time-domain input, peak normalisation; finalize events record an empty span unless
// the N = 1024 split has pieces, whose solve and finalize launches the solve and finalize
// events then time), or the persistent chunk grid followed by avz_finalize_kernel. ev: the
// (start, stop) event pairs of the solve, synthesis and finalize launches (6, may be null).
template <int N, int PF, bool SPEC = false>
static int launch_synthesis(const ChainArgs* a, hipStream_t st, hipEvent_t e0, hipEvent_t e1);
template <int N, int PF, bool SPEC = false>
static int launch_synth_finalize(const ChainArgs* a0, hipStream_t st, const hipEvent_t* ev,
                                 bool fused_solve = false) {
  ChainArgs c = *a0;
  const ChainArgs* a = &c;
  auto evt = [&](int i) -> hipEvent_t { return ev ? ev[i] : nullptr; };
  const hipEvent_t e0 = evt(2), e1 = evt(3), e2 = evt(4), e3 = evt(5);
  if (synth_per_utterance<N, PF, SPEC>(a)) {
    constexpr int UPF = (PF == PF_IBM_TARGET || PF == PF_NONE) ? PF : PF_NONE;  // instantiated
    dim3 grid((unsigned)std::min(a->batch, resident_cus()));
    c.s_whole = a->batch;
    c.s_pieces = 0;
    if constexpr (N == 1024) {
      const SynthSplit sp = synth_split(a);
      c.s_whole = sp.whole;
      c.s_pieces = sp.pieces;
      c.s_steps = sp.steps;
      c.s_ipf = sp.ipf ? 1 : 0;
      grid = dim3((unsigned)sp.grid);
    }
    if constexpr (N == 1024) {
      constexpr int lds = UttGeo::LDS_BYTES;
      // the general instance for pieces and for split analysis chunks (the whole-rounds one
      // reads only whole-chunk partials)
      const bool pc = c.s_pieces > 0 || c.a_pieces > 1;
      auto kern = fused_solve ? (pc ? avz_synthesis_utt_kernel<UPF, true, true>
                                    : avz_synthesis_utt_kernel<UPF, true, false>)
                              : (pc ? avz_synthesis_utt_kernel<UPF, false, true>
                                    : avz_synthesis_utt_kernel<UPF, false, false>);
      const bool ready = fused_solve
                             ? (pc ? lds_ready<avz_synthesis_utt_kernel<UPF, true, true>>(lds)
                                   : lds_ready<avz_synthesis_utt_kernel<UPF, true, false>>(lds))
                             : (pc ? lds_ready<avz_synthesis_utt_kernel<UPF, false, true>>(lds)
                                   : lds_ready<avz_synthesis_utt_kernel<UPF, false, false>>(lds));
      if (!ready) return -3;
      hipExtLaunchKernelGGL(kern, grid, dim3(kUttThreads), lds, st, e0, e1, 0, *a);
      if (c.s_pieces > 0 && !c.s_ipf) {
        const int T = a->max_frames;
        const int n4 = (T - 1) * (N / 2) / 4;
        const int gx = (n4 + kFinPieceU * kCThreads - 1) / (kFinPieceU * kCThreads);
        hipExtLaunchKernelGGL(avz_finalize_pieces_kernel<N>, dim3(gx, a->batch - c.s_whole),
                              dim3(kCThreads), 0, st, e2, e3, 0, *a);
      }
    } else {
      constexpr int lds = Utt512Geo::LDS_BYTES;
      auto kern = fused_solve ? avz_synthesis_utt512_kernel<UPF, true>
                              : avz_synthesis_utt512_kernel<UPF, false>;
      if (!(fused_solve ? lds_ready<avz_synthesis_utt512_kernel<UPF, true>>(lds)
                        : lds_ready<avz_synthesis_utt512_kernel<UPF, false>>(lds)))
        return -3;
      hipExtLaunchKernelGGL(kern, grid, dim3(kUtt512Threads), lds, st, e0, e1, 0, *a);
    }
    return 0;  // no finalize launch unless pieces: its events stay unrecorded (avz_chain_kernels)
  }
  if (launch_synthesis<N, PF, SPEC>(a, st, e0, e1) != 0) return -3;
  const int nch = (a->max_frames + kChunk - 1) / kChunk;
  hipExtLaunchKernelGGL(avz_finalize_kernel<N>, dim3(fin_groups<N>(nch), a->batch), dim3(kCThreads),
                        0, st, e2, e3, 0, *a);
  return 0;
}

// The synthesis launch of the chain and of the stage exports (persistent grid).
template <int N, int PF, bool SPEC>
static int launch_synthesis(const ChainArgs* a, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  const int nch = (a->max_frames + kChunk - 1) / kChunk;
  constexpr int lds = SGeo<N, kSynR<N, PF>>::LDS_BYTES;
  if (!lds_ready<avz_synthesis_kernel<N, PF, SPEC>>(lds)) return -3;
  const int n_items = nch * a->batch;
  if (n_items == 0) return 0;
  const dim3 sgrid((unsigned)std::min(n_items, KCfg<N>::SYN_BLOCKS_PER_CU * resident_cus()));
  hipExtLaunchKernelGGL((avz_synthesis_kernel<N, PF, SPEC>), sgrid, dim3(kCThreads), lds, st, e0,
                        e1, 0, *a);
  return 0;
}

#if defined(AVZ_STAMPS) || defined(AVZ_XTRACE)
#ifndef AVZ_ONE_TU
extern "C" int avz_stamps_set_ana1024(void*);
extern "C" int avz_stamps_set_ana512(void*);
extern "C" int avz_stamps_set_syn(void*);
#endif
extern "C" int avz_debug_set_stamps_chunked(void* dev_ptr) {
  int r = hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &dev_ptr, sizeof(dev_ptr)) == hipSuccess ? 0 : -3;
#ifndef AVZ_ONE_TU
  r |= avz_stamps_set_ana1024(dev_ptr) | avz_stamps_set_ana512(dev_ptr) | avz_stamps_set_syn(dev_ptr);
#endif
  return r;
}
#endif

// Compute units of the current device (cached per device id; thread-safe).
static int resident_cus() {
  static std::atomic<int> cache[64];
  int dev = 0, v = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return 256;
  if (dev < 64 && cache[dev].load(std::memory_order_relaxed) > 0)
    return cache[dev].load(std::memory_order_relaxed);
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
    v = 256;
  if (dev < 64) cache[dev].store(v, std::memory_order_relaxed);
  return v;
}

// Tail splitting of the analysis grid (analysis_items): with G resident blocks, the
// floor(n / G) G items of the full rounds run whole and the partial last round's items in
// P step-range pieces each (P <= SA, the steps of a chunk; P * tail <= G, the tail slots), so
// that round takes 1/P of an item's time instead of a whole one (B = 257: 1028 items over
// 512 blocks ran a third round of 4 items). Returns the grid.
static int analysis_tail(ChainArgs& c, int n_items, int G, int SA) {
  c.a_whole = n_items;
  c.a_pieces = 1;
  const int whole = n_items / G * G, tail = n_items - whole;
  int P = 1;
  if (tail > 0 && c.tpart != nullptr)
    for (int q = SA; q >= 2; q >>= 1)
      if ((long long)tail * q <= G && (long long)tail * q <= c.tpart_slots) {
        P = q;
        break;
      }
  if (P == 1) return std::min(n_items, G);
  c.a_whole = whole;
  c.a_pieces = P;
  return whole > 0 ? G : tail * P;
}

template <int N, int MASK, int PF>
static int launch_chunked_t(const ChainArgs* a0, hipStream_t st) {
  auto k3 = avz_finalize_kernel<N>;
  constexpr int lds = CGeo<N>::LDS_BYTES;
  ChainArgs c = *a0;  // this launch's copy (tail splitting parameters)
  const ChainArgs* a = &c;
  const int nch = (a->max_frames + kChunk - 1) / kChunk;
  if (nch > a->nchunk) return -2;
  const int n_items = nch * a->batch;
  constexpr int SA = kChunk / ((MASK == MASK_IBM) ? CGeo<N>::NSLOT / 2 : CGeo<N>::NSLOT);
  const dim3 pgrid((unsigned)analysis_tail(c, n_items, CGeo<N>::BLOCKS * resident_cus(), SA));
  const bool split = c.a_pieces > 1;  // the SPLIT instances only then
  auto k1 = split ? avz_analysis_kernel<N, MASK, PF == PF_IRM, true>
                  : avz_analysis_kernel<N, MASK, PF == PF_IRM, false>;
  const bool lanes = split && few_solve_threads<N>(a);
  auto ks = lanes ? avz_solve_lanes_kernel<N>
                  : (split ? avz_solve_kernel<N, true> : avz_solve_kernel<N, false>);
  if (!(split ? lds_ready<avz_analysis_kernel<N, MASK, PF == PF_IRM, true>>(lds)
              : lds_ready<avz_analysis_kernel<N, MASK, PF == PF_IRM, false>>(lds)))
    return -3;
  const int nsolve = solve_blocks<N>(a, lanes), nfix = solve_blocks<N>(a, false);
  // diagnostic timing: kernel i's (start, stop) events ride on its own dispatch packet
  // (hipExtLaunchKernel), so timing adds no marker packets between the launches
  hipEvent_t const* ev = reinterpret_cast<hipEvent_t const*>(a->events);
  auto evt = [&](int i) -> hipEvent_t { return (ev && i < a->n_events) ? ev[i] : nullptr; };
  const bool item_fallback = a->singular_fallback == 2 && a->beamformer == BF_MVDR;
  if (item_fallback && hipMemsetAsync(a->flag, 0, sizeof(int) * a->batch, st) != hipSuccess)
    return -3;
  hipExtLaunchKernelGGL(k1, pgrid, dim3(kCThreads), lds, st, evt(0), evt(1), 0, *a);
  const bool fused = solve_fused<N, PF>(a);  // the synthesis kernel solves (no launch here)
  if (fused) {
  } else if (item_fallback) {
    hipExtLaunchKernelGGL(ks, dim3(nsolve), dim3(kSolveThreads), 0, st, evt(2), nullptr, 0, *a);
    hipExtLaunchKernelGGL(avz_solve_fixup_kernel<N>, dim3(nfix), dim3(kSolveThreads), 0, st,
                          nullptr, evt(3), 0, *a);
  } else {
    hipExtLaunchKernelGGL(ks, dim3(nsolve), dim3(kSolveThreads), 0, st, evt(2), evt(3), 0, *a);
  }
  (void)k3;
  const hipEvent_t sev[6] = {evt(2), evt(3), evt(4), evt(5), evt(6), evt(7)};
  if (launch_synth_finalize<N, PF>(a, st, sev, fused) != 0) return -3;
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

template <int N, int MASK>
static int launch_pf(const ChainArgs* a, hipStream_t st) {
  if constexpr (MASK == MASK_IBM) {
    if (a->postfilter == PF_IBM_TARGET) return launch_chunked_t<N, MASK, PF_IBM_TARGET>(a, st);
    if (a->postfilter == PF_IRM) return launch_chunked_t<N, MASK, PF_IRM>(a, st);
  }
  if constexpr (MASK == MASK_EXTERNAL) {
    if (a->postfilter == PF_EXT_FLOOR) return launch_chunked_t<N, MASK, PF_EXT_FLOOR>(a, st);
    if (a->postfilter == PF_EXT_MUL) return launch_chunked_t<N, MASK, PF_EXT_MUL>(a, st);
  }
  if (a->postfilter == PF_NONE) return launch_chunked_t<N, MASK, PF_NONE>(a, st);
  return -4;
}

template <int N>
static int launch_srp_t(const ChainArgs* a, const SrpArgs* s, hipStream_t st) {
  auto k1 = avz_analysis_kernel<N, MASK_ONES, false>;
  constexpr int lds = CGeo<N>::LDS_BYTES;
  if (!lds_ready<avz_analysis_kernel<N, MASK_ONES, false>>(lds)) return -3;
  const int nch = (a->max_frames + kChunk - 1) / kChunk;
  if (nch > a->nchunk) return -2;
  const int n_items = nch * a->batch;
  hipLaunchKernelGGL(k1, dim3((unsigned)std::min(n_items, CGeo<N>::BLOCKS * resident_cus())), dim3(kCThreads),
                     lds, st, *a);
  hipLaunchKernelGGL(avz_srp_kernel<N>, dim3(a->batch), dim3(kSrpThreads), 0, st, *a, *s);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int avz_launch_srp(int n_fft, const ChainArgs* a, const SrpArgs* s, void* stream) {
  if (a->batch <= 0) return 0;
  if (n_fft == 1024) return launch_srp_t<1024>(a, s, (hipStream_t)stream);
  if (n_fft == 512) return launch_srp_t<512>(a, s, (hipStream_t)stream);
  return -4;
}

template <int N>
static void chain_kernels_t(const ChainArgs* a, bool& utt, bool& fused) {
  if (a->postfilter == PF_IBM_TARGET) {
    utt = synth_per_utterance<N, PF_IBM_TARGET, false>(a);
    fused = solve_fused<N, PF_IBM_TARGET>(a);
  } else if (a->postfilter == PF_NONE) {
    utt = synth_per_utterance<N, PF_NONE, false>(a);
    fused = solve_fused<N, PF_NONE>(a);
  }
}
extern "C" int avz_chain_kernels(int n_fft, const ChainArgs* a) {
  bool utt = false, fused = false;
  if (n_fft == 1024) chain_kernels_t<1024>(a, utt, fused);
  if (n_fft == 512) chain_kernels_t<512>(a, utt, fused);
  // the N = 1024 per-utterance kernel's pieces below whole rounds bring a finalize launch
  const SynthSplit sp = n_fft == 1024 ? synth_split(a) : SynthSplit{0, 0, 0, 0, false};
  const bool fin = utt && n_fft == 1024 && sp.pieces > 0 && !sp.ipf;
  return 1 | (fused ? 0 : 2) | 4 | (utt && !fin ? 0 : 8);
}

extern "C" int avz_launch_chunked(int n_fft, int mask_mode, const ChainArgs* a, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (a->batch <= 0) return 0;
  if (n_fft == 1024) {
    switch (mask_mode) {
      case MASK_IBM: return launch_pf<1024, MASK_IBM>(a, st);
      case MASK_IPD: return launch_pf<1024, MASK_IPD>(a, st);
      case MASK_EXTERNAL: return launch_pf<1024, MASK_EXTERNAL>(a, st);
      case MASK_ONES: return launch_pf<1024, MASK_ONES>(a, st);
    }
  } else if (n_fft == 512) {
    switch (mask_mode) {
      case MASK_IBM: return launch_pf<512, MASK_IBM>(a, st);
      case MASK_IPD: return launch_pf<512, MASK_IPD>(a, st);
      case MASK_EXTERNAL: return launch_pf<512, MASK_EXTERNAL>(a, st);
      case MASK_ONES: return launch_pf<512, MASK_ONES>(a, st);
    }
  }
  return -4;
}

// ================================ stage exports ================================
// Apply coefficients of caller weights w[b][k] = (Re w0, Im w0, Re w1, Im w1) (the w_out
// layout): S = conj(w0) y0 + conj(w1) y1 as alpha Z[k] + beta conj(Z[N-k]).
__global__ void __launch_bounds__(256) avz_coef_kernel(ChainArgs A, const float* w, int F) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)A.batch * F) return;
  const float4 x = reinterpret_cast<const float4*>(w)[i];
  cf al, be;
  coef_from_w(x.x, x.y, x.z, x.w, al, be, nullptr);
  reinterpret_cast<float4*>(A.coef)[i] = make_float4(al.x, al.y, be.x, be.y);
}

template <int N, int MASK>
static int launch_cov_t(const ChainArgs* a, hipStream_t st) {
  constexpr int lds = CGeo<N>::LDS_BYTES;
  if (!lds_ready<avz_analysis_kernel<N, MASK, false, true>>(lds) ||
      !lds_ready<avz_analysis_kernel<N, MASK, false, false>>(lds))
    return -3;
  const int nch = (a->max_frames + kChunk - 1) / kChunk;
  if (nch > a->nchunk) return -2;
  const int n_items = nch * a->batch;
  ChainArgs c = *a;
  c.cov_only = 1;
  // the chain's tail splitting, so the sums equal the fused call's bitwise (but where the
  // solve lanes kernel sums a small split batch: its fp64 association differs, equal up to
  // fp64 rounding)
  constexpr int SA = kChunk / ((MASK == MASK_IBM) ? CGeo<N>::NSLOT / 2 : CGeo<N>::NSLOT);
  const int grid = analysis_tail(c, n_items, CGeo<N>::BLOCKS * resident_cus(), SA);
  const bool split = c.a_pieces > 1;
  auto ka = split ? avz_analysis_kernel<N, MASK, false, true>
                  : avz_analysis_kernel<N, MASK, false, false>;
  const bool lanes = split && few_solve_threads<N>(a);
  auto ks = lanes ? avz_solve_lanes_kernel<N>
                  : (split ? avz_solve_kernel<N, true> : avz_solve_kernel<N, false>);
  hipLaunchKernelGGL(ka, dim3((unsigned)grid), dim3(kCThreads), lds, st, c);
  hipLaunchKernelGGL(ks, dim3(solve_blocks<N>(a, lanes)), dim3(kSolveThreads), 0, st, c);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int avz_launch_covariance(int n_fft, int mask_mode, const ChainArgs* a, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (a->batch <= 0) return 0;
#define AVZ_COV_CASES(NN)                                                   \
  switch (mask_mode) {                                                      \
    case MASK_IBM: return launch_cov_t<NN, MASK_IBM>(a, st);                \
    case MASK_IPD: return launch_cov_t<NN, MASK_IPD>(a, st);                \
    case MASK_EXTERNAL: return launch_cov_t<NN, MASK_EXTERNAL>(a, st);      \
    case MASK_ONES: return launch_cov_t<NN, MASK_ONES>(a, st);              \
  }
  if (n_fft == 1024) { AVZ_COV_CASES(1024) }
  if (n_fft == 512) { AVZ_COV_CASES(512) }
#undef AVZ_COV_CASES
  return -4;
}

template <int N, int PF, bool SPEC>
static int launch_synth_t(const ChainArgs* a, hipStream_t st) {
  const int nch = (a->max_frames + kChunk - 1) / kChunk;
  if (nch > a->nchunk) return -2;
  // no analysis pass in these stages: it is the analysis kernel that resets peak_u
  if (hipMemsetAsync(a->peak_u, 0, sizeof(uint32_t) * a->batch, st) != hipSuccess) return -3;
  if (a->pstate && hipMemsetAsync(a->pstate, 0, sizeof(PieceState) * a->batch, st) != hipSuccess)
    return -3;
  if (a->peak && a->normalize != NORM_PEAK &&
      hipMemsetAsync(a->peak, 0, sizeof(float) * a->batch, st) != hipSuccess)
    return -3;
  if (launch_synth_finalize<N, PF, SPEC>(a, st, nullptr) != 0) return -3;
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int avz_launch_apply_istft(int n_fft, const ChainArgs* a, const float* w, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (a->batch <= 0) return 0;
  const int F = n_fft / 2 + 1;
  const long long n = (long long)a->batch * F;
  hipLaunchKernelGGL(avz_coef_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, *a, w, F);
  const bool g = a->ext_mask != nullptr;
  if (n_fft == 1024)
    return g ? launch_synth_t<1024, PF_EXT_MUL, false>(a, st) : launch_synth_t<1024, PF_NONE, false>(a, st);
  if (n_fft == 512)
    return g ? launch_synth_t<512, PF_EXT_MUL, false>(a, st) : launch_synth_t<512, PF_NONE, false>(a, st);
  return -4;
}

extern "C" int avz_launch_istft(int n_fft, const ChainArgs* a, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (a->batch <= 0) return 0;
  if (n_fft == 1024) return launch_synth_t<1024, PF_NONE, true>(a, st);
  if (n_fft == 512) return launch_synth_t<512, PF_NONE, true>(a, st);
  return -4;
}
