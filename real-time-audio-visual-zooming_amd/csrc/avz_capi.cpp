// avz_capi.cpp — plan management, validation and dispatch behind include/avz.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <complex>
#include <limits>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/avz.h"
#include "avz_internal.h"

// Per-call device workspace of the chain (see avz_internal.h ChainArgs), carved from one
// caller-provided block (avz_mvdr_workspace_bytes) or from the plan's own arena.
struct Workspace {
  float* part;
  uint32_t* mwords;
  float* coef;               // [batch][F][4] per-bin apply coefficients
  float* heads;
  float* tails;
  uint32_t* peak_u;
  int* flag;                 // [batch] item-level fallback flags (AVZ_FALLBACK_BATCH)
  float* pf_gain;            // [batch][nchunk][32][F] IRM gains (AVZ_PF_IRM plans only)
  float* tpart;              // [tail_slots][5][F] analysis pieces' partials (tail splitting)
  int tail_slots;
  float* pheads;             // [seam_slots][H] per-utterance synthesis pieces' seam halves
  float* ptails;
  int seam_slots;
  avz::PieceState* pstate;   // [batch] in-kernel piece finalize: arrivals, 1/peak, hand-backs
  uint32_t* xpend;           // IBM plans: [units][4] exact-path records (ChainArgs)
  uint32_t* xdfr;            // IBM plans: [units][F] per-bin deferrals
  uint32_t* xunc;            // IBM plans: [units][32][32] uncertain bins of deferred frames
  uint32_t* xst;             // IBM plans: [units][2] work-sharing state (must start zero)
  size_t xst_bytes;
  long long xst_units;
  float* xres;               // IBM plans: [units][kXPieces][5][F] shared units' piece sums
};

// Tail-splitting capacity (ChainArgs a_* / s_*): analysis pieces of a partial last round
// (at most the analysis grid, 3 blocks x 256 CUs; 8 pieces per 32-frame chunk), and the
// seams of the per-utterance synthesis pieces (at most 255 piece utterances on 256 CUs,
// 32 pieces each, at most two per chunk). Launches never split beyond these.
static int tail_slots(long long B, int nchunk) { return (int)std::min<long long>(B * nchunk * 8, 768); }
static int seam_slots(long long B, int nchunk) {
  return (int)(std::min<long long>(B, 256) * std::min(32, 2 * nchunk));
}

static size_t align256(size_t n) { return (n + 255) & ~size_t(255); }

// Bytes of a workspace for `batch` utterances of at most `nchunk` 32-frame chunks; with a
// non-null base also carves it into *w. Every piece starts on a 256-byte boundary.
static size_t ws_layout(const avz_config& c, long long batch, int nchunk, char* base, Workspace* w) {
  const int F = c.n_fft / 2 + 1, H = c.n_fft / 2, CF = avz_chunk_frames();
  const long long B = batch;
  const size_t sz_part = align256(sizeof(float) * B * nchunk * 5 * F);
  const size_t sz_mw = align256(sizeof(uint32_t) * B * nchunk * F);
  const size_t sz_coef = align256(sizeof(float) * B * F * 4);
  const size_t sz_ht = align256(sizeof(float) * B * nchunk * H);
  const size_t sz_b = align256(sizeof(uint32_t) * B);
  const size_t sz_gain =
      c.postfilter == AVZ_PF_IRM ? align256(sizeof(float) * B * nchunk * CF * F) : 0;
  const int ts = tail_slots(B, nchunk), ss = seam_slots(B, nchunk);
  const size_t sz_tpart = align256(sizeof(float) * (size_t)ts * 5 * F);
  const size_t sz_seam = align256(sizeof(float) * (size_t)ss * H);
  // exact IBM path: one record per analysis unit (whole items + tail pieces)
  const long long units = c.mask_mode == AVZ_MASK_IBM ? B * nchunk + ts : 0;
  const size_t sz_xp = align256(sizeof(uint32_t) * 4 * units);
  const size_t sz_xd = align256(sizeof(uint32_t) * (size_t)F * units);
  const size_t sz_xu = align256(sizeof(uint32_t) * 32 * 32 * (size_t)units);
  const size_t sz_xs = align256(sizeof(uint32_t) * (2 * (size_t)units + (size_t)(units + 31) / 32));
  const size_t sz_xr = align256(sizeof(float) * avz::kXPieces * 5 * (size_t)F * units);

  if (base && w) {
    char* q = base;
    w->part = reinterpret_cast<float*>(q); q += sz_part;
    w->mwords = reinterpret_cast<uint32_t*>(q); q += sz_mw;
    w->coef = reinterpret_cast<float*>(q); q += sz_coef;
    w->heads = reinterpret_cast<float*>(q); q += sz_ht;
    w->tails = reinterpret_cast<float*>(q); q += sz_ht;
    w->peak_u = reinterpret_cast<uint32_t*>(q); q += sz_b;
    w->flag = reinterpret_cast<int*>(q); q += sz_b;
    w->pf_gain = sz_gain ? reinterpret_cast<float*>(q) : nullptr;
    q += sz_gain;
    w->tpart = reinterpret_cast<float*>(q); q += sz_tpart;
    w->tail_slots = ts;
    w->pheads = reinterpret_cast<float*>(q); q += sz_seam;
    w->ptails = reinterpret_cast<float*>(q); q += sz_seam;
    w->seam_slots = ss;
    w->pstate = reinterpret_cast<avz::PieceState*>(q); q += 4 * sz_b;
    w->xpend = units ? reinterpret_cast<uint32_t*>(q) : nullptr; q += sz_xp;
    w->xdfr = units ? reinterpret_cast<uint32_t*>(q) : nullptr; q += sz_xd;
    w->xunc = units ? reinterpret_cast<uint32_t*>(q) : nullptr; q += sz_xu;
    w->xst = units ? reinterpret_cast<uint32_t*>(q) : nullptr; q += sz_xs;
    w->xst_bytes = sz_xs;
    w->xst_units = units;
    w->xres = units ? reinterpret_cast<float*>(q) : nullptr; q += sz_xr;
  }
  return sz_part + sz_mw + sz_coef + 2 * sz_ht + 6 * sz_b + sz_gain + sz_tpart + 2 * sz_seam +
         sz_xp + sz_xd + sz_xu + sz_xs + sz_xr;
}

struct avz_plan {
  avz_config cfg;
  double tau1, tau2;         // far-field delays of the two mics (masked_mvdr.py:28-29)
  int max_frames;
  int nchunk;                // 32-frame chunks of a max_samples utterance
  void* arena;               // steering table, exact-IBM tables + the plan's own workspace
  double* steer;             // [F][4] steering vectors (masked_mvdr.py:22-35), fp64
  double* xtw;               // [N][2] W_N^j, fp64 (exact IBM path)
  float* xwin;               // [N] the reference's fp32 Hann window (exact IBM path)
  float ibm_cert;            // ibm_kappa * 2^-24 (0: no certificate)
  unsigned long long* xstat; // avz_plan_set_ibm_stats (diagnostic) or null
  int synth_variant;         // avz_plan_set_diagnostics (default 2)
  int dbg_ipf;               // avz_plan_set_diagnostics (default 0)
  Workspace ws;              // used by calls that pass no workspace (serialised by contract)
  // diagnostic per-kernel timing (avz_plan_set_timing): two event sets used alternately
  bool timing;
  int n_k;  // kernels timed per call: 4 (all) or 1 (analysis only)
  // per kernel a (start, stop) pair carried by the kernel's own dispatch
  // (hipExtLaunchKernel): no marker packets between the chain's launches
  hipEvent_t ev[2][8];
  bool ev_pending[2];
  int ev_kern[2];  // kernels the set's call launched (avz_chain_kernels bits; others count 0)
  int ev_next;
  int period;      // events on one avz_mvdr_batch call in `period` (avz_plan_set_timing_period)
  long long seen;  // calls since timing was enabled
  double ms_sum[4];
  int ms_calls;
};

static void timing_drain(avz_plan* p, int set) {
  if (!p->ev_pending[set]) return;
  p->ev_pending[set] = false;
  int last = 0;  // the last launched kernel's stop event
  for (int i = 0; i < p->n_k; ++i)
    if ((p->ev_kern[set] >> i) & 1) last = i;
  if (hipEventSynchronize(p->ev[set][2 * last + 1]) != hipSuccess) return;
  for (int i = 0; i < p->n_k; ++i) {
    if (!((p->ev_kern[set] >> i) & 1)) continue;  // folded into another kernel: 0 ms
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, p->ev[set][2 * i], p->ev[set][2 * i + 1]) == hipSuccess)
      p->ms_sum[i] += ms;
  }
  p->ms_calls += 1;
}

static void timing_free(avz_plan* p) {
  if (!p->timing) return;
  for (int s = 0; s < 2; ++s)
    for (int i = 0; i < 8; ++i) (void)hipEventDestroy(p->ev[s][i]);
  p->timing = false;
}

static thread_local std::string g_last_hip;

static int hip_fail(hipError_t e) {
  g_last_hip = hipGetErrorString(e);
  return AVZ_ERR_HIP;
}

extern "C" int avz_version(void) { return 3; }

extern "C" const char* avz_last_hip_error(void) { return g_last_hip.c_str(); }

extern "C" const char* avz_strerror(int code) {
  switch (code) {
    case AVZ_OK: return "ok";
    case AVZ_ERR_ARG: return "invalid argument";
    case AVZ_ERR_SHAPE: return "length, stride or batch outside the plan";
    case AVZ_ERR_HIP: return "HIP runtime error";
    case AVZ_ERR_UNSUPPORTED: return "unsupported configuration";
    case AVZ_ERR_ALIGN: return "pointer or stride not aligned to its element / vector size";
    default: return "unknown error";
  }
}

static bool misaligned(const void* ptr, uintptr_t bytes) {
  return (reinterpret_cast<uintptr_t>(ptr) & (bytes - 1)) != 0;
}

static int frames_for(int len, int hop) { return (len + hop - 1) / hop + 1; }

// scipy.signal.get_window('hann', n) cast to float32 (the reference's STFT window,
// _spectral_py.py:2083-2084): 0.5 + 0.5 cos(fac), fac = np.linspace(-pi, pi, n + 1)[:-1]
// evaluated as numpy does (i * step, then + start; no fused multiply-add).
#pragma clang fp contract(off)
static void ref_window_f32(int n, float* out) {
  const double start = -M_PI, step = (M_PI - start) / n;
  for (int i = 0; i < n; ++i) {
    double y = (double)i * step;
    y = y + start;
    const double c = std::cos(y);
    const double w = 0.5 + 0.5 * c;
    out[i] = (float)w;
  }
}
#pragma clang fp contract(on)

extern "C" int avz_ibm_window(int n, float* out) {
  if ((n != 512 && n != 1024) || !out) return AVZ_ERR_ARG;
  ref_window_f32(n, out);
  return AVZ_OK;
}

extern "C" int avz_plan_create(avz_plan** out, const avz_config* cfg) {
  if (!out || !cfg) return AVZ_ERR_ARG;
  *out = nullptr;
  const avz_config& c = *cfg;
  if (c.n_fft != 512 && c.n_fft != 1024) return AVZ_ERR_UNSUPPORTED;
  if (c.hop != c.n_fft / 2) return AVZ_ERR_UNSUPPORTED;
  if (c.fs <= 0 || c.c_sound <= 0 || !(c.sigma >= 0) || c.max_batch <= 0 ||
      c.max_samples < c.n_fft)
    return AVZ_ERR_ARG;
  if (c.mask_mode < AVZ_MASK_IBM || c.mask_mode > AVZ_MASK_ONES) return AVZ_ERR_ARG;
  if (c.postfilter < AVZ_PF_NONE || c.postfilter > AVZ_PF_IRM) return AVZ_ERR_ARG;
  if ((c.postfilter == AVZ_PF_IBM_TARGET || c.postfilter == AVZ_PF_IRM) &&
      c.mask_mode != AVZ_MASK_IBM)
    return AVZ_ERR_ARG;
  if (c.singular_fallback != AVZ_FALLBACK_MIC0 && c.singular_fallback != AVZ_FALLBACK_MEAN &&
      c.singular_fallback != AVZ_FALLBACK_BATCH)
    return AVZ_ERR_ARG;
  if ((c.postfilter == AVZ_PF_EXT_FLOOR || c.postfilter == AVZ_PF_EXT_MUL) &&
      c.mask_mode != AVZ_MASK_EXTERNAL)
    return AVZ_ERR_ARG;
  if (c.normalize != AVZ_NORM_NONE && c.normalize != AVZ_NORM_PEAK) return AVZ_ERR_ARG;
  if (c.beamformer != AVZ_BF_MVDR && c.beamformer != AVZ_BF_HYBRID_NULL) return AVZ_ERR_ARG;
  if (c.beamformer == AVZ_BF_HYBRID_NULL && !(c.cond_max >= 1.0)) return AVZ_ERR_ARG;

  avz_plan* p = new (std::nothrow) avz_plan();
  if (!p) return AVZ_ERR_ARG;
  p->cfg = c;
  // masked_mvdr.py:22-35: tau_m1 = (d/2) cos(phi) cos(theta - 0)/c, tau_m2 with theta - pi
  const double theta = c.angle_deg * (M_PI / 180.0);  // np.deg2rad
  p->tau1 = (c.mic_d / 2) * std::cos(0.0) * std::cos(theta - 0) / c.c_sound;
  p->tau2 = (c.mic_d / 2) * std::cos(0.0) * std::cos(theta - M_PI) / c.c_sound;
  p->max_frames = frames_for(c.max_samples, c.hop);
  const int F = c.n_fft / 2 + 1;
  {
    p->nchunk = (p->max_frames + avz_chunk_frames() - 1) / avz_chunk_frames();
    const int N = c.n_fft;
    const size_t sz_steer = align256(sizeof(double) * F * 4);
    const size_t sz_xtw = align256(sizeof(double) * N * 2), sz_xwin = align256(sizeof(float) * N);
    const size_t sz_tab = sz_steer + sz_xtw + sz_xwin;
    const size_t sz_ws = ws_layout(c, c.max_batch, p->nchunk, nullptr, nullptr);
    hipError_t e = hipMalloc(&p->arena, sz_tab + sz_ws);
    if (e != hipSuccess) {
      delete p;
      return hip_fail(e);
    }
    char* q = static_cast<char*>(p->arena);
    p->steer = reinterpret_cast<double*>(q);
    p->xtw = reinterpret_cast<double*>(q + sz_steer);
    p->xwin = reinterpret_cast<float*>(q + sz_steer + sz_xtw);
    ws_layout(c, c.max_batch, p->nchunk, q + sz_tab, &p->ws);
    if (p->ws.xst) {  // the exact path's work-sharing state starts closed (launches leave it so)
      e = hipMemset(p->ws.xst, 0, p->ws.xst_bytes);
      if (e != hipSuccess) {
        (void)hipFree(p->arena);
        delete p;
        return hip_fail(e);
      }
    }
    const double kappa = c.ibm_kappa == 0.0 ? AVZ_IBM_KAPPA : c.ibm_kappa;
    p->ibm_cert = kappa > 0.0 ? (float)(kappa * 0x1p-24) : 0.0f;
    p->xstat = nullptr;
    p->synth_variant = 2;
    p->dbg_ipf = 0;
    // exact IBM path: W_N^j = exp(-2 pi i j / N) (long double argument, rounded once) and the
    // reference's fp32 window
    std::vector<double> xt((size_t)N * 2);
    for (int j = 0; j < N; ++j) {
      const long double a = -2.0L * 3.141592653589793238462643383279502884L * j / N;
      xt[2 * j] = (double)cosl(a);
      xt[2 * j + 1] = (double)sinl(a);
    }
    std::vector<float> xw((size_t)N);
    ref_window_f32(N, xw.data());
    // d_m(f_k) = exp(-1j * (2 pi f_k) * tau_m), f_k = np.fft.rfftfreq(n_fft, 1/fs)[k]
    // (masked_mvdr.py:22-35); the hybrid null beamformer phase-normalises it to mic 0,
    // v / (v[0] + 1e-10) (Final_pipeline/src/inference.py:16-26).
    std::vector<double> st((size_t)F * 4);
    const double df = 1.0 / (c.n_fft * (1.0 / c.fs));
    for (int k = 0; k < F; ++k) {
      const double omega = 2 * M_PI * (k * df);
      const std::complex<double> v0 = std::exp(std::complex<double>(0.0, -omega * p->tau1));
      const std::complex<double> v1 = std::exp(std::complex<double>(0.0, -omega * p->tau2));
      std::complex<double> d0 = v0, d1 = v1;
      if (c.beamformer == AVZ_BF_HYBRID_NULL) {
        const std::complex<double> den = v0 + 1e-10;
        d0 = v0 / den;
        d1 = v1 / den;
      }
      st[4 * k + 0] = d0.real();
      st[4 * k + 1] = d0.imag();
      st[4 * k + 2] = d1.real();
      st[4 * k + 3] = d1.imag();
    }
    e = hipMemcpy(p->steer, st.data(), sizeof(double) * st.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess)
      e = hipMemcpy(p->xtw, xt.data(), sizeof(double) * xt.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess)
      e = hipMemcpy(p->xwin, xw.data(), sizeof(float) * xw.size(), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      (void)hipFree(p->arena);
      delete p;
      return hip_fail(e);
    }
  }
  *out = p;
  return AVZ_OK;
}

extern "C" int avz_plan_destroy(avz_plan* p) {
  if (!p) return AVZ_ERR_ARG;
  timing_free(p);
  if (p->arena) (void)hipFree(p->arena);
  delete p;
  return AVZ_OK;
}

extern "C" int avz_plan_get_config(const avz_plan* p, avz_config* cfg) {
  if (!p || !cfg) return AVZ_ERR_ARG;
  *cfg = p->cfg;
  return AVZ_OK;
}

extern "C" int avz_num_frames(const avz_plan* p, int len) {
  if (!p || len < p->cfg.n_fft) return AVZ_ERR_SHAPE;
  return frames_for(len, p->cfg.hop);
}

static int chunks_for(int max_len, int hop) {
  return (frames_for(max_len, hop) + avz_chunk_frames() - 1) / avz_chunk_frames();
}

extern "C" long long avz_mvdr_workspace_bytes(const avz_plan* p, int batch, int max_len) {
  if (!p || batch < 0 || batch > p->cfg.max_batch) return AVZ_ERR_SHAPE;
  if (max_len < p->cfg.n_fft || max_len > p->cfg.max_samples) return AVZ_ERR_SHAPE;
  return (long long)ws_layout(p->cfg, batch, chunks_for(max_len, p->cfg.hop), nullptr, nullptr);
}

// Solve / post-filter parameters of the plan (shared by every chain and spectral call).
static void plan_params(const avz_plan* p, avz::ChainArgs& k) {
  const avz_config& c = p->cfg;
  k.fs = c.fs;
  k.sigma = c.sigma;
  k.tau1 = p->tau1;
  k.tau2 = p->tau2;
  k.mic_d = c.mic_d;
  k.c_sound = c.c_sound;
  k.fmin_hz = c.fmin_hz;
  k.weight_eps = (float)c.weight_eps;
  k.pf_floor = (float)c.pf_floor;
  k.norm_eps = (float)c.norm_eps;
  k.postfilter = c.postfilter;
  k.normalize = c.normalize;
  k.singular_fallback = c.singular_fallback;
  k.beamformer = c.beamformer;
  k.bypass_hz = c.bypass_hz;
  k.cond_max = c.cond_max;
  k.steer = p->steer;
  k.ibm_cert = p->ibm_cert;
  k.xwin = p->xwin;
  k.xtw = p->xtw;
  k.xstat = p->xstat;
  k.synth_variant = p->synth_variant;
  k.dbg_ipf = p->dbg_ipf;
}

enum { USE_CHAIN = 0, USE_COVARIANCE = 1, USE_APPLY = 2 };

// Validates a time-domain batch call and fills the kernels' argument block: the full
// chain (avz_mvdr_batch), the covariance stage (refs / mask as the plan's mask mode
// needs; cov_out required) or the apply + iSTFT stage (mixture only; ext_mask optional).
static int prepare_chain(const avz_plan* p, const avz_batch_args* a, int use, avz::ChainArgs& k) {
  if (!p || !a) return AVZ_ERR_ARG;
  const avz_config& c = p->cfg;
  if (a->batch < 0 || a->batch > c.max_batch) return AVZ_ERR_SHAPE;
  if (!a->len || !a->mix || (use != USE_COVARIANCE && !a->out)) return AVZ_ERR_ARG;
  if (use == USE_COVARIANCE && !a->cov_out) return AVZ_ERR_ARG;
  if (a->max_len < c.n_fft || a->max_len > c.max_samples) return AVZ_ERR_SHAPE;
  if (a->ch_stride < a->max_len) return AVZ_ERR_SHAPE;
  if (a->batch > 1 && a->mix_stride < a->ch_stride + a->max_len) return AVZ_ERR_SHAPE;
  const int T = frames_for(a->max_len, c.hop);
  const int F = c.n_fft / 2 + 1;
  if (use != USE_COVARIANCE) {
    const long long out_len = (long long)(T - 1) * c.hop;
    if (a->batch > 1 && a->out_stride < out_len) return AVZ_ERR_SHAPE;
    if ((a->out_stride & 3) || (reinterpret_cast<uintptr_t>(a->out) & 15)) return AVZ_ERR_ALIGN;
  }
  if (use != USE_APPLY && c.mask_mode == AVZ_MASK_IBM) {
    if (!a->ref_tgt || !a->ref_int) return AVZ_ERR_ARG;
    if (a->batch > 1 && a->ref_stride < a->max_len) return AVZ_ERR_SHAPE;
  }
  const bool needs_mask = use == USE_APPLY ? a->ext_mask != nullptr
                                           : c.mask_mode == AVZ_MASK_EXTERNAL;
  if (use != USE_APPLY && c.mask_mode == AVZ_MASK_EXTERNAL && !a->ext_mask) return AVZ_ERR_ARG;
  // the kernels read M[b][k][t] for every bin and every frame of the longest utterance
  if (needs_mask && (a->mask_bins < F || a->mask_frames < T)) return AVZ_ERR_SHAPE;
  Workspace ws = p->ws;
  int nchunk = p->nchunk;
  if (a->workspace) {
    nchunk = chunks_for(a->max_len, c.hop);
    if (reinterpret_cast<uintptr_t>(a->workspace) & 255) return AVZ_ERR_ALIGN;
    if (a->workspace_bytes < (long long)ws_layout(c, a->batch, nchunk, nullptr, nullptr))
      return AVZ_ERR_SHAPE;
    ws_layout(c, a->batch, nchunk, static_cast<char*>(a->workspace), &ws);
  }
  k = avz::ChainArgs{};
  k.xst_reset = (a->workspace && ws.xst) ? (long long)ws.xst_bytes : 0;
  plan_params(p, k);
  k.batch = a->batch;
  k.len = a->len;
  k.max_len = a->max_len;
  k.mix = a->mix;
  k.mix_stride = a->mix_stride;
  k.ch_stride = a->ch_stride;
  k.ref_tgt = a->ref_tgt;
  k.ref_int = a->ref_int;
  k.ref_stride = a->ref_stride;
  k.ext_mask = needs_mask ? a->ext_mask : nullptr;
  k.mask_sb = a->mask_stride_b;
  k.mask_sf = a->mask_stride_f;
  k.mask_st = a->mask_stride_t;
  k.out = a->out;
  k.out_stride = a->out_stride;
  k.peak = a->peak;
  k.cov_out = a->cov_out;
  k.w_out = a->w_out;
  k.max_frames = T;
  k.nchunk = nchunk;
  k.part = ws.part;
  k.mwords = ws.mwords;
  k.coef = ws.coef;
  k.heads = ws.heads;
  k.tails = ws.tails;
  k.peak_u = ws.peak_u;
  k.flag = ws.flag;
  k.pf_gain = ws.pf_gain;
  k.tpart = ws.tpart;
  k.tpart_slots = ws.tail_slots;
  k.pheads = ws.pheads;
  k.ptails = ws.ptails;
  k.pseam_slots = ws.seam_slots;
  k.pstate = ws.pstate;
  k.xpend = ws.xpend;
  k.xdfr = ws.xdfr;
  k.xunc = ws.xunc;
  k.xst = ws.xst;
  k.xres = ws.xres;
  k.xhint = ws.xst ? ws.xst + 2 * (ws.xst_units) : nullptr;
  if (use == USE_COVARIANCE) {  // that stage produces cov_out only: leave the caller's
    k.out = nullptr;            // out / peak / w buffers untouched (the analysis kernel
    k.peak = nullptr;           // would otherwise zero peak[b] as the atomicMax target)
    k.w_out = nullptr;
  }
  return AVZ_OK;
}

static int hip_rc(int rc) {
  if (rc == AVZ_ERR_HIP) g_last_hip = hipGetErrorString(hipGetLastError());
  return rc;
}

extern "C" int avz_mvdr_batch(const avz_plan* p, const avz_batch_args* a, void* stream) {
  if (p && a && a->batch == 0) return AVZ_OK;
  avz::ChainArgs k;
  const int e = prepare_chain(p, a, USE_CHAIN, k);
  if (e != AVZ_OK) return e;
  avz_plan* mp = const_cast<avz_plan*>(p);  // diagnostic timing state only (not thread-safe)
  void* evs[8];
  int set = -1;
  if (mp->timing && (mp->seen++ % mp->period) == 0) {
    set = mp->ev_next;
    mp->ev_next ^= 1;
    timing_drain(mp, set);  // the call two back: the previous call keeps the GPU busy
    for (int i = 0; i < 8; ++i) evs[i] = mp->ev[set][i];
    k.events = evs;
    k.n_events = 2 * mp->n_k;
  }
  if (k.xst_reset && hipMemsetAsync(k.xst, 0, (size_t)k.xst_reset, (hipStream_t)stream) != hipSuccess)
    return hip_rc(AVZ_ERR_HIP);
  const int rc = hip_rc(avz_launch_chunked(p->cfg.n_fft, p->cfg.mask_mode, &k, stream));
  if (set >= 0 && rc == AVZ_OK) {
    mp->ev_pending[set] = true;
    mp->ev_kern[set] = avz_chain_kernels(p->cfg.n_fft, &k);
  }
  return rc;
}

extern "C" int avz_mvdr_covariance(const avz_plan* p, const avz_batch_args* a, void* stream) {
  if (p && a && a->batch == 0) return AVZ_OK;
  avz::ChainArgs k;
  const int e = prepare_chain(p, a, USE_COVARIANCE, k);
  if (e != AVZ_OK) return e;
  if (k.xst_reset && hipMemsetAsync(k.xst, 0, (size_t)k.xst_reset, (hipStream_t)stream) != hipSuccess)
    return hip_rc(AVZ_ERR_HIP);
  return hip_rc(avz_launch_covariance(p->cfg.n_fft, p->cfg.mask_mode, &k, stream));
}

extern "C" int avz_apply_istft(const avz_plan* p, const avz_batch_args* a, const float* w,
                               void* stream) {
  if (p && a && a->batch == 0) return AVZ_OK;
  if (!w || (reinterpret_cast<uintptr_t>(w) & 15)) return w ? AVZ_ERR_ALIGN : AVZ_ERR_ARG;
  avz::ChainArgs k;
  const int e = prepare_chain(p, a, USE_APPLY, k);
  if (e != AVZ_OK) return e;
  return hip_rc(avz_launch_apply_istft(p->cfg.n_fft, &k, w, stream));
}

extern "C" int avz_istft(const avz_plan* p, int batch, int frames, const float* S,
                         long long s_stride_b, long long s_stride_f, float* out,
                         long long out_stride, float* peak, void* workspace,
                         long long workspace_bytes, void* stream) {
  if (!p) return AVZ_ERR_ARG;
  const avz_config& c = p->cfg;
  if (batch < 0 || batch > c.max_batch || frames < 0) return AVZ_ERR_SHAPE;
  if (batch == 0) return AVZ_OK;
  if (!S || !out) return AVZ_ERR_ARG;
  if (misaligned(S, 8)) return AVZ_ERR_ALIGN;
  const long long len = (long long)(frames - 1) * c.hop;  // scipy.signal.istft output length
  if (len < c.n_fft || len > c.max_samples) return AVZ_ERR_SHAPE;
  const int F = c.n_fft / 2 + 1;
  if (s_stride_f < frames || (batch > 1 && s_stride_b < (long long)F * s_stride_f))
    return AVZ_ERR_SHAPE;
  if (batch > 1 && out_stride < len) return AVZ_ERR_SHAPE;
  if ((out_stride & 3) || (reinterpret_cast<uintptr_t>(out) & 15)) return AVZ_ERR_ALIGN;
  Workspace ws = p->ws;
  int nchunk = p->nchunk;
  if (workspace) {
    nchunk = chunks_for((int)len, c.hop);
    if (reinterpret_cast<uintptr_t>(workspace) & 255) return AVZ_ERR_ALIGN;
    if (workspace_bytes < (long long)ws_layout(c, batch, nchunk, nullptr, nullptr))
      return AVZ_ERR_SHAPE;
    ws_layout(c, batch, nchunk, static_cast<char*>(workspace), &ws);
  }
  avz::ChainArgs k{};
  plan_params(p, k);
  k.postfilter = AVZ_PF_NONE;
  k.batch = batch;
  k.len = nullptr;  // every item is (frames - 1) hop samples
  k.max_len = (int)len;
  k.max_frames = frames;
  k.spec = S;
  k.spec_sb = s_stride_b;
  k.spec_sf = s_stride_f;
  k.spec_frames = frames;
  k.out = out;
  k.out_stride = out_stride;
  k.peak = peak;
  k.nchunk = nchunk;
  k.heads = ws.heads;
  k.tails = ws.tails;
  k.peak_u = ws.peak_u;
  return hip_rc(avz_launch_istft(c.n_fft, &k, stream));
}

extern "C" int avz_beamform_spectral(const avz_plan* p, const avz_spectral_args* a, void* stream) {
  if (!p || !a) return AVZ_ERR_ARG;
  const avz_config& c = p->cfg;
  if (a->batch < 0 || a->batch > c.max_batch || a->frames < 1) return AVZ_ERR_SHAPE;
  if (a->batch == 0) return AVZ_OK;
  if (!a->Y || !a->mask || !a->S) return AVZ_ERR_ARG;
  // complex64 Y / S (8 B), float mask (4 B): element-aligned, or a GPU fault
  if (misaligned(a->Y, 8) || misaligned(a->S, 8) || misaligned(a->mask, 4))
    return AVZ_ERR_ALIGN;
  if (c.mask_mode != AVZ_MASK_EXTERNAL) return AVZ_ERR_ARG;  // the mask is a target probability
  const int F = c.n_fft / 2 + 1;
  if (a->y_stride_f < a->frames || a->y_stride_m < (long long)F * a->y_stride_f ||
      a->mask_stride_f < a->frames || a->s_stride_f < a->frames)
    return AVZ_ERR_SHAPE;
  if (a->batch > 1 && (a->y_stride_b < 2 * a->y_stride_m ||
                       a->mask_stride_b < (long long)F * a->mask_stride_f ||
                       a->s_stride_b < (long long)F * a->s_stride_f))
    return AVZ_ERR_SHAPE;
  avz::ChainArgs k{};
  plan_params(p, k);
  avz::SpecArgs s{};
  s.batch = a->batch;
  s.frames = a->frames;
  s.Y = a->Y;
  s.y_sb = a->y_stride_b;
  s.y_sm = a->y_stride_m;
  s.y_sf = a->y_stride_f;
  s.M = a->mask;
  s.m_sb = a->mask_stride_b;
  s.m_sf = a->mask_stride_f;
  s.steer = a->steer ? a->steer : p->steer;
  s.S = a->S;
  s.s_sb = a->s_stride_b;
  s.s_sf = a->s_stride_f;
  s.cov_out = a->cov_out;
  s.w_out = a->w_out;
  s.flag = a->fallback ? a->fallback : p->ws.flag;
  return hip_rc(avz_launch_spectral(c.n_fft, &s, &k, stream));
}

extern "C" int avz_solve_covariance(const avz_plan* p, int batch, const double* cov, float* w,
                                    const double* steer, int* fallback, void* stream) {
  if (!p) return AVZ_ERR_ARG;
  if (batch < 0 || batch > p->cfg.max_batch) return AVZ_ERR_SHAPE;
  if (batch == 0) return AVZ_OK;
  if (!cov || !w) return AVZ_ERR_ARG;
  if (misaligned(cov, 8) || misaligned(w, 16) || misaligned(steer, 8)) return AVZ_ERR_ALIGN;
  avz::ChainArgs k{};
  plan_params(p, k);
  avz::SpecArgs s{};
  s.batch = batch;
  s.cov_in = cov;
  s.w_out = w;
  s.steer = steer ? steer : p->steer;
  s.flag = fallback ? fallback : p->ws.flag;
  return hip_rc(avz_launch_solve_cov(p->cfg.n_fft, &s, &k, stream));
}

extern "C" int avz_plan_set_timing(avz_plan* p, int enable) {
  if (!p) return AVZ_ERR_ARG;
  timing_free(p);
  p->ev_pending[0] = p->ev_pending[1] = false;
  p->ev_next = 0;
  p->ms_calls = 0;
  p->seen = 0;
  if (p->period < 1) p->period = 1;
  for (double& m : p->ms_sum) m = 0.0;
  if (!enable) return AVZ_OK;
  if (enable != 1 && enable != 2) return AVZ_ERR_ARG;
  p->n_k = enable == 2 ? 1 : 4;
  for (int s = 0; s < 2; ++s)
    for (int i = 0; i < 8; ++i) {
      const hipError_t e = hipEventCreateWithFlags(&p->ev[s][i], hipEventDisableSystemFence);
      if (e != hipSuccess) {
        for (int t = 0; t <= s; ++t)
          for (int j = 0; j < (t < s ? 8 : i); ++j) (void)hipEventDestroy(p->ev[t][j]);
        return hip_fail(e);
      }
    }
  p->timing = true;
  return AVZ_OK;
}

extern "C" int avz_plan_set_ibm_stats(avz_plan* p, unsigned long long* counts) {
  if (!p) return AVZ_ERR_ARG;
  if (misaligned(counts, 8)) return AVZ_ERR_ALIGN;
  p->xstat = counts;
  return AVZ_OK;
}

extern "C" int avz_plan_set_diagnostics(avz_plan* p, int synth_variant, int ipf_mode) {
  if (!p || synth_variant < 0 || synth_variant > 2 || ipf_mode < 0 || ipf_mode > 2)
    return AVZ_ERR_ARG;
  p->synth_variant = synth_variant;
  p->dbg_ipf = ipf_mode;
  return AVZ_OK;
}

extern "C" int avz_plan_set_timing_period(avz_plan* p, int period) {
  if (!p || period < 1) return AVZ_ERR_ARG;
  p->period = period;
  p->seen = 0;
  return AVZ_OK;
}

extern "C" int avz_plan_get_timing(avz_plan* p, double* ms_avg, int* calls) {
  if (!p || !ms_avg) return AVZ_ERR_ARG;
  if (!p->timing) return AVZ_ERR_ARG;
  timing_drain(p, p->ev_next);
  timing_drain(p, p->ev_next ^ 1);
  for (int i = 0; i < 4; ++i)
    ms_avg[i] = i >= p->n_k ? std::numeric_limits<double>::quiet_NaN()
                                 : (p->ms_calls ? p->ms_sum[i] / p->ms_calls : 0.0);
  if (calls) *calls = p->ms_calls;
  return AVZ_OK;
}

extern "C" int avz_stft(const avz_plan* p, int batch, int channels, const int* len, int max_len,
                        const float* x, long long x_stride, long long ch_stride, float* Y,
                        long long y_stride_b, long long y_stride_c, long long y_stride_f,
                        void* stream) {
  if (!p || !len || !x || !Y) return AVZ_ERR_ARG;
  if (channels != 1 && channels != 2) return AVZ_ERR_ARG;
  if (batch < 0) return AVZ_ERR_SHAPE;
  if (batch == 0) return AVZ_OK;
  if (max_len < p->cfg.n_fft) return AVZ_ERR_SHAPE;
  const int T = frames_for(max_len, p->cfg.hop);
  if (y_stride_f < T) return AVZ_ERR_SHAPE;
  avz::StftArgs s{};
  s.batch = batch;
  s.channels = channels;
  s.len = len;
  s.x = x;
  s.x_stride = x_stride;
  s.ch_stride = ch_stride;
  s.Y = Y;
  s.y_stride_b = y_stride_b;
  s.y_stride_c = y_stride_c;
  s.y_stride_f = y_stride_f;
  s.max_frames = T;
  s.max_len = max_len;
  const int rc = avz_launch_stft(p->cfg.n_fft, &s, stream);
  if (rc == AVZ_ERR_HIP) g_last_hip = hipGetErrorString(hipGetLastError());
  return rc;
}

extern "C" int avz_chunk_split(int n_items, int channels, int chunk, const int* item_utt,
                               const int* item_start, const int* len, const float* x,
                               long long x_stride, long long x_ch_stride, float* items,
                               long long item_stride, long long item_ch_stride, void* stream) {
  if (n_items < 0 || chunk <= 0 || (channels != 1 && channels != 2)) return AVZ_ERR_SHAPE;
  if (n_items == 0) return AVZ_OK;
  if (!item_utt || !item_start || !len || !x || !items) return AVZ_ERR_ARG;
  if (item_ch_stride < chunk && channels > 1) return AVZ_ERR_SHAPE;
  if (n_items > 1 && item_stride < (long long)channels * chunk) return AVZ_ERR_SHAPE;
  avz::ChunkSplitArgs s{};
  s.n_items = n_items;
  s.channels = channels;
  s.chunk = chunk;
  s.item_utt = item_utt;
  s.item_start = item_start;
  s.len = len;
  s.x = x;
  s.x_stride = x_stride;
  s.x_ch_stride = x_ch_stride;
  s.items = items;
  s.item_stride = item_stride;
  s.item_ch_stride = item_ch_stride;
  const int rc = avz_launch_chunk_split(&s, stream);
  if (rc == AVZ_ERR_HIP) g_last_hip = hipGetErrorString(hipGetLastError());
  return rc;
}

extern "C" int avz_chunk_merge(int batch, int max_len, int hop, int item_out_len, const int* len,
                               const int* item_base, const float* item_out,
                               long long item_out_stride, float* y, long long y_stride,
                               float* peak, int normalize, double norm_eps, void* stream) {
  if (batch < 0 || max_len < 0 || hop <= 0 || item_out_len <= 0) return AVZ_ERR_SHAPE;
  if (batch == 0 || max_len == 0) return AVZ_OK;
  if (!len || !item_base || !item_out || !y || !peak) return AVZ_ERR_ARG;
  if (item_out_stride < item_out_len || (batch > 1 && y_stride < max_len)) return AVZ_ERR_SHAPE;
  avz::ChunkMergeArgs m{};
  m.batch = batch;
  m.max_len = max_len;
  m.hop = hop;
  m.item_out_len = item_out_len;
  m.len = len;
  m.item_base = item_base;
  m.item_out = item_out;
  m.item_out_stride = item_out_stride;
  m.y = y;
  m.y_stride = y_stride;
  m.peak = peak;
  m.normalize = normalize != 0;
  m.norm_eps = (float)norm_eps;
  const int rc = avz_launch_chunk_merge(&m, stream);
  if (rc == AVZ_ERR_HIP) g_last_hip = hipGetErrorString(hipGetLastError());
  return rc;
}

extern "C" int avz_mask_features(const avz_plan* p, int layout, int batch, const int* len,
                                 int max_len, const float* x, long long x_stride,
                                 long long ch_stride, float* feat, long long s_b, long long s_c,
                                 long long s_f, long long s_t, void* stream) {
  if (!p || !len || !x || !feat) return AVZ_ERR_ARG;
  if (layout != AVZ_FEAT_LOGMAG_IPD && layout != AVZ_FEAT_TFLITE) return AVZ_ERR_ARG;
  if (batch < 0) return AVZ_ERR_SHAPE;
  if (batch == 0) return AVZ_OK;
  if (max_len < p->cfg.n_fft || max_len > p->cfg.max_samples) return AVZ_ERR_SHAPE;
  if (ch_stride < max_len) return AVZ_ERR_SHAPE;
  avz::StftArgs s{};
  s.batch = batch;
  s.channels = 2;
  s.len = len;
  s.x = x;
  s.x_stride = x_stride;
  s.ch_stride = ch_stride;
  s.max_frames = frames_for(max_len, p->cfg.hop);
  s.max_len = max_len;
  s.feat = layout;
  s.F_out = feat;
  s.f_sb = s_b;
  s.f_sc = s_c;
  s.f_sf = s_f;
  s.f_st = s_t;
  const int rc = avz_launch_stft(p->cfg.n_fft, &s, stream);
  if (rc == AVZ_ERR_HIP) g_last_hip = hipGetErrorString(hipGetLastError());
  return rc;
}

extern "C" int avz_srp_scan(const avz_plan* p, int batch, const int* len, int max_len,
                            const float* mix, long long mix_stride, long long ch_stride,
                            int n_angles, double angle_lo, double angle_hi, double f_lo,
                            double f_hi, double* power_db, void* stream) {
  if (!p || !len || !mix || !power_db) return AVZ_ERR_ARG;
  const avz_config& c = p->cfg;
  if (batch < 0 || batch > c.max_batch || n_angles < 1) return AVZ_ERR_SHAPE;
  if (batch == 0) return AVZ_OK;
  if (max_len < c.n_fft || max_len > c.max_samples || ch_stride < max_len) return AVZ_ERR_SHAPE;
  if (batch > 1 && mix_stride < ch_stride + max_len) return AVZ_ERR_SHAPE;
  avz::ChainArgs k{};
  k.batch = batch;
  k.len = len;
  k.mix = mix;
  k.mix_stride = mix_stride;
  k.ch_stride = ch_stride;
  k.fs = c.fs;
  k.mic_d = c.mic_d;
  k.c_sound = c.c_sound;
  k.max_frames = frames_for(max_len, c.hop);
  k.max_len = max_len;
  k.nchunk = p->nchunk;
  k.part = p->ws.part;
  k.mwords = p->ws.mwords;
  k.peak_u = p->ws.peak_u;
  avz::SrpArgs s{};
  s.n_angles = n_angles;
  s.angle_lo = angle_lo;
  s.angle_hi = angle_hi;
  s.f_lo = f_lo;
  s.f_hi = f_hi;
  s.power_db = power_db;
  const int rc = avz_launch_srp(c.n_fft, &k, &s, stream);
  if (rc == AVZ_ERR_HIP) g_last_hip = hipGetErrorString(hipGetLastError());
  return rc;
}

extern "C" long long avz_scene_workspace_bytes(int batch, int n_src, int n) {
  if (batch <= 0 || n_src <= 0 || n <= 0) return 0;
  return avz_scene_mix_ws(batch, n_src, n);
}

static int scene_check(int batch, int n_src, int n, double fs, double c_sound, float* mix,
                       long long mix_stride, long long ch_stride, float* tgt, float* itf,
                       long long ref_stride, void* workspace) {
  if (batch < 0 || n_src < 1 || n < 2 || (n & 1)) return AVZ_ERR_SHAPE;  // irfft pairs: n even
  if (batch == 0) return AVZ_OK;
  if (!mix || !tgt || !itf || !workspace) return AVZ_ERR_ARG;
  if (!(fs > 0) || !(c_sound > 0)) return AVZ_ERR_ARG;
  if (ch_stride < n || (batch > 1 && (mix_stride < ch_stride + n || ref_stride < n)))
    return AVZ_ERR_SHAPE;
  if (batch > 65535) return AVZ_ERR_UNSUPPORTED;  // grid.y
  return AVZ_OK;
}

static avz::SceneArgs scene_args(int batch, int n_src, int n, double mic_d, double c_sound,
                                 double fs, double sir_db, double snr_db, float* mix,
                                 long long mix_stride, long long ch_stride, float* tgt,
                                 float* itf, long long ref_stride) {
  avz::SceneArgs s{};
  s.batch = batch;
  s.n_src = n_src;
  s.n = n;
  s.mic_d = mic_d;
  s.c_sound = c_sound;
  s.fs = fs;
  s.sir_db = sir_db;
  s.snr_db = snr_db;
  s.mix = mix;
  s.mix_stride = mix_stride;
  s.ch_stride = ch_stride;
  s.tgt = tgt;
  s.itf = itf;
  s.ref_stride = ref_stride;
  return s;
}

extern "C" int avz_scene_mix(int batch, int n_src, int n, const float* src,
                             const double* angles_deg, const float* noise, double mic_d,
                             double c_sound, double fs, double sir_db, double snr_db, float* mix,
                             long long mix_stride, long long ch_stride, float* tgt, float* itf,
                             long long ref_stride, void* workspace, long long workspace_bytes,
                             void* stream) {
  const int rc0 = scene_check(batch, n_src, n, fs, c_sound, mix, mix_stride, ch_stride, tgt, itf,
                              ref_stride, workspace);
  if (rc0 != AVZ_OK || batch == 0) return rc0;
  if (!src || !angles_deg || !noise) return AVZ_ERR_ARG;
  if (workspace_bytes < avz_scene_workspace_bytes(batch, n_src, n)) return AVZ_ERR_SHAPE;
  if (!avz_scene_fft_len(n) && (long long)batch * n_src * 2 > 65535)  // O(n^2) path grid.y
    return AVZ_ERR_UNSUPPORTED;
  avz::SceneArgs s = scene_args(batch, n_src, n, mic_d, c_sound, fs, sir_db, snr_db, mix,
                                mix_stride, ch_stride, tgt, itf, ref_stride);
  s.src = src;
  s.angles_deg = angles_deg;
  s.noise = noise;
  const int rc = avz_launch_scene(&s, workspace, stream);
  if (rc == AVZ_ERR_HIP) g_last_hip = hipGetErrorString(hipGetLastError());
  return rc;
}

extern "C" long long avz_scene_generate_workspace_bytes(int batch, int n_interferers, int n) {
  if (batch <= 0 || n_interferers < 0 || n <= 0) return 0;
  return avz_scene_gen_ws(batch, 1 + n_interferers, n);
}

// source s draws Philox stream s (s <= 255 with 255 interferers) and the mic noise draws
// streams 0x100 + mic, so every stream stays distinct
constexpr int kMaxInterferers = 255;

extern "C" int avz_scene_generate(int batch, long long start_idx, int n_interferers, int n,
                                  unsigned seed, double mic_d, double c_sound, double fs,
                                  double sir_db, double snr_db, float* mix, long long mix_stride,
                                  long long ch_stride, float* tgt, float* itf,
                                  long long ref_stride, void* workspace,
                                  long long workspace_bytes, void* stream) {
  if (n_interferers < 0 || start_idx < 0) return AVZ_ERR_ARG;
  // at most kMaxInterferers (disjoint Philox streams); fs >= 4 keeps the 0.25-s envelope
  // block non-empty
  if (n_interferers > kMaxInterferers || !(fs >= 4.0)) return AVZ_ERR_ARG;
  const int n_src = 1 + n_interferers;
  const int rc0 = scene_check(batch, n_src, n, fs, c_sound, mix, mix_stride, ch_stride, tgt, itf,
                              ref_stride, workspace);
  if (rc0 != AVZ_OK || batch == 0) return rc0;
  if (workspace_bytes < avz_scene_generate_workspace_bytes(batch, n_interferers, n))
    return AVZ_ERR_SHAPE;
  if (!avz_scene_fft_len(n) && (long long)batch * n_src * 2 > 65535)  // O(n^2) path grid.y
    return AVZ_ERR_UNSUPPORTED;
  avz::SceneArgs s = scene_args(batch, n_src, n, mic_d, c_sound, fs, sir_db, snr_db, mix,
                                mix_stride, ch_stride, tgt, itf, ref_stride);
  const int rc = avz_launch_scene_generate(&s, start_idx, seed, workspace, stream);
  if (rc == AVZ_ERR_HIP) g_last_hip = hipGetErrorString(hipGetLastError());
  return rc;
}

extern "C" int avz_projection_metrics_scaled(int batch, int max_len, const int* len,
                                             const float* est, long long est_stride,
                                             const float* est_peak, double est_eps,
                                             const float* tgt, long long tgt_stride,
                                             const float* itf, long long itf_stride,
                                             double* sums, double* metrics, void* stream) {
  if (batch < 0 || max_len < 0) return AVZ_ERR_SHAPE;
  if (batch == 0) return AVZ_OK;
  if (!len || !est || !tgt || !itf || !sums || !metrics) return AVZ_ERR_ARG;
  if (batch > 1 && (est_stride < max_len || tgt_stride < max_len || itf_stride < max_len))
    return AVZ_ERR_SHAPE;
  avz::MetricsArgs m{};
  m.batch = batch;
  m.max_len = max_len;
  m.len = len;
  m.est = est;
  m.tgt = tgt;
  m.itf = itf;
  m.est_stride = est_stride;
  m.tgt_stride = tgt_stride;
  m.itf_stride = itf_stride;
  m.sums = sums;
  m.metrics = metrics;
  m.est_peak = est_peak;
  m.est_eps = est_eps;
  const int rc = avz_launch_metrics(&m, stream);
  if (rc == AVZ_ERR_HIP) g_last_hip = hipGetErrorString(hipGetLastError());
  return rc;
}

extern "C" int avz_projection_metrics(int batch, int max_len, const int* len, const float* est,
                                      long long est_stride, const float* tgt,
                                      long long tgt_stride, const float* itf,
                                      long long itf_stride, double* sums, double* metrics,
                                      void* stream) {
  return avz_projection_metrics_scaled(batch, max_len, len, est, est_stride, nullptr, 0.0, tgt,
                                       tgt_stride, itf, itf_stride, sums, metrics, stream);
}
