// avz_internal.h — host/device shared argument blocks (not part of the public ABI).
#pragma once
#include <stdint.h>

namespace avz {

enum : int { MASK_IBM = 0, MASK_IPD = 1, MASK_EXTERNAL = 2, MASK_ONES = 3 };
enum : int { PF_NONE = 0, PF_IBM_TARGET = 1, PF_EXT_FLOOR = 2, PF_EXT_MUL = 3, PF_IRM = 4 };
enum : int { NORM_NONE = 0, NORM_PEAK = 1 };

enum : int { BF_MVDR = 0, BF_HYBRID_NULL = 1 };

// Everything the analysis / solve / synthesis / finalize chain needs, passed by value.
struct PieceState {
  uint32_t cnt, fin;
  unsigned long long st;
};
static_assert(sizeof(PieceState) == 16, "one 16-B store resets it");

// Pieces a shared unit of the exact IBM path splits into at most (avz_chunked_k.hpp XPieces).
constexpr int kXPieces = 8;

struct ChainArgs {
  int batch;
  const int* len;             // [B] samples per utterance (device; kernels clamp to max_len)
  int max_len;                // host-validated upper bound of len[] (the buffers' extent)
  const float* mix;           // [B][2][..] planar
  long long mix_stride;       // floats between utterances
  long long ch_stride;        // floats between the two mic channels
  const float* ref_tgt;       // [B][..] or null
  const float* ref_int;       // [B][..] or null
  long long ref_stride;
  const float* ext_mask;      // target-probability mask M[b][k][t] or null
  long long mask_sb, mask_sf, mask_st;
  float* out;                 // [B][out_stride]
  long long out_stride;
  float* peak;                // [B] or null: max|out| before normalisation
  double* cov_out;            // [B][F][5] or null: sum m|y0|^2, sum m|y1|^2, Re/Im sum m y0 y1*, sum m
  float* w_out;               // [B][F][4] or null: Re w0, Im w0, Re w1, Im w1
  double fs, sigma, tau1, tau2, fmin_hz;
  double mic_d, c_sound;
  float weight_eps, pf_floor, norm_eps;
  int postfilter, normalize;
  int beamformer;             // BF_*
  double bypass_hz, cond_max; // hybrid null: mic-0 bypass below, delay-and-sum above
  // chunked path workspace (plan-owned)
  int max_frames;             // frames of the longest utterance (grid extent)
  int nchunk;                 // allocated 32-frame chunks per utterance (workspace stride)
  float* part;                // [B][nchunk][5][F] masked covariance partials (fp32)
  uint32_t* mwords;           // [B][nchunk][F] IBM bits, bit i = frame 32 c + i is noise
  const double* steer;        // [F][4] steering vector d0 (re, im), d1 (re, im), fp64
  float* coef;                // [B][F][4] apply coefficients alpha (re, im), beta (re, im)
  float* heads;               // [B][nchunk][H] chunk's first frame, first-half contribution
  float* tails;               // [B][nchunk][H] chunk's last frame, second-half contribution
  uint32_t* peak_u;           // [B] max |out| over chunk interiors (float bits, atomicMax)
  float* pf_gain;             // [B][nchunk][32][F] IRM post-filter gain (PF_IRM) or null
  int singular_fallback;      // 0: w = [1, 0]; 1: w = [1/2, 1/2]
  // spectrum-input synthesis (avz_istft): S[b][k][t] complex64 replaces the forward FFT of
  // the mixture and the apply step (post-filter still applied); len == null means every
  // utterance is max_len samples long
  const float* spec;
  long long spec_sb, spec_sf; // complex elements; t stride 1
  int spec_frames;            // frames present in S (frames >= spec_frames read as zero)
  int cov_only;               // solve kernel: write cov_out only (the covariance stage export)
  int* flag;                  // [B] item-level (batch_mvdr) fallback flags, zeroed per call
  // Tail splitting of the persistent grids (set per launch by the launcher; zero = off).
  // Analysis: items [0, a_whole) run whole, each later (chunk, utterance) item in a_pieces
  // step-range pieces whose partials go to tpart[(item - a_whole) * a_pieces + p][5][F]
  // (the solve sums them in fp64) and whose IBM bits are merged into mwords atomically.
  int a_whole, a_pieces;
  float* tpart;               // [tpart_slots][5][F]
  int tpart_slots;
  // Per-utterance synthesis: utterances [0, s_whole) whole (in-block seams, peak, rescale),
  // utterances [s_whole, batch) in s_pieces pieces of s_steps steps each, whose boundary
  // half-frames go to pheads / ptails[(b - s_whole) * s_pieces + p][H] for the piece
  // finalize kernel (seams, peak, rescale).
  int s_whole, s_pieces, s_steps;
  float* pheads;
  float* ptails;
  int pseam_slots;
  int b_lo;                   // solve launches: first utterance solved (0 in the chain)
  // In-kernel piece finalize (s_ipf = 1; batches with whole rounds): the piece units run
  // first, the last piece of utterance b to arrive (pstate[b].cnt) forms its seams and peak
  // and publishes 1/peak in pstate[b].fin (float bits, 0 = not yet); each piece rescales its
  // own interior during its block's next utterance, or hands it back to that last arriver
  // (pstate[b].st: bit p = piece p handed back, bit 32 + p = the last arriver has passed
  // it). Reset with peak_u by the analysis kernel.
  int s_ipf;
  PieceState* pstate;
  int dbg_ipf;                // diagnostic (avz_plan_set_diagnostics): 1 = every piece but the
                              // last arriver hands itself back at once, 2 = pieces ignore 1/peak
                              // until their next utterance's end (the protocol's rare paths)
  // Reference-exact IBM decisions (avz_ibm_exact.hpp): ibm_cert = kappa * 2^-24, the error
  // bound of the fp32 reference transform per unit of frame norm (0: every decision from the
  // fp32 transform); xwin [N] the reference's fp32 Hann window, xtw [N][2] W_N^j in fp64
  // (plan tables); xstat (optional, [2]): deferred (bin, frame) decisions, exact noise ones.
  float ibm_cert;
  const float* xwin;
  const double* xtw;
  unsigned long long* xstat;
  uint32_t* xpend;            // [units][4] per analysis unit (item b * gx + c, or piece
                              // gx * B + q): frames with a deferred decision, frames deferred
                              // whole, the Nyquist bin's deferrals (IBM plans' workspace)
  uint32_t* xdfr;             // [units][F] per-bin deferred frames (IBM without the
                              // reference-bit hand-off), written only for units with deferrals
  uint32_t* xunc;             // [units][32 frames][32] reference-bit path: the frame's
                              // uncertain bins (word l bit k: bin l + 32 k), deferred frames only
  uint32_t* xst;              // [units][2] exact-path work sharing: state, arrivals (closed
                              // between launches; avz_chunked_k.hpp kXOpen)
  float* xres;                // [units][kXPieces][5][F] a shared unit's piece sums
  uint32_t* xhint;            // [units / 32] published units (one bit each)
  long long xst_reset;        // host-only: bytes of xst to zero before the launch (a caller's
                              // workspace, whose contents the library does not know)
  int synth_variant;          // host-only (avz_plan_set_diagnostics): synthesis path, 2 default
  void* const* events;        // host-only: (start, stop) hipEvent_t pairs of the 4 launches, or null
  int n_events;               // host-only: how many of them to use (8, or 2: analysis only)
};

// Spectral-domain beamformer (avz_beamform_spectral) and the solve stage export
// (avz_solve_covariance). Solve parameters come from a ChainArgs (fs, sigma, fmin_hz,
// weight_eps, singular_fallback, bypass_hz, cond_max, postfilter, pf_floor).
struct SpecArgs {
  int batch, frames;
  const float* Y;             // complex64 Y[b][m][k][t], m = 0, 1 (t contiguous)
  long long y_sb, y_sm, y_sf; // complex elements
  const float* M;             // target probability M[b][k][t] (t contiguous)
  long long m_sb, m_sf;
  const double* steer;        // [F][4] d0 (re, im), d1 (re, im)
  float* S;                   // complex64 S[b][k][t] (t contiguous)
  long long s_sb, s_sf;
  double* cov_out;            // [B][F][5] or null
  float* w_out;               // [B][F][4] or null
  const double* cov_in;       // solve stage: [B][F][5] covariance sums
  int* flag;                  // [B] item-level fallback flags (zeroed by the launcher)
};

struct StftArgs {
  int batch, channels;        // channels 1 or 2
  const int* len;             // clamped to max_len in the kernel
  int max_len;
  const float* x;             // [B][C][..]
  long long x_stride, ch_stride;
  float* Y;                   // complex64 [B][C][F][t_stride] as float2
  long long y_stride_b, y_stride_c, y_stride_f;  // in complex elements
  int max_frames;
  int feat;                   // 0: write Y; FEAT_*: mask-model features into `F_out`
  float* F_out;
  long long f_sb, f_sc, f_sf, f_st;  // feature strides in floats
};
enum : int { FEAT_NONE = 0, FEAT_LOGMAG_IPD = 1, FEAT_TFLITE = 2 };

struct SrpArgs {
  int n_angles;
  double angle_lo, angle_hi;  // np.linspace(angle_lo, angle_hi, n_angles)
  double f_lo, f_hi;          // bins with f_lo <= f <= f_hi
  double* power_db;           // [B][n_angles]
};

struct MetricsArgs {
  int batch, max_len;
  const int* len;             // [B] samples to score (the aligned minimum length)
  const float* est;           // [B][est_stride] output
  const float* tgt;           // [B][tgt_stride] target reference
  const float* itf;           // [B][itf_stride] interference reference
  long long est_stride, tgt_stride, itf_stride;
  double* sums;               // [B][6] workspace
  double* metrics;            // [B][4] OSINR, OSIR, SDR, SIR (dB)
  const float* est_peak;      // [B] or null: score est / (est_peak[b] + est_eps)
  double est_eps;
};

struct ChunkSplitArgs {
  int n_items, channels, chunk;
  const int* item_utt;        // [n_items] source utterance
  const int* item_start;      // [n_items] first sample
  const int* len;             // [B] utterance lengths
  const float* x;             // [B][channels][..]
  long long x_stride, x_ch_stride;
  float* items;               // [n_items][channels][..]
  long long item_stride, item_ch_stride;
};

struct ChunkMergeArgs {
  int batch, max_len, hop, item_out_len;
  const int* len;             // [B]
  const int* item_base;       // [B] index of each utterance's first item
  const float* item_out;      // [n_items][item_out_stride]
  long long item_out_stride;
  float* y;                   // [B][y_stride]
  long long y_stride;
  float* peak;                // [B] max |y| before normalisation
  int normalize;
  float norm_eps;
};

struct SceneArgs {
  int batch, n_src, n;        // utterances, sources per utterance (target first), samples
  const float* src;           // [B][n_src][n]
  const double* angles_deg;   // [B][n_src] azimuths
  const float* noise;         // [B][2][n] unit-normal AWGN draws
  double mic_d, c_sound, fs, sir_db, snr_db;
  float* hk;                  // O(n^2) fallback workspace [B][n_src][2][n] delay kernels
  float* img;                 // O(n^2) fallback workspace [B][n_src][2][n] source images
  float* mix;                 // [B][mix_stride]: mic channels at ch_stride
  long long mix_stride, ch_stride;
  float* tgt;                 // [B][ref_stride] mic-1 target image / peak
  float* itf;                 // [B][ref_stride] mic-1 interference image / peak
  long long ref_stride;
};

}  // namespace avz

extern "C" {
int avz_launch_scene(const avz::SceneArgs* a, void* ws, void* stream);
int avz_launch_scene_generate(avz::SceneArgs* a, long long start, uint32_t seed, void* ws,
                              void* stream);
long long avz_scene_mix_ws(int batch, int n_src, int n);
int avz_scene_fft_len(int n);  // 1: n factors into 8, 4, 2, 5, 3 (the FFT path)
long long avz_scene_gen_ws(int batch, int n_src, int n);
int avz_launch_chunk_split(const avz::ChunkSplitArgs* a, void* stream);
int avz_launch_metrics(const avz::MetricsArgs* a, void* stream);
int avz_launch_chunk_merge(const avz::ChunkMergeArgs* a, void* stream);
int avz_launch_chunked(int n_fft, int mask_mode, const avz::ChainArgs* a, void* stream);
// Kernels avz_launch_chunked launches for these arguments, bit i = kernel i (analysis,
// solve, synthesis, finalize): the per-utterance synthesis folds finalize in (bit 3 clear)
// and, for plain MVDR plans, the solve too (bit 1 clear); unlaunched kernels' events stay
// unrecorded.
int avz_chain_kernels(int n_fft, const avz::ChainArgs* a);
// stage exports: analysis + partial sums -> cov_out; w [B][F][4] -> coef -> synthesis +
// finalize (post-filter PF_NONE or PF_EXT_MUL with ext_mask as the gain); S -> synthesis
// (spectrum input) + finalize
int avz_launch_covariance(int n_fft, int mask_mode, const avz::ChainArgs* a, void* stream);
int avz_launch_apply_istft(int n_fft, const avz::ChainArgs* a, const float* w, void* stream);
int avz_launch_istft(int n_fft, const avz::ChainArgs* a, void* stream);
int avz_launch_spectral(int n_fft, const avz::SpecArgs* s, const avz::ChainArgs* p, void* stream);
int avz_launch_solve_cov(int n_fft, const avz::SpecArgs* s, const avz::ChainArgs* p, void* stream);
int avz_launch_srp(int n_fft, const avz::ChainArgs* a, const avz::SrpArgs* s, void* stream);
int avz_chunk_frames(void);
int avz_launch_stft(int n_fft, const avz::StftArgs* a, void* stream);
}
