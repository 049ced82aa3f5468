/* avz.h — C ABI of the MI355X-native mask-driven MVDR engine (libavz.so).
 *
 * The reference (Senpai-sama06/real-time-audio-visual-zooming) is pure Python and
 * binds no FFI; its operator surface for this path is a set of module-level
 * functions. Each entry point below states the reference interface it replaces
 * (paths relative to the reference root). Host code reaches it through ctypes
 * (real-time-audio-visual-zooming_amd/avz/_lib.py); see INTEGRATION.md.
 *
 * Conventions
 *  - Plain pointers and sizes only. Array pointers are DEVICE pointers (HBM),
 *    caller-owned; strides are in elements. No allocation on the hot call.
 *  - Every function returns 0 on success or a negative AVZ_ERR_* code and never
 *    throws across the ABI (the reference reports errors by print-and-return,
 *    e.g. oracle_debug.py:31-33; singular solves fall back to w = [1, 0],
 *    oracle_debug.py:78-79 — the kernels reproduce that fallback per bin).
 *  - A plan's configuration and steering table are immutable after creation. Every
 *    avz_mvdr_batch call needs a per-call device workspace (chunk partials, mask words,
 *    apply coefficients, seam halves, peak words). A call that passes its own
 *    (avz_batch_args.workspace, sized by avz_mvdr_workspace_bytes) shares nothing
 *    mutable with other calls, so calls with distinct workspaces may run concurrently
 *    on different streams. A call that passes workspace = NULL uses the plan's own
 *    workspace: such calls (and avz_srp_scan, which always uses it) must be ordered
 *    on one stream or otherwise serialised by the caller. The diagnostic timing state
 *    (avz_plan_set_timing) is not thread-safe.
 *  - Device lengths len[b] are clamped to the call's host-validated max_len in every
 *    kernel, so an inconsistent len[] cannot move an access outside the caller's rows.
 */
#ifndef AVZ_H_
#define AVZ_H_

#ifdef __cplusplus
extern "C" {
#endif

#define AVZ_OK 0
#define AVZ_ERR_ARG (-1)         /* null/invalid argument                       */
#define AVZ_ERR_SHAPE (-2)       /* length/stride/batch outside the plan        */
#define AVZ_ERR_HIP (-3)         /* HIP runtime error (launch / allocation)     */
#define AVZ_ERR_UNSUPPORTED (-4) /* configuration not implemented              */
#define AVZ_ERR_ALIGN (-5)       /* pointer/stride below its element/vector alignment */

/* mask sources */
#define AVZ_MASK_IBM 0      /* oracle ideal binary mask from refs, oracle_debug.py:49-53  */
#define AVZ_MASK_IPD 1      /* heuristic phase mask, masked_mvdr.py:37-46                 */
#define AVZ_MASK_EXTERNAL 2 /* caller-provided target probability M, noise = 1 - M,
                               full_audio_generating_pipeline/inference.py:99-106          */
#define AVZ_MASK_ONES 3     /* every bin weight 1: full-signal covariance (MPDR; the SRP
                               scan's R, scripts/debug_srp.py:56-59)                       */

/* post-filters (A10) */
#define AVZ_PF_NONE 0       /* masked_mvdr.py: none                                      */
#define AVZ_PF_IBM_TARGET 1 /* x (1 - mask_noise), oracle_debug.py:84-90                 */
#define AVZ_PF_EXT_FLOOR 2  /* x max(M, floor), full_audio.../inference.py:116           */
#define AVZ_PF_EXT_MUL 3    /* x M, Final_pipeline/src/inference.py:219                  */
#define AVZ_PF_IRM 4        /* x sqrt(|S_t|^2 / (|S_t|^2 + |S_i|^2 + 1e-10)) from the two
                               references (AVZ_MASK_IBM only), oracle_reverb.py:143-156   */

/* weights of a bin whose loaded covariance is singular (A8) */
#define AVZ_FALLBACK_MIC0 0 /* w = [1, 0], oracle_debug.py:78-79, masked_mvdr.py:120-122  */
#define AVZ_FALLBACK_MEAN 1 /* w = ones/2, oracle_reverb.py:133-135                       */
#define AVZ_FALLBACK_BATCH 2 /* batch_mvdr (tf_lite_version/inference.py:143-157): one
                               np.linalg.solve over all bins of a call, so a singular bin sends
                               EVERY bin of that item to w~ = [1, 0]^T, which is then
                               normalised like the others: w = [1/(conj(d0) + 1e-10), 0]     */

/* beamformers (A8 / A14) */
#define AVZ_BF_MVDR 0       /* (R/(sum m + 1e-6) + sigma I)^-1 d, normalised; oracle_debug.py:66-79 */
#define AVZ_BF_HYBRID_NULL 1 /* principal eigenvector of the noise covariance as a hard null
                               next to the phase-normalised target steering vector; delay-and-sum
                               when cond([v_tgt, v_int]) > cond_max; mic 0 below bypass_hz;
                               Final_pipeline/src/inference.py:16-98                          */

/* output normalisation (A12) */
#define AVZ_NORM_NONE 0     /* un-normalised; peak[] reports max|out|                     */
#define AVZ_NORM_PEAK 1     /* out /= (max|out| + norm_eps), oracle_debug.py:94 (eps 0),
                               masked_mvdr.py:128 (eps 1e-6)                              */

typedef struct avz_config {
  int fs;            /* sample rate, masked_mvdr.py:9 (16000)                         */
  int n_fft;         /* 512 (rt_av_zoom core) or 1024 (Final_pipeline/config.py:15)   */
  int hop;           /* must be n_fft/2 (every reference call site uses 50% overlap)  */
  double sigma;      /* diagonal loading: 1 (oracle_debug.py:24), 1e-7, 1e-5          */
  double angle_deg;  /* target direction, 90 (masked_mvdr.py:12)                     */
  double mic_d;      /* mic spacing in m: 0.01 (masked_mvdr.py:10), 0.04, 0.08        */
  double c_sound;    /* 343 (masked_mvdr.py:11)                                      */
  double fmin_hz;    /* bins with f < fmin get w = 0 (oracle_debug.py:67: 100)       */
  int mask_mode;     /* AVZ_MASK_*                                                   */
  int postfilter;    /* AVZ_PF_*                                                     */
  double pf_floor;   /* floor for AVZ_PF_EXT_FLOOR (0.05)                           */
  double weight_eps; /* covariance weight sqrt(m + eps)^2: 0, or 1e-10 as in
                        tf_lite_version/inference.py:109                            */
  int normalize;     /* AVZ_NORM_*                                                   */
  double norm_eps;   /* 0 (oracle_debug), 1e-6 (masked_mvdr), 1e-9 (oracle_reverb)   */
  int max_batch;     /* utterances per call                                          */
  int max_samples;   /* longest utterance (samples)                                  */
  int beamformer;    /* AVZ_BF_*                                                     */
  double bypass_hz;  /* AVZ_BF_HYBRID_NULL: bins with f < bypass_hz pass mic 0 (200)  */
  double cond_max;   /* AVZ_BF_HYBRID_NULL: delay-and-sum above this 2-norm condition
                        number of [v_tgt, v_int] (10, inference.py:80)               */
  int singular_fallback; /* AVZ_FALLBACK_*                                            */
  double ibm_kappa;  /* AVZ_MASK_IBM, reference-exact decisions (oracle_debug.py:42-53):
                        every (bin, frame) decision of the fp32 reference transform must
                        clear an error bound of ibm_kappa * 2^-24 * ||windowed frame||, or
                        the frame's decision is recomputed from fp64 reference spectra
                        rounded to complex64 with numpy's |.|.
                        0 = AVZ_IBM_KAPPA; < 0 = no certificate (fp32 decisions only). */
} avz_config;
/* 16: the bound 3.9 kappa eps ||z|| max|Z| covers the largest fp32-transform error seen in
 * 1.5 M decisions of the configs[1] generator (49 eps ||z|| max|Z|, tools/dbg/kappa_sweep.py
 * and DESIGN.md section 2) by 1.27x; each doubling of kappa adds ~1 % of the frames. */
#define AVZ_IBM_KAPPA 16.0

typedef struct avz_plan avz_plan;

/* Fused batch call. Replaces, per utterance b, the body of
 * rt_av_zoom/core/oracle_debug.py:42-94 (IBM), rt_av_zoom/core/masked_mvdr.py:76-128
 * (IPD) and full_audio_generating_pipeline/inference.py:88-118 (external mask):
 * STFT -> mask -> masked covariance -> MVDR solve -> apply + post-filter -> iSTFT
 * (-> peak normalise). out[b] has (ceil(len[b]/hop)) * hop samples
 * (scipy.signal.istft length). */
typedef struct avz_batch_args {
  int batch;
  const int* len;          /* [batch] samples per utterance (device), n_fft <= len <= max_samples */
  int max_len;             /* host-side upper bound of len[] (validated against strides)         */
  const float* mix;        /* [batch][2][ch_stride]: mic channels planar (y_mix [2,S])          */
  long long mix_stride;    /* elements between utterances                                       */
  long long ch_stride;     /* elements between the two mic channels                             */
  const float* ref_tgt;    /* [batch][ref_stride] target reference (IBM) or NULL                */
  const float* ref_int;    /* [batch][ref_stride] interference reference (IBM) or NULL          */
  long long ref_stride;
  const float* ext_mask;   /* target probability M[b][k][t] (EXTERNAL) or NULL                   */
  long long mask_stride_b, mask_stride_f, mask_stride_t;
  float* out;              /* [batch][out_stride], out_stride % 4 == 0, 16-byte aligned          */
  long long out_stride;
  float* peak;             /* [batch] max|out| before normalisation, or NULL                    */
  double* cov_out;         /* debug: [batch][F][5] sum m|y0|^2, sum m|y1|^2, Re/Im sum m y0 y1*,
                              sum m   (or NULL)                                                  */
  float* w_out;            /* debug: [batch][F][4] Re w0, Im w0, Re w1, Im w1 (or NULL)         */
  int mask_bins;           /* EXTERNAL: bins of ext_mask (>= F) and frames (>= frames of max_len) */
  int mask_frames;
  void* workspace;         /* per-call device workspace (256-byte aligned), or NULL: the plan's */
  long long workspace_bytes; /* >= avz_mvdr_workspace_bytes(plan, batch, max_len)              */
} avz_batch_args;

int avz_plan_create(avz_plan** plan, const avz_config* cfg);
int avz_plan_destroy(avz_plan* plan);
int avz_plan_get_config(const avz_plan* plan, avz_config* cfg);
/* Frames of an utterance of len samples: ceil(len/hop) + 1 (scipy padded/boundary). */
int avz_num_frames(const avz_plan* plan, int len);
int avz_mvdr_batch(const avz_plan* plan, const avz_batch_args* args, void* hip_stream);
/* Device bytes of a per-call workspace for `batch` utterances of at most max_len samples
 * (negative AVZ_ERR_* on bad arguments). */
long long avz_mvdr_workspace_bytes(const avz_plan* plan, int batch, int max_len);

/* ------------------------------------------------------------------ stage exports
 * The chain of avz_mvdr_batch, one stage at a time (stage-wise parity with
 * rt_av_zoom/core/oracle_debug.py:42-64 / :66-79 / :80-94):
 *  avz_mvdr_covariance  STFT -> mask -> masked covariance sums, args->cov_out[b][F][5]
 *                       (sum m|y0|^2, sum m|y1|^2, Re/Im sum m y0 y1*, sum m; fp64);
 *                       args->out unused. Inputs as avz_mvdr_batch for the plan's mask mode.
 *  avz_solve_covariance cov[b][F][5] -> weights w[b][F][4] (Re w0, Im w0, Re w1, Im w1;
 *                       16-byte aligned) with the plan's beamformer, sigma, fmin and
 *                       fallback; steer = optional [F][2] complex128 steering vectors
 *                       (NULL: the plan's); fallback = optional [batch] flags (NULL: the
 *                       plan's own buffer, calls then serialised).
 *  avz_apply_istft      STFT of args->mix -> S = w^H y (x args->ext_mask as a gain when
 *                       non-NULL, mask_bins / mask_frames as for EXTERNAL) -> iSTFT/OLA ->
 *                       args->out (peak-normalised per the plan), args->peak.
 * Device arrays; the same workspace rules as avz_mvdr_batch. */
int avz_mvdr_covariance(const avz_plan* plan, const avz_batch_args* args, void* hip_stream);
int avz_solve_covariance(const avz_plan* plan, int batch, const double* cov, float* w,
                         const double* steer, int* fallback, void* hip_stream);
int avz_apply_istft(const avz_plan* plan, const avz_batch_args* args, const float* w,
                    void* hip_stream);

/* ------------------------------------------------------------------ spectral domain
 * For callers that already hold an STFT. avz_beamform_spectral replaces, per item b,
 *  - beamformer AVZ_BF_MVDR: batch_mvdr(Y, mask, f_bins, d_vectors, sigma)
 *    (rt_av_zoom/core/tf_lite_version/inference.py:85-179; plan: weight_eps 1e-10,
 *    fmin_hz 0, singular_fallback AVZ_FALLBACK_BATCH, sigma = SIGMA);
 *  - beamformer AVZ_BF_HYBRID_NULL: hybrid_hard_null_bf(Y, mask, f_bins)
 *    (Final_pipeline/src/inference.py:28-98; plan: weight_eps 0, bypass_hz 200,
 *    cond_max 10),
 * with the plan's post-filter fused (AVZ_PF_EXT_FLOOR: x max(M, pf_floor), the TFLite
 * driver's S_out * np.maximum(mask, 0.05), inference.py:350; AVZ_PF_EXT_MUL: x M,
 * Final_pipeline/src/inference.py:219; AVZ_PF_NONE: the bare operator). The plan's mask
 * mode must be AVZ_MASK_EXTERNAL (mask = target probability, noise weight 1 - M).
 * Y: complex64 [b][m][k][t] (interleaved re/im; m = mic 0, 1; t contiguous), strides in
 * complex elements; mask [b][k][t] float; S: complex64 [b][k][t]. steer: optional [F][2]
 * complex128 (batch_mvdr's d_vectors; NULL: the plan's table). Y and S 8-byte, mask 4-byte
 * aligned (else AVZ_ERR_ALIGN). cov_out / w_out: optional
 * per-bin covariance sums / weights; fallback: optional [batch] int flags (1 where an
 * item took the item-level fallback; NULL: the plan's own buffer). */
typedef struct avz_spectral_args {
  int batch;               /* items (one reference call each)                              */
  int frames;              /* T frames per item                                            */
  const float* Y;
  long long y_stride_b, y_stride_m, y_stride_f;
  const float* mask;
  long long mask_stride_b, mask_stride_f;
  const double* steer;
  float* S;
  long long s_stride_b, s_stride_f;
  double* cov_out;
  float* w_out;
  int* fallback;
} avz_spectral_args;
int avz_beamform_spectral(const avz_plan* plan, const avz_spectral_args* args, void* hip_stream);

/* scipy.signal.istft(S, fs, nperseg=n_fft, noverlap=n_fft/2) of complex64 S[b][k][t]
 * (t contiguous; strides in complex elements) for `frames` frames per item: out[b] gets
 * (frames - 1) * hop samples (<= max_samples), peak-normalised per the plan; peak[b] =
 * max|out| before normalisation (or NULL). The same workspace rules as avz_mvdr_batch
 * (workspace bytes: avz_mvdr_workspace_bytes(plan, batch, (frames - 1) * hop)). Replaces
 * the istft calls at oracle_debug.py:93, tf_lite_version/inference.py:352,
 * Final_pipeline/src/inference.py:222. */
int avz_istft(const avz_plan* plan, int batch, int frames, const float* S, long long s_stride_b,
              long long s_stride_f, float* out, long long out_stride, float* peak,
              void* workspace, long long workspace_bytes, void* hip_stream);

/* Diagnostics: time the kernels of every avz_mvdr_batch call on this plan with HIP
 * events carried by the kernels' own dispatches (hipExtLaunchKernel start / stop events,
 * no marker packets between launches): enable 1 = all four (analysis, solve, synthesis,
 * finalize), 2 = the analysis kernel only, 0 = off; enabling also resets the sums.
 * avz_plan_get_timing waits for the outstanding calls and returns the average
 * milliseconds per kernel over the calls recorded since enabling (NaN for kernels not
 * timed; a kernel folded into another counts 0: with N = 512 or 1024, peak normalisation
 * and the IBM or no post-filter the per-utterance synthesis kernel folds finalize in, and
 * for plain MVDR plans without the item-level fallback or cov / w outputs the solve too --
 * except that a batch below the CU count that the N = 1024 kernel splits into step pieces
 * launches a piece finalize, which the finalize slot then times; the pieces of a partial
 * last round after whole rounds finalize inside the synthesis kernel). Not thread-safe. */
int avz_plan_set_timing(avz_plan* plan, int enable);
/* Time one avz_mvdr_batch call in `period` (>= 1; default 1): the calls in between carry no
 * events, so a sampled timing run costs the other calls nothing. */
int avz_plan_set_timing_period(avz_plan* plan, int period);
int avz_plan_get_timing(avz_plan* plan, double* ms_avg /*[4]*/, int* calls);
/* Diagnostics of the reference-exact IBM path (avz_config.ibm_kappa): every later call on
 * this plan adds to counts[0] the frames decided on the exact path and to counts[1] the
 * (bin, frame) decisions taken there (device array of two unsigned long long, zeroed by the
 * caller; NULL = off). Not thread-safe with calls on the plan. */
int avz_plan_set_ibm_stats(avz_plan* plan, unsigned long long* counts);
/* Diagnostics: kernel-path A/B of this plan's later calls (tests and tools only; the
 * results are the same up to the fp32 association of the partial sums):
 *  synth_variant 2 (default) = the per-utterance synthesis kernel solving its own bins,
 *  1 = the same after the solve kernel, 0 = the two-block chunk grid + finalize kernel;
 *  ipf_mode 0 (default) = the in-kernel piece finalize as shipped, 1 = every piece but its
 *  utterance's last arriver hands its interior back at once, 2 = pieces ignore the published
 *  1/peak until their next utterance's end (the protocol's rare paths, forced).
 * Not thread-safe with calls on the plan. */
int avz_plan_set_diagnostics(avz_plan* plan, int synth_variant, int ipf_mode);
/* The reference's fp32 analysis window, np.float32(scipy.signal.get_window('hann', n)), as the
 * exact IBM path uses it (n = 512 or 1024; host memory; for tests). */
int avz_ibm_window(int n, float* out);

/* Stage API: STFT of [batch][channels][x_stride] real signals into complex64
 * Y[b][c][k][t] (interleaved re/im floats) with element strides; replaces the
 * reference's scipy.signal.stft(x, fs, nperseg=n_fft, noverlap=n_fft/2) calls
 * (oracle_debug.py:42-44, masked_mvdr.py:76, Final_pipeline/src/inference.py:198). */
int avz_stft(const avz_plan* plan, int batch, int channels, const int* len, int max_len,
             const float* x, long long x_stride, long long ch_stride, float* Y,
             long long y_stride_b, long long y_stride_c, long long y_stride_f,
             void* hip_stream);

/* Final_pipeline driver chunking (Final_pipeline/src/inference.py:171-188): copy
 * item i = samples [item_start[i], item_start[i] + chunk) of utterance item_utt[i]
 * (zero beyond len[utt], the driver's np.pad of the tail chunk) for each of
 * `channels` planar channels into items[i][c][0..chunk). Device arrays. */
int avz_chunk_split(int n_items, int channels, int chunk, const int* item_utt,
                    const int* item_start, const int* len, const float* x, long long x_stride,
                    long long x_ch_stride, float* items, long long item_stride,
                    long long item_ch_stride, void* hip_stream);

/* Final_pipeline driver overlap-add (inference.py:224-236): for utterance b with
 * chunks c = 0 .. ceil(len[b]/hop) - 1 stored as items item_base[b] + c, each adding
 * item_out[...][0 .. min(item_out_len, len[b] - c hop)) at sample c hop:
 * y[b][n] = (sum of the covering chunk outputs) / max(count, 1); peak[b] = max|y[b]|;
 * with normalize != 0, y[b] /= peak[b] + norm_eps (1e-9 in the reference). */
int avz_chunk_merge(int batch, int max_len, int hop, int item_out_len, const int* len,
                    const int* item_base, const float* item_out, long long item_out_stride,
                    float* y, long long y_stride, float* peak, int normalize, double norm_eps,
                    void* hip_stream);

/* Mask-model input features straight from the time-domain mic pair (device arrays):
 *  AVZ_FEAT_LOGMAG_IPD: feat[b*s_b + c*s_c + k*s_f + t*s_t], c = 0: log(|Y0| + 1e-7),
 *    c = 1: angle(Y0) - angle(Y1) — the U-Net input of
 *    full_audio_generating_pipeline/inference.py:90-94 (NCHW with s_t = 1);
 *  AVZ_FEAT_TFLITE: c = 0..3: log_mag, sin(ipd), cos(ipd), linspace(0, 1, F)[k] — the
 *    TFLite input of Final_pipeline/src/inference.py:198-203, 117-128 (NHWC: s_c = 1,
 *    s_t = 4, s_f = 4 T).
 * Y = scipy.signal.stft(x, nperseg=n_fft, noverlap=n_fft/2) of the plan's n_fft. */
#define AVZ_FEAT_LOGMAG_IPD 1
#define AVZ_FEAT_TFLITE 2
int avz_mask_features(const avz_plan* plan, int layout, int batch, const int* len, int max_len,
                      const float* x, long long x_stride, long long ch_stride, float* feat,
                      long long s_b, long long s_c, long long s_f, long long s_t,
                      void* hip_stream);

/* Steered response power scan, scripts/debug_srp.py:46-62 for a batch: for the
 * angles np.linspace(angle_lo, angle_hi, n_angles) (degrees, the plan's mic_d and
 * c_sound, debug_srp.py:17-23 geometry), P = sum over bins f_lo <= f <= f_hi and all
 * frames of |d^H y|^2; power_db[b][i] = 10 log10(P_i) - max_j 10 log10(P_j) (device). */
int avz_srp_scan(const avz_plan* plan, int batch, const int* len, int max_len,
                 const float* mix, long long mix_stride, long long ch_stride, int n_angles,
                 double angle_lo, double angle_hi, double f_lo, double f_hi, double* power_db,
                 void* hip_stream);

/* Projection metrics of a batch (device arrays, float32 signals of len[b] samples, the
 * caller having aligned them to the minimum length as metrics.py:91-98 does):
 * metrics[b] = { OSINR, OSIR } of Final_pipeline/src/metrics.py:102-123
 *              (calculate_osnr_osir; output not normalised) and
 *              { SDR, SIR } of scripts/run_metrics.py:6-36 (calculate_metrics_manual),
 * in dB, from fp64 inner products; sums[b][6] is caller-provided workspace
 * (<o,o>, <t,t>, <i,i>, <o,t>, <o,i>, <t,i> on return). */
int avz_projection_metrics(int batch, int max_len, const int* len, const float* est,
                           long long est_stride, const float* tgt, long long tgt_stride,
                           const float* itf, long long itf_stride, double* sums,
                           double* metrics, void* hip_stream);
/* The same metrics of est[b] / (est_peak[b] + est_eps): an un-normalised output (a plan
 * with AVZ_NORM_NONE, whose peak[] it returns) scored as the peak-normalised one without
 * the normalisation pass over the samples (the scale enters the fp64 sums). */
int avz_projection_metrics_scaled(int batch, int max_len, const int* len, const float* est,
                                  long long est_stride, const float* est_peak, double est_eps,
                                  const float* tgt, long long tgt_stride, const float* itf,
                                  long long itf_stride, double* sums, double* metrics,
                                  void* hip_stream);

/* Synthetic scene mixing on the device — the anechoic far-field generator of
 * full_audio_generating_pipeline/world_building.py:47-59 (per-mic fractional delay by an
 * rfft phase shift over the whole signal, d = mic_d, c = c_sound) with the SIR gain
 * (Final_pipeline/src/simulation.py:167-179, on mic 1), AWGN at snr_db per channel
 * (world.py:93-98, noise = sqrt(mean(clean^2)/10^(snr/10)) * z) and the shared peak
 * normalisation of simulation.py:197-202 (peak = max|mix| + 1e-9).
 * src[b][s][0..n) are the mono sources (s = 0 the target, 1..n_src-1 interferers) at
 * angles_deg[b][s]; noise[b][c][0..n) unit-normal draws for mic c. Writes
 * mix[b][c] (at mix_stride / ch_stride), tgt[b] = mic-1 target image / peak,
 * itf[b] = mic-1 interference image / peak. `workspace` holds
 * avz_scene_workspace_bytes(batch, n_src, n) bytes. All arrays device-resident.
 * n even. When n factors into 2, 3 and 5 the delays run as fp64 mixed-radix FFTs
 * (O(n log n)); otherwise as the exact O(n^2) circular convolution. */
long long avz_scene_workspace_bytes(int batch, int n_src, int n);
int avz_scene_mix(int batch, int n_src, int n, const float* src, const double* angles_deg,
                  const float* noise, double mic_d, double c_sound, double fs, double sir_db,
                  double snr_db, float* mix, long long mix_stride, long long ch_stride,
                  float* tgt, float* itf, long long ref_stride, void* workspace,
                  long long workspace_bytes, void* hip_stream);

/* The whole scene on the device (the sharded batch driver's input path): utterance
 * start_idx + b draws from counter-based Philox4x32-10 streams keyed by (start_idx + b,
 * 0x5CE7E5ED ^ seed) — Box-Muller normals for the speech-like sources (AR(2) poles 0.9 /
 * 0.5, |sin(2 pi 4 t + phi)| envelope, 25 % of 250-ms blocks silenced: synth.speech_like)
 * and the AWGN, uniforms for the envelope phases, the kept blocks and the azimuths of
 * interferers 2.. (target 90 deg, interferer 1 at 40 deg) — then avz_scene_mix's model.
 * avz/synth.py make_scene_philox is the host restatement. `workspace` holds
 * avz_scene_generate_workspace_bytes(batch, n_interferers, n) bytes. */
long long avz_scene_generate_workspace_bytes(int batch, int n_interferers, int n);
int avz_scene_generate(int batch, long long start_idx, int n_interferers, int n, unsigned seed,
                       double mic_d, double c_sound, double fs, double sir_db, double snr_db,
                       float* mix, long long mix_stride, long long ch_stride, float* tgt,
                       float* itf, long long ref_stride, void* workspace,
                       long long workspace_bytes, void* hip_stream);

const char* avz_strerror(int code);
/* Last HIP error string recorded by the library on this thread (diagnostics). */
const char* avz_last_hip_error(void);
int avz_version(void);

#ifdef __cplusplus
}
#endif
#endif /* AVZ_H_ */
