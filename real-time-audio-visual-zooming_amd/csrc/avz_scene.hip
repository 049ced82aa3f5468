// avz_scene.hip — on-device synthetic scene generation and mixing (gfx950): the
// reference's anechoic far-field generator, full_audio_generating_pipeline/
// world_building.py:47-59 (per-mic fractional delay by an rfft phase shift over the WHOLE
// signal) with the SIR / AWGN / shared-peak conventions of Final_pipeline/src/
// simulation.py:167-202 (the bench's generator, avz/synth.py make_scene).
//
// Two entry points share the mixing back end:
//  * avz_scene_mix      — sources, angles and unit-normal noise given (the host RNG draws
//                         of synth.scene_draws, so the device scene is the host scene);
//  * avz_scene_generate — everything on the device: counter-based Philox4x32-10 draws
//                         (Box-Muller normals, 53-bit uniforms), the speech-like AR(2)
//                         source model with its syllabic envelope (synth.speech_like), the
//                         interferer azimuths; synth.make_scene_philox is its host restatement.
//
// Fractional delay, O(n log n). Real sources are packed two per complex signal, run
// through a mixed-radix (8, 4, 2, 5, 3) Stockham FFT in fp64, split, multiplied by the
// per-mic phase ramps exp(-2 pi i f tau) with irfft's conventions (DC and Nyquist imaginary
// parts dropped), summed into the target and interference images, packed two mics per
// complex signal and inverse transformed: four length-n FFTs per utterance for up to four
// sources. A length with another prime factor takes the exact O(n^2) circular convolution
// with the periodic kernel h[d] = -(1/n) (-1)^d sin(pi delta) cot(pi (d - delta) / n).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "avz_internal.h"

namespace avz {

// ================================================================ Philox4x32-10 draws
struct U4 {
  uint32_t x, y, z, w;
};
// Random123's philox4x32 with 10 rounds: ctr (c0..c3), key (k0, k1).
__device__ __forceinline__ U4 philox4x32(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                         uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return {c0, c1, c2, c3};
}

// Draw streams of utterance idx (key = (idx, kSceneKey ^ seed)); synth.py mirrors these.
constexpr uint32_t kSceneKey = 0x5CE7E5EDu;
constexpr uint32_t kStreamNoise = 0x100u;  // + mic
constexpr uint32_t kStreamUnif = 0x200u;
constexpr uint32_t kUnifPhase = 0x1000u;     // + source: envelope phase
constexpr uint32_t kUnifKeep = 0x100000u;    // * (1 + source) + block: keep flags
constexpr int kSegLen = 256;                 // AR(2) segment (even: normal pairs stay whole)

__device__ __forceinline__ double u53(uint32_t hi, uint32_t lo) {
  return (double)((((uint64_t)hi << 32) | lo) >> 11) * 0x1p-53;
}
// Normal pair i of a stream: Box-Muller on (u1 in (0, 1], u2 in [0, 1)).
__device__ __forceinline__ void normal_pair(uint32_t k0, uint32_t k1, uint32_t stream, uint32_t i,
                                            double& z0, double& z1) {
  const U4 r = philox4x32(i, stream, 0u, 0u, k0, k1);
  const double u1 = (double)(((((uint64_t)r.x << 32) | r.y) >> 11) + 1) * 0x1p-53;
  const double u2 = u53(r.z, r.w);
  const double rr = sqrt(-2.0 * log(u1));
  double s, c;
  sincospi(2.0 * u2, &s, &c);
  z0 = rr * c;
  z1 = rr * s;
}
__device__ __forceinline__ double uniform(uint32_t k0, uint32_t k1, uint32_t j) {
  const U4 r = philox4x32(j, kStreamUnif, 0u, 0u, k0, k1);
  return u53(r.x, r.y);
}

struct GenArgs {
  int batch, n_src, n, nseg;
  long long start;
  uint32_t seed;
  double fs;
  float* src;          // [B][n_src][n] speech-like sources
  float* noise;        // [B][2][n] unit normals
  double* angles;      // [B][n_src]
  double* zs;          // [B][n_src][nseg][2] zero-state final (y[e], y[e-1]) per segment
  double* sin_;        // [B][n_src][nseg][2] true state entering each segment
};

__device__ __forceinline__ void gen_key(const GenArgs& G, int b, uint32_t& k0, uint32_t& k1) {
  const unsigned long long idx = (unsigned long long)(G.start + b);
  k0 = (uint32_t)idx;
  k1 = (uint32_t)(idx >> 32) ^ kSceneKey ^ G.seed;
}

// AR(2) x -> y[m] = x[m] + 1.4 y[m-1] - 0.45 y[m-2] (lfilter([1], [1, -1.4, 0.45])) over
// segment `seg` from state (y1, y2); FINAL: write source * envelope, else the final state.
template <bool FINAL>
__global__ void __launch_bounds__(256) scene_ar_kernel(GenArgs G) {
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long tot = (long long)G.batch * G.n_src * G.nseg;
  if (t >= tot) return;
  const int seg = (int)(t % G.nseg);
  const int s = (int)((t / G.nseg) % G.n_src);
  const int b = (int)(t / ((long long)G.nseg * G.n_src));
  uint32_t k0, k1;
  gen_key(G, b, k0, k1);
  double y1 = 0.0, y2 = 0.0;
  const long long so = (((long long)b * G.n_src + s) * G.nseg + seg) * 2;
  if (FINAL) {
    y1 = G.sin_[so];
    y2 = G.sin_[so + 1];
  }
  const int m0 = seg * kSegLen, m1 = min(G.n, m0 + kSegLen);
  // envelope |sin(2 pi 4 t + phi)| with phi ~ U(0, pi); 250-ms blocks kept with p = 0.75
  const double phi = M_PI * uniform(k0, k1, kUnifPhase + (uint32_t)s);
  const int blk = (int)(0.25 * G.fs);
  float* out = G.src + ((long long)b * G.n_src + s) * G.n;
  int keep_blk = -1;
  bool keep = true;
  for (int m = m0; m < m1; m += 2) {
    double x[2];
    normal_pair(k0, k1, (uint32_t)s, (uint32_t)(m >> 1), x[0], x[1]);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const double y = x[q] + 1.4 * y1 - 0.45 * y2;
      y2 = y1;
      y1 = y;
      if (FINAL) {
        const int mm = m + q;
        if (mm / blk != keep_blk) {
          keep_blk = mm / blk;
          keep = uniform(k0, k1, kUnifKeep * (1u + (uint32_t)s) + (uint32_t)keep_blk) >= 0.25;
        }
        const double env = keep ? fabs(sin(2.0 * M_PI * 4.0 * ((double)mm / G.fs) + phi)) : 0.0;
        out[mm] = (float)(y * env);
      }
    }
  }
  if (!FINAL) {
    G.zs[so] = y1;
    G.zs[so + 1] = y2;
  }
}

// Segment states: S_j = A^L S_{j-1} + Z_j (A the AR(2) companion matrix); one thread per
// source. Thread s = 0 also draws the utterance's azimuths (target 90, interferer 1 at 40,
// further ones U(0, 180), as synth.make_scene).
__global__ void __launch_bounds__(64) scene_ar_scan_kernel(GenArgs G) {
  const int t = blockIdx.x * 64 + threadIdx.x;
  if (t >= G.batch * G.n_src) return;
  const int b = t / G.n_src, s = t % G.n_src;
  uint32_t k0, k1;
  gen_key(G, b, k0, k1);
  if (s == 0) {
    double* ang = G.angles + (long long)b * G.n_src;
    ang[0] = 90.0;
    if (G.n_src > 1) ang[1] = 40.0;
    for (int k = 2; k < G.n_src; ++k) ang[k] = 180.0 * uniform(k0, k1, (uint32_t)(k - 2));
  }
  // M = A^kSegLen, A = [[1.4, -0.45], [1, 0]]
  double m00 = 1.0, m01 = 0.0, m10 = 0.0, m11 = 1.0;
  for (int i = 0; i < kSegLen; ++i) {
    const double a00 = 1.4 * m00 - 0.45 * m10, a01 = 1.4 * m01 - 0.45 * m11;
    m10 = m00;
    m11 = m01;
    m00 = a00;
    m01 = a01;
  }
  double y1 = 0.0, y2 = 0.0;
  const long long so = ((long long)b * G.n_src + s) * G.nseg * 2;
  for (int j = 0; j < G.nseg; ++j) {
    G.sin_[so + 2 * j] = y1;
    G.sin_[so + 2 * j + 1] = y2;
    const double n1 = m00 * y1 + m01 * y2 + G.zs[so + 2 * j];
    const double n2 = m10 * y1 + m11 * y2 + G.zs[so + 2 * j + 1];
    y1 = n1;
    y2 = n2;
  }
}

__global__ void __launch_bounds__(256) scene_noise_kernel(GenArgs G) {
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  const int half = G.n / 2;
  if (t >= (long long)G.batch * 2 * half) return;
  const int i = (int)(t % half);
  const int c = (int)((t / half) & 1);
  const int b = (int)(t / (2LL * half));
  uint32_t k0, k1;
  gen_key(G, b, k0, k1);
  double z0, z1;
  normal_pair(k0, k1, kStreamNoise + (uint32_t)c, (uint32_t)i, z0, z1);
  float* z = G.noise + ((long long)b * 2 + c) * G.n + 2 * i;
  z[0] = (float)z0;
  z[1] = (float)z1;
}

// ================================================================ mixed-radix FFT (fp64)
struct Rad {
  static constexpr double C8 = 0.70710678118654752440;
  static constexpr double S3 = 0.86602540378443864676;
  static constexpr double C5a = 0.30901699437494742410, S5a = 0.95105651629515357212;
  static constexpr double C5b = -0.80901699437494742410, S5b = 0.58778525229247312917;
};
// cos / sin of 2 pi m / R for the radices used
template <int R>
__device__ __forceinline__ void rad_cs(int m, double& c, double& s) {
  m %= R;
  if constexpr (R == 2) {
    c = m ? -1.0 : 1.0; s = 0.0;
  } else if constexpr (R == 4) {
    const double cc[4] = {1, 0, -1, 0}, ss[4] = {0, 1, 0, -1};
    c = cc[m]; s = ss[m];
  } else if constexpr (R == 8) {
    const double cc[8] = {1, Rad::C8, 0, -Rad::C8, -1, -Rad::C8, 0, Rad::C8};
    const double ss[8] = {0, Rad::C8, 1, Rad::C8, 0, -Rad::C8, -1, -Rad::C8};
    c = cc[m]; s = ss[m];
  } else if constexpr (R == 3) {
    const double cc[3] = {1, -0.5, -0.5}, ss[3] = {0, Rad::S3, -Rad::S3};
    c = cc[m]; s = ss[m];
  } else {
    static_assert(R == 5, "radix");
    const double cc[5] = {1, Rad::C5a, Rad::C5b, Rad::C5b, Rad::C5a};
    const double ss[5] = {0, Rad::S5a, Rad::S5b, -Rad::S5b, -Rad::S5a};
    c = cc[m]; s = ss[m];
  }
}

// One Stockham pass (Govindaraju et al.): for j < n/R, v[r] = in[j + r n/R] W^{r (j mod Ns)},
// length-R DFT, out[(j / Ns) Ns R + j mod Ns + r Ns] = V[r]; W = exp(dir 2 pi i / (Ns R)).
// Signals: grid.y utterances (stride sb elements) x grid.z signals (stride n).
template <int R>
__global__ void __launch_bounds__(256) scene_fft_pass(const double2* __restrict__ in,
                                                      double2* __restrict__ out, int n, int Ns,
                                                      long long sb, double dir) {
  const int nr = n / R;
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= nr) return;
  const long long base = (long long)blockIdx.y * sb + (long long)blockIdx.z * n;
  const int jm = j % Ns;
  double2 v[R];
#pragma unroll
  for (int r = 0; r < R; ++r) v[r] = in[base + j + (long long)r * nr];
  if (Ns > 1) {
#pragma unroll
    for (int r = 1; r < R; ++r) {
      double s, c;
      sincospi(2.0 * (double)(r * jm) / (double)(Ns * R), &s, &c);
      s *= dir;
      v[r] = make_double2(v[r].x * c - v[r].y * s, v[r].x * s + v[r].y * c);
    }
  }
  double2 o[R];
#pragma unroll
  for (int k = 0; k < R; ++k) {
    double ax = 0.0, ay = 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      double c, s;
      rad_cs<R>(r * k, c, s);
      s *= dir;
      ax += v[r].x * c - v[r].y * s;
      ay += v[r].x * s + v[r].y * c;
    }
    o[k] = make_double2(ax, ay);
  }
  const int d0 = (j / Ns) * Ns * R + jm;
#pragma unroll
  for (int r = 0; r < R; ++r) out[base + d0 + (long long)r * Ns] = o[r];
}

// n = product of radices in {8, 4, 2, 5, 3}; returns the count (0: another prime factor).
static int fft_factor(int n, int* rad) {
  int k = 0;
  for (int r : {8, 4, 2, 5, 3})
    while (n % r == 0 && k < 32) {
      rad[k++] = r;
      n /= r;
    }
  return n == 1 ? k : 0;
}

// Transform `nz` signals per utterance in place of the ping-pong pair; returns the buffer
// holding the result.
static double2* fft_run(double2* a, double2* b, int n, int batch, int nz, long long sb,
                        double dir, hipStream_t st) {
  int rad[32];
  const int np = fft_factor(n, rad);
  int Ns = 1;
  for (int p = 0; p < np; ++p) {
    const int R = rad[p];
    const dim3 grid((unsigned)((n / R + 255) / 256), (unsigned)batch, (unsigned)nz);
    switch (R) {
      case 8: hipLaunchKernelGGL(scene_fft_pass<8>, grid, dim3(256), 0, st, a, b, n, Ns, sb, dir); break;
      case 4: hipLaunchKernelGGL(scene_fft_pass<4>, grid, dim3(256), 0, st, a, b, n, Ns, sb, dir); break;
      case 2: hipLaunchKernelGGL(scene_fft_pass<2>, grid, dim3(256), 0, st, a, b, n, Ns, sb, dir); break;
      case 5: hipLaunchKernelGGL(scene_fft_pass<5>, grid, dim3(256), 0, st, a, b, n, Ns, sb, dir); break;
      default: hipLaunchKernelGGL(scene_fft_pass<3>, grid, dim3(256), 0, st, a, b, n, Ns, sb, dir); break;
    }
    Ns *= R;
    double2* t = a;
    a = b;
    b = t;
  }
  return a;
}

// delta of (utterance b, source s, mic c): tau_mic * fs with world_building.py:47-51
// tau_1 = (d/2) cos(theta)/c, tau_2 = (d/2) cos(theta - pi)/c
__device__ __forceinline__ double scene_tau(const SceneArgs& A, int b, int s, int mic) {
  const double th = A.angles_deg[(long long)b * A.n_src + s] * (M_PI / 180.0);
  return (A.mic_d / 2) * cos(th - (mic ? M_PI : 0.0)) / A.c_sound;
}

// Sources packed two per complex signal: z[b][p][m] = src[2p][m] + i src[2p + 1][m].
__global__ void __launch_bounds__(256) scene_pack_kernel(SceneArgs A, double2* z, long long sb) {
  const int m = blockIdx.x * 256 + threadIdx.x;
  if (m >= A.n) return;
  const int b = blockIdx.y, p = blockIdx.z;
  const float* y = A.src + (long long)b * A.n_src * A.n;
  const double re = (double)y[(long long)(2 * p) * A.n + m];
  const double im = (2 * p + 1 < A.n_src) ? (double)y[(long long)(2 * p + 1) * A.n + m] : 0.0;
  z[(long long)b * sb + (long long)p * A.n + m] = make_double2(re, im);
}

// Frequency-domain mixing, thread per bin k <= n/2 of utterance b: source spectra from the
// packed transforms, per-mic phase ramps (irfft: imaginary parts of DC and Nyquist
// dropped), target / summed-interference images packed two mics per signal, both halves
// of the Hermitian spectrum written: zo[b][0] = T0 + i T1, zo[b][1] = I0 + i I1.
__global__ void __launch_bounds__(256) scene_phase_kernel(SceneArgs A, const double2* zf,
                                                          double2* zo, long long sb) {
  const int n = A.n, half = n / 2;
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k > half) return;
  const int b = blockIdx.y;
  const int kp = (n - k) % n;
  const double f = (double)k * (1.0 / ((double)n * (1.0 / A.fs)));  // np.fft.rfftfreq
  double2 T[2] = {{0, 0}, {0, 0}}, I[2] = {{0, 0}, {0, 0}};
  for (int s = 0; s < A.n_src; ++s) {
    const double2* zp = zf + (long long)b * sb + (long long)(s >> 1) * n;
    const double2 z = zp[k], zc = zp[kp];  // Z[k], Z[n - k]
    double2 Y;
    if ((s & 1) == 0)
      Y = make_double2(0.5 * (z.x + zc.x), 0.5 * (z.y - zc.y));  // (Z + conj Zc) / 2
    else
      Y = make_double2(0.5 * (z.y + zc.y), 0.5 * (zc.x - z.x));  // (Z - conj Zc) / 2i
#pragma unroll
    for (int mic = 0; mic < 2; ++mic) {
      double sn, cs;
      sincospi(2.0 * f * scene_tau(A, b, s, mic), &sn, &cs);  // exp(-2 pi i f tau)
      double2 h = make_double2(Y.x * cs + Y.y * sn, Y.y * cs - Y.x * sn);
      if (k == 0 || k == half) h.y = 0.0;
      double2& acc = (s == 0) ? T[mic] : I[mic];
      acc.x += h.x;
      acc.y += h.y;
    }
  }
  double2* o = zo + (long long)b * sb;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const double2 a = q ? I[0] : T[0], c = q ? I[1] : T[1];
    o[(long long)q * n + k] = make_double2(a.x - c.y, a.y + c.x);  // a + i c
    if (k != 0 && k != half)
      o[(long long)q * n + (n - k)] = make_double2(a.x + c.y, c.x - a.y);  // conj a + i conj c
  }
}

// ================================================================ O(n^2) fallback
constexpr int kConvThreads = 256;
constexpr int kConvOut = 8;                          // outputs per thread
constexpr int kConvM = kConvThreads * kConvOut;      // 2048 outputs per block
constexpr int kConvJ = 256;                          // inputs per LDS tile
constexpr int kConvH = kConvM + kConvJ;              // kernel values per tile (2304)

// h tables: one per (utterance, source, mic) signal, h[d] in fp64 -> fp32
__global__ void __launch_bounds__(256) avz_scene_kernel_fill(SceneArgs A) {
  const long long n = A.n;
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long nsig = (long long)A.batch * A.n_src * 2;
  if (idx >= nsig * n) return;
  const int sig = (int)(idx / n);
  const int d = (int)(idx % n);
  const int mic = sig & 1, s = (sig >> 1) % A.n_src, b = (sig >> 1) / A.n_src;
  const double delta = scene_tau(A, b, s, mic) * A.fs;
  const double x = ((double)d - delta) / (double)n;
  double sn, cs;
  sincospi(x, &sn, &cs);
  const double sd = sinpi(delta);
  const double h = -(1.0 / (double)n) * ((d & 1) ? -1.0 : 1.0) * sd * (cs / sn);
  A.hk[idx] = (float)h;
}

// image[sig][m] = sum_j src[b][s][j] h[sig][(m - j) mod n]; grid (ceil(n/2048), nsig).
// Thread t owns outputs M0 + 8t .. M0 + 8t + 7; per 256-input tile the block stages the
// inputs and the 2304 kernel values they meet, and each thread slides an 8-output window
// over 16 kernel values per 8 inputs (4 ds_read_b128 + 2 broadcast reads per 64 FMAs).
__global__ void __launch_bounds__(kConvThreads) avz_scene_conv_kernel(SceneArgs A) {
  __shared__ __align__(16) float y_t[kConvJ];
  __shared__ __align__(16) float h_t[kConvH];
  const int n = A.n;
  const int sig = blockIdx.y;
  const int mic = sig & 1, s = (sig >> 1) % A.n_src, b = (sig >> 1) / A.n_src;
  const float* y = A.src + ((long long)b * A.n_src + s) * n;
  float* img = A.img + (long long)sig * n;
  const int M0 = blockIdx.x * kConvM;
  const int tid = threadIdx.x;
  // broadside (sin(pi delta) ~ 0): the phase shift is 1 to within fp64 rounding
  if (fabs(sinpi(scene_tau(A, b, s, mic) * A.fs)) < 1e-12) {
    for (int m = M0 + tid; m < min(M0 + kConvM, n); m += kConvThreads) img[m] = y[m];
    return;
  }
  const float* h = A.hk + (long long)sig * n;
  float acc[kConvOut];
#pragma unroll
  for (int r = 0; r < kConvOut; ++r) acc[r] = 0.0f;
  for (int j0 = 0; j0 < n; j0 += kConvJ) {
    __syncthreads();
    y_t[tid] = (j0 + tid < n) ? y[j0 + tid] : 0.0f;
    // h_t[i] = h[(M0 - j0 - 255 + i) mod n]
    int base = (M0 - j0 - (kConvJ - 1)) % n;
    if (base < 0) base += n;
    for (int i = tid; i < kConvH; i += kConvThreads) {
      int d = base + i;
      if (d >= n) d -= n;
      if (d >= n) d -= n;
      h_t[i] = h[d];
    }
    __syncthreads();
#pragma unroll 2
    for (int q0 = 0; q0 < kConvJ; q0 += 8) {
      const int hb = kConvOut * tid - q0 + (kConvJ - 8);  // multiple of 8: 16-B aligned
      float hw[16];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const float4 t4 = *reinterpret_cast<const float4*>(h_t + hb + 4 * v);
        hw[4 * v] = t4.x; hw[4 * v + 1] = t4.y; hw[4 * v + 2] = t4.z; hw[4 * v + 3] = t4.w;
      }
      const float4 ya = *reinterpret_cast<const float4*>(y_t + q0);
      const float4 yb = *reinterpret_cast<const float4*>(y_t + q0 + 4);
      const float yq[8] = {ya.x, ya.y, ya.z, ya.w, yb.x, yb.y, yb.z, yb.w};
#pragma unroll
      for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int r = 0; r < kConvOut; ++r) acc[r] = fmaf(yq[q], hw[r - q + 7], acc[r]);
    }
  }
#pragma unroll
  for (int r = 0; r < kConvOut; ++r) {
    const int m = M0 + kConvOut * tid + r;
    if (m < n) img[m] = acc[r];
  }
}

// Per-source images -> the packed target / interference layout of the FFT path (times n,
// so the mix kernel scales both paths alike).
__global__ void __launch_bounds__(256) scene_conv_pack_kernel(SceneArgs A, double2* zo,
                                                              long long sb) {
  const int m = blockIdx.x * 256 + threadIdx.x;
  if (m >= A.n) return;
  const int b = blockIdx.y;
  const long long n = A.n;
  const float* im = A.img + (long long)b * A.n_src * 2 * n;  // [src][mic][n]
  double t[2], i[2] = {0.0, 0.0};
#pragma unroll
  for (int mic = 0; mic < 2; ++mic) {
    t[mic] = (double)im[mic * n + m];
    for (int k = 1; k < A.n_src; ++k) i[mic] += (double)im[(k * 2 + mic) * n + m];
  }
  const double sc = (double)n;
  zo[(long long)b * sb + m] = make_double2(t[0] * sc, t[1] * sc);
  zo[(long long)b * sb + n + m] = make_double2(i[0] * sc, i[1] * sc);
}

// ================================================================ mixing
// One block per utterance: simulation.py:167-202 on the images.
//   tgt_m = image(target), int_m = g * sum_k image(interferer k), g for SIR sir_db on mic 1;
//   noisy = clean + sqrt(mean(clean^2) / 10^(snr/10)) * z  (world.py:93-98 add_awgn);
//   peak = max |noisy| + 1e-9 over both mics; outputs / peak.
// Images: ti[b][0][m] = n (T0 + i T1), ti[b][1][m] = n (I0 + i I1).
constexpr int kMixThreads = 256;
__device__ __forceinline__ double block_sum(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int w = 0; w < kMixThreads / 64; ++w) t += red[w];
  return t;
}
__device__ __forceinline__ float block_max(float v, float* red) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float t = 0.0f;
#pragma unroll
  for (int w = 0; w < kMixThreads / 64; ++w) t = fmaxf(t, red[w]);
  return t;
}

__global__ void __launch_bounds__(kMixThreads) avz_scene_mix_kernel(SceneArgs A, const double2* ti,
                                                                    long long sb) {
  __shared__ double red[kMixThreads / 64];
  __shared__ float redf[kMixThreads / 64];
  const int b = blockIdx.x, tid = threadIdx.x, n = A.n, K = A.n_src - 1;
  const double2* T = ti + (long long)b * sb;
  const double2* I = T + n;
  const double sc = 1.0 / (double)n;
  auto tgt_img = [&](int mic, int m) -> double { return (mic ? T[m].y : T[m].x) * sc; };
  auto int_img = [&](int mic, int m) -> double { return (mic ? I[m].y : I[m].x) * sc; };
  double st = 0.0, si = 0.0;
  for (int m = tid; m < n; m += kMixThreads) {
    const double t = tgt_img(0, m), i = int_img(0, m);
    st += t * t;
    si += i * i;
  }
  const double p_t = block_sum(st, red) / n;
  const double p_i = block_sum(si, red) / n;
  const double g = (K > 0 && p_i > 0) ? sqrt(p_t / (p_i * pow(10.0, A.sir_db / 10.0))) : 1.0;
  double scl[2] = {0.0, 0.0};
  for (int m = tid; m < n; m += kMixThreads) {
#pragma unroll
    for (int mic = 0; mic < 2; ++mic) {
      const double cl = tgt_img(mic, m) + g * int_img(mic, m);
      scl[mic] += cl * cl;
    }
  }
  double sig_n[2];
#pragma unroll
  for (int mic = 0; mic < 2; ++mic) {
    const double p = block_sum(scl[mic], red) / n;
    sig_n[mic] = (p == 0.0) ? 0.0 : sqrt(p / pow(10.0, A.snr_db / 10.0));
  }
  const float* z = A.noise + (long long)b * 2 * n;
  float pk = 0.0f;
  for (int m = tid; m < n; m += kMixThreads) {
#pragma unroll
    for (int mic = 0; mic < 2; ++mic) {
      const double v = tgt_img(mic, m) + g * int_img(mic, m) + sig_n[mic] * (double)z[(long long)mic * n + m];
      pk = fmaxf(pk, (float)fabs(v));
    }
  }
  // the peak in fp64 would need a second reduction type; |v| rounded to fp32 first
  // changes 1/(peak + 1e-9) by < 1 ulp of fp32
  const double peak = (double)block_max(pk, redf) + 1e-9;
  float* mix = A.mix + (long long)b * A.mix_stride;
  for (int m = tid; m < n; m += kMixThreads) {
#pragma unroll
    for (int mic = 0; mic < 2; ++mic) {
      const double v = tgt_img(mic, m) + g * int_img(mic, m) + sig_n[mic] * (double)z[(long long)mic * n + m];
      mix[(long long)mic * A.ch_stride + m] = (float)(v / peak);
    }
    A.tgt[(long long)b * A.ref_stride + m] = (float)(tgt_img(0, m) / peak);
    A.itf[(long long)b * A.ref_stride + m] = (float)(g * int_img(0, m) / peak);
  }
}

}  // namespace avz

using namespace avz;

extern "C" int avz_scene_fft_len(int n) {
  int rad[32];
  return n > 1 && fft_factor(n, rad) > 0;
}

// Workspace of the mixing back end: FFT path 2 x [B][max(ceil(n_src/2), 2)][n] double2;
// fallback: fp32 kernels + images [B][n_src][2][n] each, and [B][2][n] double2.
extern "C" long long avz_scene_mix_ws(int batch, int n_src, int n) {
  int rad[32];
  const long long B = batch, N = n;
  if (fft_factor(n, rad) > 0) {
    const long long nz = std::max((n_src + 1) / 2, 2);
    return 2 * B * nz * N * (long long)sizeof(double2);
  }
  return 2 * B * n_src * 2 * N * (long long)sizeof(float) + B * 2 * N * (long long)sizeof(double2);
}

extern "C" int avz_launch_scene(const SceneArgs* a, void* ws, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int B = a->batch, n = a->n;
  int rad[32];
  if (fft_factor(n, rad) > 0) {
    const int nz = std::max((a->n_src + 1) / 2, 2);
    const long long sb = (long long)nz * n;
    double2* z0 = static_cast<double2*>(ws);
    double2* z1 = z0 + (long long)B * sb;
    const int P = (a->n_src + 1) / 2;
    hipLaunchKernelGGL(scene_pack_kernel, dim3((n + 255) / 256, B, P), dim3(256), 0, st, *a, z0, sb);
    double2* f = fft_run(z0, z1, n, B, P, sb, -1.0, st);
    double2* o = (f == z0) ? z1 : z0;
    hipLaunchKernelGGL(scene_phase_kernel, dim3((n / 2 + 1 + 255) / 256, B), dim3(256), 0, st, *a,
                       (const double2*)f, o, sb);
    double2* t = fft_run(o, f, n, B, 2, sb, 1.0, st);
    hipLaunchKernelGGL(avz_scene_mix_kernel, dim3(B), dim3(kMixThreads), 0, st, *a,
                       (const double2*)t, sb);
  } else {
    SceneArgs c = *a;
    const long long per = (long long)B * a->n_src * 2 * n;
    c.hk = static_cast<float*>(ws);
    c.img = c.hk + per;
    double2* zo = reinterpret_cast<double2*>(c.img + per);
    const long long nsig = (long long)B * a->n_src * 2;
    hipLaunchKernelGGL(avz_scene_kernel_fill, dim3((unsigned)((nsig * n + 255) / 256)), dim3(256), 0,
                       st, c);
    hipLaunchKernelGGL(avz_scene_conv_kernel, dim3((n + kConvM - 1) / kConvM, (unsigned)nsig),
                       dim3(kConvThreads), 0, st, c);
    hipLaunchKernelGGL(scene_conv_pack_kernel, dim3((n + 255) / 256, B), dim3(256), 0, st, c, zo,
                       2LL * n);
    hipLaunchKernelGGL(avz_scene_mix_kernel, dim3(B), dim3(kMixThreads), 0, st, c,
                       (const double2*)zo, 2LL * n);
  }
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// Generation scratch: sources, noise, angles and the AR(2) segment states; the mixing
// back end's workspace follows it.
static long long gen_scratch(int batch, int n_src, int n) {
  const long long nseg = (n + kSegLen - 1) / kSegLen;
  auto al = [](long long x) { return (x + 255) & ~255LL; };
  return al((long long)batch * n_src * n * 4) + al((long long)batch * 2 * n * 4) +
         al((long long)batch * n_src * 8) + 2 * al((long long)batch * n_src * nseg * 16);
}

extern "C" long long avz_scene_gen_ws(int batch, int n_src, int n) {
  return gen_scratch(batch, n_src, n) + avz_scene_mix_ws(batch, n_src, n);
}

extern "C" int avz_launch_scene_generate(SceneArgs* a, long long start, uint32_t seed, void* ws,
                                         void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int B = a->batch, S = a->n_src, n = a->n;
  auto al = [](long long x) { return (x + 255) & ~255LL; };
  char* p = static_cast<char*>(ws);
  GenArgs g{};
  g.batch = B;
  g.n_src = S;
  g.n = n;
  g.nseg = (n + kSegLen - 1) / kSegLen;
  g.start = start;
  g.seed = seed;
  g.fs = a->fs;
  g.src = reinterpret_cast<float*>(p);
  p += al((long long)B * S * n * 4);
  g.noise = reinterpret_cast<float*>(p);
  p += al((long long)B * 2 * n * 4);
  g.angles = reinterpret_cast<double*>(p);
  p += al((long long)B * S * 8);
  g.zs = reinterpret_cast<double*>(p);
  p += al((long long)B * S * g.nseg * 16);
  g.sin_ = reinterpret_cast<double*>(p);
  p += al((long long)B * S * g.nseg * 16);
  const long long nar = (long long)B * S * g.nseg;
  hipLaunchKernelGGL(scene_ar_kernel<false>, dim3((unsigned)((nar + 255) / 256)), dim3(256), 0, st, g);
  hipLaunchKernelGGL(scene_ar_scan_kernel, dim3((B * S + 63) / 64), dim3(64), 0, st, g);
  hipLaunchKernelGGL(scene_ar_kernel<true>, dim3((unsigned)((nar + 255) / 256)), dim3(256), 0, st, g);
  const long long nn = (long long)B * n;  // B * 2 * (n / 2) normal pairs
  hipLaunchKernelGGL(scene_noise_kernel, dim3((unsigned)((nn + 255) / 256)), dim3(256), 0, st, g);
  a->src = g.src;
  a->noise = g.noise;
  a->angles_deg = g.angles;
  if (hipGetLastError() != hipSuccess) return -3;
  return avz_launch_scene(a, p, stream);
}
