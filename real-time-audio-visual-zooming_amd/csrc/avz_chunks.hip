// avz_chunks.hip — time-domain chunking of the Final_pipeline driver (gfx950).
//
// Final_pipeline/src/inference.py:171-237 processes an utterance as 2-s chunks
// (WIN_SIZE = 32000 samples every 16000, zero-padded tail), beamforms each chunk
// independently, and overlap-adds the chunk outputs divided by the per-sample count.
// Here every chunk of every utterance is one batch item of the MVDR chain; these
// kernels cut the items out of the utterances and merge the item outputs back.
// Both are HBM streaming kernels: one float4 per thread, grid-stride free (one
// block row per item / utterance slice).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "avz_internal.h"

namespace avz {

constexpr int kCopyThreads = 256;

// items[i][c][n] = x[utt][c][start + n] for start + n < len[utt], else 0.
// grid (ceil(chunk / (4 * 256)), n_items * channels)
__global__ void __launch_bounds__(kCopyThreads) avz_chunk_split_kernel(ChunkSplitArgs A) {
  const int ic = blockIdx.y;
  const int i = ic / A.channels, c = ic % A.channels;
  const int utt = A.item_utt[i];
  const int start = A.item_start[i];
  const int L = A.len[utt];
  const float* src = A.x + (long long)utt * A.x_stride + (long long)c * A.x_ch_stride;
  float* dst = A.items + (long long)i * A.item_stride + (long long)c * A.item_ch_stride;
  const int n0 = 4 * (blockIdx.x * kCopyThreads + threadIdx.x);
  if (n0 >= A.chunk) return;
  float v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + j;
    const long long s = (long long)start + n;
    v[j] = (n < A.chunk && s < L) ? src[s] : 0.0f;
  }
  if (n0 + 4 <= A.chunk && ((reinterpret_cast<uintptr_t>(dst + n0) & 15) == 0)) {
    *reinterpret_cast<float4*>(dst + n0) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (n0 + j < A.chunk) dst[n0 + j] = v[j];
  }
}

// y[b][n] = sum_c item_out[base[b] + c][n - c hop] / count(n) over the chunks c of
// utterance b whose output window [c hop, c hop + item_out_len) covers n
// (inference.py:224-229: w_len = min(len(chunk_out), len(out_buf[start:]))).
// Block max |y| -> atomicMax on the float bits (non-negative) of peak[b].
// grid (ceil(max_len / (4 * 256)), batch)
__global__ void __launch_bounds__(kCopyThreads) avz_chunk_merge_kernel(ChunkMergeArgs A) {
  __shared__ float red[kCopyThreads / 64];
  const int b = blockIdx.y;
  const int L = min(A.len[b], A.max_len);
  const int nch = (L + A.hop - 1) / A.hop;
  const float* io = A.item_out + (long long)A.item_base[b] * A.item_out_stride;
  float* y = A.y + (long long)b * A.y_stride;
  const int n0 = 4 * (blockIdx.x * kCopyThreads + threadIdx.x);
  float pk = 0.0f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + j;
    if (n >= L) break;
    // chunks c with c hop <= n < c hop + item_out_len
    int c_lo = (n - A.item_out_len) / A.hop + 1;
    if (n < A.item_out_len) c_lo = 0;
    const int c_hi = min(n / A.hop, nch - 1);
    float acc = 0.0f;
    int cnt = 0;
    for (int c = c_lo; c <= c_hi; ++c) {
      acc += io[(long long)c * A.item_out_stride + (n - c * A.hop)];
      ++cnt;
    }
    const float v = acc / (float)max(cnt, 1);
    y[n] = v;
    pk = fmaxf(pk, fabsf(v));
  }
  for (int o = 32; o > 0; o >>= 1) pk = fmaxf(pk, __shfl_xor(pk, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = pk;
  __syncthreads();
  if (threadIdx.x == 0) {
    float m = red[0];
#pragma unroll
    for (int w = 1; w < kCopyThreads / 64; ++w) m = fmaxf(m, red[w]);
    atomicMax(reinterpret_cast<unsigned int*>(A.peak) + b, __float_as_uint(m));
  }
}

// y[b][n] /= peak[b] + norm_eps (inference.py:236). grid as the merge kernel.
__global__ void __launch_bounds__(kCopyThreads) avz_chunk_scale_kernel(ChunkMergeArgs A) {
  const int b = blockIdx.y;
  const int L = min(A.len[b], A.max_len);
  const float s = 1.0f / (A.peak[b] + A.norm_eps);
  float* y = A.y + (long long)b * A.y_stride;
  const int n0 = 4 * (blockIdx.x * kCopyThreads + threadIdx.x);
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (n0 + j < L) y[n0 + j] *= s;
}

}  // namespace avz

using namespace avz;

extern "C" int avz_launch_chunk_split(const ChunkSplitArgs* a, void* stream) {
  if (a->n_items <= 0) return 0;
  const dim3 grid((a->chunk + 4 * kCopyThreads - 1) / (4 * kCopyThreads), a->n_items * a->channels);
  hipLaunchKernelGGL(avz_chunk_split_kernel, grid, dim3(kCopyThreads), 0, (hipStream_t)stream, *a);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int avz_launch_chunk_merge(const ChunkMergeArgs* a, void* stream) {
  if (a->batch <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(a->peak, 0, sizeof(float) * a->batch, st) != hipSuccess) return -3;
  const dim3 grid((a->max_len + 4 * kCopyThreads - 1) / (4 * kCopyThreads), a->batch);
  hipLaunchKernelGGL(avz_chunk_merge_kernel, grid, dim3(kCopyThreads), 0, st, *a);
  if (a->normalize) hipLaunchKernelGGL(avz_chunk_scale_kernel, grid, dim3(kCopyThreads), 0, st, *a);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
