// avz_chunked_inst.hpp — the chain kernels' instantiations, one list for both sides: the
// kernel translation units (avz_chunked_{ana1024,ana512,syn}.hip) define them
// (AVZ_INST = template), avz_chunked.hip declares them (AVZ_INST = extern template) so its
// launchers reference the other units' kernels instead of compiling them again. Split only to
// compile the device code in parallel; one list keeps the two sides in step.
#pragma once
#define AVZ_ANALYSIS_INST(N)                                                         \
  AVZ_INST __global__ void avz_analysis_kernel<N, MASK_IBM, false, false>(ChainArgs);      \
  AVZ_INST __global__ void avz_analysis_kernel<N, MASK_IBM, false, true>(ChainArgs);       \
  AVZ_INST __global__ void avz_analysis_kernel<N, MASK_IBM, true, false>(ChainArgs);       \
  AVZ_INST __global__ void avz_analysis_kernel<N, MASK_IBM, true, true>(ChainArgs);        \
  AVZ_INST __global__ void avz_analysis_kernel<N, MASK_IPD, false, false>(ChainArgs);      \
  AVZ_INST __global__ void avz_analysis_kernel<N, MASK_IPD, false, true>(ChainArgs);       \
  AVZ_INST __global__ void avz_analysis_kernel<N, MASK_EXTERNAL, false, false>(ChainArgs); \
  AVZ_INST __global__ void avz_analysis_kernel<N, MASK_EXTERNAL, false, true>(ChainArgs);  \
  AVZ_INST __global__ void avz_analysis_kernel<N, MASK_ONES, false, false>(ChainArgs);     \
  AVZ_INST __global__ void avz_analysis_kernel<N, MASK_ONES, false, true>(ChainArgs);
#define AVZ_UTT_INST                                                                  \
  AVZ_INST __global__ void avz_synthesis_utt_kernel<PF_NONE, false, false>(ChainArgs);       \
  AVZ_INST __global__ void avz_synthesis_utt_kernel<PF_NONE, false, true>(ChainArgs);        \
  AVZ_INST __global__ void avz_synthesis_utt_kernel<PF_NONE, true, false>(ChainArgs);        \
  AVZ_INST __global__ void avz_synthesis_utt_kernel<PF_NONE, true, true>(ChainArgs);         \
  AVZ_INST __global__ void avz_synthesis_utt_kernel<PF_IBM_TARGET, false, false>(ChainArgs); \
  AVZ_INST __global__ void avz_synthesis_utt_kernel<PF_IBM_TARGET, false, true>(ChainArgs);  \
  AVZ_INST __global__ void avz_synthesis_utt_kernel<PF_IBM_TARGET, true, false>(ChainArgs);  \
  AVZ_INST __global__ void avz_synthesis_utt_kernel<PF_IBM_TARGET, true, true>(ChainArgs);   \
  AVZ_INST __global__ void avz_synthesis_utt512_kernel<PF_NONE, false>(ChainArgs);           \
  AVZ_INST __global__ void avz_synthesis_utt512_kernel<PF_NONE, true>(ChainArgs);            \
  AVZ_INST __global__ void avz_synthesis_utt512_kernel<PF_IBM_TARGET, false>(ChainArgs);     \
  AVZ_INST __global__ void avz_synthesis_utt512_kernel<PF_IBM_TARGET, true>(ChainArgs);
#define AVZ_SYN_INST(N)                                                              \
  AVZ_INST __global__ void avz_synthesis_kernel<N, PF_NONE, false>(ChainArgs);       \
  AVZ_INST __global__ void avz_synthesis_kernel<N, PF_NONE, true>(ChainArgs);        \
  AVZ_INST __global__ void avz_synthesis_kernel<N, PF_IBM_TARGET, false>(ChainArgs); \
  AVZ_INST __global__ void avz_synthesis_kernel<N, PF_EXT_FLOOR, false>(ChainArgs);  \
  AVZ_INST __global__ void avz_synthesis_kernel<N, PF_EXT_MUL, false>(ChainArgs);    \
  AVZ_INST __global__ void avz_synthesis_kernel<N, PF_IRM, false>(ChainArgs);
