// avz_chunked_utt.hip — per-utterance synthesis kernels: device code of the chain kernels compiled in parallel with the other units
// (instantiation list: avz_chunked_inst.hpp; kernels: avz_chunked_k.hpp).
#include "avz_chunked_k.hpp"
#include "avz_chunked_inst.hpp"

namespace avz {
#define AVZ_INST template
AVZ_UTT_INST
#undef AVZ_INST
}  // namespace avz

#ifdef AVZ_STAMPS
extern "C" int avz_stamps_set_utt(void* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(avz::g_stamps), &p, sizeof(p)) == hipSuccess ? 0 : -3;
}
#endif
