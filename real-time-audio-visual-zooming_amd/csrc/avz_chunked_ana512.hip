// avz_chunked_ana512.hip — N = 512 analysis kernels: device code of the chain kernels compiled in parallel with the other units
// (instantiation list: avz_chunked_inst.hpp; kernels: avz_chunked_k.hpp).
#include "avz_chunked_k.hpp"
#include "avz_chunked_inst.hpp"

namespace avz {
#define AVZ_INST template
AVZ_ANALYSIS_INST(512)
#undef AVZ_INST
}  // namespace avz

#if defined(AVZ_STAMPS) || defined(AVZ_XTRACE)
extern "C" int avz_stamps_set_ana512(void* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(avz::g_stamps), &p, sizeof(p)) == hipSuccess ? 0 : -3;
}
#endif
