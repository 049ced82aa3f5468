// avz_chunked_ana1024.hip — N = 1024 analysis kernels: device code of the chain kernels compiled in parallel with the other units
// (instantiation list: avz_chunked_inst.hpp; kernels: avz_chunked_k.hpp).
#include "avz_chunked_k.hpp"
#include "avz_chunked_inst.hpp"

namespace avz {
#define AVZ_INST template
AVZ_ANALYSIS_INST(1024)
#undef AVZ_INST
}  // namespace avz

#if defined(AVZ_STAMPS) || defined(AVZ_XTRACE)
extern "C" int avz_stamps_set_ana1024(void* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(avz::g_stamps), &p, sizeof(p)) == hipSuccess ? 0 : -3;
}
#endif
