// avz_chunked_syn.hip — chunk-grid synthesis kernels: device code of the chain kernels compiled in parallel with the other units
// (instantiation list: avz_chunked_inst.hpp; kernels: avz_chunked_k.hpp).
#include "avz_chunked_k.hpp"
#include "avz_chunked_inst.hpp"

namespace avz {
#define AVZ_INST template
AVZ_SYN_INST(1024)
AVZ_SYN_INST(512)
#undef AVZ_INST
}  // namespace avz

#if defined(AVZ_STAMPS) || defined(AVZ_XTRACE)
extern "C" int avz_stamps_set_syn(void* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(avz::g_stamps), &p, sizeof(p)) == hipSuccess ? 0 : -3;
}
#endif
