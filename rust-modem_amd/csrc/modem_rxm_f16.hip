// rust-modem_amd/csrc/modem_rxm_f16.hip — RX matrix-core variants (modem_rxm.h) for
//   f16 samples in and out, complex mix (the C5 f16 sweep) and their channel batches.
#include "modem_rxm.h"

namespace mk {
template hipError_t rxm_sel<__half, MIX_COMPLEX, __half>(const RxParams&, int, int, const void*, hipStream_t);
template hipError_t rxm_sel_batch<__half>(const RxBatch&, int, int, const void*, hipStream_t);
}  // namespace mk
