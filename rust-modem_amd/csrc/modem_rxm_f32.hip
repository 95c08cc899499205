// rust-modem_amd/csrc/modem_rxm_f32.hip — RX matrix-core variants (modem_rxm.h) for
//   f32 samples in and out, complex mix (the loopback: C2, C3, C4, C5) and their channel batches.
#include "modem_rxm.h"

namespace mk {
template hipError_t rxm_sel<float, MIX_COMPLEX, float>(const RxParams&, int, int, const void*, hipStream_t);
template hipError_t rxm_sel_batch<float>(const RxBatch&, int, int, const void*, hipStream_t);
}  // namespace mk
