// rust-modem_amd/csrc/modem_txm_real.hip — TX matrix-core variants (modem_txm.h)
//   for the real passband output (modulate's default form), f32 and f16.
#include "modem_txm.h"

namespace mk {
template hipError_t txm_sel<OUT_REAL, float>(const TxParams&, int, int, const void*, hipStream_t);
template hipError_t txm_sel<OUT_REAL, __half>(const TxParams&, int, int, const void*, hipStream_t);
}  // namespace mk
