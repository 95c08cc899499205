// rust-modem_amd/csrc/modem_txm_bb.hip — TX matrix-core variants (modem_txm.h)
//   for baseband I/Q (no carrier), f32 and f16.
#include "modem_txm.h"

namespace mk {
template hipError_t txm_sel<OUT_IQ_BASEBAND, float>(const TxParams&, int, int, const void*, hipStream_t);
template hipError_t txm_sel<OUT_IQ_BASEBAND, __half>(const TxParams&, int, int, const void*, hipStream_t);
}  // namespace mk
