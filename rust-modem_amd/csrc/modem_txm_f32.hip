// rust-modem_amd/csrc/modem_txm_f32.hip — TX matrix-core variants (modem_txm.h)
//   for the loopback's f32 samples (C2, C3, C4, C5) and their channel batches.
#include "modem_txm.h"

namespace mk {
template hipError_t txm_sel<OUT_IQ_MIXED, float>(const TxParams&, int, int, const void*, hipStream_t);
template hipError_t txm_sel_batch<float>(const TxBatch&, int, int, const void*, hipStream_t);
}  // namespace mk
