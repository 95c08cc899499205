// rust-modem_amd/csrc/modem_txm_f16.hip — TX matrix-core variants (modem_txm.h)
//   for f16 samples (the C5 f16 sweep) and their channel batches.
#include "modem_txm.h"

namespace mk {
template hipError_t txm_sel<OUT_IQ_MIXED, __half>(const TxParams&, int, int, const void*, hipStream_t);
template hipError_t txm_sel_batch<__half>(const TxBatch&, int, int, const void*, hipStream_t);
}  // namespace mk
