// rust-modem_amd/csrc/modem_rxm_mixed.hip — RX matrix-core variants (modem_rxm.h) for the other
//   element types and mixes: f32 / f16 in and out in every combination with the reference's real
//   mix (demodulator.rs:46,53-54), and the complex mix across dtypes.
#include "modem_rxm.h"

namespace mk {
template hipError_t rxm_sel<float, MIX_COMPLEX, __half>(const RxParams&, int, int, const void*, hipStream_t);
template hipError_t rxm_sel<__half, MIX_COMPLEX, float>(const RxParams&, int, int, const void*, hipStream_t);
template hipError_t rxm_sel<float, MIX_REFERENCE_REAL, float>(const RxParams&, int, int, const void*, hipStream_t);
template hipError_t rxm_sel<float, MIX_REFERENCE_REAL, __half>(const RxParams&, int, int, const void*, hipStream_t);
template hipError_t rxm_sel<__half, MIX_REFERENCE_REAL, float>(const RxParams&, int, int, const void*, hipStream_t);
template hipError_t rxm_sel<__half, MIX_REFERENCE_REAL, __half>(const RxParams&, int, int, const void*, hipStream_t);
}  // namespace mk
