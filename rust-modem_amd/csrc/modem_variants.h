// rust-modem_amd/csrc/modem_variants.h — the filter shapes the matrix-core kernels are
// instantiated for (one place for the TX, RX and their k-step selection).
//   TX (sps, k-steps): W = 32 * nks >= 16 / sps + K - 1 symbols (K = taps per phase);
//   RX (decim, k-steps): W = 32 * nks >= 15 * decim + ntaps.
// A filter with no variant runs on the VALU kernels (tx_fast / rx_fast / *_generic).
// MODEM_VARIANTS_MIN is a build option for experiment builds only (tools/build_var.sh,
// DESIGN.md §5): the BASELINE configurations' filters alone (C2 / C4: 65 taps sps 4, C3: 129
// taps sps 4, C5: 513 taps sps 8), which compiles in a fraction of the time. The product
// library (Makefile, __graft_entry__.build) never defines it.
#pragma once

#ifdef MODEM_VARIANTS_MIN
#define MODEM_TXM_TABLE(X) X(4, 1) X(4, 2) X(8, 3)
#define MODEM_RXM_TABLE(X) X(4, 4) X(4, 6) X(8, 20)
#else
#define MODEM_TXM_TABLE(X) X(2, 1) X(2, 2) X(2, 3) X(2, 5) X(4, 1) X(4, 2) X(4, 3) X(4, 5) X(4, 9) \
                           X(8, 1) X(8, 2) X(8, 3) X(8, 5) X(8, 9) X(16, 1) X(16, 2) X(16, 3) X(16, 5)
#define MODEM_RXM_TABLE(X) X(2, 2) X(2, 3) X(2, 5) X(2, 8) X(4, 3) X(4, 4) X(4, 6) X(4, 8) X(8, 5) X(8, 6) \
                           X(8, 9) X(8, 20)
#endif
