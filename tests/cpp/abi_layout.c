/* tests/cpp/abi_layout.c — the C ABI's descriptor layouts (LP64: x86_64 / aarch64 Linux), pinned.
 *
 * Compiled as C11 and as C++17 (tests/cpp/Makefile): every static_assert below is the table in
 * INTEGRATION.md ("Descriptor layouts"), which the Rust #[repr(C)] structs there must match
 * field for field. Run, it prints the same table (tests/test_capi_host.py compares the two).
 */
#include <assert.h>
#include <stddef.h>
#include <stdio.h>

#include "modem_hip.h"

#define SZ(T, s, a) static_assert(sizeof(T) == (s) && _Alignof(T) == (a), #T " size / alignment");
#define OF(T, m, o) static_assert(offsetof(T, m) == (o), #T "." #m " offset");

#ifdef __cplusplus
#define _Alignof alignof
#endif

static_assert(MODEM_HIP_ABI_VERSION == 6, "the layouts below are ABI version 6 (unchanged since 4)");

SZ(modem_ring, 12, 4)
OF(modem_ring, start, 0) OF(modem_ring, end, 1) OF(modem_ring, radius, 4) OF(modem_ring, phase, 8)

SZ(modem_phasor_desc, 48, 8)
OF(modem_phasor_desc, kind, 0) OF(modem_phasor_desc, bits_per_symbol, 4) OF(modem_phasor_desc, phase, 8)
OF(modem_phasor_desc, amplitude, 12) OF(modem_phasor_desc, nrings, 16) OF(modem_phasor_desc, rings, 24)
OF(modem_phasor_desc, freq, 32) OF(modem_phasor_desc, samples_per_symbol, 36) OF(modem_phasor_desc, shift, 40)
OF(modem_phasor_desc, mfsk_map, 44)

SZ(modem_slicer_desc, 32, 8)
OF(modem_slicer_desc, kind, 0) OF(modem_slicer_desc, bits_per_symbol, 4) OF(modem_slicer_desc, lut, 8)
OF(modem_slicer_desc, bits_per_carrier, 16) OF(modem_slicer_desc, inv_scale, 20) OF(modem_slicer_desc, max_symbol, 24)

SZ(modem_tx_desc, 72, 8)
OF(modem_tx_desc, bits_per_symbol, 0) OF(modem_tx_desc, lut, 8) OF(modem_tx_desc, samples_per_symbol, 16)
OF(modem_tx_desc, taps, 24) OF(modem_tx_desc, ntaps, 32) OF(modem_tx_desc, sample_freq, 36) OF(modem_tx_desc, s0, 40)
OF(modem_tx_desc, dtype, 48) OF(modem_tx_desc, out_mode, 52) OF(modem_tx_desc, q_offset, 56) OF(modem_tx_desc, phasor, 64)

SZ(modem_rx_desc, 88, 8)
OF(modem_rx_desc, sample_freq, 0) OF(modem_rx_desc, s0, 8) OF(modem_rx_desc, taps, 16) OF(modem_rx_desc, ntaps, 24)
OF(modem_rx_desc, decim, 28) OF(modem_rx_desc, decim_offset, 32) OF(modem_rx_desc, mix, 36)
OF(modem_rx_desc, in_dtype, 40) OF(modem_rx_desc, out_dtype, 44) OF(modem_rx_desc, slicer, 48)
OF(modem_rx_desc, phase_offset, 80)

#define PS(T) printf("%s %zu %zu\n", #T, sizeof(T), (size_t)_Alignof(T));
#define PF(T, m) printf("%s.%s %zu\n", #T, #m, offsetof(T, m));

int main(void) {
    PS(modem_ring) PF(modem_ring, start) PF(modem_ring, end) PF(modem_ring, radius) PF(modem_ring, phase)
    PS(modem_phasor_desc) PF(modem_phasor_desc, kind) PF(modem_phasor_desc, bits_per_symbol)
    PF(modem_phasor_desc, phase) PF(modem_phasor_desc, amplitude) PF(modem_phasor_desc, nrings)
    PF(modem_phasor_desc, rings) PF(modem_phasor_desc, freq) PF(modem_phasor_desc, samples_per_symbol)
    PF(modem_phasor_desc, shift) PF(modem_phasor_desc, mfsk_map)
    PS(modem_slicer_desc) PF(modem_slicer_desc, kind) PF(modem_slicer_desc, bits_per_symbol)
    PF(modem_slicer_desc, lut) PF(modem_slicer_desc, bits_per_carrier) PF(modem_slicer_desc, inv_scale)
    PF(modem_slicer_desc, max_symbol)
    PS(modem_tx_desc) PF(modem_tx_desc, bits_per_symbol) PF(modem_tx_desc, lut) PF(modem_tx_desc, samples_per_symbol)
    PF(modem_tx_desc, taps) PF(modem_tx_desc, ntaps) PF(modem_tx_desc, sample_freq) PF(modem_tx_desc, s0)
    PF(modem_tx_desc, dtype) PF(modem_tx_desc, out_mode) PF(modem_tx_desc, q_offset) PF(modem_tx_desc, phasor)
    PS(modem_rx_desc) PF(modem_rx_desc, sample_freq) PF(modem_rx_desc, s0) PF(modem_rx_desc, taps)
    PF(modem_rx_desc, ntaps) PF(modem_rx_desc, decim) PF(modem_rx_desc, decim_offset) PF(modem_rx_desc, mix)
    PF(modem_rx_desc, in_dtype) PF(modem_rx_desc, out_dtype) PF(modem_rx_desc, slicer) PF(modem_rx_desc, phase_offset)
    return 0;
}
