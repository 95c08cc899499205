"""Time-segment sharding of one long stream.

Channels shard with no exchange; a single long stream shards too, by time segment, because
the carrier phase is a pure function of the absolute sample index (carrier.rs:17-19: a
handle created with `Carrier.sample = s0` continues the stream at s0) and the FIRs only look
back (fir.rs:18-34: y[n] = sum h[k] x[n-k]). Segment g of G is processed by its own handle,
started a halo early so that its FIR history holds the real samples, and the halo's outputs
are dropped:

* TX segment [a, b) symbols: a handle at symbol a - H (carrier s0 = (a - H) * sps) is fed the
  bits of symbols [a - H, b) and returns samples [(a - H) * sps, b * sps); the first H * sps
  are dropped. H >= ceil((L - 1) / sps) symbols.
* RX segment [na, nb) samples: a handle at sample n0 = na - Hs (carrier s0 = n0, same
  decimation offset D = L - 1) is fed samples [n0, nb); global kept instant k (sample
  k * sps + D) is local instant k - n0 / sps. Hs >= L - 1 samples.

Halo starts are rounded to the kernels' alignment (the TX's row-blocks repeat every
16 / sps symbols, the RX's rows every 16 kept instants; both kernels align them to the
handle's own index), so every segment computes each output with the same operands at the
same MFMA positions as one long call: the concatenated segments are bit-identical to it
(tests/test_gpu_parity.py::test_time_segments_equal_one_stream). Each rank of a node can take
one segment (no collective: the halo is re-read input, not exchanged state).
"""
from __future__ import annotations

from typing import List, Tuple

# One alignment unit covers both kernels: 64 symbols is a multiple of the RX rows (16 kept
# instants) and of the TX row-blocks (16 / sps symbols, every sps dividing 16).
ALIGN_SYMBOLS = 64


def _round_down(x: int, m: int) -> int:
    return x // m * m


def segment_bounds(nsym: int, nseg: int, align: int = ALIGN_SYMBOLS) -> List[Tuple[int, int]]:
    """Symbol ranges [a_g, b_g) covering [0, nsym) in nseg contiguous pieces of (almost)
    equal length, every interior boundary a multiple of `align` (empty pieces possible when
    nsym is small)."""
    if nseg < 1 or nsym < 0 or align < 1:
        raise ValueError("segment_bounds: nseg >= 1, nsym >= 0, align >= 1")
    cuts = [0] + [_round_down(nsym * g // nseg, align) for g in range(1, nseg)] + [nsym]
    cuts = [min(max(c, 0), nsym) for c in cuts]
    for i in range(1, len(cuts)):
        cuts[i] = max(cuts[i], cuts[i - 1])
    return [(cuts[g], cuts[g + 1]) for g in range(nseg)]


def tx_halo_symbols(ntaps: int, sps: int, align: int = ALIGN_SYMBOLS) -> int:
    """Symbols a TX segment starts early: the FIR span ceil((L - 1) / sps), rounded up to
    `align` so the segment's first symbol keeps the long call's row alignment."""
    need = (max(ntaps, 1) - 1 + sps - 1) // sps
    return (need + align - 1) // align * align


def rx_halo_samples(ntaps: int, sps: int, align: int = ALIGN_SYMBOLS) -> int:
    """Samples an RX segment starts early: L - 1, rounded up to `align` symbols of samples."""
    unit = align * sps
    return (max(ntaps, 1) - 1 + unit - 1) // unit * unit


def first_kept(n: int, sps: int, D: int) -> int:
    """Kept instants (samples k * sps + D) with sample index < n."""
    return 0 if n <= D else (n - D + sps - 1) // sps


def tx_segment(a: int, b: int, ntaps: int, sps: int, bps: int, align: int = ALIGN_SYMBOLS) -> dict:
    """Plan of TX segment [a, b) symbols: the handle's start symbol, its carrier s0, the bit
    range to feed and the samples to drop."""
    h = min(tx_halo_symbols(ntaps, sps, align), a)
    start = a - h
    return {"start_symbol": start, "s0": start * sps, "bits": (start * bps, b * bps), "drop": h * sps,
            "samples": (a * sps, b * sps)}


def rx_segment(na: int, nb: int, ntaps: int, sps: int, align: int = ALIGN_SYMBOLS) -> dict:
    """Plan of RX segment [na, nb) samples (na a multiple of align * sps): the handle's carrier
    s0, the input range to feed, the local outputs to drop and the global kept-instant range
    it yields (decimation offset D = L - 1, the loopback contract)."""
    D = ntaps - 1
    if na % (align * sps):
        raise ValueError("rx_segment: the segment start must be a multiple of align * sps samples")
    n0 = na - min(rx_halo_samples(ntaps, sps, align), na)
    k_lo, k_hi = first_kept(na, sps, D), first_kept(nb, sps, D)
    # local instant j is global instant j + n0 / sps (n0 is a multiple of sps)
    return {"s0": n0, "input": (n0, nb), "drop": k_lo - n0 // sps, "instants": (k_lo, k_hi)}


# Phasors that carry state from symbol to symbol in f32 (DMPSK phase, dmpsk.rs:29-33; MFSK
# cur_coef / phase_offset, mfsk.rs:68-75; BFSK phase / previous bit, bfsk.rs:43-55): a handle
# started a halo early begins from the initial state, not the state the long stream has at the
# halo, so a time segment other than the first would come out wrong. They are not sharded.
SERIAL_STATE_PHASORS = ("DMPSK", "MFSK", "BFSK")


def _to_device(x, device):
    """The slice on `device` (a handle's kernels only read their own device's memory)."""
    if type(x).__module__.startswith("torch") and x.is_cuda and x.device.index != device:
        return x.to(f"cuda:{device}")
    return x


def run_tx_segment(pkg, carrier_freq, phasor, taps, sps, bits, a, b, dtype=0, device=0, stream=None):
    """TX samples [a * sps, b * sps) of the stream whose bits are `bits` (one byte per bit,
    the whole stream's buffer), through a fresh DigitalModulator started a halo early.
    Raises ValueError for phasors with serial symbol state (SERIAL_STATE_PHASORS) unless the
    segment starts at symbol 0."""
    if type(phasor).__name__ in SERIAL_STATE_PHASORS and a > 0:
        raise ValueError(f"{type(phasor).__name__} carries its phase from symbol to symbol: "
                         "a time segment cannot start mid-stream")
    plan = tx_segment(a, b, len(taps), sps, phasor.bits_per_symbol())
    mod = pkg.DigitalModulator(pkg.Carrier(carrier_freq, plan["s0"]), phasor, sps, taps=taps, dtype=dtype,
                               device=device)
    lo, hi = plan["bits"]
    y = mod.process(_to_device(bits[lo:hi], device), stream=stream)
    return y[plan["drop"]:]


def run_rx_segment(pkg, carrier_freq, taps, sps, slicer, x, na, nb, in_dtype=0, device=0, stream=None):
    """RX decimated I/Q and decisions of the kept instants whose sample lies in [na, nb), from the
    stream `x` (the whole stream's (n, 2) buffer), through a fresh DemodulatorRx started a
    halo early; returns (iq, sym, (k_lo, k_hi))."""
    plan = rx_segment(na, nb, len(taps), sps)
    rx = pkg.DemodulatorRx(pkg.Carrier(carrier_freq, plan["s0"]), taps, decim=sps, decim_offset=len(taps) - 1,
                           mix=pkg.MIX_COMPLEX, slicer=slicer, in_dtype=in_dtype, out_dtype=in_dtype, device=device)
    lo, hi = plan["input"]
    iq, sym = rx.process(_to_device(x[lo:hi], device), stream=stream)
    d = plan["drop"]
    return iq[d:], sym[d:], plan["instants"]
