"""The `demodulate` front-end: demodulate.rs:29-43 — analytic signal
(x, Hilbert(x)), Demodulator with the 64-sample PLL lock (demodulator.rs:32-36, pll.rs:16-22)
and the full-rate real-input mix + low-pass (demodulator.rs:44-56) — on the GPU (Hilbert on
modem_fir, the demodulator on modem_rx with the locked phase offset) against the oracle's
restatement with the same filters.

The binary's own coefficient tables (demodulate.rs:47-150) are not copied here: the filters
are designed in this file (a 23-tap windowed Hilbert and a 64-tap windowed-sinc low-pass with
the binary's 1 kHz pass band at 10 kHz), so parity covers the structure, not those numbers.
Tolerance: the PLL offset (host, glibc) bit-exact; outputs within 1e-5 of their maximum.
"""
import ctypes

import numpy as np
import pytest


def hilbert_taps(n=23):
    k = np.arange(n) - (n - 1) // 2
    h = np.where(k % 2 != 0, 2.0 / (np.pi * np.where(k == 0, 1, k)), 0.0)
    return (h * np.hamming(n)).astype(np.float32)


def lowpass_taps(n=64, fc=1250.0, sr=10000.0):
    t = np.arange(n) - (n - 1) / 2.0
    h = 2 * fc / sr * np.sinc(2 * fc / sr * t) * np.hamming(n)
    return (h / h.sum()).astype(np.float32)


def test_pll_lock_matches_oracle(m, o):
    """modem_pll_lock (host) == the oracle's PLL over the same 64 analytic samples."""
    rng = np.random.default_rng(5)
    x = rng.standard_normal((64, 2)).astype(np.float32)
    w = o.sample_freq(900, 10000)
    off = (ctypes.c_float * 1)(0.0)
    assert m.load_library().modem_pll_lock(w, 0, m._fptr(np.ascontiguousarray(x)), 64, off) == 0
    p = (ctypes.c_float * 1)(0.0)
    for k in range(64):
        o.lib().or_pll_handle(p, o.carrier_phases(w, k, 1)[0], float(x[k, 0]), float(x[k, 1]))
    assert np.float32(off[0]).view(np.uint32) == np.float32(p[0]).view(np.uint32)


@pytest.mark.gpu
@pytest.mark.parametrize("chunks", [None, [1000, 1, 5000]])
def test_demodulate_front_end(m, o, torch_cuda, chunks):
    torch = torch_cuda
    sr, cf = 10000, 900
    w = o.sample_freq(cf, sr)
    # input: a BPSK passband (the modulator's real output, modulate.rs:128-133) scaled to i16
    # and back, as `demodulate` reads i16 (demodulate.rs:29)
    bits = o.prng_bits(77, 300)
    y = o.tx_chain(o.new_phasor(o.BPSK, np.float32(np.pi / 4), 1.0), bits, 45, None, w, 0,
                   out_mode=o.OUT_REAL)
    x = np.round(y * 12000.0).astype(np.int16).astype(np.float32)
    ht, lp = hilbert_taps(), lowpass_taps()
    ref_i, ref_q, ref_off = o.demodulate_front(w, x, ht, lp)

    xd = torch.from_numpy(x).cuda()
    hil = m.FIRFilter(ht).process(xd)                       # analytic imag (demodulate.rs:32-34)
    sig = torch.stack([xd, hil], dim=1).contiguous()
    dem = m.Demodulator(m.Carrier(m.Freq(cf, sr)), lp)
    rest = dem.lock_phase(sig)
    assert np.float32(dem.phase_offset).view(np.uint32) == np.float32(ref_off).view(np.uint32)
    if chunks is None:
        got = dem.process(rest.contiguous()).cpu().numpy()
    else:
        parts, pos = [], 0
        for c in chunks + [rest.shape[0] - sum(chunks)]:
            parts.append(dem.process(rest[pos:pos + c].contiguous()))
            pos += c
        got = torch.cat(parts).cpu().numpy()
    assert got.shape == (len(ref_i), 2)
    ref = np.stack([ref_i, ref_q], 1)
    assert np.abs(got - ref).max() <= 1e-5 * np.abs(ref).max()
