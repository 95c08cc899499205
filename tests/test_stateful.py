"""Phasors whose (i, q) depend on the symbol count or the sample index:
DCQPSK (dcqpsk.rs), CPFSK (cpfsk.rs), MSK over EvenOddOffset (msk.rs + data.rs:81-123), on
the GPU's per-sample phasor kernel (tx_phasor) against the oracle's DigitalModulator
(modulator.rs:85-100, which passes the post-increment carrier sample to the phasor).

DCQPSK's values come from a host table built with the reference's f32 formulas: bit-exact.
CPFSK and MSK take sin/cos of a per-sample argument: the f32 sample tolerance.
"""
import ctypes

import numpy as np
import pytest

SEED = 0x57A7E000


def test_sample_dependent_phasors_have_no_table(m):
    with pytest.raises(m.ModemError) as e:
        m.DCQPSK(1.0).lut()
    assert e.value.status == m.ERR_UNSUPPORTED
    with pytest.raises(m.ModemPanic):
        m.MSK(1.0, 45)                                     # msk.rs:14
    L = m.load_library()
    d = m.DCQPSK(1.0)._desc()
    out = np.zeros(16, np.float32)
    assert L.modem_phasor_lut(ctypes.byref(d), m._fptr(out)) == m.ERR_UNSUPPORTED
    assert m.CPFSK(4, m.Rates(250, 10000), 1.0, 1).bits_per_symbol() == 4


def _gpu(m, torch, phasor, bits, sps, s0, w, out_mode=1, offset=False, chunks=None):
    tx = m.DigitalModulator(m.Carrier(w, s0), phasor, sps, None, out_mode=out_mode, even_odd_offset=offset)
    if chunks is None:
        return tx.process(torch.from_numpy(bits).cuda()).cpu().numpy()
    parts, pos = [], 0
    for c in chunks:
        parts.append(tx.process(torch.from_numpy(bits[pos:pos + c].copy()).cuda()))
        pos += c
    return torch.cat(parts).cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("sps", [1, 4, 45])
def test_dcqpsk_bit_exact(m, o, torch_cuda, sps):
    bits = o.prng_bits(SEED + sps, 2 * 777 + 1)
    got = _gpu(m, torch_cuda, m.DCQPSK(1.0), bits, sps, 0, 0.5)
    ref = o.tx_chain(o.new_phasor(o.DCQPSK, 1.0), bits, sps, None, 0.5, 0, out_mode=o.OUT_IQ_BASEBAND)
    assert got.shape == ref.shape
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.gpu
def test_dcqpsk_parity_continues_across_calls(m, o, torch_cuda):
    bits = o.prng_bits(SEED + 1, 2 * 1000 + 1)
    one = _gpu(m, torch_cuda, m.DCQPSK(1.0), bits, 8, 0, 0.5)
    many = _gpu(m, torch_cuda, m.DCQPSK(1.0), bits, 8, 0, 0.5, chunks=[3, 0, 2, 995, 1, len(bits) - 1001])
    assert np.array_equal(one.view(np.uint32), many.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("s0", [0, (1 << 20) + 5])
def test_cpfsk(m, o, torch_cuda, s0):
    br, sr = 250, 10000
    sps = sr // br
    bits = o.prng_bits(SEED + 2, 4 * 600 + 3)
    w = o.sample_freq(1000, sr)
    ph = m.CPFSK(4, m.Rates(br, sr), 1.0, 1)
    for out_mode in (1, 0):
        got = _gpu(m, torch_cuda, ph, bits, sps, s0, w, out_mode=out_mode)
        ref = o.tx_chain(o.new_phasor(o.CPFSK, 4, br, sr, 1.0, 1), bits, sps, None, w, s0, out_mode=out_mode)
        assert got.shape == ref.shape
        assert np.abs(got - ref).max() <= 1e-5 * np.abs(ref).max(), out_mode
    chunked = _gpu(m, torch_cuda, ph, bits, sps, s0, w, chunks=[5, 1000, 7, len(bits) - 1012])
    assert np.array_equal(chunked.view(np.uint32), _gpu(m, torch_cuda, ph, bits, sps, s0, w).view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("sps", [2, 8, 40])
def test_msk_even_odd(m, o, torch_cuda, sps):
    bits = o.prng_bits(SEED + 3, 2 * 500 + 1)
    w = o.sample_freq(1000, 10000)
    got = _gpu(m, torch_cuda, m.MSK(1.0, sps), bits, sps, 0, w, offset=True)
    ref = o.tx_chain(o.new_phasor(o.MSK, 1.0, sps), bits, sps, None, w, 0, out_mode=o.OUT_IQ_BASEBAND,
                     even_odd=True)
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() <= 1e-5 * np.abs(ref).max()
    chunked = _gpu(m, torch_cuda, m.MSK(1.0, sps), bits, sps, 0, w, offset=True,
                   chunks=[1, 2, 3, 500, len(bits) - 506])
    one = _gpu(m, torch_cuda, m.MSK(1.0, sps), bits, sps, 0, w, offset=True)
    assert np.array_equal(chunked.view(np.uint32), one.view(np.uint32))
