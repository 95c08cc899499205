"""Phasors whose (i, q) depend on the symbol count, the sample index or a phase carried from
symbol to symbol: DCQPSK (dcqpsk.rs), CPFSK (cpfsk.rs), MSK over
EvenOddOffset (msk.rs + data.rs:81-123), DMPSK (dmpsk.rs), MFSK (mfsk.rs), BFSK (bfsk.rs), on
the GPU's per-sample phasor kernel (tx_phasor; the last three after the serial state scan
tx_scan) against the oracle's DigitalModulator (modulator.rs:85-100, which passes the
post-increment carrier sample to the phasor).

DCQPSK's values come from a host table built with the reference's f32 formulas: bit-exact.
The others take sin/cos of a per-sample argument: the f32 sample tolerance. The scanned
phases must follow the reference's f32 rounding exactly — long streams (20 000 symbols, where
a phase that drifted by an ulp per step would be off by far more than the tolerance) check it.
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


SCANNED = {
    "dqpsk": (lambda m: m.DMPSK(2, 1.0, 0.7853982, 1.5707964),
              lambda o: o.new_phasor(o.DMPSK, 2, 1.0, 0.7853982, 1.5707964), 2),
    "dbpsk": (lambda m: m.DMPSK(1, 1.0, 0.7853982, 3.1415927),
              lambda o: o.new_phasor(o.DMPSK, 1, 1.0, 0.7853982, 3.1415927), 1),
    "mfsk": (lambda m: m.MFSK(4, m.Freq(50, 10000), 1.0, "increase"),
             lambda o: o.new_phasor(o.MFSK, 4, o.sample_freq(50, 10000), 1.0, 1), 4),
    "mfsk_default": (lambda m: m.MFSK(3, m.Freq(120, 10000), 0.5, "default"),
                     lambda o: o.new_phasor(o.MFSK, 3, o.sample_freq(120, 10000), 0.5, 0), 3),
    "bfsk": (lambda m: m.BFSK(m.Freq(200, 10000), 1.0),
             lambda o: o.new_phasor(o.BFSK, o.sample_freq(200, 10000), 1.0), 1),
}


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(SCANNED))
def test_scanned_phasors(m, o, torch_cuda, name):
    mk, ok, bps = SCANNED[name]
    sps = 4
    bits = o.prng_bits(SEED + 4, bps * 20000 + 1)
    w = o.sample_freq(1000, 10000)
    got = _gpu(m, torch_cuda, mk(m), bits, sps, 3, w, out_mode=1)
    ref = o.tx_chain(ok(o), bits, sps, None, w, 3, out_mode=o.OUT_IQ_BASEBAND)
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() <= 1e-5 * np.abs(ref).max()
    # the state carries across calls (the scan resumes from the handle's state)
    chunked = _gpu(m, torch_cuda, mk(m), bits, sps, 3, w, out_mode=1,
                   chunks=[bps * 3 + 1, 0, bps * 7000, len(bits) - bps * 7003 - 1])
    assert np.array_equal(chunked.view(np.uint32), got.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(SCANNED))
def test_scanned_batch_equals_single_calls(m, o, torch_cuda, name):
    """A bank of channels of one scanned phasor through DigitalModulator.process_batch (the
    channel-parallel scan, tx_scan_batch: one lane per channel) equals one process() per channel
    bit for bit, over two calls (the handles' carried states resume) with ragged lengths (leftover
    bits, an empty channel) and different carrier offsets; the first call's samples are also within
    the f32 tolerance of the oracle for two channels. DMPSK runs the 64-channel bank of the
    VERDICT r05 item 7 (dmpsk.rs:29-33), the other kinds 9 channels (two waves' worth of lanes
    is the same code)."""
    torch = torch_cuda
    mk, ok, bps = SCANNED[name]
    nch = 64 if name == "dqpsk" else 9
    sps = 4
    w = o.sample_freq(1000, 10000)
    lens = [[bps * (1500 + 37 * c) + c % bps, bps * (900 + 11 * c)] for c in range(nch)]
    lens[5] = [0, bps * 300]
    streams = [o.prng_bits(SEED + 100 + c, sum(lens[c])) for c in range(nch)]
    s0s = [3 + 17 * c for c in range(nch)]
    bank = [m.DigitalModulator(m.Carrier(w, s0s[c]), mk(m), sps, None, out_mode=1) for c in range(nch)]
    singles = [m.DigitalModulator(m.Carrier(w, s0s[c]), mk(m), sps, None, out_mode=1) for c in range(nch)]
    pos = [0] * nch
    for call in range(2):
        chunks = [torch.from_numpy(streams[c][pos[c]:pos[c] + lens[c][call]].copy()).cuda() for c in range(nch)]
        got = m.DigitalModulator.process_batch(bank, chunks)
        for c in range(nch):
            want = singles[c].process(chunks[c])
            assert got[c].shape == want.shape, (c, call)
            assert np.array_equal(got[c].cpu().numpy().view(np.uint32), want.cpu().numpy().view(np.uint32)), (c, call)
            assert bank[c].carrier.sample == singles[c].carrier.sample
            if call == 0 and c in (0, nch - 1):
                ref = o.tx_chain(ok(o), streams[c][:lens[c][0]], sps, None, w, s0s[c], out_mode=o.OUT_IQ_BASEBAND)
                g = got[c].cpu().numpy()
                assert g.shape == ref.shape and np.abs(g - ref).max() <= 1e-5 * np.abs(ref).max()
            pos[c] += lens[c][call]
