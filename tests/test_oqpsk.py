"""OQPSK through the EvenOddOffset source: oqpsk.rs:16-26 over
data.rs:81-123, as `modulate` builds it (modulate.rs:85,101-107).

CPU: the oracle's TX chain with the offset source equals the oracle's restatement of the
`modulate --iq` CLI path on the same bits (both follow the reference structure), and the C ABI
rejects what EvenOddOffset::new asserts (data.rs:91-92).
GPU: sample-and-hold output bit-exact to the oracle (reference semantics, including Q = bit 0
before the first Q tick); pulse-shaped output (GLUE: Q impulses at the Q ticks) within the
f32 tolerance; chunked calls equal one call; loopback decisions from the I and Q decision
instants (L-1 and L-1+sps/2) equal the bits sent.
"""
import ctypes

import numpy as np
import pytest

SEED = 0x0DD0E0E0


def oq_oracle(o):
    return o.new_phasor(o.OQPSK, 1.0)


def test_oracle_chain_equals_cli_iq(o):
    """or_tx_chain_src(even_odd) == or_modulate_cli('oqpsk', --iq) on the same bits."""
    sr, br = 10000, 1250                    # sps 8
    bits = o.prng_bits(SEED, 2 * 300)
    text = "".join("1" if b else "0" for b in bits)
    n = 2 * len(bits) // 2 * 8 + 16
    out = np.zeros(2 * n, np.float32)
    k = o.lib().or_modulate_cli(b"oqpsk", sr, br, 1000, 0, 1, text.encode(), len(text),
                                out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), len(out))
    assert k > 0
    cli = out[:k].reshape(-1, 2)
    chain = o.tx_chain(oq_oracle(o), bits, 8, None, o.sample_freq(1000, sr), 0,
                       out_mode=o.OUT_IQ_BASEBAND, even_odd=True)
    assert np.array_equal(cli.view(np.uint32), chain.view(np.uint32))
    # Q before the first Q tick is bit 0 -> -sqrt(1/2) (data.rs:84, oqpsk.rs:23-25)
    assert np.all(chain[:4, 1] == np.float32(-np.sqrt(np.float32(0.5))))


def test_offset_source_arguments(m):
    """EvenOddOffset::new asserts bps == 2 and an even sps (data.rs:91-92)."""
    with pytest.raises(m.ModemPanic):
        m.DigitalModulator(m.Carrier(m.Freq(1, 4)), m.QPSK(0.0, 1.0), 5, None, even_odd_offset=True)
    with pytest.raises(m.ModemPanic):
        m.DigitalModulator(m.Carrier(m.Freq(1, 4)), m.QAM(4, 0.0, 1.0), 4, None, even_odd_offset=True)
    L = m.load_library()
    lut = m.OQPSK(1.0).lut()
    d = m._TxDesc()
    d.bits_per_symbol, d.lut, d.samples_per_symbol = 2, m._fptr(lut), 8
    d.ntaps, d.sample_freq, d.s0, d.dtype, d.out_mode = 0, 0.5, 0, 0, 0
    h = ctypes.c_void_p()
    d.q_offset = 3                          # only samples_per_symbol / 2 is a source the crate has
    assert L.modem_tx_create(ctypes.byref(d), 0, ctypes.byref(h)) == m.ERR_INVALID_ARG


# ------------------------------------------------------------------------------ GPU ----
def _gpu_tx(m, torch, bits, sps, taps, w, out_mode, flush=False, chunks=None):
    tx = m.DigitalModulator(m.Carrier(w), m.OQPSK(1.0), sps, taps, out_mode=out_mode, even_odd_offset=True)
    parts = []
    if chunks is None:
        parts.append(tx.process(torch.from_numpy(bits).cuda()))
    else:
        pos = 0
        for c in chunks:
            parts.append(tx.process(torch.from_numpy(bits[pos:pos + c].copy()).cuda()))
            pos += c
    if flush:
        parts.append(tx.flush(like=parts[0]))
    return torch.cat(parts).cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("sps", [2, 4, 8, 16, 44])
def test_oqpsk_sample_and_hold_bit_exact(m, o, torch_cuda, sps):
    bits = o.prng_bits(SEED + sps, 2 * 401 + 1)     # ragged tail bit is dropped
    got = _gpu_tx(m, torch_cuda, bits, sps, None, 0.5, out_mode=1)
    ref = o.tx_chain(oq_oracle(o), bits, sps, None, 0.5, 0, out_mode=o.OUT_IQ_BASEBAND, even_odd=True)
    assert got.shape == ref.shape
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.gpu
def test_oqpsk_sample_and_hold_mixed(m, o, torch_cuda):
    w = o.sample_freq(1000, 10000)
    bits = o.prng_bits(SEED + 1, 2 * 500)
    got = _gpu_tx(m, torch_cuda, bits, 8, None, w, out_mode=0)
    ref = o.tx_chain(oq_oracle(o), bits, 8, None, w, 0, out_mode=o.OUT_IQ_MIXED, even_odd=True)
    assert np.abs(got - ref).max() <= 1e-5 * np.abs(ref).max()


@pytest.mark.gpu
@pytest.mark.parametrize("sps,L", [(4, 65), (8, 129), (2, 33)])
def test_oqpsk_pulse_shaped(m, o, torch_cuda, sps, L):
    bits = o.prng_bits(SEED + 2, 2 * 1500)
    taps = m.rrc_taps(L, sps, 0.35)
    w = o.sample_freq(1, 4)
    got = _gpu_tx(m, torch_cuda, bits, sps, taps, w, out_mode=0, flush=True)
    nflush = (L - 1 + sps // 2 + sps - 1) // sps
    ref = o.tx_chain(oq_oracle(o), bits, sps, taps, w, 0, flush_syms=nflush, out_mode=o.OUT_IQ_MIXED,
                     even_odd=True)
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() <= 1e-5 * np.abs(ref).max()


@pytest.mark.gpu
@pytest.mark.parametrize("taps_L", [0, 65])
def test_oqpsk_streaming_equals_one_call(m, o, torch_cuda, taps_L):
    sps = 8
    bits = o.prng_bits(SEED + 3, 2 * 2000 + 1)
    taps = None if taps_L == 0 else m.rrc_taps(taps_L, sps, 0.35)
    one = _gpu_tx(m, torch_cuda, bits, sps, taps, 0.25, out_mode=1)
    chunks = [1, 0, 3, 998, 7, 2000, len(bits) - 3009]
    many = _gpu_tx(m, torch_cuda, bits, sps, taps, 0.25, out_mode=1, chunks=chunks)
    assert np.array_equal(one.view(np.uint32), many.view(np.uint32))


@pytest.mark.gpu
def test_oqpsk_loopback_decisions(m, o, torch_cuda):
    """I decided at n = k*sps + L-1, Q half a symbol later: the signs equal the bits sent."""
    torch = torch_cuda
    sps, L = 8, 129
    nsym = 4000
    bits = o.prng_bits(SEED + 4, 2 * nsym)
    taps = m.rrc_taps(L, sps, 0.35)
    w = m.Freq(1, 4).sample_freq()
    y = torch.from_numpy(_gpu_tx(m, torch, bits, sps, taps, w, out_mode=0, flush=True)).cuda()
    iq = []
    for off in (L - 1, L - 1 + sps // 2):
        rx = m.DemodulatorRx(m.Carrier(w), taps, decim=sps, decim_offset=off, mix=m.MIX_COMPLEX)
        got, _ = rx.process(y, want_sym=False)
        iq.append(got.cpu().numpy())
    b = bits.reshape(-1, 2)
    i_dec = (iq[0][:nsym, 0] > 0).astype(np.uint8)
    q_dec = (iq[1][:nsym, 1] > 0).astype(np.uint8)
    assert np.array_equal(i_dec, b[:, 0]) and np.array_equal(q_dec, b[:, 1])
