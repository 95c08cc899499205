"""Time-segment sharding of one long stream (rust-modem_amd/segments.py).

CPU: the segment plans (halo, carrier s0, dropped outputs) reproduce one long stream exactly
when the segments run through the oracle (the reference loop restated in C, the checker).
GPU: the same plans through the product handles give samples, I/Q and decisions bit-identical
to one long call, and equal to the oracle within the f32 tolerance.
"""
import numpy as np
import pytest

from conftest import CONFIGS, graft, oracle_phasor, oracle_slicer, product_phasor, sent_symbols

SEED = 0x5EED5E60


def seg():
    graft.package()
    import rust_modem_amd.segments as s
    return s


def test_segment_bounds_cover_and_align():
    s = seg()
    for nsym, G in [(0, 1), (10, 4), (4096, 3), (1 << 20, 8), (1000003, 7)]:
        b = s.segment_bounds(nsym, G)
        assert len(b) == G and b[0][0] == 0 and b[-1][1] == nsym
        assert all(b[i][1] == b[i + 1][0] for i in range(G - 1))
        assert all(a % s.ALIGN_SYMBOLS == 0 for a, _ in b)
        if nsym >= 64 * G * 4:
            sizes = [hi - lo for lo, hi in b]
            assert max(sizes) - min(sizes) <= 2 * s.ALIGN_SYMBOLS
    with pytest.raises(ValueError):
        s.segment_bounds(10, 0)
    with pytest.raises(ValueError):
        s.rx_segment(4, 100, 129, 4)          # not on the alignment grid


def test_halo_sizes():
    s = seg()
    for L, sps in [(33, 4), (65, 4), (129, 4), (513, 8), (1, 4)]:
        h = s.tx_halo_symbols(L, sps)
        assert h % s.ALIGN_SYMBOLS == 0 and h * sps >= L - 1
        hs = s.rx_halo_samples(L, sps)
        assert hs % (s.ALIGN_SYMBOLS * sps) == 0 and hs >= L - 1


@pytest.mark.parametrize("cfg,G", [("c3_qam16", 3), ("c2_qpsk", 4), ("c5_qam256", 2)])
def test_segments_reproduce_one_stream_oracle(o, cfg, G):
    """Oracle TX and RX run segment by segment per the plans == one oracle call, bit-exact."""
    s = seg()
    name, bps, L, sps = CONFIGS[cfg]
    nsym = 3000 + 17
    bits = o.prng_bits(SEED, nsym * bps)
    taps = o.rrc_taps(L, sps, 0.35)
    w = o.sample_freq(1, 4)
    s0 = 0
    y = o.tx_chain(oracle_phasor(o, name), bits, sps, taps, w, s0)
    iq, sym = o.rx_chain(y, w, s0, o.MIX_COMPLEX, taps, sps, L - 1, oracle_slicer(o, name, bps))
    ys, iqs, syms = [], [], []
    for a, b in s.segment_bounds(nsym, G):
        p = s.tx_segment(a, b, L, sps, bps)
        lo, hi = p["bits"]
        yg = o.tx_chain(oracle_phasor(o, name), bits[lo:hi], sps, taps, w, p["s0"])
        ys.append(yg[p["drop"]:])
        assert len(ys[-1]) == (b - a) * sps
        r = s.rx_segment(a * sps, b * sps, L, sps)
        lo, hi = r["input"]
        gi, gs = o.rx_chain(y[lo:hi], w, r["s0"], o.MIX_COMPLEX, taps, sps, L - 1, oracle_slicer(o, name, bps))
        iqs.append(gi[r["drop"]:])
        syms.append(gs[r["drop"]:])
        assert len(syms[-1]) == r["instants"][1] - r["instants"][0]
    assert np.array_equal(np.concatenate(ys), y)
    assert np.array_equal(np.concatenate(iqs), iq)
    assert np.array_equal(np.concatenate(syms), sym)
    # kept instant k sits at sample k * sps + L - 1, the peak of symbol k's TX * RX pulse
    assert np.array_equal(sym, sent_symbols(bits, bps)[: len(sym)])


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,G,dtype", [("c3_qam16", 4, 0), ("c2_qpsk", 3, 0), ("c5_qam256", 2, 0),
                                         ("c3_qam16", 3, 1)])
def test_time_segments_equal_one_stream(m, o, torch_cuda, cfg, G, dtype):
    """Segments through fresh handles (halo, carrier s0, drop) == one long call, bit-exact on
    the device (TX samples, RX I/Q, decisions); decisions also equal the symbols sent."""
    torch = torch_cuda
    s = seg()
    name, bps, L, sps = CONFIGS[cfg]
    nsym = (1 << 16) + 37
    bits = torch.from_numpy(o.prng_bits(SEED + 1, nsym * bps)).cuda()
    taps = m.rrc_taps(L, sps, 0.35)
    w = o.sample_freq(1, 4)
    s0 = 0
    tx = m.DigitalModulator(m.Carrier(w, s0), product_phasor(m, name), sps, taps, dtype=dtype)
    y = tx.process(bits)
    rx = m.DemodulatorRx(m.Carrier(w, s0), taps, decim=sps, decim_offset=L - 1, mix=m.MIX_COMPLEX,
                         slicer=product_phasor(m, name).slicer(), in_dtype=dtype, out_dtype=dtype)
    iq, sym = rx.process(y)
    ys, iqs, syms = [], [], []
    for a, b in s.segment_bounds(nsym, G):
        ys.append(s.run_tx_segment(m, w, product_phasor(m, name), taps, sps, bits, a, b, dtype=dtype))
        gi, gs, (k_lo, k_hi) = s.run_rx_segment(m, w, taps, sps, product_phasor(m, name).slicer(), y,
                                               a * sps, b * sps, in_dtype=dtype)
        assert gs.shape[0] == k_hi - k_lo
        iqs.append(gi)
        syms.append(gs)
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(ys), y)
    assert torch.equal(torch.cat(iqs), iq)
    assert torch.equal(torch.cat(syms), sym)
    sent = torch.from_numpy(sent_symbols(bits.cpu().numpy(), bps)).cuda()
    assert torch.equal(sym, sent[: sym.shape[0]])
