"""GPU parity of the split-f16 range machinery and at full size (SURVEY.md §8c tolerances).

The matrix-core FIRs split every operand into f16 hi + lo halves, so the magnitude of the
data is part of correctness:
  * RX: each tile of mixed samples is used as it is when its max lies in [2^-3, 2^15), else
    scaled by 2^ka (tile_ka: steps of 8 binades) — on the fast path with a predicted exponent
    that must match, otherwise on the general path. Inputs at 2^-8 .. 2^17 of the unit
    constellation, and a stream whose amplitude steps by 2^10 inside a tile, against the
    oracle (demodulator.rs:44-56 mix, fir.rs:18-34 fold).
  * TX: the LUT and the taps are scaled into range on the host (lut_scale_exp /
    tap_scale_exp): constellations at 1e-3 and 1e5, taps scaled by 1e-4, and a non-integer
    LUT (8-PSK at phase 0.1), against the oracle (modulator.rs:45-48, fir.rs:18-34).
  * Full size: C3 (2^24 samples) TX samples and RX I/Q compared sample by sample with the
    oracle, C5 (513 taps, sps 8) over a 2^20-sample prefix in f32 and f16 storage.
Each test prints the observed max|d| / max|y_ref| beside its bound.
"""
import numpy as np
import pytest

from conftest import CONFIGS, oracle_phasor, oracle_slicer, product_phasor, sent_symbols

pytestmark = pytest.mark.gpu

SEED = 0x5EED1000


def host(t):
    return t.detach().cpu().numpy()


def rel_err(got, ref):
    return float(np.abs(got.astype(np.float64) - ref).max() / np.abs(ref).max())


def report(what, err, bound):
    print(f"\n[range] {what}: max|d|/max|y| = {err:.3g} (bound {bound:.3g})", flush=True)
    assert err <= bound, f"{what}: {err} > {bound}"


def qam16_rx(m, taps, w, amp, s0=0):
    name, bps, L, sps = CONFIGS["c3_qam16"]
    return m.DemodulatorRx(m.Carrier(w, s0), taps, decim=sps, decim_offset=L - 1, mix=m.MIX_COMPLEX,
                           slicer=m.QAM(4, 0.0, amp).slicer())


@pytest.fixture(scope="module")
def c3_stream(o):
    """2^21 C3 samples from the oracle TX (about 500 RX tiles of 1024 instants: more than one
    tile per workgroup, so the fast path's exponent prediction carries across tiles)."""
    name, bps, L, sps = CONFIGS["c3_qam16"]
    nsym = (1 << 21) // sps
    bits = o.prng_bits(SEED, nsym * bps)
    taps = o.rrc_taps(L, sps, 0.35)
    w = o.sample_freq(1, 4)
    x = o.tx_chain(oracle_phasor(o, name), bits, sps, taps, w, 0, flush_syms=(L - 1 + sps - 1) // sps)
    return bits, taps, w, x


@pytest.mark.parametrize("k", [-8, -4, 16, 17])
def test_rx_scaled_input(m, o, torch_cuda, c3_stream, k):
    """RX input at 2^k of the unit-amplitude stream: I/Q within 1e-5 of the oracle's max,
    decisions bit-exact (the slicer scaled with the constellation)."""
    name, bps, L, sps = CONFIGS["c3_qam16"]
    bits, taps, w, x0 = c3_stream
    amp = float(2.0 ** k)
    x = (x0 * np.float32(amp)).astype(np.float32)
    riq, rsym = o.rx_chain(x, w, 0, o.MIX_COMPLEX, taps, sps, L - 1, o.qam_axis_slicer(bps, amp))
    giq, gsym = qam16_rx(m, taps, w, amp).process(torch_cuda.from_numpy(x).cuda())
    giq, gsym = host(giq), host(gsym)
    assert giq.shape == riq.shape
    report(f"RX input x 2^{k}", rel_err(giq, riq), 1e-5)
    assert np.array_equal(gsym, rsym)
    assert np.array_equal(gsym[: len(bits) // bps], sent_symbols(bits, bps))


def test_rx_amplitude_step_inside_a_tile(m, o, torch_cuda, c3_stream):
    """Amplitude steps by 2^10 at a sample that is not a tile boundary: I/Q within 1e-5 of the
    global max, each side within 1e-5 of its own max away from the tile that holds the step,
    decisions equal the oracle's (its slicer follows the unit constellation)."""
    name, bps, L, sps = CONFIGS["c3_qam16"]
    bits, taps, w, x0 = c3_stream
    step = 1_000_003
    x = x0.copy()
    x[step:] *= np.float32(1024.0)
    riq, rsym = o.rx_chain(x, w, 0, o.MIX_COMPLEX, taps, sps, L - 1, o.qam_axis_slicer(bps, 1.0))
    giq, gsym = qam16_rx(m, taps, w, 1.0).process(torch_cuda.from_numpy(x).cuda())
    giq, gsym = host(giq), host(gsym)
    report("RX 2^10 step, whole stream", rel_err(giq, riq), 1e-5)
    k_step = (step - (L - 1)) // sps                  # first instant whose window sees the step
    lo, hi = slice(0, k_step - 2048), slice(k_step + (L - 1) // sps + 2048, None)
    report("RX 2^10 step, before", rel_err(giq[lo], riq[lo]), 1e-5)
    report("RX 2^10 step, after", rel_err(giq[hi], riq[hi]), 1e-5)
    assert np.array_equal(gsym, rsym)


@pytest.mark.parametrize("phasor,amp,tap_scale", [("qam16", 1e-3, 1.0), ("qam16", 1e5, 1.0),
                                                  ("qam16", 1.0, 1e-4), ("8psk", 1e-3, 1.0),
                                                  ("8psk", 1.0, 1e4)])
def test_tx_operand_scales(m, o, torch_cuda, phasor, amp, tap_scale):
    """TX constellations and taps outside the f16 window (host-side exact power-of-two
    scales of the split operands) against the oracle; the samples round trip through the RX."""
    name, bps, L, sps = CONFIGS["c3_qam16"]
    nsym = 20000
    if phasor == "qam16":
        pp, op, bps = m.QAM(4, 0.0, amp), o.new_phasor(o.QAM, 4, 0.0, amp), 4
    else:
        pp, op, bps = m.MPSK(3, 0.1, amp), o.new_phasor(o.MPSK, 3, 0.1, amp), 3
    bits = o.prng_bits(SEED + 1, nsym * bps)
    taps = (o.rrc_taps(L, sps, 0.35) * np.float32(tap_scale)).astype(np.float32)
    w = o.sample_freq(1, 4)
    flush = (L - 1 + sps - 1) // sps
    tx = m.DigitalModulator(m.Carrier(w), pp, sps, taps)
    y = tx.process(torch_cuda.from_numpy(bits).cuda())
    y = host(torch_cuda.cat([y, tx.flush(like=y)]))
    ref = o.tx_chain(op, bits, sps, taps, w, 0, flush_syms=flush)
    assert y.shape == ref.shape
    report(f"TX {phasor} amp {amp:g} taps x{tap_scale:g}", rel_err(y, ref), 1e-5)


def test_c3_full_size_against_oracle(m, o, torch_cuda):
    """BASELINE config 3 at full size (2^24 samples): every TX sample and every RX I/Q against
    the oracle (1e-5 of max), every decision bit-exact to the oracle and to the symbols sent."""
    torch = torch_cuda
    name, bps, L, sps = CONFIGS["c3_qam16"]
    N = 1 << 24
    bits_t = m.prng_bits(0x5EED0000, N // sps * bps)
    bits = host(bits_t)
    taps = m.rrc_taps(L, sps, 0.35)
    w = o.sample_freq(1, 4)
    tx = m.DigitalModulator(m.Carrier(w), product_phasor(m, name), sps, taps)
    y = tx.process(bits_t)
    rx = m.DemodulatorRx(m.Carrier(w), taps, decim=sps, decim_offset=L - 1, mix=m.MIX_COMPLEX,
                         slicer=product_phasor(m, name).slicer())
    giq, gsym = rx.process(y)
    ref = o.tx_chain(oracle_phasor(o, name), bits, sps, taps, w, 0)
    report("C3 2^24 TX samples", rel_err(host(y), ref), 1e-5)
    riq, rsym = o.rx_chain(ref, w, 0, o.MIX_COMPLEX, taps, sps, L - 1, oracle_slicer(o, name, bps))
    giq, gsym = host(giq), host(gsym)
    assert giq.shape == riq.shape
    report("C3 2^24 RX I/Q", rel_err(giq, riq), 1e-5)
    assert np.array_equal(gsym, rsym)
    assert np.array_equal(gsym, sent_symbols(bits, bps)[: len(gsym)])


@pytest.mark.parametrize("dtype", [0, 1])
def test_c5_prefix_against_oracle(m, o, torch_cuda, dtype):
    """Config 5 (256-QAM, 513 taps, sps 8) over a 2^20-sample prefix: TX samples and RX I/Q
    within 4e-5 (f32) or 2^-10 (f16 storage) of the oracle's max, decisions bit-exact."""
    torch = torch_cuda
    name, bps, L, sps = CONFIGS["c5_qam256"]
    N = 1 << 20
    bits = o.prng_bits(0x5EED0000, N // sps * bps)
    taps = m.rrc_taps(L, sps, 0.35)
    w = o.sample_freq(1, 4)
    tx = m.DigitalModulator(m.Carrier(w), product_phasor(m, name), sps, taps, dtype=dtype)
    y = tx.process(torch.from_numpy(bits).cuda())
    ref = o.tx_chain(oracle_phasor(o, name), bits, sps, taps, w, 0)
    bound = 2.0 ** -10 if dtype else 4e-5
    report(f"C5 2^20 TX samples dtype {dtype}", rel_err(host(y).astype(np.float32), ref), bound)
    rx = m.DemodulatorRx(m.Carrier(w), taps, decim=sps, decim_offset=L - 1, mix=m.MIX_COMPLEX,
                         slicer=product_phasor(m, name).slicer(), in_dtype=dtype, out_dtype=dtype)
    giq, gsym = rx.process(y)
    # the oracle RX reads what the GPU stored (f16 storage rounds the TX samples)
    xin = host(y).astype(np.float32)
    riq, rsym = o.rx_chain(xin, w, 0, o.MIX_COMPLEX, taps, sps, L - 1, oracle_slicer(o, name, bps))
    report(f"C5 2^20 RX I/Q dtype {dtype}", rel_err(host(giq).astype(np.float32), riq), bound)
    assert np.array_equal(host(gsym), rsym)
    assert np.array_equal(host(gsym), sent_symbols(bits, bps)[: len(rsym)])


@pytest.mark.parametrize("sps,L,phasor", [(4, 129, "c3_qam16"), (4, 65, "c2_qpsk"), (2, 129, "c3_qam16")])
def test_rx_f16_large_tiles_against_oracle(m, o, torch_cuda, sps, L, phasor):
    """f16 samples in and out of the RX on its 1024-instant tiles (>= 4 tiles per CU) at decim 4
    (129 and 65 taps) and decim 2 (129 taps): the tile's partial last staging slot is staged one
    sample per lane into the two f16 planes. I/Q within 2^-10 of the oracle's max (the oracle
    reads the same f16-rounded input), decisions bit-exact to the oracle and the symbols sent."""
    torch = torch_cuda
    name, bps, _, _ = CONFIGS[phasor]
    ninst = (4 * 1024 * 256) + 3 * 1024 + 77            # past rx_small_tiles on 256 CUs, ragged end
    nsym = ninst + (L - 1) // sps + 1
    bits = o.prng_bits(SEED + 7 + sps + L, nsym * bps)
    taps = o.rrc_taps(L, sps, 0.35)
    w = o.sample_freq(1, 4)
    x = o.tx_chain(oracle_phasor(o, name), bits, sps, taps, w, 0).astype(np.float16)
    xin = x.astype(np.float32)
    riq, rsym = o.rx_chain(xin, w, 0, o.MIX_COMPLEX, taps, sps, L - 1, oracle_slicer(o, name, bps))
    rx = m.DemodulatorRx(m.Carrier(w), taps, decim=sps, decim_offset=L - 1, mix=m.MIX_COMPLEX,
                         slicer=product_phasor(m, name).slicer(), in_dtype=1, out_dtype=1)
    giq, gsym = rx.process(torch.from_numpy(x).cuda())
    giq, gsym = host(giq).astype(np.float32), host(gsym)
    assert giq.shape == riq.shape and len(rsym) >= 4 * 1024 * 256
    report(f"RX f16->f16 decim {sps} {L} taps, {len(rsym)} instants", rel_err(giq, riq), 2.0 ** -10)
    assert np.array_equal(gsym, rsym)
    assert np.array_equal(gsym, sent_symbols(bits, bps)[: len(gsym)])


def test_rx_streaming_across_scales_equals_one_call(m, o, torch_cuda, c3_stream):
    """A stream whose amplitude jumps between 2^-20 and 2^12 in segments, cut into calls of
    ragged sizes (many tiles per call; each call's first exponent is predicted from where the
    previous one ended, often wrongly here). Where every tile is inside the f16 window (tile_ka
    0: the segments at 1, 2^3, 2^12) the outputs are bitwise those of one call; a scaled tile's
    low bits depend on which samples share its tile (f16 subnormal lo halves), so elsewhere
    streamed and one-call outputs agree within 1e-6 of the segment's max. Each segment, away
    from its edges, is within 1e-5 of the oracle relative to its own max."""
    torch = torch_cuda
    name, bps, L, sps = CONFIGS["c3_qam16"]
    bits, taps, w, x0 = c3_stream
    x = x0.copy()
    bounds = [0, 300_001, 700_003, 1_100_005, 1_500_007, len(x)]
    scales = [2.0 ** -8, 2.0 ** 12, 1.0, 2.0 ** -20, 2.0 ** 3]
    for (a, b), s in zip(zip(bounds, bounds[1:]), scales):
        x[a:b] *= np.float32(s)
    xt = torch.from_numpy(x).cuda()

    def rx():
        return qam16_rx(m, taps, w, 1.0)
    iq1, s1 = rx().process(xt)
    r = rx()
    iqs, ss, pos = [], [], 0
    rng = np.random.RandomState(7)
    while pos < len(x):
        c = int(rng.randint(1, 300_000))
        i_, s_ = r.process(xt[pos:pos + c])
        iqs.append(host(i_)); ss.append(host(s_)); pos += c
    siq, ssym = np.concatenate(iqs), np.concatenate(ss)
    giq, gsym = host(iq1), host(s1)
    assert siq.shape == giq.shape and ssym.shape == gsym.shape
    riq, _ = o.rx_chain(x, w, 0, o.MIX_COMPLEX, taps, sps, L - 1, o.qam_axis_slicer(bps, 1.0))
    for (a, b), s in zip(zip(bounds, bounds[1:]), scales):
        # clear of the tiles that hold an edge (a tile spanning 2^20 of dynamic range is used
        # at its max's scale: its small samples keep only their f16 hi halves)
        lo, hi = a // sps + 2048, b // sps - 2048
        report(f"RX streamed vs one call, segment x {s:g}", rel_err(siq[lo:hi], giq[lo:hi].astype(np.float64)), 1e-6)
        report(f"RX streamed segment x {s:g} vs oracle", rel_err(siq[lo:hi], riq[lo:hi]), 1e-5)
        if 1.0 <= s < 2.0 ** 15 / 2:                         # in the window: call-split invariant
            assert np.array_equal(siq[lo:hi].view(np.uint32), giq[lo:hi].view(np.uint32)), s
            assert np.array_equal(ssym[lo:hi], gsym[lo:hi]), s


def test_rx_chunk_tails(m, o, torch_cuda, c3_stream):
    """Calls whose last tile is partial at every offset class (the fast path's bounded loads and
    stores): chunk lengths around tile multiples, bitwise equal to one call."""
    torch = torch_cuda
    name, bps, L, sps = CONFIGS["c3_qam16"]
    bits, taps, w, x0 = c3_stream
    xt = torch.from_numpy(x0[: 1 << 19]).cuda()
    iq1, s1 = qam16_rx(m, taps, w, 1.0).process(xt)
    r = qam16_rx(m, taps, w, 1.0)
    iqs, ss, pos = [], [], 0
    for c in [4096 * 4 - 1, 4096 * 4 + 1, 4 * 1024 * 5 + 3, 17, 4 * 1024 * 16 - 4, 4 * 1024 * 16 + 64,
              65537, 2, 4 * 1024 * 9 + 61, 131071]:
        i_, s_ = r.process(xt[pos:pos + c])
        iqs.append(host(i_)); ss.append(host(s_)); pos += c
    i_, s_ = r.process(xt[pos:])
    iqs.append(host(i_)); ss.append(host(s_))
    assert np.array_equal(np.concatenate(iqs).view(np.uint32), host(iq1).view(np.uint32))
    assert np.array_equal(np.concatenate(ss), host(s1))


def test_tx_f16_output_only_4_byte_aligned(m, o, torch_cuda):
    """An f16 TX output that is only 4-byte aligned (a row-sliced (n, 2) float16 tensor): the
    whole-line pair stores need 8-byte alignment, so such a call takes the one-sample stores;
    the samples equal, bit for bit, those of a call into an aligned buffer."""
    torch = torch_cuda
    name, bps, L, sps = CONFIGS["c3_qam16"]
    nsym = 300_001
    bits = torch.from_numpy(o.prng_bits(SEED + 11, nsym * bps)).cuda()
    taps = m.rrc_taps(L, sps, 0.35)
    w = o.sample_freq(1, 4)

    def tx():
        return m.DigitalModulator(m.Carrier(w), product_phasor(m, name), sps, taps, dtype=1)
    ref = tx().process(bits)
    big = torch.zeros((ref.shape[0] + 1, 2), dtype=torch.float16, device="cuda")
    out = big[1:]
    assert out.data_ptr() % 8 == 4
    got = tx().process(bits, out=out)
    assert torch.equal(got.view(torch.int16), ref.view(torch.int16))
    assert torch.equal(big[0], torch.zeros(2, dtype=torch.float16, device="cuda"))


@pytest.mark.parametrize("nsamp,cuts", [
    (1 << 19, [4096 * 4 - 1, 4096 * 4 + 1, 17, 4 * 1024 * 16 - 4, 65537, 2, 4 * 1024 * 9 + 61, 131071]),
    ((1 << 23) + 4 * 1024 * 5 + 6, [(1 << 22) + 4 * 37 + 3]),
])
def test_rx_f16_chunk_tails(m, o, torch_cuda, nsamp, cuts):
    """f16 samples in and out: calls whose last tile is partial at odd offsets, bitwise equal to one
    call, on the small tiles (2^19 samples) and on the 1024-instant tiles (calls of >= 2^22
    samples). The fast path stores f16 I/Q two instants per lane (whole 128-B lines): a pair
    straddling a call's last instant must still write its first (per-dword range check)."""
    torch = torch_cuda
    name, bps, L, sps = CONFIGS["c3_qam16"]
    bits = torch.from_numpy(o.prng_bits(SEED + 21, nsamp // sps * bps)).cuda()
    taps = m.rrc_taps(L, sps, 0.35)
    w = o.sample_freq(1, 4)
    x = m.DigitalModulator(m.Carrier(w), product_phasor(m, name), sps, taps, dtype=1).process(bits)

    def rx():
        return m.DemodulatorRx(m.Carrier(w), taps, decim=sps, decim_offset=L - 1, mix=m.MIX_COMPLEX,
                               slicer=product_phasor(m, name).slicer(), in_dtype=1, out_dtype=1)
    iq1, s1 = rx().process(x)
    r = rx()
    iqs, ss, pos = [], [], 0
    for c in cuts + [x.shape[0] - sum(cuts)]:
        i_, s_ = r.process(x[pos:pos + c])
        iqs.append(host(i_)); ss.append(host(s_)); pos += c
    assert np.array_equal(np.concatenate(iqs).view(np.uint16), host(iq1).view(np.uint16))
    assert np.array_equal(np.concatenate(ss), host(s1))
