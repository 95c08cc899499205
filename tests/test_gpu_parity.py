"""GPU parity: the HIP path through the C ABI against the CPU oracle.

Tolerances (stated per SURVEY.md §8c):
  * symbol indices (TX map, RX decisions), carrier phase, sample-and-hold baseband: bit-exact;
  * TX/RX f32 samples: max|d| <= 1e-5 * max|y_ref| for ntaps <= 129, 4e-5 for 513
    (FIR summation order and the hardware sin/cos differ from glibc by a few ulp);
  * f16 sample storage: max|d| <= 2^-10 * max|y_ref| with decisions still bit-exact.
"""
import numpy as np
import pytest

from conftest import CONFIGS, oracle_phasor, oracle_slicer, product_phasor, sent_symbols

pytestmark = pytest.mark.gpu

SEED = 0x5EED0000
W_QUARTER = None   # Freq::new(1, 4).sample_freq(), set lazily


def tol_for(ntaps):
    return 1e-5 if ntaps <= 129 else 4e-5


def w_quarter(o):
    return o.sample_freq(1, 4)


def host(t):
    return t.detach().cpu().numpy()


def gpu_tx(m, torch, name, bits_np, sps, taps, w, s0=0, dtype=0, out_mode=0, flush=False):
    tx = m.DigitalModulator(m.Carrier(w, s0), product_phasor(m, name), sps, taps, dtype=dtype,
                            out_mode=out_mode)
    y = tx.process(torch.from_numpy(bits_np).cuda())
    if flush:
        y = torch.cat([y, tx.flush(like=y)])
    return y


# ------------------------------------------------------------------------ phase ----
@pytest.mark.parametrize("hz,sr", [(1, 4), (1000, 10000), (900, 10000), (220, 10000), (7, 48000)])
@pytest.mark.parametrize("s0", [0, 2**20 - 1000, 2**24 - 4096, 2**26 - 4096, 2**32 - 3000, 2**40 + 11])
def test_carrier_phase_bit_exact(m, o, torch_cuda, hz, sr, s0):
    """carrier.rs:17-19 + util.rs:3-6 reproduced bit for bit by the kernels' phase path."""
    w = o.sample_freq(hz, sr)
    n = 8192
    got = host(m.Carrier(w).phases(s0, n))
    ref = o.carrier_phases(w, s0, n)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


# ------------------------------------------------------------------------ TX ----
@pytest.fixture(params=["auto", "valu"])
def fir_path(request, monkeypatch):
    """TX FIR on the matrix pipe (default where instantiated) and forced onto the VALU."""
    if request.param == "valu":
        monkeypatch.setenv("MODEM_HIP_FIR", "valu")
    else:
        monkeypatch.delenv("MODEM_HIP_FIR", raising=False)
    return request.param


@pytest.mark.parametrize("cfg", list(CONFIGS))
@pytest.mark.parametrize("out_mode", [0, 1, 2])
def test_tx_matches_oracle(m, o, torch_cuda, cfg, out_mode, fir_path):
    name, bps, L, sps = CONFIGS[cfg]
    nsym = 3000
    bits = o.prng_bits(SEED + 1, nsym * bps)
    taps = m.rrc_taps(L, sps, 0.35)
    w = w_quarter(o)
    got = host(gpu_tx(m, torch_cuda, name, bits, sps, taps, w, out_mode=out_mode, flush=True))
    ref = o.tx_chain(oracle_phasor(o, name), bits, sps, taps, w, 0, flush_syms=(L - 1 + sps - 1) // sps,
                     out_mode=out_mode)
    assert got.shape == ref.shape
    err = np.abs(got - ref).max()
    assert err <= tol_for(L) * np.abs(ref).max(), f"{cfg} mode {out_mode}: max|d|={err}"


@pytest.mark.parametrize("name,bps", [("bpsk", 1), ("qpsk", 2), ("qam16", 4), ("qam256", 8)])
@pytest.mark.parametrize("sps", [1, 4, 8, 45])
def test_tx_sample_and_hold_bit_exact(m, o, torch_cuda, name, bps, sps):
    """ntaps=0: the reference DigitalModulator's held (i,q) — what `modulate --iq` writes."""
    nsym = 700
    bits = o.prng_bits(SEED + 2, nsym * bps + (bps - 1))        # ragged tail is dropped
    got = host(gpu_tx(m, torch_cuda, name, bits, sps, None, 0.5, out_mode=1))
    ref = o.tx_chain(oracle_phasor(o, name), bits, sps, None, 0.5, 0, out_mode=1)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("sps,L", [(3, 31), (5, 40), (45, 91), (16, 129), (2, 17), (1, 23), (8, 129),
                                   (4, 257), (4, 9), (2, 65), (16, 33)])
def test_tx_other_rates(m, o, torch_cuda, sps, L, fir_path):
    """Generic and remaining specialised samples-per-symbol paths (e.g. sr/br = 45)."""
    bits = o.prng_bits(SEED + 3, 500 * 2)
    taps = m.rrc_taps(L, sps, 0.25)
    w = o.sample_freq(1000, 10000)
    got = host(gpu_tx(m, torch_cuda, "qpsk", bits, sps, taps, w, flush=True))
    ref = o.tx_chain(oracle_phasor(o, "qpsk"), bits, sps, taps, w, 0, flush_syms=(L - 1 + sps - 1) // sps)
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() <= 1e-5 * np.abs(ref).max()


def test_tx_streaming_equals_one_call(m, o, torch_cuda, fir_path):
    """Ragged chunks (0, 1, non-multiples of bps) give the same samples as one call."""
    torch = torch_cuda
    name, bps, L, sps = CONFIGS["c3_qam16"]
    bits = o.prng_bits(SEED + 4, 40001)
    taps = m.rrc_taps(L, sps, 0.35)
    w = w_quarter(o)
    one = host(gpu_tx(m, torch, name, bits, sps, taps, w, s0=123))
    tx = m.DigitalModulator(m.Carrier(w, 123), product_phasor(m, name), sps, taps)
    parts, pos = [], 0
    for c in [0, 1, 3, 4, 5, 1000, 1, 2, 7, 13001, 0, 9, 26000]:
        chunk = torch.from_numpy(bits[pos:pos + c].copy()).cuda()
        parts.append(host(tx.process(chunk)))
        pos += c
    parts.append(host(tx.process(torch.from_numpy(bits[pos:].copy()).cuda())))
    got = np.concatenate(parts)
    assert np.array_equal(got.view(np.uint32), one.view(np.uint32))
    assert tx.carrier.sample == 123 + len(one)


def test_tx_host_buffers(m, o, torch_cuda):
    """Host (numpy) in/out goes through the handle's staging and gives the same samples."""
    name, bps, L, sps = CONFIGS["c2_qpsk"]
    bits = o.prng_bits(SEED + 5, 2000)
    taps = m.rrc_taps(L, sps, 0.35)
    w = w_quarter(o)
    dev = host(gpu_tx(m, torch_cuda, name, bits, sps, taps, w))
    tx = m.DigitalModulator(m.Carrier(w), product_phasor(m, name), sps, taps)
    hst = tx.process(bits)
    assert isinstance(hst, np.ndarray)
    assert np.array_equal(dev, hst)


def test_tx_f16(m, o, torch_cuda, fir_path):
    name, bps, L, sps = CONFIGS["c5_qam256"]
    bits = o.prng_bits(SEED + 6, 2000 * bps)
    taps = m.rrc_taps(L, sps, 0.35)
    w = w_quarter(o)
    got = host(gpu_tx(m, torch_cuda, name, bits, sps, taps, w, dtype=1)).astype(np.float32)
    ref = o.tx_chain(oracle_phasor(o, name), bits, sps, taps, w, 0)
    assert np.abs(got - ref).max() <= 2.0 ** -10 * np.abs(ref).max()


# ------------------------------------------------------------------------ RX ----
@pytest.mark.parametrize("cfg", list(CONFIGS))
def test_rx_matches_oracle(m, o, torch_cuda, cfg, fir_path):
    """Oracle TX samples in; decimated I/Q within tolerance, decisions bit-exact."""
    name, bps, L, sps = CONFIGS[cfg]
    nsym = 3000
    bits = o.prng_bits(SEED + 7, nsym * bps)
    taps = m.rrc_taps(L, sps, 0.35)
    w = w_quarter(o)
    flush = (L - 1 + sps - 1) // sps
    x = o.tx_chain(oracle_phasor(o, name), bits, sps, taps, w, 0, flush_syms=flush)
    riq, rsym = o.rx_chain(x, w, 0, o.MIX_COMPLEX, taps, sps, L - 1, oracle_slicer(o, name, bps))
    rx = m.DemodulatorRx(m.Carrier(w), taps, decim=sps, decim_offset=L - 1, mix=m.MIX_COMPLEX,
                         slicer=product_phasor(m, name).slicer())
    giq, gsym = rx.process(torch_cuda.from_numpy(x).cuda())
    giq, gsym = host(giq), host(gsym)
    assert giq.shape == riq.shape and gsym.shape == rsym.shape
    assert np.abs(giq - riq).max() <= tol_for(L) * np.abs(riq).max()
    assert np.array_equal(gsym, rsym)
    assert np.array_equal(gsym[:nsym], sent_symbols(bits, bps))


def test_rx_reference_demodulator(m, o, torch_cuda, fir_path):
    """decim=1, real mix, 2x gain: Demodulator::next (demodulator.rs:44-56) at every sample."""
    rng = np.random.RandomState(11)
    n = 20000
    x = np.zeros((n, 2), np.float32)
    x[:, 0] = rng.randn(n).astype(np.float32)
    x[:, 1] = rng.randn(n).astype(np.float32)       # ignored by the reference (x.re only)
    taps = m.rrc_taps(64, 4, 0.2)
    w = o.sample_freq(900, 10000)
    ri, rq = o.demodulate(w, 0, 0.0, taps, x[:, 0].copy())
    rx = m.DemodulatorRx(m.Carrier(w), taps, decim=1, decim_offset=0, mix=m.MIX_REFERENCE_REAL)
    giq, _ = rx.process(torch_cuda.from_numpy(x).cuda(), want_sym=False)
    giq = host(giq)
    ref = np.stack([ri, rq], 1)
    assert giq.shape == ref.shape
    assert np.abs(giq - ref).max() <= 1e-5 * np.abs(ref).max()


def test_rx_streaming_equals_one_call(m, o, torch_cuda, fir_path):
    torch = torch_cuda
    name, bps, L, sps = CONFIGS["c3_qam16"]
    bits = o.prng_bits(SEED + 8, 5000 * bps)
    taps = m.rrc_taps(L, sps, 0.35)
    w = w_quarter(o)
    x = torch.from_numpy(o.tx_chain(oracle_phasor(o, name), bits, sps, taps, w, 0)).cuda()

    def rx():
        return m.DemodulatorRx(m.Carrier(w), taps, decim=sps, decim_offset=L - 1, mix=m.MIX_COMPLEX,
                               slicer=product_phasor(m, name).slicer())
    a = rx()
    iq1, s1 = a.process(x)
    b = rx()
    iqs, ss, pos = [], [], 0
    for c in [1, 0, 2, 3, 127, 128, 129, 5, 4096, 1, 7777]:
        i_, s_ = b.process(x[pos:pos + c])
        iqs.append(host(i_)); ss.append(host(s_)); pos += c
    i_, s_ = b.process(x[pos:])
    iqs.append(host(i_)); ss.append(host(s_))
    assert np.array_equal(np.concatenate(ss), host(s1))
    assert np.array_equal(np.concatenate(iqs).view(np.uint32), host(iq1).view(np.uint32))


def test_rx_flush_drains(m, o, torch_cuda):
    """TX without flush + RX flush recovers every symbol but the FIR-tail ones of TX."""
    name, bps, L, sps = CONFIGS["c2_qpsk"]
    nsym = 2000
    bits = o.prng_bits(SEED + 9, nsym * bps)
    taps = m.rrc_taps(L, sps, 0.35)
    w = w_quarter(o)
    y = gpu_tx(m, torch_cuda, name, bits, sps, taps, w, flush=True)
    rx = m.DemodulatorRx(m.Carrier(w), taps, decim=sps, decim_offset=L - 1, mix=m.MIX_COMPLEX,
                         slicer=product_phasor(m, name).slicer())
    _, s1 = rx.process(y)
    _, s2 = rx.flush(like=y)
    got = np.concatenate([host(s1), host(s2)])
    assert np.array_equal(got[:nsym], sent_symbols(bits, bps))


def test_rx_f16_decisions(m, o, torch_cuda, fir_path):
    """C5 with f16 I/Q storage: samples within 2^-10, decisions bit-exact."""
    name, bps, L, sps = CONFIGS["c5_qam256"]
    nsym = 3000
    bits = o.prng_bits(SEED + 10, nsym * bps)
    taps = m.rrc_taps(L, sps, 0.35)
    w = w_quarter(o)
    y = gpu_tx(m, torch_cuda, name, bits, sps, taps, w, dtype=1, flush=True)
    rx = m.DemodulatorRx(m.Carrier(w), taps, decim=sps, decim_offset=L - 1, mix=m.MIX_COMPLEX,
                         slicer=product_phasor(m, name).slicer(), in_dtype=1, out_dtype=1)
    _, s = rx.process(y)
    assert np.array_equal(host(s)[:nsym], sent_symbols(bits, bps))


@pytest.mark.parametrize("decim,L", [(3, 31), (45, 91), (16, 129), (2, 17), (4, 33), (4, 65), (2, 65),
                                     (2, 129), (8, 129), (8, 257), (4, 130)])
def test_rx_other_rates(m, o, torch_cuda, decim, L, fir_path):
    name, bps = "qpsk", 2
    bits = o.prng_bits(SEED + 12, 400 * bps)
    taps = m.rrc_taps(L, decim, 0.25)
    w = o.sample_freq(1000, 10000)
    x = o.tx_chain(oracle_phasor(o, name), bits, decim, taps, w, 0, flush_syms=(L - 1 + decim - 1) // decim)
    riq, rsym = o.rx_chain(x, w, 0, o.MIX_COMPLEX, taps, decim, L - 1, oracle_slicer(o, name, bps))
    rx = m.DemodulatorRx(m.Carrier(w), taps, decim=decim, decim_offset=L - 1, mix=m.MIX_COMPLEX,
                         slicer=product_phasor(m, name).slicer())
    giq, gsym = rx.process(torch_cuda.from_numpy(x).cuda())
    assert np.abs(host(giq) - riq).max() <= 1e-5 * np.abs(riq).max()
    assert np.array_equal(host(gsym), rsym)


@pytest.mark.parametrize("s0", [2**32 - 5000, 2**40 + 3, 2**53 - 6000])
def test_long_stream_carrier_index(m, o, torch_cuda, s0, fir_path):
    """Carrier indices past 2^32 (a stream older than 4.3 Gsamples) take the same fast kernels
    (the index is kept in f64, exact below 2^53); a call that reaches 2^53 takes the general
    path's u64 -> f32 conversion. TX and RX against the oracle started at the same index."""
    name, bps, L, sps = CONFIGS["c3_qam16"]
    nsym = 3000
    bits = o.prng_bits(SEED + 13, nsym * bps)
    taps = m.rrc_taps(L, sps, 0.35)
    w = w_quarter(o)
    flush = (L - 1 + sps - 1) // sps
    y = gpu_tx(m, torch_cuda, name, bits, sps, taps, w, s0=s0, flush=True)
    x = o.tx_chain(oracle_phasor(o, name), bits, sps, taps, w, s0, flush_syms=flush)
    assert y.shape[0] == x.shape[0]
    assert np.abs(host(y) - x).max() <= tol_for(L) * np.abs(x).max()
    riq, rsym = o.rx_chain(x, w, s0, o.MIX_COMPLEX, taps, sps, L - 1, oracle_slicer(o, name, bps))
    rx = m.DemodulatorRx(m.Carrier(w, s0), taps, decim=sps, decim_offset=L - 1, mix=m.MIX_COMPLEX,
                         slicer=product_phasor(m, name).slicer())
    giq, gsym = rx.process(torch_cuda.from_numpy(x).cuda())
    assert np.abs(host(giq) - riq).max() <= tol_for(L) * np.abs(riq).max()
    assert np.array_equal(host(gsym), rsym)
    assert np.array_equal(host(gsym)[:nsym], sent_symbols(bits, bps))


# ------------------------------------------------------------------- FIRFilter ----
@pytest.mark.parametrize("L", [1, 2, 23, 64, 129, 1000])
def test_fir_filter(m, o, torch_cuda, L):
    rng = np.random.RandomState(L)
    taps = rng.randn(L).astype(np.float32)
    x = rng.randn(30000).astype(np.float32)
    ref = o.fir_block(taps, x)
    f = m.FIRFilter(taps)
    xt = torch_cuda.from_numpy(x).cuda()
    y = np.concatenate([host(f.process(xt[:777])), host(f.process(xt[777:12345])), host(f.process(xt[12345:]))])
    scale = np.abs(taps).sum() * np.abs(x).max()
    assert np.abs(y - ref).max() <= 1e-6 * scale


# ------------------------------------------------------------ full-size properties ----
def test_c3_full_size_loopback(m, o, torch_cuda):
    """BASELINE config 3 at full size (16 M samples): every decision equals the symbol sent."""
    torch = torch_cuda
    name, bps, L, sps = CONFIGS["c3_qam16"]
    N = 1 << 24
    bits = m.prng_bits(SEED, N // sps * bps)
    taps = m.rrc_taps(L, sps, 0.35)
    w = w_quarter(o)
    tx = m.DigitalModulator(m.Carrier(w), product_phasor(m, name), sps, taps)
    y = tx.process(bits)
    assert y.shape[0] == N
    y = torch.cat([y, tx.flush(like=y)])
    rx = m.DemodulatorRx(m.Carrier(w), taps, decim=sps, decim_offset=L - 1, mix=m.MIX_COMPLEX,
                         slicer=product_phasor(m, name).slicer())
    _, s = rx.process(y)
    b = bits.view(-1, bps).to(torch.int64)
    sent = (b * torch.tensor([8, 4, 2, 1], device=b.device)).sum(1).to(torch.uint8)
    assert torch.equal(s[: N // sps], sent)


def test_prng_matches_oracle(m, o, torch_cuda):
    for nbits in [1, 63, 64, 65, 1000, 4096 + 17]:
        assert np.array_equal(host(m.prng_bits(SEED + 3, nbits)), o.prng_bits(SEED + 3, nbits))


def test_errors_on_device(m, o, torch_cuda):
    with pytest.raises(m.ModemError):
        m.DigitalModulator(m.Carrier(0.5), m.QPSK(0.0, 1.0), 4, None, device=99)
    tx = m.DigitalModulator(m.Carrier(0.5), m.QPSK(0.0, 1.0), 4, None)
    out = torch_cuda.empty((3, 2), device="cuda")
    with pytest.raises(m.ModemError):     # 8 bits -> 4 symbols -> 16 samples > cap 3
        tx.process(torch_cuda.zeros(8, dtype=torch_cuda.uint8, device="cuda"), out=out)


# ------------------------------------------------------------- channel batches ----
@pytest.mark.parametrize("cfg,dtype", [("c2_qpsk", 0), ("c3_qam16", 0), ("c3_qam16", 1), ("c5_qam256", 0)])
def test_batch_equals_single_calls(m, o, torch_cuda, cfg, dtype):
    """process_batch (one launch per 8 channels) gives bit-identical samples, I/Q and
    decisions to per-channel process() calls on separate handles, over two streaming calls;
    10 channels with distinct carrier indices, ragged lengths and leftover bits exercise the
    chunking (8 + 2), the per-channel state and the bit carry (one channel's first call is
    shorter than a symbol: it produces nothing and only carries its bits)."""
    torch = torch_cuda
    name, bps, L, sps = CONFIGS[cfg]
    taps = m.rrc_taps(L, sps, 0.35)
    w = w_quarter(o)
    nch = 10
    s0s = [c * 1000003 + (c % 3) for c in range(nch)]

    def mk(c):
        tx = m.DigitalModulator(m.Carrier(w, s0s[c]), product_phasor(m, name), sps, taps, dtype=dtype)
        rx = m.DemodulatorRx(m.Carrier(w, s0s[c]), taps, decim=sps, decim_offset=L - 1, mix=m.MIX_COMPLEX,
                             slicer=product_phasor(m, name).slicer(), in_dtype=dtype, out_dtype=dtype)
        return tx, rx

    single, batch = [mk(c) for c in range(nch)], [mk(c) for c in range(nch)]
    for rnd in range(2):
        # channel 0 gets fewer bits than one symbol in the first call (no samples, only carry)
        nb = [(bps - 1 if (rnd == 0 and c == 0) else (1500 + 97 * c) * bps + c % bps) for c in range(nch)]
        bits = [torch.from_numpy(o.prng_bits(SEED + 200 + 10 * rnd + c, nb[c])).cuda() for c in range(nch)]
        ys = [t.process(b) for (t, _), b in zip(single, bits)]
        yb = m.DigitalModulator.process_batch([t for t, _ in batch], bits)
        for c in range(nch):
            assert yb[c].shape == ys[c].shape
            assert torch.equal(yb[c], ys[c]), (rnd, c)
            assert batch[c][0].carrier.sample == single[c][0].carrier.sample
        rs = [r.process(y) for (_, r), y in zip(single, ys)]
        rb = m.DemodulatorRx.process_batch([r for _, r in batch], yb)
        for c in range(nch):
            assert torch.equal(rb[c][0], rs[c][0]) and torch.equal(rb[c][1], rs[c][1]), (rnd, c)


def test_batch_mixed_configs_fall_back(m, o, torch_cuda):
    """Handles of different configurations in one batch run one call at a time, with the same
    results as separate process() calls."""
    torch = torch_cuda
    w = w_quarter(o)
    specs = [CONFIGS["c2_qpsk"], CONFIGS["c3_qam16"]]
    mods, ref = [], []
    for name, bps, L, sps in specs:
        taps = m.rrc_taps(L, sps, 0.35)
        mods.append(m.DigitalModulator(m.Carrier(w), product_phasor(m, name), sps, taps))
        ref.append(m.DigitalModulator(m.Carrier(w), product_phasor(m, name), sps, taps))
    bits = [torch.from_numpy(o.prng_bits(SEED + 300 + i, 2000 * bps)).cuda() for i, (_, bps, _, _) in enumerate(specs)]
    yb = m.DigitalModulator.process_batch(mods, bits)
    for i in range(2):
        assert torch.equal(yb[i], ref[i].process(bits[i]))


def test_batch_plans_equal_single_calls(m, o, torch_cuda):
    """TxBatchPlan / RxBatchPlan (prepared batch calls over fixed buffers, run every period)
    give the same samples, I/Q and decisions as per-channel process() calls, period after
    period."""
    torch = torch_cuda
    name, bps, L, sps = CONFIGS["c3_qam16"]
    taps = m.rrc_taps(L, sps, 0.35)
    w = w_quarter(o)
    nch, nsym = 3, 2048

    def mk(c):
        tx = m.DigitalModulator(m.Carrier(w, 777 * c), product_phasor(m, name), sps, taps)
        rx = m.DemodulatorRx(m.Carrier(w, 777 * c), taps, decim=sps, decim_offset=L - 1, mix=m.MIX_COMPLEX,
                             slicer=product_phasor(m, name).slicer())
        return tx, rx

    single, batch = [mk(c) for c in range(nch)], [mk(c) for c in range(nch)]
    bits = [torch.from_numpy(o.prng_bits(SEED + 400 + c, nsym * bps)).cuda() for c in range(nch)]
    ys = [torch.empty((nsym * sps, 2), device="cuda") for _ in range(nch)]
    iqs = [torch.empty((nsym, 2), device="cuda") for _ in range(nch)]
    syms = [torch.empty(nsym, dtype=torch.uint8, device="cuda") for _ in range(nch)]
    txp = m.TxBatchPlan([t for t, _ in batch], bits, ys)
    rxp = m.RxBatchPlan([r for _, r in batch], ys, iqs, syms)
    for period in range(3):
        assert txp.run() == [nsym * sps] * nch
        got = rxp.run()
        for c in range(nch):
            y = single[c][0].process(bits[c])
            assert torch.equal(ys[c], y), (period, c)
            giq, gsym = single[c][1].process(y)
            assert got[c] == giq.shape[0]
            assert torch.equal(iqs[c][: got[c]], giq) and torch.equal(syms[c][: got[c]], gsym), (period, c)


# ------------------------------------------------------------------ C host ----
def test_c_host_loopback():
    """tests/cpp/loopback.c: the C ABI from a plain C program (host buffers, split calls,
    flushes), every decision equal to the symbol sent."""
    import os
    import subprocess
    from conftest import ROOT
    exe = os.path.join(ROOT, "tests", "cpp", "loopback")
    assert os.path.exists(exe), "tests/cpp/loopback not built (build())"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=90)
    print(r.stdout, r.stderr)
    assert r.returncode == 0
    assert "0 wrong" in r.stdout


@pytest.mark.parametrize("src", ["bits", "evenodd", "ascii"])
def test_rust_source_binding(o, tmp_path, src):
    """tests/cpp/rust_source.c: the Rust binding's Source-driven HipModulator
    restated in C — the handle created from the Rust TxDesc layout (q_offset = sps / 2 for the
    EvenOddOffset source), the bits gathered from data.rs's Bits / EvenOddOffset / AsciiBits state
    machines at their Changed events, chunked modem_tx_process calls — against the oracle's
    DigitalModulator over the same source (`modulate --iq` of qpsk and oqpsk), bit for bit."""
    import os
    import subprocess
    from conftest import ROOT
    exe = os.path.join(ROOT, "tests", "cpp", "rust_source")
    assert os.path.exists(exe), "tests/cpp/rust_source not built (build())"
    out = str(tmp_path / "y.f32")
    r = subprocess.run([exe, src, out], capture_output=True, text=True, timeout=90)
    print(r.stdout, r.stderr)
    assert r.returncode == 0
    got = np.fromfile(out, dtype=np.float32).reshape(-1, 2)
    bits = np.fromfile(out + ".bits", dtype=np.uint8)
    eo = src == "evenodd"
    ph = o.new_phasor(o.OQPSK, 1.0) if eo else o.new_phasor(o.QPSK, 0.0, 1.0)
    ref = o.tx_chain(ph, bits, 8, None, o.sample_freq(1000, 10000), 0, out_mode=o.OUT_IQ_BASEBAND, even_odd=eo)
    assert got.shape == ref.shape == ((len(bits) // 2) * 8, 2)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("cfg,dtype", [("c3_qam16", 0), ("c2_qpsk", 0), ("c5_qam256", 1)])
def test_chain_plan_equals_separate_calls(m, o, torch_cuda, cfg, dtype):
    """modem_chain_run (ChainPlan: the bench's step) equals modem_tx_process followed by
    modem_rx_process on separate handles, bit for bit, over three periods of a stream whose bit
    buffer leaves a carry (bits not a multiple of the symbol size); the handles' carrier samples
    advance alike, and the decisions of the last period equal the symbols sent."""
    torch = torch_cuda
    name, bps, L, sps = CONFIGS[cfg]
    taps = m.rrc_taps(L, sps, 0.35)
    w = w_quarter(o)
    nsym = 3000
    nb = nsym * bps + (1 if bps > 1 else 0)
    hb = o.prng_bits(SEED + 300, nb)
    bits = torch.from_numpy(hb).cuda()
    tdt = torch.float16 if dtype else torch.float32

    def mk():
        tx = m.DigitalModulator(m.Carrier(w, 12345), product_phasor(m, name), sps, taps, dtype=dtype)
        rx = m.DemodulatorRx(m.Carrier(w, 12345), taps, decim=sps, decim_offset=L - 1, mix=m.MIX_COMPLEX,
                             slicer=product_phasor(m, name).slicer(), in_dtype=dtype, out_dtype=dtype)
        return tx, rx
    (tx1, rx1), (tx2, rx2) = mk(), mk()
    cap = (nb + bps) // bps * sps
    y = torch.empty((cap, 2), dtype=tdt, device="cuda")
    oiq = torch.empty((cap // sps + 1, 2), dtype=tdt, device="cuda")
    osym = torch.empty(cap // sps + 1, dtype=torch.uint8, device="cuda")
    plan = m.ChainPlan(tx2, rx2, bits, y, oiq, osym)
    for rnd in range(3):
        ys = tx1.process(bits)
        riq, rsym = rx1.process(ys)
        n, k = plan.run()
        torch.cuda.synchronize()
        assert n == ys.shape[0] and k == rsym.shape[0], (rnd, n, k)
        assert torch.equal(y[:n], ys) and torch.equal(oiq[:k], riq) and torch.equal(osym[:k], rsym), rnd
        assert tx2.carrier.sample == tx1.carrier.sample and rx2.carrier.sample == rx1.carrier.sample
    # sanity: the decisions are the symbols of the (continuing) stream
    stream_bits = np.concatenate([hb] * 3)
    sent = sent_symbols(stream_bits[: (len(stream_bits) // bps) * bps], bps)
    got = osym[:k].cpu().numpy()
    c_prev = rx2.carrier.sample - 12345 - n                 # samples the RX consumed before the last call
    k0 = max(0, -(-(c_prev - (L - 1)) // sps))              # its first kept instant (n = K sps + L - 1)
    assert np.array_equal(got, sent[k0: k0 + k])
