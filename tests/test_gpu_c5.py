"""BASELINE config 5's own launch shape (VERDICT r03 Missing 3): ONE period of 256-QAM, 513-tap RRC
at sps 8 over 2^26 complex f32 samples through the bench's step (ChainPlan: modem_chain_run), so
the TX is a single 512 MiB launch with non-temporal stores (modem_capi.cpp tx_nt_below) and the
RX a single launch over it with 2^23 - 64 kept instants in one grid walk.

  * every decision equals the symbol sent (the loopback property of SURVEY.md §8c; reference
    loop: modulator.rs:85-100 -> fir.rs:18-34 -> demodulator.rs:44-56);
  * three 2^16-sample windows — near the start, past 2^25 and at the end of the call — against
    the oracle's TX chain at that carrier index within 4e-5 of max (the 513-tap f32 bound of
    tests/test_gpu_parity.py), and the oracle's RX chain fed with the oracle's samples: RX I/Q
    within 4e-5 of max, decisions bit-exact.
"""
import numpy as np
import pytest

from conftest import CONFIGS, oracle_phasor, oracle_slicer, sent_symbols

pytestmark = pytest.mark.gpu

N = 1 << 26
WIN = 1 << 16
BOUND = 4e-5


def host(t):
    return t.detach().cpu().numpy()


def rel_err(got, ref):
    return float(np.abs(got.astype(np.float64) - ref).max() / np.abs(ref).max())


def test_c5_f32_single_launch_full_size(m, o, torch_cuda):
    torch = torch_cuda
    name, bps, L, sps = CONFIGS["c5_qam256"]
    nsym = N // sps
    H = (L - 1 + sps - 1) // sps                       # FIR halo in symbols (64)
    w = o.sample_freq(1, 4)
    taps = m.rrc_taps(L, sps, 0.35)
    bits = m.prng_bits(0x5EED0000, nsym * bps)         # bench.channel_seed(0, 1, 0)
    hb = host(bits)
    tx = m.DigitalModulator(m.Carrier(w), m.QAM(8, 0.0, 1.0), sps, taps)
    rx = m.DemodulatorRx(m.Carrier(w), taps, decim=sps, decim_offset=L - 1, mix=m.MIX_COMPLEX,
                         slicer=m.QAM(8, 0.0, 1.0).slicer())
    y = torch.empty((N, 2), dtype=torch.float32, device="cuda")
    oiq = torch.empty((nsym, 2), dtype=torch.float32, device="cuda")
    osym = torch.empty(nsym, dtype=torch.uint8, device="cuda")
    plan = m.ChainPlan(tx, rx, bits, y, oiq, osym)
    n, k = plan.run()
    torch.cuda.synchronize()
    assert plan.fused == 0                              # at size: the TX and RX launches
    assert n == N and k == nsym - H
    got = host(osym[:k])
    sent = sent_symbols(hb, bps)
    assert np.array_equal(got, sent[:k]), f"{int((got != sent[:k]).sum())} decisions differ"
    op = oracle_phasor(o, name)
    osl = oracle_slicer(o, name, bps)
    worst_tx = worst_rx = 0.0
    for A in (sps * 4096, (1 << 25) + sps * 777, N - WIN):
        s_a = A // sps
        # oracle TX over symbols [s_a - 2H, s_a + WIN/sps): the first H symbols' samples are
        # its warm-up, the next H the RX halo
        wb = hb[(s_a - 2 * H) * bps:(s_a + WIN // sps) * bps]
        ref = o.tx_chain(op, wb, sps, taps, w, (s_a - 2 * H) * sps)
        ref_win = ref[2 * H * sps:]                     # stream samples [A, A + WIN)
        e = rel_err(host(y[A: A + WIN]), ref_win)
        worst_tx = max(worst_tx, e)
        assert e <= BOUND, f"TX window at {A}: {e}"
        # oracle RX from stream sample A - (L - 1): outputs at n = A + 8j, instants s_a - H + j
        riq, rsym = o.rx_chain(ref[H * sps:], w, A - (L - 1), o.MIX_COMPLEX, taps, sps, L - 1, osl)
        K0 = s_a - H
        cnt = min(len(rsym), k - K0)
        assert cnt >= WIN // sps - H
        e = rel_err(host(oiq[K0: K0 + cnt]), riq[:cnt])
        worst_rx = max(worst_rx, e)
        assert e <= BOUND, f"RX window at {A}: {e}"
        assert np.array_equal(host(osym[K0: K0 + cnt]), rsym[:cnt]), f"RX decisions at {A}"
    print(f"\n[c5] one 2^26-sample period: {k} decisions = symbols sent; TX max|d|/max|y| "
          f"{worst_tx:.3g}, RX I/Q {worst_rx:.3g} (bound {BOUND})")


def test_c5_ksplit_equals_small_tile_calls(m, o, torch_cuda):
    """The K-split RX launch (RxMfma KS = 2: C5 f32's 1024-instant tiles, 8 waves, two per 16-row
    block over half of the k-steps each) against the same stream cut into calls small enough for
    the 256-instant tiles (one filter wave, KS = 1): I/Q and decisions bit for bit — every launch
    of this configuration sums the two halves of the k-steps the same way (RxMfma::KSO), so a
    result never depends on how a stream is cut into calls (demodulator.rs:44-56, fir.rs:18-34)."""
    torch = torch_cuda
    name, bps, L, sps = CONFIGS["c5_qam256"]
    n = 1 << 24                                         # 2^21 instants: the 1024-instant tiles
    parts = 16                                          # 2^17 instants per call: 256-instant tiles
    w = o.sample_freq(1, 4)
    taps = m.rrc_taps(L, sps, 0.35)
    bits = m.prng_bits(0x5EED0005, (n // sps) * bps)
    tx = m.DigitalModulator(m.Carrier(w), m.QAM(8, 0.0, 1.0), sps, taps)
    y = tx.process(bits)
    torch.cuda.synchronize()

    def rx():
        return m.DemodulatorRx(m.Carrier(w), taps, decim=sps, decim_offset=L - 1, mix=m.MIX_COMPLEX,
                               slicer=m.QAM(8, 0.0, 1.0).slicer())
    iq1, sy1 = rx().process(y[:n])
    r = rx()
    outs = [r.process(y[i * (n // parts):(i + 1) * (n // parts)]) for i in range(parts)]
    torch.cuda.synchronize()
    iq2 = torch.cat([a for a, _ in outs])
    sy2 = torch.cat([b for _, b in outs])
    assert iq1.shape == iq2.shape and sy1.shape == sy2.shape
    assert torch.equal(iq1.view(torch.int32), iq2.view(torch.int32)), "I/Q differ between the launch shapes"
    assert torch.equal(sy1, sy2)
    H = (L - 1 + sps - 1) // sps
    sent = sent_symbols(host(bits), bps)
    assert np.array_equal(host(sy1), sent[:len(sy1)]) and len(sy1) == n // sps - H
