"""BASELINE config 4's per-GPU workload at size: 8 independent QPSK / 65-tap
channels of 2^22 samples each through the channel-batch plans (TxBatchPlan / RxBatchPlan, one TX
and one RX launch per period, the bench's C4 path), for two periods of a continuing stream.

  * every channel's decisions equal the symbols that channel sent, in both periods (the second
    period's RX calls decide symbols whose filter spans the period boundary);
  * windows of 2^16 samples of every channel — early in period 1, at the period boundary and
    deep into period 2 — against the oracle's TX chain (modulator.rs:85-100 + fir.rs:18-34, at
    that channel's carrier index) within 1e-5 of max, and the oracle's RX chain
    (demodulator.rs:44-56 with the complex mix, fir.rs:18-34, decimation, slicer) fed with the
    oracle's samples: RX I/Q within 1e-5 of max, decisions bit-exact.
"""
import numpy as np
import pytest

from conftest import CONFIGS, oracle_phasor, oracle_slicer, sent_symbols

pytestmark = pytest.mark.gpu

NCH, N = 8, 1 << 22
WIN = 1 << 16


def host(t):
    return t.detach().cpu().numpy()


def rel_err(got, ref):
    return float(np.abs(got.astype(np.float64) - ref).max() / np.abs(ref).max())


def test_c4_per_gpu_workload_two_periods(m, o, torch_cuda):
    torch = torch_cuda
    name, bps, L, sps = CONFIGS["c4_qpsk"]
    nsym = N // sps
    H = (L - 1 + sps - 1) // sps                       # FIR halo in symbols (16)
    w = o.sample_freq(1, 4)
    taps = m.rrc_taps(L, sps, 0.35)
    seeds = [0x5EED0000 + c for c in range(NCH)]       # bench.channel_seed(0, 8, c)
    bits = [m.prng_bits(s, nsym * bps) for s in seeds]
    hbits = [host(b) for b in bits]
    sent = [sent_symbols(b, bps) for b in hbits]
    txs = [m.DigitalModulator(m.Carrier(w), m.QPSK(0.0, 1.0), sps, taps) for _ in range(NCH)]
    rxs = [m.DemodulatorRx(m.Carrier(w), taps, decim=sps, decim_offset=L - 1, mix=m.MIX_COMPLEX,
                           slicer=m.QPSK(0.0, 1.0).slicer()) for _ in range(NCH)]
    ys = [torch.empty((N, 2), dtype=torch.float32, device="cuda") for _ in range(NCH)]
    oiq = [torch.empty((nsym, 2), dtype=torch.float32, device="cuda") for _ in range(NCH)]
    osym = [torch.empty(nsym, dtype=torch.uint8, device="cuda") for _ in range(NCH)]
    txp = m.TxBatchPlan(txs, bits, ys)
    rxp = m.RxBatchPlan(rxs, ys, oiq, osym)
    op = oracle_phasor(o, name)
    osl = oracle_slicer(o, name, bps)
    # windows (stream sample index A, a multiple of sps) checked after the period holding them
    windows = {0: [sps * 5000, N - WIN], 1: [N, N + sps * (nsym // 2) + 4 * 777]}
    worst_tx = worst_rx = 0.0
    for period in range(2):
        assert txp.run() == [N] * NCH
        prod = rxp.run()
        torch.cuda.synchronize()
        # kept instants K (n = K sps + L - 1) of this period's RX call decide stream symbol K
        k_first = 0 if period == 0 else period * nsym - H
        for c in range(NCH):
            got = host(osym[c][: prod[c]])
            assert prod[c] == (nsym - H if period == 0 else nsym)
            want = sent[c][(np.arange(k_first, k_first + prod[c])) % nsym]
            assert np.array_equal(got, want), f"channel {c} period {period}: decisions differ"
        for A in windows[period]:
            s_a = A // sps
            for c in range(NCH):
                # oracle TX over symbols [s_a - 2H, s_a + WIN/sps) of the periodic stream: the
                # first H symbols' samples are its warm-up, the next H the RX halo
                idx = np.arange(s_a - 2 * H, s_a + WIN // sps) % nsym
                wb = hbits[c].reshape(nsym, bps)[idx].reshape(-1)
                ref = o.tx_chain(op, wb, sps, taps, w, (s_a - 2 * H) * sps)
                ref_win = ref[2 * H * sps:]                       # stream samples [A, A + WIN)
                gpu_win = host(ys[c][A - period * N: A - period * N + WIN])
                e = rel_err(gpu_win, ref_win)
                worst_tx = max(worst_tx, e)
                assert e <= 1e-5, f"channel {c} TX window at {A}: {e}"
                # oracle RX from stream sample A - (L - 1): outputs at n = A + 4k, instants
                # K = s_a - H + k
                riq, rsym = o.rx_chain(ref[H * sps:], w, A - (L - 1), o.MIX_COMPLEX, taps, sps, L - 1, osl)
                K = s_a - H + np.arange(len(rsym))
                i = K - k_first
                sel = (i >= 0) & (i < prod[c])
                assert sel.sum() >= WIN // sps - H
                giq = host(oiq[c][int(i[sel][0]): int(i[sel][-1]) + 1])
                gsym = host(osym[c][int(i[sel][0]): int(i[sel][-1]) + 1])
                e = rel_err(giq, riq[sel])
                worst_rx = max(worst_rx, e)
                assert e <= 1e-5, f"channel {c} RX window at {A}: {e}"
                assert np.array_equal(gsym, rsym[sel]), f"channel {c} RX decisions at {A}"
    print(f"\n[c4] 8 ch x 2^22, 2 periods: TX max|d|/max|y| {worst_tx:.3g}, RX I/Q {worst_rx:.3g} (bound 1e-5)")
