"""The RX fast path's window reads at the history boundary.

A call's tiles whose window starts inside the chunk read it through a buffer descriptor
(RxMfma::window_rsrc); the tiles whose window reaches back into the history (a call's first
tiles) take the general path, which patches the history in. The split is the walk's tile
classification (Walk::nfull), and the descriptor is bounded by the call's buffer itself (a
window starting before it gets no records). Here a stream is cut after n1 samples for n1 over
every offset class around that boundary — the second call's first tile window starting before,
at and after the chunk's first sample, at every row alignment — and the two calls must equal
one call bit for bit (I/Q as raw bits, decisions), with small tiles (a short second call) and
with the 1024-instant tiles (a second call at size), for C3's filter (decim 4, 129 taps,
W = 192) and C5's (decim 8, 513 taps, W = 640, the K-split kernel at size).
Reference: demodulator.rs:44-56 (the stream's first samples meet a zero history)."""
import numpy as np
import pytest

from conftest import CONFIGS, product_phasor

pytestmark = pytest.mark.gpu

SEED = 0x5EED6000


def _host(t):
    return t.detach().cpu().numpy()


def _stream(m, o, torch, cfg, nsamp):
    name, bps, L, sps = CONFIGS[cfg]
    bits = o.prng_bits(SEED + nsamp % 977, nsamp // sps * bps)
    taps = m.rrc_taps(L, sps, 0.35)
    w = o.sample_freq(1, 4)
    tx = m.DigitalModulator(m.Carrier(w, 5), product_phasor(m, name), sps, taps)
    x = tx.process(torch.from_numpy(bits).cuda())
    torch.cuda.synchronize()

    def rx():
        return m.DemodulatorRx(m.Carrier(w, 5), taps, decim=sps, decim_offset=L - 1, mix=m.MIX_COMPLEX,
                               slicer=product_phasor(m, name).slicer())
    return x, rx


def _check_cuts(torch, x, rx, cuts):
    one = rx()
    iq1, s1 = one.process(x)
    iq1, s1 = _host(iq1), _host(s1)
    for n1 in cuts:
        r = rx()
        ia, sa = r.process(x[:n1])
        ib, sb = r.process(x[n1:])
        iq = np.concatenate([_host(ia), _host(ib)])
        sy = np.concatenate([_host(sa), _host(sb)])
        assert np.array_equal(sy, s1), f"decisions differ for the cut at {n1}"
        assert np.array_equal(iq.view(np.uint32), iq1.view(np.uint32)), f"I/Q differ for the cut at {n1}"


@pytest.mark.parametrize("cfg", ["c3_qam16", "c5_qam256"])
def test_small_tiles_every_offset_class(m, o, torch_cuda, cfg):
    """Second call on the 256-instant tiles: n1 over W + 2 rows of samples, every residue."""
    name, bps, L, sps = CONFIGS[cfg]
    W = 192 if sps == 4 else 640
    x, rx = _stream(m, o, torch_cuda, cfg, 1 << 16)
    cuts = list(range(1, W + 32 * sps, 3 if sps == 4 else 11)) + [W - 1, W, W + 1, 16 * sps * 7]
    _check_cuts(torch_cuda, x, rx, sorted(set(cuts)))


@pytest.mark.parametrize("cfg,nsamp", [("c3_qam16", (1 << 22) + 8192), ("c5_qam256", (1 << 23) + 16384)])
def test_large_tiles_history_boundary(m, o, torch_cuda, cfg, nsamp):
    """Second call at size (1024-instant tiles, C5: the K-split kernel): cuts around the window."""
    name, bps, L, sps = CONFIGS[cfg]
    W = 192 if sps == 4 else 640
    x, rx = _stream(m, o, torch_cuda, cfg, nsamp)
    cuts = [1, sps - 1, 16 * sps - 1, 16 * sps, W - 16 * sps, W - 1, W, W + 1, W + 16 * sps + 3, 4096 + 5]
    _check_cuts(torch_cuda, x, rx, cuts)
