"""GPU parity against the committed golden fixtures (tests/golden/) — no oracle at run time.

Tolerances as in test_gpu_parity.py: carrier phase and decisions bit-exact; f32 samples
max|d| <= 1e-5 * max|y_ref| (ntaps <= 129) or 4e-5 (513 taps).
"""
import ctypes
import os

import numpy as np
import pytest

from conftest import ROOT, product_phasor

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(ROOT, "tests", "golden")
NAMES = {"c1": "bpsk", "c2": "qpsk", "c3": "qam16", "c5": "qam256"}


def load(fname):
    with np.load(os.path.join(GOLDEN, fname)) as z:
        return {k: z[k] for k in z.files}


def host(t):
    return t.detach().cpu().numpy()


def tol_for(ntaps):
    return 1e-5 if ntaps <= 129 else 4e-5


def test_carrier_phases_fixture(m, torch_cuda):
    z = load("carrier_phases.npz")
    for tag in ("fs4", "1k_10k"):
        w = float(z[f"w_{tag}"][0])
        for key in [k for k in z if k.startswith(tag + "_")]:
            s0 = int(key.split("_")[-1])
            ref = z[key]
            got = host(m.Carrier(w).phases(s0, len(ref)))
            assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), key


@pytest.mark.parametrize("cfg", list(NAMES))
@pytest.mark.parametrize("window", [False, True])
def test_chain_fixture(m, torch_cuda, cfg, window):
    """TX from the stored bits (at s0 = 0 and at s0 = 2^24 - 4096), then RX of the stored TX
    samples: samples within tolerance, decisions bit-exact."""
    torch = torch_cuda
    z = load(f"chain_{cfg}.npz")
    sps, taps = int(z["sps"][0]), z["taps"]
    pre = "win_" if window else ""
    bits, tx_ref = z[pre + "bits"], z[pre + "tx"]
    rx_iq_ref, rx_sym_ref = z[pre + "rx_iq"], z[pre + "rx_sym"]
    s0 = int(z["win_s0"][0]) if window else 0
    w = m.Freq(1, 4).sample_freq()
    ph = product_phasor(m, NAMES[cfg])
    tx = m.DigitalModulator(m.Carrier(w, s0), ph, sps, taps)
    y = host(tx.process(torch.from_numpy(bits).cuda()))
    assert y.shape == tx_ref.shape
    assert np.abs(y - tx_ref).max() <= tol_for(len(taps)) * np.abs(tx_ref).max()
    rx = m.DemodulatorRx(m.Carrier(w, s0), taps, decim=sps, decim_offset=len(taps) - 1,
                         mix=m.MIX_COMPLEX, slicer=ph.slicer())
    giq, gsym = rx.process(torch.from_numpy(tx_ref).cuda())
    giq, gsym = host(giq), host(gsym)
    assert gsym.shape == rx_sym_ref.shape and np.array_equal(gsym, rx_sym_ref)
    assert np.abs(giq - rx_iq_ref).max() <= tol_for(len(taps)) * np.abs(rx_iq_ref).max()


def test_cli_c1_fixture_iq(m, torch_cuda):
    """`modulate --iq` for config 1 (bpsk, sr 10000, br 220): the sample-and-hold (i, q) pairs
    of DigitalModulator are bit-exact on the GPU (ntaps = 0, modulate.rs:109-113)."""
    z = load("cli_c1.npz")
    bits = (z["text"] - ord("0")).astype(np.uint8)
    sps = m.Rates(220, 10000).samples_per_symbol
    w = m.Freq(1000, 10000).sample_freq()
    tx = m.DigitalModulator(m.Carrier(w), m.BPSK(float(np.float32(np.pi) / np.float32(4)), 1.0), sps, None,
                            out_mode=m.OUT_IQ_BASEBAND)
    y = host(tx.process(torch_cuda.from_numpy(bits).cuda())).reshape(-1)
    assert np.array_equal(y.view(np.uint32), z["iq"].view(np.uint32))


def test_cli_c1_fixture_passband(m, torch_cuda):
    """`modulate` passband `.re` for config 1 (modulate.rs:128-133): hardware sin/cos within 1e-6."""
    z = load("cli_c1.npz")
    bits = (z["text"] - ord("0")).astype(np.uint8)
    sps = m.Rates(220, 10000).samples_per_symbol
    w = m.Freq(1000, 10000).sample_freq()
    tx = m.DigitalModulator(m.Carrier(w), m.BPSK(float(np.float32(np.pi) / np.float32(4)), 1.0), sps, None,
                            out_mode=m.OUT_REAL)
    y = host(tx.process(torch_cuda.from_numpy(bits).cuda())).reshape(-1)
    assert y.shape == z["passband"].shape
    assert np.abs(y - z["passband"]).max() <= 1e-6


@pytest.mark.parametrize("bps", [4, 8])
def test_slicer_special_values(m, o, torch_cuda, bps):
    """The QAM slicer on the GPU (RX with one unit tap at w = 0 is the identity) equals the
    oracle's on clamps, ties, huge, infinite and NaN inputs."""
    pts = np.array([[0.6, -0.6], [-0.6, 0.6], [0, 0], [1e9, -1e9], [0.5, 0.5], [-0.5, -0.5],
                    [np.nan, -np.inf], [np.inf, np.nan], [1 / 6, -1 / 6], [1e-30, -1e-30],
                    [1 / 30, 1 / 30], [-1 / 30, 7 / 30]], np.float32)
    rng = np.random.default_rng(bps)
    pts = np.concatenate([pts, rng.uniform(-0.7, 0.7, (4000, 2)).astype(np.float32)])
    sl = o.qam_axis_slicer(bps, 1.0)
    one = np.ones(1, np.float32)
    want_iq, want = o.rx_chain(pts, 0.0, 0, o.MIX_COMPLEX, one, 1, 0, sl)   # same mix + slicer on the CPU
    rx = m.DemodulatorRx(m.Carrier(0.0), one, decim=1, decim_offset=0,
                         mix=m.MIX_COMPLEX, slicer=m.QAM(bps, 0.0, 1.0).slicer())
    giq, gsym = rx.process(torch_cuda.from_numpy(pts).cuda())
    assert np.array_equal(host(giq), want_iq, equal_nan=True)
    assert np.array_equal(host(gsym), want)
