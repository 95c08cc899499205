#!/usr/bin/env python3
"""Regenerate tests/golden/*.npz from the CPU oracle (SURVEY.md §8c "golden fixtures").

The reference's own tests pin only the bit→symbol map and symbol timing (its KATs are
restated in tests/test_oracle_kats.py); nothing upstream pins the FIR, the carrier, the mix
or the RX. These fixtures freeze the oracle's outputs for exactly those, after the oracle was
cross-checked against independent numpy restatements (tests/test_oracle_numpy.py), so that
(a) any later change of the oracle is caught on the CPU and (b) the GPU parity tests can
compare the HIP path against stored vectors without running the oracle.

    python tests/golden/make_golden.py      # rewrites the .npz files next to this script
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as o  # noqa: E402

SEED = 0x5EED0000
PI_4 = float(np.float32(np.float32(np.pi) / np.float32(4.0)))
# name: (phasor ctor, bps, ntaps, sps) — BASELINE.json configs 1, 2, 3, 5
CONFIGS = {
    "c1": (lambda: o.new_phasor(o.BPSK, PI_4, 1.0), 1, 33, 4),
    "c2": (lambda: o.new_phasor(o.QPSK, 0.0, 1.0), 2, 65, 4),
    "c3": (lambda: o.new_phasor(o.QAM, 4, 0.0, 1.0), 4, 129, 4),
    "c5": (lambda: o.new_phasor(o.QAM, 8, 0.0, 1.0), 8, 513, 8),
}
NTX = 8192            # first TX samples per config
NWIN = 4096           # TX window starting at s0 = 2^24 - 4096
PHASE_RANGES = [(0, 256), ((1 << 24) - 256, 512), ((1 << 26) - 256, 512)]


def slicer_for(name, bps, p):
    if name in ("c3", "c5"):
        return o.qam_axis_slicer(bps, 1.0)
    return o.make_slicer(o.SLICER_NEAREST, bps, o.phasor_lut(p))


def build_fixtures():
    """{file name: {array name: array}} for every fixture."""
    files = {}
    # (2) bits -> index -> LUT tables
    luts = {"bpsk_pi4": o.phasor_lut(o.new_phasor(o.BPSK, PI_4, 1.0)),
            "qpsk": o.phasor_lut(o.new_phasor(o.QPSK, 0.0, 1.0)),
            "qam16": o.phasor_lut(o.new_phasor(o.QAM, 4, 0.0, 1.0)),
            "qam256": o.phasor_lut(o.new_phasor(o.QAM, 8, 0.0, 1.0))}
    files["luts.npz"] = luts
    # (3) carrier phases at w = 2π/4 and 2π·1000/10000
    ph = {}
    for tag, (hz, sr) in (("fs4", (1, 4)), ("1k_10k", (1000, 10000))):
        w = o.sample_freq(hz, sr)
        ph[f"w_{tag}"] = np.array([w], np.float32)
        for s0, n in PHASE_RANGES:
            ph[f"{tag}_{s0}"] = o.carrier_phases(w, s0, n)
    files["carrier_phases.npz"] = ph
    # (4) per config: taps, first NTX TX samples, TX window at 2^24 - NWIN, RX decisions
    w = o.sample_freq(1, 4)
    for name, (mk, bps, L, sps) in CONFIGS.items():
        p = mk()
        taps = o.rrc_taps(L, sps, 0.35)
        bits = o.prng_bits(SEED, NTX // sps * bps)
        y = o.tx_chain(p, bits, sps, taps, w, 0)
        s0w = (1 << 24) - NWIN
        bw = o.prng_bits(SEED + 1, NWIN // sps * bps)
        yw = o.tx_chain(mk(), bw, sps, taps, w, s0w)
        iq, sym = o.rx_chain(y, w, 0, o.MIX_COMPLEX, taps, sps, L - 1, slicer_for(name, bps, p))
        iqw, symw = o.rx_chain(yw, w, s0w, o.MIX_COMPLEX, taps, sps, L - 1, slicer_for(name, bps, p))
        files[f"chain_{name}.npz"] = dict(
            seed=np.array([SEED], np.uint64), bps=np.array([bps]), sps=np.array([sps]),
            taps=taps, bits=bits, tx=y, rx_iq=iq, rx_sym=sym,
            win_s0=np.array([s0w], np.uint64), win_bits=bw, win_tx=yw, win_rx_iq=iqw, win_rx_sym=symw)
    # (5) config 1 through the `modulate` CLI (bpsk, sr 10000, br 220, fc 1000, passband f32 .re)
    text = "".join("01"[b] for b in o.prng_bits(SEED, 1024)).encode()
    cli = o.modulate_cli("bpsk", text)
    cli_iq = o.modulate_cli("bpsk", text, iq=True)
    files["cli_c1.npz"] = dict(text=np.frombuffer(text, np.uint8), passband=cli, iq=cli_iq)
    return files


if __name__ == "__main__":
    for fname, arrays in build_fixtures().items():
        np.savez_compressed(os.path.join(HERE, fname), **arrays)
        print(fname, {k: v.shape for k, v in arrays.items()})
    total = sum(os.path.getsize(os.path.join(HERE, f)) for f in os.listdir(HERE) if f.endswith(".npz"))
    print(f"{total / 1024:.0f} KiB of fixtures")
