#!/usr/bin/env python3
"""BASELINE config 5: 256-QAM, 513-tap RRC, 8x oversampling — f32 vs f16 I/Q storage sweep.

For each storage type: the observed max error of the TX samples and the RX decimated I/Q
against the CPU oracle (f32, the reference loop) on a 2^16-sample prefix, whether the RX
decisions equal the oracle's, and a full-size (2^26 samples) loopback whose decisions must
equal the symbols sent. The oracle runs here only as the checker. Writes one JSON line.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import __graft_entry__ as g  # noqa: E402


def main():
    m, o = g.package(), g.oracle()
    L, sps, bps = 513, 8, 8
    taps = m.rrc_taps(L, sps, 0.35)
    w = m.Freq(1, 4).sample_freq()
    op = o.new_phasor(o.QAM, 8, 0.0, 1.0)
    nsym = 8192
    bits = o.prng_bits(0x5EED0000, nsym * bps)
    y_ref = o.tx_chain(op, bits, sps, taps, w, 0)
    iq_ref, sym_ref = o.rx_chain(y_ref, w, 0, o.MIX_COMPLEX, taps, sps, L - 1, o.qam_axis_slicer(bps, 1.0))
    res = {"config": "c5: 256-QAM, 513-tap RRC, sps 8", "prefix_samples": len(y_ref)}
    for name, dt in (("f32", 0), ("f16", 1)):
        qam = m.QAM(8, 0.0, 1.0)
        tx = m.DigitalModulator(m.Carrier(w), qam, sps, taps, dtype=dt)
        y = tx.process(torch.from_numpy(bits).cuda())
        rx = m.DemodulatorRx(m.Carrier(w), taps, decim=sps, decim_offset=L - 1, mix=m.MIX_COMPLEX,
                             slicer=qam.slicer(), in_dtype=dt, out_dtype=dt)
        iq, sym = rx.process(y)
        torch.cuda.synchronize()
        yh = y.float().cpu().numpy()
        iqh = iq.float().cpu().numpy()
        tx_err = float(np.abs(yh - y_ref).max() / np.abs(y_ref).max())
        rx_err = float(np.abs(iqh - iq_ref[: len(iqh)]).max() / np.abs(iq_ref).max())
        dec_eq = bool(np.array_equal(sym.cpu().numpy(), sym_ref[: len(iqh)]))
        # full size: 2^26 samples, decisions against the symbols sent
        nfull = (1 << 26) // sps
        fb = m.prng_bits(0x5EED0001, nfull * bps)
        tx2 = m.DigitalModulator(m.Carrier(w), qam, sps, taps, dtype=dt)
        rx2 = m.DemodulatorRx(m.Carrier(w), taps, decim=sps, decim_offset=L - 1, mix=m.MIX_COMPLEX,
                              slicer=qam.slicer(), in_dtype=dt, out_dtype=dt)
        _, s2 = rx2.process(tx2.process(fb), want_iq=False)
        b = fb.view(-1, bps).to(torch.int64)
        sent = (b * torch.tensor([1 << (bps - 1 - k) for k in range(bps)], device=b.device)).sum(1)
        full_ok = bool(torch.equal(s2.to(torch.int64), sent[: s2.shape[0]]))
        res[name] = {"tx_max_rel_err": tx_err, "rx_iq_max_rel_err": rx_err,
                     "decisions_equal_oracle": dec_eq, "full_size_decisions_equal_sent": full_ok,
                     "full_size_symbols": int(s2.shape[0])}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
