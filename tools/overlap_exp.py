#!/usr/bin/env python3
"""Experiment: TX of batch k+1 on one stream while RX of batch k runs on another (double-
buffered sample buffers), against the single-stream chain. Prints wall us/step for each.
Grid caps per kernel come from MODEM_TX_WGS_PER_CU / MODEM_RX_WGS_PER_CU (read once per
process), so run one process per setting."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import __graft_entry__ as g  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--mode", choices=["seq", "pipe"], default="seq")
    a = ap.parse_args()
    m = g.package()
    L, sps, nsamp = 129, 4, 1 << 24
    taps = m.rrc_taps(L, sps, 0.35)
    w = m.Freq(1, 4).sample_freq()
    bits = m.prng_bits(0x5EED0000, nsamp // sps * 4, device=0)
    tx = m.DigitalModulator(m.Carrier(w), m.QAM(4, 0.0, 1.0), sps, taps)
    rx = m.DemodulatorRx(m.Carrier(w), taps, decim=sps, decim_offset=L - 1, mix=m.MIX_COMPLEX,
                         slicer=m.QAM(4, 0.0, 1.0).slicer())
    ys = [torch.empty((nsamp, 2), dtype=torch.float32, device="cuda") for _ in range(2)]
    oiq = torch.empty((nsamp // sps, 2), dtype=torch.float32, device="cuda")
    osym = torch.empty(nsamp // sps, dtype=torch.uint8, device="cuda")
    s_tx = torch.cuda.Stream()
    s_rx = torch.cuda.Stream() if a.mode == "pipe" else s_tx
    tx_done = [torch.cuda.Event() for _ in range(2)]
    rx_done = [torch.cuda.Event() for _ in range(2)]

    def run(nsteps):
        # step k: TX batch k into ys[k%2] (after RX of batch k-2 has read it), RX batch k
        for k in range(nsteps):
            b = k & 1
            if a.mode == "pipe" and k >= 2:
                s_tx.wait_event(rx_done[b])
            tx.process(bits, out=ys[b], stream=s_tx)
            if a.mode == "pipe":
                tx_done[b].record(s_tx)
                s_rx.wait_event(tx_done[b])
            rx.process(ys[b], out_iq=oiq, out_sym=osym, stream=s_rx)
            if a.mode == "pipe":
                rx_done[b].record(s_rx)

    run(20)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(a.steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"mode": a.mode, "tx_cap": os.environ.get("MODEM_TX_WGS_PER_CU"),
                      "rx_cap": os.environ.get("MODEM_RX_WGS_PER_CU"),
                      "us_per_step": round(dt / a.steps * 1e6, 2),
                      "gsps": round(nsamp * a.steps / dt / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
