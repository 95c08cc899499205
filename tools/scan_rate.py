#!/usr/bin/env python3
"""Rates of the scanned phasors (DMPSK / MFSK / BFSK: a serial f32 state recurrence per stream,
DESIGN.md §8): one channel through DigitalModulator.process (tx_scan: one lane runs the
recurrence) against a bank of channels through DigitalModulator.process_batch (tx_scan_batch:
one lane per channel), in Msymbols/s by HIP events around the calls (scan + the per-sample
phasor kernel), median of 3. Run under rocprofv3 --kernel-trace --stats for the scan kernels
alone. Usage: tools/scan_rate.py [--nsym N] [--nch C] [--sps S]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nsym", type=int, default=1 << 16)
    ap.add_argument("--nch", type=int, default=64)
    ap.add_argument("--sps", type=int, default=1)
    a = ap.parse_args()
    import torch
    import __graft_entry__ as g
    m = g.package()
    w = m.Freq(1000, 10000).sample_freq()
    kinds = {"dqpsk": (lambda: m.DMPSK(2, 1.0, 0.7853982, 1.5707964), 2),
             "mfsk16": (lambda: m.MFSK(4, m.Freq(50, 10000), 1.0, "increase"), 4),
             "bfsk": (lambda: m.BFSK(m.Freq(200, 10000), 1.0), 1)}

    def timed(fn, reps=3):
        ts = []
        for _ in range(reps):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            torch.cuda.synchronize()
            ev[0].record()
            fn()
            ev[1].record()
            torch.cuda.synchronize()
            ts.append(ev[0].elapsed_time(ev[1]) * 1e-3)
        return sorted(ts)[len(ts) // 2]

    for name, (mk, bps) in kinds.items():
        bits = [m.prng_bits(0x5CA40000 + c, a.nsym * bps) for c in range(a.nch)]
        one = m.DigitalModulator(m.Carrier(w), mk(), a.sps, None, out_mode=1)
        out1 = torch.empty((a.nsym * a.sps, 2), dtype=torch.float32, device="cuda")
        one.process(bits[0], out=out1)                     # warm
        t1 = timed(lambda: one.process(bits[0], out=out1))
        bank = [m.DigitalModulator(m.Carrier(w), mk(), a.sps, None, out_mode=1) for _ in range(a.nch)]
        outs = [torch.empty((a.nsym * a.sps, 2), dtype=torch.float32, device="cuda") for _ in range(a.nch)]
        m.DigitalModulator.process_batch(bank, bits, outs)
        tb = timed(lambda: m.DigitalModulator.process_batch(bank, bits, outs))
        print(json.dumps({"phasor": name, "nsym_per_channel": a.nsym, "sps": a.sps,
                          "single_channel_msym_s": round(a.nsym / t1 / 1e6, 2),
                          "bank_channels": a.nch, "bank_msym_s": round(a.nch * a.nsym / tb / 1e6, 2),
                          "bank_speedup": round(a.nch * a.nsym / tb / (a.nsym / t1), 1)}), flush=True)


if __name__ == "__main__":
    main()
