#!/usr/bin/env python3
"""Kernel legs of ad-hoc workloads (experiment tooling): bench.GpuRunner on a workload tuple
given on the command line, its TX / RX / chain legs by HIP events (bench's kernel_times_ms).
Usage: tools/wl_probe.py phasor bps ntaps sps nsamp nch [dtype] [--no-batch | --batch] [--group G]
e.g.   tools/wl_probe.py qpsk 2 65 4 16777216 1     (C4's filter on one 2^24-sample channel)"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("phasor")
    ap.add_argument("bps", type=int)
    ap.add_argument("ntaps", type=int)
    ap.add_argument("sps", type=int)
    ap.add_argument("nsamp", type=int)
    ap.add_argument("nch", type=int)
    ap.add_argument("dtype", type=int, nargs="?", default=0)
    ap.add_argument("--no-batch", action="store_true")
    ap.add_argument("--batch", action="store_true", help="the batch path even for one channel")
    ap.add_argument("--group", type=int, default=0)
    ap.add_argument("--label", default="")
    a = ap.parse_args()
    wl = (a.phasor, a.bps, a.ntaps, a.sps, a.nsamp, a.nch, a.dtype, "probe")
    batch = (a.nch > 1 or a.batch) and not a.no_batch
    r = bench.GpuRunner(wl, 0, 0, streams=1, batch=batch, group=a.group)
    bench.settle_clocks(r, 200.0)
    tx, rx, ch = r.kernel_times_ms(budget_ms=10.0, rounds=5)
    per = r.launch_channels()
    n = a.nsamp * per
    print(json.dumps({"label": a.label, "wl": wl[:7], "batch": batch, "channels_per_launch": per,
                      "tx_us": round(tx * 1e3, 2), "rx_us": round(rx * 1e3, 2), "chain_us": round(ch * 1e3, 2),
                      "chain_gsps": round(n / (ch * 1e-3) / 1e9, 1), "ok": r.check()}), flush=True)


if __name__ == "__main__":
    main()
