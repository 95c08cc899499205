#!/usr/bin/env python3
"""Profiling driver: run the TX and RX kernels of one bench workload `--reps` times
(device-resident buffers, no oracle). Used under rocprofv3 for traces and PMC counters."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3", choices=sorted(bench.WORKLOADS))
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", choices=["tx", "rx", "both", "chain"], default="both",
                    help="chain: the bench's step (ChainPlan: the fused launch where it applies)")
    ap.add_argument("--amplitude", type=float, default=1.0)
    # multi-channel configs: the bench's batch launches over groups of --group channels (0: the
    # config's default), as bench.py runs them; --no-batch: one launch per channel
    ap.add_argument("--group", type=int, default=0)
    ap.add_argument("--no-batch", action="store_true")
    a = ap.parse_args()
    wl, _ = bench.rank_workload(a.config, 1)
    batch = wl[5] > 1 and not a.no_batch
    group = a.group if a.group > 0 else bench.GROUP_DEFAULT.get(a.config, 0)
    r = bench.GpuRunner(wl, 0, 0, amplitude=a.amplitude, batch=batch, group=group)
    for _ in range(a.reps):
        if a.only == "chain" or batch:
            r.step()
            continue
        for c in range(r.nch):
            if a.only in ("tx", "both"):
                r.tx(c)
            if a.only in ("rx", "both"):
                r.rx(c)
    r.sync()
    # coverage: poison the outputs, run the chain once more, then check every decision
    for d in r.ch:
        d["y"].fill_(float("nan"))
        d["osym"].fill_(255)
    r.step()
    r.sync()
    print("ok", r.check())


if __name__ == "__main__":
    main()
