#!/usr/bin/env python3
"""C4 channel-batch probe (experiment tooling): does the placement of the channels' sample
buffers set the batch launches' per-sample cost? The channels' (nsamp, 2) sample buffers are
carved from one arena at a pitch of nsamp * 8 + stagger bytes (stagger 0: back to back, the
same address bits modulo the buffer size for every channel; else each channel shifted by c *
stagger against that), or left to torch's allocator (--separate). Prints the first group's
TX / RX / chain legs (HIP events, bench.kernel_times_ms) and the whole job's step time.
Usage: tools/c4_layout_probe.py [--group G] [--stagger BYTES | --separate] [--nch N]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--group", type=int, default=8)
    ap.add_argument("--nch", type=int, default=64)
    ap.add_argument("--nsamp", type=int, default=1 << 22)
    ap.add_argument("--stagger", type=int, default=0)
    ap.add_argument("--separate", action="store_true")
    ap.add_argument("--steps", type=int, default=100)
    a = ap.parse_args()
    import torch
    real_empty = torch.empty
    arena = {}
    if not a.separate:
        pitch = a.nsamp * 8 + a.stagger
        assert pitch % 256 == 0
        buf = real_empty(pitch * a.nch + 4096, dtype=torch.uint8, device="cuda:0")
        arena["buf"], arena["next"], arena["pitch"] = buf, 0, pitch

        def empty(*shape, **kw):
            shp = shape[0] if len(shape) == 1 and isinstance(shape[0], tuple) else shape
            if tuple(shp) == (a.nsamp, 2) and kw.get("dtype") == torch.float32 and arena["next"] < a.nch:
                off = arena["next"] * arena["pitch"]
                arena["next"] += 1
                return arena["buf"][off:off + a.nsamp * 8].view(torch.float32).view(a.nsamp, 2)
            return real_empty(*shape, **kw)
        torch.empty = empty
    wl = ("qpsk", 2, 65, 4, a.nsamp, a.nch, 0, "c4 layout probe")
    r = bench.GpuRunner(wl, 0, 0, streams=1, batch=True, group=a.group)
    torch.empty = real_empty
    ptrs = [d["y"].data_ptr() for d in r.ch[:4]]
    bench.settle_clocks(r, 200.0)
    tx, rx, ch = r.kernel_times_ms(budget_ms=10.0, rounds=5)
    for _ in range(20):
        r.step()
    r.sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        r.step()
    r.sync()
    dt = (time.perf_counter() - t0) / a.steps
    print(json.dumps({"group": a.group, "stagger": None if a.separate else a.stagger,
                      "ptr_mod_32MiB": [p % (32 << 20) for p in ptrs], "ptr_deltas": [p - ptrs[0] for p in ptrs],
                      "tx_us": round(tx * 1e3, 2), "rx_us": round(rx * 1e3, 2), "chain_us": round(ch * 1e3, 2),
                      "group_gsps": round(a.nsamp * a.group / (ch * 1e-3) / 1e9, 1),
                      "step_ms": round(dt * 1e3, 4), "job_gsps": round(a.nsamp * a.nch / dt / 1e9, 1),
                      "ok": r.check()}), flush=True)


if __name__ == "__main__":
    main()
