#!/usr/bin/env python3
"""Where the driver's short timed region (bench.py --steps 20 --warmup 5) loses time: for a
20-step region after different preambles, the wall clock per step beside the device time of
each step (HIP events between steps on the launch stream), the gap from t0 to the first step's
start and from the last step's end to the host's return from synchronize.
Usage: python tools/region_probe.py [--spin] [--preamble none|legs|w2000]"""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spin", action="store_true")
    ap.add_argument("--preamble", default="none")
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--config", default="c3")
    a = ap.parse_args()
    if a.spin:
        hip = ctypes.CDLL("libamdhip64.so")
        print("hipSetDeviceFlags(spin):", hip.hipSetDeviceFlags(ctypes.c_uint(1)))
    import torch
    import bench
    r = bench.GpuRunner(bench.WORKLOADS[a.config], 0, 0)
    if a.preamble == "legs":
        r.kernel_times_ms()
    elif a.preamble == "settle":
        print(bench.settle_clocks(r, 300.0))
    elif a.preamble == "w2000":
        for _ in range(2000):
            r.step()
    for rep in range(a.reps):
        for _ in range(5):
            r.step()
        r.sync()
        r.sync()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(21)]
        t0 = time.perf_counter()
        ev[0].record(r.stream)
        for k in range(20):
            r.step()
            ev[k + 1].record(r.stream)
        t1 = time.perf_counter()
        r.sync()
        t2 = time.perf_counter()
        d = [ev[k].elapsed_time(ev[k + 1]) * 1e3 for k in range(20)]
        print(f"[{a.preamble}{' spin' if a.spin else ''}] rep {rep}: wall/step {(t2 - t0) / 20 * 1e6:.2f} us, "
              f"device sum {sum(d):.1f} us (wall {(t2 - t0) * 1e6:.1f}), enqueue {(t1 - t0) * 1e6:.1f} us; "
              f"steps: " + " ".join(f"{x:.1f}" for x in d), flush=True)


if __name__ == "__main__":
    main()
