#!/usr/bin/env python3
"""Fixed cost of the driver's short timed region (bench.py --steps 20 --warmup 5): wall time of
K steps after a W-step warmup, for K = 20 and 200, several repeats, with the host's wait mode
as given (--spin: hipSetDeviceFlags(hipDeviceScheduleSpin) before the context exists)."""
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
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    if a.spin:
        hip = ctypes.CDLL("libamdhip64.so")
        print("hipSetDeviceFlags(spin):", hip.hipSetDeviceFlags(ctypes.c_uint(1)))
    import bench
    r = bench.GpuRunner(bench.WORKLOADS["c3"], 0, 0)
    for K in (20, 200, 20):
        ts = []
        for _ in range(a.reps):
            for _ in range(5):
                r.step()
            r.sync()
            r.sync()
            t0 = time.perf_counter()
            for _ in range(K):
                r.step()
            r.sync()
            ts.append((time.perf_counter() - t0) / K * 1e6)
        print(f"K={K}: us/step", " ".join(f"{t:.2f}" for t in ts))
    # host cost of one step (ChainPlan.run), device idle-free: enqueue 200 steps, time the loop
    r.sync()
    t0 = time.perf_counter()
    for _ in range(50):
        r.step()
    t1 = time.perf_counter()
    r.sync()
    print(f"host enqueue per step {(t1 - t0) / 50 * 1e6:.2f} us")


if __name__ == "__main__":
    main()
