#!/usr/bin/env python3
"""C2's fused launch (chain_small) by phase, from per-workgroup s_memrealtime stamps (100 MHz) of a
probe build: round 6 built it with a temporary MODEM_PROBE_STAMPS switch in modem_chain.hip (a
__device__ g_stamps[4096 * 16] array, thread 0 storing the stamps and each wave's HW_ID / XCC_ID at
slots 0-4, 5 and 8-11, and an exported modem_probe_stamps(out, n) copying it back), removed after the
measurement (profiles/r06_c2_stamps.txt); the library is taken from RUST_MODEM_AMD_LIB. Stamps per workgroup (thread 0): 0 entry, 1 the TX part done (its
stores issued), 2 the RX tap tables in LDS, 3 the RX part done (its stores issued), 4 every store
acknowledged. For isolated launches (step; synchronize) and the last of a back-to-back run, the
percentiles over the 1024 workgroups of each phase and of the entry skew, in us.
Usage: RUST_MODEM_AMD_LIB=... python3 tools/c2_stamps.py [--reps 10]"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import numpy as np
    import bench
    r = bench.GpuRunner(bench.WORKLOADS["c2"], 0, 0)
    lib = ctypes.CDLL(os.environ["RUST_MODEM_AMD_LIB"])
    lib.modem_probe_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    nwg = 1024
    buf = np.zeros(4096 * 16, dtype=np.uint64)

    def read():
        assert lib.modem_probe_stamps(buf.ctypes.data, buf.size) == 0
        s = buf[:nwg * 16].reshape(nwg, 16).astype(np.int64)
        return s[:, :5] * 10e-3, s[:, 5], s[:, 8:12]   # 100 MHz ticks -> us; XCC_ID; HW_ID per wave

    def report(tag, runs):
        cols = {"entry skew": [], "tx part": [], "tables wait": [], "rx part": [], "store drain": [], "span": []}
        for s, _, _ in runs:
            t0 = s[:, 0].min()
            cols["entry skew"].append(s[:, 0] - t0)
            cols["tx part"].append(s[:, 1] - s[:, 0])
            cols["tables wait"].append(s[:, 2] - s[:, 1])
            cols["rx part"].append(s[:, 3] - s[:, 2])
            cols["store drain"].append(s[:, 4] - s[:, 3])
            cols["span"].append(np.array([s[:, 4].max() - t0]))
        print(f"== {tag} ({len(runs)} launches, us; p10 / p50 / p90 / max over workgroups and launches)")
        for k, v in cols.items():
            x = np.concatenate(v)
            print(f"  {k:12s} {np.percentile(x, 10):7.2f} {np.percentile(x, 50):7.2f} {np.percentile(x, 90):7.2f} {x.max():7.2f}")
        sys.stdout.flush()

    for _ in range(2000):                       # clocks up
        r.step()
    r.sync()
    iso = []
    for _ in range(a.reps):
        r.step()
        r.sync()
        iso.append(read())
    report("isolated launches", iso)
    b2b = []
    for _ in range(a.reps):
        for _ in range(200):
            r.step()
        r.sync()
        b2b.append(read())
    report("last of 200 back-to-back launches", b2b)
    # where the waves ran (gfx9 HW_ID: wave 3:0, SIMD 5:4, CU 11:8, SH 12, SE 15:13): the SIMD of each
    # workgroup's wave 0, and how many workgroups' wave 0 share a SIMD of one CU
    _, xcc, hw = b2b[-1]
    simd = (hw >> 4) & 3
    cu = (xcc << 16) | (hw[:, 0] & 0xFF00)
    print("wave -> SIMD of the first 8 workgroups:", [list(map(int, simd[i])) for i in range(8)])
    import collections
    per = collections.defaultdict(list)
    for i in range(nwg):
        per[int(cu[i])].append(int(simd[i, 0]))
    hist = collections.Counter(max(collections.Counter(v).values()) for v in per.values())
    print("CUs:", len(per), " workgroups per CU:", collections.Counter(len(v) for v in per.values()),
          " largest number of wave 0s on one SIMD of a CU:", dict(hist))


if __name__ == "__main__":
    main()
