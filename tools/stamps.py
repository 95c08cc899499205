#!/usr/bin/env python3
"""Where the RX tile loop spends its cycles: runs a MODEM_STAMPS build (tools/build_var.sh
<name> -DMODEM_STAMPS) on C3 and prints each segment's share of the stamped wave-cycles
(read shares, not lengths: the stamps fence overlaps). Needs RUST_MODEM_AMD_LIB."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import bench  # noqa: E402

SEGS = ["loop", "wait-samples", "stage+max", "prefetch", "fir", "epilogue", "end-barrier", "general"]


def main():
    r = bench.GpuRunner(bench.WORKLOADS["c3"], 0, 0)
    for _ in range(5):
        r.tx(0)
        r.rx(0)
    r.sync()
    lib = ctypes.CDLL(os.environ["RUST_MODEM_AMD_LIB"])
    n = 4096 * 4 * 12
    buf = (ctypes.c_ulonglong * n)()
    assert lib.modem_debug_stamps(buf, ctypes.c_size_t(n)) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 12).astype(np.float64)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.save(os.path.join(ROOT, "gpurun_out", "stamps.npy"), a)
    a = a[a[:, :8].sum(1) > 0]
    rt = a[:, 8:10] - a[:, 8].min()
    print(f"realtime (100 MHz ticks): entry spread {rt[:, 0].max():.0f}, exit min {rt[:, 1].min():.0f} "
          f"median {np.median(rt[:, 1]):.0f} max {rt[:, 1].max():.0f}")
    a = a[:, :8]
    tot = a.sum(1)
    print(f"waves {len(a)}  mean stamped cycles/wave {tot.mean():.0f} (min {tot.min():.0f} max {tot.max():.0f})")
    for k, name in enumerate(SEGS):
        print(f"  {name:13s} {a[:, k].mean():10.0f} cyc  {100 * a[:, k].sum() / tot.sum():5.1f} %")


if __name__ == "__main__":
    main()
