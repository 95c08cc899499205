#!/usr/bin/env python3
"""RX phase timeline from a -DMODEM_STAMPS diagnostic build (tools/build_var.sh stamps -DMODEM_STAMPS):
per wave and tile, s_memtime at staging start / end, after the first barrier, after the matched
filter, after the stores and after the second barrier (rx_mfma's loop; the general-path tile is
bracketed by points 6 and 7). Runs the C3 chain warm, clears the stamps, runs one TX + RX step and
saves the raw stamps to gpurun_out/stamps_<tag>.npz with a printed summary (cycles).

    RUST_MODEM_AMD_LIB=rust-modem_amd/build/var/stamps/libmodem_hip.so python3 tools/stamps.py --tag base
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import bench  # noqa: E402

W, T, P = 8192, 8, 8


def grab(lib, clear, kernel="rx"):
    buf = np.zeros(W * T * P, dtype=np.uint64)
    fn = lib.modem_debug_rx_stamps if kernel == "rx" else lib.modem_debug_tx_stamps
    n = fn(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes), int(clear))
    assert n > 0, n
    return buf.reshape(W, T, P)


def summary(s, grid_waves, kernel="rx"):
    s = s[:grid_waves].astype(np.int64)
    hdr = s[:, 7]
    xcc = hdr[:, 3] & 0xF
    out = []
    phases = (("stage", 0, 1), ("bar1", 1, 2), ("fir", 2, 3), ("emit", 3, 4), ("bar2", 4, 5)) if kernel == "rx" else \
        (("stage", 0, 1), ("bar1", 1, 2), ("fir+emit", 2, 4), ("bar2", 4, 5))
    for name, a, b in phases:
        d = s[:, :7, b] - s[:, :7, a]
        ok = (s[:, :7, a] > 0) & (s[:, :7, b] > 0)
        v = d[ok]
        out.append(f"{name:6s} n {v.size:6d} med {np.median(v):8.0f} p10 {np.percentile(v, 10):8.0f} "
                   f"p90 {np.percentile(v, 90):8.0f} mean {v.mean():8.0f}")
    sl = s[:, :7, 7] - s[:, :7, 6]
    ok = (s[:, :7, 6] > 0) & (s[:, :7, 7] > 0)
    if ok.any():
        out.append(f"slow   n {ok.sum():6d} cycles {sl[ok].tolist()[:8]}")
    # kernel span per XCD (s_memtime is per XCD): first entry .. last exit
    for x in np.unique(xcc):
        m = xcc == x
        e0, e1 = hdr[m, 0].min(), hdr[m, 4].max()
        life = hdr[m, 4] - hdr[m, 0]
        out.append(f"xcc {x}: waves {m.sum()} span {e1 - e0} cyc; wave life med {np.median(life):.0f} "
                   f"min {life.min()} max {life.max()}; entry spread {np.ptp(hdr[m, 0])}")
    rt = hdr[:, 5] - hdr[:, 1]
    out.append(f"realtime (100 MHz) wave life med {np.median(rt):.0f} max {rt.max()} "
               f"-> clock ~ {np.median((hdr[:, 4] - hdr[:, 0]) / np.maximum(rt, 1)) * 100:.0f} MHz")
    return "\n".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="base")
    ap.add_argument("--config", default="c3")
    ap.add_argument("--warm", type=int, default=400)
    ap.add_argument("--kernel", choices=["rx", "tx"], default="rx")
    a = ap.parse_args()
    r = bench.GpuRunner(bench.WORKLOADS[a.config], 0, 0)
    m = r._m
    lib = m.load_library()
    getattr(lib, f"modem_debug_{a.kernel}_stamps").restype = ctypes.c_int
    for _ in range(a.warm):
        r.step()
    r.sync()
    runs = []
    for k in range(3):
        grab(lib, True, a.kernel)
        r.tx(0)
        r.rx(0)
        r.sync()
        runs.append(grab(lib, False, a.kernel))
    s = np.stack(runs)
    hw = s[0, :, 7, 2]
    nw = int((hw != 0).sum())
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"stamps_{a.tag}_{a.kernel}.npz"), stamps=s[:, :max(nw, 1)])
    for k in range(s.shape[0]):
        print(f"== run {k} ({nw} waves)")
        print(summary(s[k], nw, a.kernel))
    print("ok", r.check())


if __name__ == "__main__":
    main()
