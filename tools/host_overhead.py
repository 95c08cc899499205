#!/usr/bin/env python3
"""Host-side cost per process() call (no sync in the loop), and its parts, on the GPU box."""
import cProfile
import ctypes
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def per_call(fn, n=400):
    fn()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    import torch
    r = bench.GpuRunner(bench.WORKLOADS["c2"], 0, 0)     # small kernels: host cost dominates
    d = r.ch[0]
    m = sys.modules["rust_modem_amd"]
    L = m.load_library()
    print("tx.process  us/call", round(per_call(lambda: r.tx(0)), 2))
    print("rx.process  us/call", round(per_call(lambda: r.rx(0)), 2))
    torch.cuda.synchronize()
    print("current_stream() us", round(per_call(lambda: torch.cuda.current_stream().cuda_stream), 2))
    print("raw stream us", round(per_call(lambda: torch._C._cuda_getCurrentRawStream(0)), 2))
    print("data_ptr us", round(per_call(lambda: d["y"].data_ptr()), 2))
    print("slice us", round(per_call(lambda: d["y"][: 1000]), 2))
    lib = ctypes.CDLL(m.lib_path())
    lib.modem_tx_sample.restype = ctypes.c_uint64
    lib.modem_tx_sample.argtypes = [ctypes.c_void_p]
    h = d["tx"]._h
    print("ctypes trivial call us", round(per_call(lambda: lib.modem_tx_sample(h)), 2))
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(300):
        r.tx(0)
        r.rx(0)
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(14)


if __name__ == "__main__":
    main()
