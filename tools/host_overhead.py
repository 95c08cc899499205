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
    # the C entry points alone, arguments prepared once
    L.modem_tx_process.restype = ctypes.c_int
    prod = ctypes.c_size_t()
    st = torch._C._cuda_getCurrentRawStream(0)
    bp, yp, nb = d["bits"].data_ptr(), d["y"].data_ptr(), int(d["bits"].numel())
    ny = int(d["y"].shape[0])
    targs = (d["tx"]._h, ctypes.c_void_p(bp), ctypes.c_size_t(nb), ctypes.c_void_p(yp), ctypes.c_size_t(ny),
             ctypes.byref(prod), ctypes.c_void_p(st))
    print("C modem_tx_process us", round(per_call(lambda: L.modem_tx_process(*targs)), 2))
    rargs = (d["rx"]._h, ctypes.c_void_p(yp), ctypes.c_size_t(ny), ctypes.c_void_p(d["oiq"].data_ptr()),
             ctypes.c_void_p(d["osym"].data_ptr()), ctypes.c_size_t(int(d["oiq"].shape[0])), ctypes.byref(prod),
             ctypes.c_void_p(st))
    print("C modem_rx_process us", round(per_call(lambda: L.modem_rx_process(*rargs)), 2))
    hip = ctypes.CDLL("libamdhip64.so")
    attr = (ctypes.c_char * 256)()
    print("hipPointerGetAttributes us", round(per_call(lambda: hip.hipPointerGetAttributes(attr, ctypes.c_void_p(yp))), 2))
    dev = ctypes.c_int()
    print("hipGetDevice us", round(per_call(lambda: hip.hipGetDevice(ctypes.byref(dev))), 2))
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
