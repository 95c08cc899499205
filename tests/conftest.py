"""Shared fixtures. `-m gpu` tests need a gfx950 device; everything else runs on the CPU."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import __graft_entry__ as graft  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device")


@pytest.fixture(scope="session")
def m():
    """The product package (rust-modem_amd/) with its HIP library loaded."""
    mod = graft.package()
    mod.load_library()
    return mod


@pytest.fixture(scope="session")
def o():
    """The CPU oracle (test infrastructure)."""
    ora = graft.oracle()
    ora.lib()
    return ora


@pytest.fixture(scope="session")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test without a visible GPU")
    return torch


# The BASELINE.json configurations: name, phasor, bps, ntaps, sps.
CONFIGS = {
    "c1_bpsk": ("bpsk", 1, 33, 4),
    "c2_qpsk": ("qpsk", 2, 65, 4),
    "c3_qam16": ("qam16", 4, 129, 4),
    "c4_qpsk": ("qpsk", 2, 65, 4),
    "c5_qam256": ("qam256", 8, 513, 8),
}
PI_4 = float(np.float32(np.float32(np.pi) / np.float32(4.0)))   # PI / 4.0 in f32 (modulate.rs:76)


def product_phasor(m, name):
    return {"bpsk": lambda: m.BPSK(PI_4, 1.0), "qpsk": lambda: m.QPSK(0.0, 1.0),
            "qam16": lambda: m.QAM(4, 0.0, 1.0), "qam256": lambda: m.QAM(8, 0.0, 1.0)}[name]()


def oracle_phasor(o, name):
    return {"bpsk": lambda: o.new_phasor(o.BPSK, PI_4, 1.0), "qpsk": lambda: o.new_phasor(o.QPSK, 0.0, 1.0),
            "qam16": lambda: o.new_phasor(o.QAM, 4, 0.0, 1.0),
            "qam256": lambda: o.new_phasor(o.QAM, 8, 0.0, 1.0)}[name]()


def oracle_slicer(o, name, bps):
    if name.startswith("qam"):
        return o.qam_axis_slicer(bps, 1.0)
    return o.make_slicer(o.SLICER_NEAREST, bps, o.phasor_lut(oracle_phasor(o, name)))


def sent_symbols(bits, bps):
    return (bits.reshape(-1, bps).astype(np.int64) @ (1 << np.arange(bps)[::-1])).astype(np.uint8)
