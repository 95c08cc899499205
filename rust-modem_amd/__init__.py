"""rust_modem_amd — Python mirror of ramtej/rust-modem's modem API over the gfx950 backend.

The product is `lib/libmodem_hip.so` (HIP kernels + the C ABI of include/modem_hip.h); this
module is a thin ctypes layer that keeps the reference crate's names and argument meanings
so callers (and the parity tests) read like the reference:

    reference (src/modem)                          here
    Freq::new(hz, sr).sample_freq()  freq.rs:19-26  Freq(hz, sr).sample_freq()
    Rates::new(br, sr)               rates.rs:12-18 Rates(br, sr).samples_per_symbol
    Carrier::new(freq), .sample      carrier.rs:4-26 Carrier(freq), .sample, .next()
    BPSK/QPSK/QAM/BASK/MPSK/APSK/OQPSK digital/*.rs BPSK(...)... (.i/.q/.bits_per_symbol)
    DigitalModulator::new(&mut c, phasor, src)      DigitalModulator(carrier, phasor, sps, taps)
        modulator.rs:64-101                             .process(bits) -> samples (device)
    FIRFilter::new(&taps).add(x)     fir.rs:3-35    FIRFilter(taps).add(x) / .process(block)
    Demodulator::new(c, sig, lp)     demodulator.rs DemodulatorRx(carrier, taps, ...)
                                                        .process(iq) -> (decimated iq, symbols)

Where the reference panics (assert!, unwrap, index out of range) this layer raises
`ModemPanic`. The HIP library is required: importing works without a GPU (host-only
entry points such as the LUT builders run on the CPU), but every device entry point raises
if the library is missing or no gfx950 device is present — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import Optional, Sequence, Tuple

import numpy as np

__all__ = [
    "ModemPanic", "ModemError", "lib_path", "load_library",
    "Freq", "Rates", "Carrier", "Ring",
    "BPSK", "QPSK", "QAM", "BASK", "MPSK", "APSK", "OQPSK",
    "rrc_taps", "DigitalModulator", "DemodulatorRx", "FIRFilter", "prng_bits",
    "MIX_COMPLEX", "MIX_REFERENCE_REAL", "MIX_REFERENCE_REAL_EXACT", "OUT_IQ_MIXED", "OUT_IQ_BASEBAND", "OUT_REAL",
    "TxBatchPlan", "RxBatchPlan", "SLICER_NONE", "SLICER_NEAREST", "SLICER_QAM_AXIS", "DTYPE_F32", "DTYPE_F16", "DTYPE_I16",
]

PI32 = float(np.float32(math.pi))      # std::f32::consts::PI

MODEM_OK, ERR_INVALID_ARG, ERR_UNSUPPORTED, ERR_HIP, ERR_NO_DEVICE, ERR_CAPACITY, ERR_ALLOC = (
    0, -1, -2, -3, -4, -5, -6)
DTYPE_F32, DTYPE_F16, DTYPE_I16 = 0, 1, 2   # I16: real samples, RX input (demodulate)
OUT_IQ_MIXED, OUT_IQ_BASEBAND, OUT_REAL = 0, 1, 2
MIX_COMPLEX, MIX_REFERENCE_REAL, MIX_REFERENCE_REAL_EXACT = 0, 1, 2
SLICER_NONE, SLICER_NEAREST, SLICER_QAM_AXIS = 0, 1, 2
_PH_BPSK, _PH_QPSK, _PH_QAM, _PH_BASK, _PH_MPSK, _PH_APSK, _PH_OQPSK = 1, 2, 3, 4, 5, 6, 7


class ModemError(RuntimeError):
    """A backend failure (HIP error, no device, capacity)."""

    def __init__(self, status: int, what: str = ""):
        self.status = status
        super().__init__(f"{what}: {status_str(status)} ({status})" if what else status_str(status))


class ModemPanic(ModemError):
    """Raised where the reference crate would panic (assert!/unwrap/index)."""


# ------------------------------------------------------------------------- library ----
_HERE = os.path.dirname(os.path.abspath(__file__))


def lib_path() -> str:
    # RUST_MODEM_AMD_LIB: an alternative build (profiling ablations, tools/ablate.sh)
    return os.environ.get("RUST_MODEM_AMD_LIB") or os.path.join(_HERE, "lib", "libmodem_hip.so")


class _Ring(ctypes.Structure):
    _fields_ = [("start", ctypes.c_uint8), ("end", ctypes.c_uint8),
                ("radius", ctypes.c_float), ("phase", ctypes.c_float)]


class _PhasorDesc(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("bits_per_symbol", ctypes.c_uint32),
                ("phase", ctypes.c_float), ("amplitude", ctypes.c_float),
                ("nrings", ctypes.c_uint32), ("rings", ctypes.POINTER(_Ring)),
                ("freq", ctypes.c_float), ("samples_per_symbol", ctypes.c_uint32),
                ("shift", ctypes.c_float), ("mfsk_map", ctypes.c_uint32)]


class _SlicerDesc(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("bits_per_symbol", ctypes.c_uint32),
                ("lut", ctypes.POINTER(ctypes.c_float)), ("bits_per_carrier", ctypes.c_uint32),
                ("inv_scale", ctypes.c_float), ("max_symbol", ctypes.c_float)]


class _TxDesc(ctypes.Structure):
    _fields_ = [("bits_per_symbol", ctypes.c_uint32), ("lut", ctypes.POINTER(ctypes.c_float)),
                ("samples_per_symbol", ctypes.c_uint32), ("taps", ctypes.POINTER(ctypes.c_float)),
                ("ntaps", ctypes.c_uint32), ("sample_freq", ctypes.c_float),
                ("s0", ctypes.c_uint64), ("dtype", ctypes.c_int32), ("out_mode", ctypes.c_int32),
                ("q_offset", ctypes.c_uint32), ("phasor", ctypes.POINTER(_PhasorDesc))]


class _RxDesc(ctypes.Structure):
    _fields_ = [("sample_freq", ctypes.c_float), ("s0", ctypes.c_uint64),
                ("taps", ctypes.POINTER(ctypes.c_float)), ("ntaps", ctypes.c_uint32),
                ("decim", ctypes.c_uint32), ("decim_offset", ctypes.c_uint32),
                ("mix", ctypes.c_int32), ("in_dtype", ctypes.c_int32),
                ("out_dtype", ctypes.c_int32), ("slicer", _SlicerDesc),
                ("phase_offset", ctypes.c_float)]


_lib = None
_lib_err: Optional[str] = None


def load_library():
    """Load lib/libmodem_hip.so (raises if it was not built)."""
    global _lib, _lib_err
    if _lib is not None:
        return _lib
    path = lib_path()
    if not os.path.exists(path):
        _lib_err = f"{path} not built (run __graft_entry__.build() or `make -C rust-modem_amd`)"
        raise ModemError(ERR_UNSUPPORTED, _lib_err)
    # One HIP runtime per process: torch ships its own libamdhip64 (soname libamdhip64.so.7,
    # loaded by its NEEDED name "libamdhip64.so"). Loading torch first lets our NEEDED
    # libamdhip64.so.7 resolve to that already-loaded runtime, so device pointers and
    # streams from torch are valid here. Without torch, /opt/rocm's runtime is used.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(path)
    c = ctypes
    vp, sz, u64, u32, f32, st = c.c_void_p, c.c_size_t, c.c_uint64, c.c_uint32, c.c_float, c.c_int
    fp = c.POINTER(c.c_float)
    sig = {
        "modem_status_str": (c.c_char_p, [st]),
        "modem_abi_version": (c.c_int32, []),
        "modem_freq_sample_freq": (f32, [u64, u64]),
        "modem_rates_sps": (st, [u64, u64, c.POINTER(u64)]),
        "modem_pll_lock": (st, [f32, u64, fp, sz, fp]),
        "modem_carrier_phase": (f32, [f32, u64]),
        "modem_carrier_phases": (st, [f32, u64, sz, vp, c.c_int, vp]),
        "modem_phasor_bits": (st, [c.POINTER(_PhasorDesc), c.POINTER(u32)]),
        "modem_phasor_lut": (st, [c.POINTER(_PhasorDesc), fp]),
        "modem_phasor_slicer": (st, [c.POINTER(_PhasorDesc), fp, c.POINTER(_SlicerDesc)]),
        "modem_rrc_taps": (st, [u32, u32, c.c_double, fp]),
        "modem_tx_create": (st, [c.POINTER(_TxDesc), c.c_int, c.POINTER(vp)]),
        "modem_tx_process": (st, [vp, vp, sz, vp, sz, c.POINTER(sz), vp]),
        "modem_tx_flush": (st, [vp, vp, sz, c.POINTER(sz), vp]),
        "modem_tx_process_batch": (st, [c.POINTER(vp), sz, c.POINTER(vp), c.POINTER(sz), c.POINTER(vp),
                                        c.POINTER(sz), c.POINTER(sz), vp]),
        "modem_tx_sample": (u64, [vp]),
        "modem_tx_destroy": (st, [vp]),
        "modem_rx_create": (st, [c.POINTER(_RxDesc), c.c_int, c.POINTER(vp)]),
        "modem_rx_process": (st, [vp, vp, sz, vp, vp, sz, c.POINTER(sz), vp]),
        "modem_rx_flush": (st, [vp, vp, vp, sz, c.POINTER(sz), vp]),
        "modem_rx_process_batch": (st, [c.POINTER(vp), sz, c.POINTER(vp), c.POINTER(sz), c.POINTER(vp),
                                        c.POINTER(vp), c.POINTER(sz), c.POINTER(sz), vp]),
        "modem_rx_sample": (u64, [vp]),
        "modem_rx_destroy": (st, [vp]),
        "modem_fir_create": (st, [fp, u32, c.c_int, c.POINTER(vp)]),
        "modem_fir_process": (st, [vp, vp, vp, sz, vp]),
        "modem_fir_destroy": (st, [vp]),
        "modem_prng_bits": (st, [u64, vp, sz, c.c_int, vp]),
        "modem_chain_create": (st, [vp, vp, vp, sz, vp, sz, vp, vp, sz, c.POINTER(vp)]),
        "modem_chain_run": (st, [vp, c.POINTER(sz), c.POINTER(sz), vp]),
        "modem_chain_fused": (c.c_int, [vp]),
        "modem_chain_destroy": (st, [vp]),
        "modem_chain_batch_create": (st, [c.POINTER(vp), c.POINTER(vp), sz, sz, c.POINTER(vp), c.POINTER(sz),
                                          c.POINTER(vp), c.POINTER(sz), c.POINTER(vp), c.POINTER(vp),
                                          c.POINTER(sz), c.POINTER(vp)]),
        "modem_chain_batch_run": (st, [vp, c.POINTER(sz), c.POINTER(sz), vp]),
        "modem_chain_batch_destroy": (st, [vp]),
    }
    for name, (res, args) in sig.items():
        try:
            fn = getattr(L, name)
        except AttributeError:
            if name.startswith("modem_chain_"):   # ABI 5; experiment builds of older sources lack it
                continue
            raise
        fn.restype, fn.argtypes = res, args
    _lib = L
    return L


def status_str(s: int) -> str:
    try:
        return load_library().modem_status_str(s).decode()
    except ModemError:
        return f"status {s}"


def _check(status: int, what: str):
    if status == MODEM_OK:
        return
    if status == ERR_INVALID_ARG:
        raise ModemPanic(status, what)
    raise ModemError(status, what)


def _fptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


# --------------------------------------------------------------- timebase (B4) ----
class Freq:
    """freq.rs:3-27 — cycles per second at a sample rate."""

    def __init__(self, hz: int, sr: int):
        self.hz, self.sr = int(hz), int(sr)

    def ang_freq(self) -> float:
        return float(np.float32(2.0) * np.float32(PI32) * np.float32(self.hz))

    def sample_freq(self) -> float:
        return float(load_library().modem_freq_sample_freq(self.hz, self.sr))


class Rates:
    """rates.rs:1-19 — samples_per_symbol = sr / br (integer division)."""

    def __init__(self, br: int, sr: int):
        if br == 0:
            raise ModemPanic(ERR_INVALID_ARG, "Rates::new: attempt to divide by zero")
        self.baud_rate, self.sample_rate = int(br), int(sr)
        self.samples_per_symbol = int(sr) // int(br)


class Carrier:
    """carrier.rs:3-27 — phase(n) = mod_trig(sample_freq * (n as f32)); `sample` is the next n."""

    def __init__(self, freq: Freq, sample: int = 0):
        self.sample_freq = freq.sample_freq() if isinstance(freq, Freq) else float(freq)
        self.sample = int(sample)

    def inner(self, s: int) -> float:
        return float(load_library().modem_carrier_phase(self.sample_freq, int(s)))

    def next(self) -> float:
        s = self.sample
        self.sample += 1
        return self.inner(s)

    def phases(self, s0: int, n: int, device: int = 0, stream=None):
        """inner(s0 .. s0+n-1) on the device (the kernels' phase code path), a CUDA tensor."""
        import torch
        out = torch.empty(int(n), dtype=torch.float32, device=f"cuda:{device}")
        _check(load_library().modem_carrier_phases(self.sample_freq, int(s0), int(n),
                                                   out.data_ptr() if n else None, device,
                                                   _stream_handle(stream, device)), "Carrier.phases")
        return out


# ------------------------------------------------------------ DigitalPhasor (B2) ----
class _Phasor:
    """Memoryless DigitalPhasor (digital/phasor.rs:1-12) as a host-built (I,Q) table."""

    _kind = 0

    def _desc(self) -> _PhasorDesc:
        d = _PhasorDesc()
        d.kind = self._kind
        d.bits_per_symbol = getattr(self, "_bps", 0)
        d.phase = getattr(self, "_phase", 0.0)
        d.amplitude = self.amplitude
        d.nrings = 0
        return d

    def bits_per_symbol(self) -> int:
        b = ctypes.c_uint32()
        _check(load_library().modem_phasor_bits(ctypes.byref(self._desc()), ctypes.byref(b)),
               type(self).__name__)
        return int(b.value)

    def lut(self) -> np.ndarray:
        """(2^bps, 2) float32: row s = (i, q) of the bits of s, MSB first."""
        n = 1 << self.bits_per_symbol()
        out = np.zeros((n, 2), dtype=np.float32)
        _check(load_library().modem_phasor_lut(ctypes.byref(self._desc()), _fptr(out)),
               type(self).__name__)
        return out

    def _index(self, b: Sequence[int]) -> int:
        s = 0
        for v in b:
            s = (s << 1) | (int(v) & 1)   # bytes_to_bits, digital/util.rs:5-11
        return s

    def i(self, s: int, b: Sequence[int]) -> float:
        return float(self.lut()[self._index(b), 0])

    def q(self, s: int, b: Sequence[int]) -> float:
        return float(self.lut()[self._index(b), 1])

    def next(self, s: int, b: Sequence[int]) -> Tuple[float, float]:
        return self.i(s, b), self.q(s, b)

    def slicer(self) -> _SlicerDesc:
        lut = self.lut()
        self._slicer_lut = lut          # keep alive until handed to a handle
        sd = _SlicerDesc()
        _check(load_library().modem_phasor_slicer(ctypes.byref(self._desc()), _fptr(lut),
                                                  ctypes.byref(sd)), "slicer")
        return sd


class BPSK(_Phasor):
    """bpsk.rs:4-32."""
    _kind = _PH_BPSK

    def __init__(self, phase: float, amplitude: float):
        self._phase, self.amplitude = float(phase), float(amplitude)


class QPSK(_Phasor):
    """qpsk.rs:4-36."""
    _kind = _PH_QPSK

    def __init__(self, phase: float, amplitude: float):
        self._phase, self.amplitude = float(phase), float(amplitude)


class QAM(_Phasor):
    """qam.rs:4-61 (natural-binary per axis; I from the MSB half)."""
    _kind = _PH_QAM

    def __init__(self, bits_per_symbol: int, phase: float, amplitude: float):
        if not bits_per_symbol > 1:
            raise ModemPanic(ERR_INVALID_ARG, "QAM::new: assertion failed: bits_per_symbol > 1")
        self._bps, self._phase, self.amplitude = int(bits_per_symbol), float(phase), float(amplitude)


class BASK(_Phasor):
    """bask.rs:3-25."""
    _kind = _PH_BASK

    def __init__(self, a: float):
        self.amplitude = float(a)


class MPSK(_Phasor):
    """mpsk.rs:6-42."""
    _kind = _PH_MPSK

    def __init__(self, bits_per_symbol: int, phase_offset: float, amplitude: float):
        self._bps, self._phase, self.amplitude = int(bits_per_symbol), float(phase_offset), float(amplitude)


class OQPSK(_Phasor):
    """oqpsk.rs:4-26 (the symbol map; pair it with DigitalModulator(even_odd_offset=True),
    the EvenOddOffset source modulate uses, modulate.rs:101-107)."""
    _kind = _PH_OQPSK

    def __init__(self, amplitude: float):
        self.amplitude = float(amplitude)


class Ring:
    """apsk.rs:60-82."""

    def __init__(self, rng: range, radius: float, phase: float):
        if not (0.0 <= radius <= 1.0):
            raise ModemPanic(ERR_INVALID_ARG, "Ring::new: assertion failed: radius in [0, 1]")
        self.range, self.radius, self.phase = rng, float(radius), float(phase)


class APSK(_Phasor):
    """apsk.rs:12-57."""
    _kind = _PH_APSK

    def __init__(self, amplitude: float, bits_per_symbol: int, rings: Sequence[Ring]):
        self.amplitude, self._bps, self.rings = float(amplitude), int(bits_per_symbol), list(rings)
        self.lut()   # verify() (apsk.rs:26) raises ModemPanic on bad rings

    def _desc(self):
        d = super()._desc()
        arr = (_Ring * len(self.rings))()
        for k, r in enumerate(self.rings):
            arr[k].start, arr[k].end = r.range.start, r.range.stop
            arr[k].radius, arr[k].phase = r.radius, r.phase
        self._rings_c = arr
        d.nrings = len(self.rings)
        d.rings = ctypes.cast(arr, ctypes.POINTER(_Ring))
        return d


class _SamplePhasor(_Phasor):
    """A DigitalPhasor whose (i, q) also depend on the symbol count or the sample index: no
    bits-only table; DigitalModulator evaluates it per sample on the GPU (tx_phasor)."""
    sample_dependent = True

    def lut(self) -> np.ndarray:
        raise ModemError(ERR_UNSUPPORTED, f"{type(self).__name__} has no bits-only (I,Q) table")

    def slicer(self):
        raise ModemError(ERR_UNSUPPORTED, f"{type(self).__name__}: no memoryless slicer")

    def i(self, s, b):
        raise ModemError(ERR_UNSUPPORTED, "evaluated per sample inside DigitalModulator")

    q = i


class DCQPSK(_SamplePhasor):
    """dcqpsk.rs:8-53 (pi/4-QPSK: the constellation turns by pi/4 at every symbol)."""
    _kind = 8

    def __init__(self, amplitude: float):
        self.amplitude = float(amplitude)


class CPFSK(_SamplePhasor):
    """cpfsk.rs:9-45: CPFSK::new(bits_per_symbol, rates, amplitude, deviation)."""
    _kind = 10

    def __init__(self, bits_per_symbol: int, rates: "Rates", amplitude: float, deviation: int):
        self._bps, self.amplitude = int(bits_per_symbol), float(amplitude)
        self._freq = Freq(int(deviation) * rates.baud_rate // 2, rates.sample_rate).sample_freq()

    def _desc(self):
        d = super()._desc()
        d.freq = self._freq
        return d


class MSK(_SamplePhasor):
    """msk.rs:6-37: MSK::new(amplitude, samples_per_symbol) (modulate pairs it with the
    EvenOddOffset source, modulate.rs:101-107: DigitalModulator(even_odd_offset=True))."""
    _kind = 11

    def __init__(self, amplitude: float, samples_per_symbol: int):
        if int(samples_per_symbol) % 2 != 0:
            raise ModemPanic(ERR_INVALID_ARG, "MSK::new: assertion failed: samples_per_symbol % 2 == 0")
        self.amplitude, self._sps = float(amplitude), int(samples_per_symbol)

    def _desc(self):
        d = super()._desc()
        d.samples_per_symbol = self._sps
        return d


class DMPSK(_SamplePhasor):
    """dmpsk.rs:7-43: DMPSK::new(bits_per_symbol, amplitude, phase, shift); the phase is carried
    in f32 from symbol to symbol (a serial scan on the device)."""
    _kind = 9

    def __init__(self, bits_per_symbol: int, amplitude: float, phase: float, shift: float):
        self._bps, self.amplitude, self._phase, self._shift = int(bits_per_symbol), float(amplitude), \
            float(phase), float(shift)

    def _desc(self):
        d = super()._desc()
        d.shift = self._shift
        return d


class MFSK(_SamplePhasor):
    """mfsk.rs:37-85: MFSK::new(bits_per_symbol, deviation: Freq, amplitude, map);
    map "increase" (IncreaseMap, 2s) or "default" (DefaultMap, 2s - max_symbol)."""
    _kind = 12

    def __init__(self, bits_per_symbol: int, deviation: "Freq", amplitude: float, map: str = "default"):
        self._bps, self.amplitude = int(bits_per_symbol), float(amplitude)
        self._freq, self._map = deviation.sample_freq(), 1 if map == "increase" else 0

    def _desc(self):
        d = super()._desc()
        d.freq, d.mfsk_map = self._freq, self._map
        return d


class BFSK(_SamplePhasor):
    """bfsk.rs:4-56: BFSK::new(deviation: Freq, amplitude)."""
    _kind = 13

    def __init__(self, deviation: "Freq", amplitude: float):
        self.amplitude, self._freq = float(amplitude), deviation.sample_freq()

    def _desc(self):
        d = super()._desc()
        d.freq = self._freq
        return d


def rrc_taps(ntaps: int, sps: int, beta: float = 0.35) -> np.ndarray:
    """Root-raised-cosine taps (GLUE: absent from the reference), unit energy."""
    out = np.zeros(int(ntaps), dtype=np.float32)
    _check(load_library().modem_rrc_taps(int(ntaps), int(sps), float(beta), _fptr(out)), "rrc_taps")
    return out


# ------------------------------------------------------------- buffers / streams ----
def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch")


_TORCH = None


def _torch_cuda():
    """torch when it has a GPU, else False (looked up once: is_available() costs ~1 us)."""
    global _TORCH
    if _TORCH is None:
        try:
            import torch
            _TORCH = torch if torch.cuda.is_available() else False
        except ImportError:
            _TORCH = False
    return _TORCH


def _stream_handle(stream, device: Optional[int] = None) -> Optional[int]:
    """The raw HIP stream a call is queued on: `stream` (a torch Stream or a raw handle), else
    torch's current stream of `device` (the handle's GPU; None: the current device), so that
    a handle on another GPU never launches on this device's stream."""
    if stream is not None:
        sdev = getattr(stream, "device_index", None)
        if device is not None and sdev is not None and int(sdev) != int(device):
            raise ValueError(f"stream of cuda:{sdev} given to a handle on cuda:{device}")
        return int(getattr(stream, "cuda_stream", stream))
    t = _torch_cuda()
    if t:
        # the current stream's raw handle (current_stream() builds a Stream object: ~3 us)
        return t._C._cuda_getCurrentRawStream(t._C._cuda_getDevice() if device is None else int(device))
    return None


def _ptr(x) -> int:
    if x is None:
        return 0
    if _is_torch(x):
        if not x.is_contiguous():
            raise ValueError("tensor must be contiguous")
        return int(x.data_ptr())
    if not x.flags["C_CONTIGUOUS"]:
        raise ValueError("array must be C-contiguous")
    return int(x.ctypes.data)


def _empty_like_input(ref, shape, np_dtype):
    """Allocate an output on the same side (device tensor / host ndarray) as `ref`."""
    if _is_torch(ref):
        import torch
        tdt = {np.float32: torch.float32, np.float16: torch.float16, np.uint8: torch.uint8}[np_dtype]
        return torch.empty(shape, dtype=tdt, device=ref.device)
    return np.empty(shape, dtype=np_dtype)


def _device_of(x, default: int) -> int:
    if _is_torch(x) and x.is_cuda:
        return int(x.device.index or 0)
    return default


# ------------------------------------------------------------------- TX (B3+B5) ----
class DigitalModulator:
    """DigitalModulator (modulator.rs:64-101) + pulse shaping + IQSample::modulate.

    `process(bits)` takes one byte per bit (values 0/1, data.rs:36) — a CUDA uint8 tensor
    (asynchronous, on the current stream) or a numpy array — and returns the samples of
    every complete symbol: (n, 2) interleaved (i, q) for the IQ modes, (n,) for OUT_REAL.
    `taps=None` keeps the reference's sample-and-hold (bit-compatible with `modulate --iq`).
    `carrier.sample` advances by the samples produced, as the shared `&mut Carrier` does.
    `even_odd_offset=True` is the `EvenOddOffset` source (data.rs:81-123) that `modulate`
    puts under OQPSK (modulate.rs:101-107): Q changes half a symbol after I; it panics
    (ModemPanic) unless the phasor has 2 bits per symbol and samples_per_symbol is even.
    """

    def __init__(self, carrier: Carrier, phasor: _Phasor, samples_per_symbol: int,
                 taps: Optional[np.ndarray] = None, dtype: int = DTYPE_F32,
                 out_mode: int = OUT_IQ_MIXED, device: int = 0, even_odd_offset: bool = False):
        L = load_library()
        self.carrier, self.phasor = carrier, phasor
        self.sps, self.dtype, self.out_mode, self.device = int(samples_per_symbol), dtype, out_mode, device
        self.bps = phasor.bits_per_symbol()
        sample_dep = getattr(phasor, "sample_dependent", False)
        self._lut = None if sample_dep else phasor.lut()
        self.taps = None if taps is None else np.ascontiguousarray(taps, dtype=np.float32)
        d = _TxDesc()
        d.bits_per_symbol = self.bps
        d.lut = _fptr(self._lut) if self._lut is not None else None
        if sample_dep:
            self._pdesc = phasor._desc()
            d.phasor = ctypes.pointer(self._pdesc)
        d.samples_per_symbol = self.sps
        d.taps = _fptr(self.taps) if self.taps is not None else None
        d.ntaps = 0 if self.taps is None else len(self.taps)
        d.sample_freq = carrier.sample_freq
        d.s0 = carrier.sample
        d.dtype, d.out_mode = dtype, out_mode
        d.q_offset = self._q_offset = self.sps // 2 if even_odd_offset else 0
        if even_odd_offset and (self.bps != 2 or self.sps % 2):
            raise ModemPanic(-1, "EvenOddOffset: bits_per_symbol == 2 and an even samples_per_symbol")
        h = ctypes.c_void_p()
        _check(L.modem_tx_create(ctypes.byref(d), device, ctypes.byref(h)), "DigitalModulator")
        self._h = h
        self._ncarry = 0

    def _alloc(self, ref, nsamp: int):
        npd = np.float16 if self.dtype == DTYPE_F16 else np.float32
        shape = (nsamp,) if self.out_mode == OUT_REAL else (nsamp, 2)
        return _empty_like_input(ref, shape, npd)

    def nsamples(self, nbits: int) -> int:
        return ((self._ncarry + nbits) // self.bps) * self.sps

    def process(self, bits, out=None, stream=None):
        n = int(bits.numel() if _is_torch(bits) else bits.size)
        ns = self.nsamples(n)
        if out is None:
            out = self._alloc(bits, ns)
        cap = int(out.shape[0])
        prod = ctypes.c_size_t()
        _check(load_library().modem_tx_process(self._h, _ptr(bits), n, _ptr(out), cap,
                                               ctypes.byref(prod), _stream_handle(stream, self.device)),
               "DigitalModulator.process")
        self._ncarry = (self._ncarry + n) % self.bps
        self.carrier.sample += prod.value        # = modem_tx_sample(h): one sample per output
        return out if prod.value == cap else out[: prod.value]

    @staticmethod
    def process_batch(mods, bits, outs=None, stream=None):
        """`m.process(b)` for every (modulator, bits) pair in order, as one call
        (modem_tx_process_batch): independent channels of one configuration with device
        buffers share one kernel launch per 8 channels. Returns the outputs, as process does."""
        mods, bits = list(mods), list(bits)
        if len(mods) != len(bits) or len(set(map(id, mods))) != len(mods):
            raise ValueError("one bits buffer per distinct modulator")
        n = len(mods)
        nb = [int(b.numel() if _is_torch(b) else b.size) for b in bits]
        if outs is None:
            outs = [m._alloc(b, m.nsamples(k)) for m, b, k in zip(mods, bits, nb)]
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        hs = (vp * n)(*[m._h.value for m in mods])
        prod = (sz * n)()
        _check(load_library().modem_tx_process_batch(
            hs, n, (vp * n)(*[_ptr(b) for b in bits]), (sz * n)(*nb), (vp * n)(*[_ptr(o) for o in outs]),
            (sz * n)(*[int(o.shape[0]) for o in outs]), prod, _stream_handle(stream, mods[0].device)),
            "DigitalModulator.process_batch")
        for m, k in zip(mods, nb):
            m._ncarry = (m._ncarry + k) % m.bps
            m.carrier.sample = int(load_library().modem_tx_sample(m._h))
        return [o[: prod[i]] for i, o in enumerate(outs)]

    def flush(self, like=None, stream=None):
        ntaps = 0 if self.taps is None else len(self.taps)
        tail = ntaps - 1 + self._q_offset if ntaps else 0     # the delayed Q rail drains later
        ns = ((tail + self.sps - 1) // self.sps) * self.sps
        ref = like if like is not None else np.zeros(1, np.uint8)
        out = self._alloc(ref, ns)
        prod = ctypes.c_size_t()
        _check(load_library().modem_tx_flush(self._h, _ptr(out), int(out.shape[0]), ctypes.byref(prod),
                                             _stream_handle(stream, self.device)), "DigitalModulator.flush")
        self.carrier.sample = int(load_library().modem_tx_sample(self._h))
        return out[: prod.value]

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.modem_tx_destroy(self._h)
            self._h = None


class TxBatchPlan:
    """A prepared `DigitalModulator.process_batch` over fixed buffers: bits[c] -> outs[c] for
    every channel, the ctypes argument arrays built once, so that each `run()` is one C call
    (modem_tx_process_batch) plus the per-channel bookkeeping. For a channel bank that streams
    through the same device buffers every period."""

    def __init__(self, mods, bits, outs):
        self.mods, self.bits, self.outs = list(mods), list(bits), list(outs)
        n = self.n = len(self.mods)
        if len(self.bits) != n or len(self.outs) != n or len(set(map(id, self.mods))) != n:
            raise ValueError("one bits and one output buffer per distinct modulator")
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        self._nb = [int(b.numel() if _is_torch(b) else b.size) for b in self.bits]
        self._hs = (vp * n)(*[m._h.value for m in self.mods])
        self._bits = (vp * n)(*[_ptr(b) for b in self.bits])
        self._nbits = (sz * n)(*self._nb)
        self._outs = (vp * n)(*[_ptr(o) for o in self.outs])
        self._caps = (sz * n)(*[int(o.shape[0]) for o in self.outs])
        self._prod = (sz * n)()
        self._fn = load_library().modem_tx_process_batch

    def run(self, stream=None):
        """Returns the samples produced per channel (written to outs[c][:produced[c]])."""
        _check(self._fn(self._hs, self.n, self._bits, self._nbits, self._outs, self._caps, self._prod,
                        _stream_handle(stream, self.mods[0].device)), "TxBatchPlan.run")
        L = load_library()
        for m, k in zip(self.mods, self._nb):
            m._ncarry = (m._ncarry + k) % m.bps
            m.carrier.sample = int(L.modem_tx_sample(m._h))
        return list(self._prod)


# ------------------------------------------------------------------- RX (B6+B5) ----
_IN_DTYPE_NAME = {DTYPE_F32: "float32", DTYPE_F16: "float16", DTYPE_I16: "int16"}


def _dtype_name(x) -> str:
    return str(getattr(x, "dtype", "")).replace("torch.", "")


def _check_rx_input(x, in_dtype: int, what: str) -> int:
    """The input must be what the handle was created for — (n, 2) float32 / float16 (i, q) or
    (n,) int16 real samples — else the C side would read n samples of the wrong width.
    Returns n."""
    want = _IN_DTYPE_NAME.get(in_dtype)
    got = _dtype_name(x)
    shape = tuple(int(d) for d in x.shape)
    ok_shape = len(shape) == 1 if in_dtype == DTYPE_I16 else (len(shape) == 2 and shape[1] == 2)
    if got != want or not ok_shape:
        form = "(n,) int16" if in_dtype == DTYPE_I16 else f"(n, 2) {want}"
        raise ValueError(f"{what}: input must be {form} (the handle's in_dtype), got {shape} {got}")
    return shape[0]


class DemodulatorRx:
    """Demodulator (demodulator.rs:7-56) + matched filter + decimation + slicer.

    mix=MIX_REFERENCE_REAL, decim=1 is the reference Demodulator exactly (real input
    x.re, (2*FIR(x cos), 2*FIR(-x sin)) at every sample, PLL offset 0). The loopback
    contract uses MIX_COMPLEX with decim = samples/symbol and decim_offset = ntaps-1.
    """

    def __init__(self, carrier: Carrier, taps: np.ndarray, decim: int = 1, decim_offset: int = 0,
                 mix: int = MIX_REFERENCE_REAL, slicer: Optional[_SlicerDesc] = None,
                 in_dtype: int = DTYPE_F32, out_dtype: int = DTYPE_F32, device: int = 0,
                 phase_offset: float = 0.0):
        L = load_library()
        self.carrier, self.decim, self.out_dtype, self.in_dtype = carrier, int(decim), out_dtype, in_dtype
        self.device = device
        self.taps = np.ascontiguousarray(taps, dtype=np.float32)
        self.decim_offset = int(decim_offset)
        d = _RxDesc()
        d.sample_freq = carrier.sample_freq
        d.s0 = carrier.sample
        d.taps = _fptr(self.taps)
        d.ntaps = len(self.taps)
        d.decim, d.decim_offset, d.mix = self.decim, self.decim_offset, mix
        d.in_dtype, d.out_dtype = in_dtype, out_dtype
        d.phase_offset = float(phase_offset)
        if slicer is not None:
            d.slicer = slicer
        else:
            d.slicer.kind = SLICER_NONE
        self._slicer = slicer
        h = ctypes.c_void_p()
        _check(L.modem_rx_create(ctypes.byref(d), device, ctypes.byref(h)), "Demodulator")
        self._h = h
        self._consumed = 0

    def noutputs(self, n: int) -> int:
        def first(x):
            return 0 if x <= self.decim_offset else (x - self.decim_offset + self.decim - 1) // self.decim
        a, b = first(self._consumed), first(self._consumed + n)
        return max(0, b - a)

    def process(self, iq, want_iq: bool = True, want_sym: bool = True, stream=None,
                out_iq=None, out_sym=None):
        n = _check_rx_input(iq, self.in_dtype, "Demodulator.process")
        nout = self.noutputs(n)
        npd = np.float16 if self.out_dtype == DTYPE_F16 else np.float32
        oiq = out_iq if out_iq is not None else (_empty_like_input(iq, (nout, 2), npd) if want_iq else None)
        osym = out_sym if out_sym is not None else (
            _empty_like_input(iq, (nout,), np.uint8) if (want_sym and self._slicer is not None) else None)
        cap = min(int(oiq.shape[0]) if oiq is not None else nout, int(osym.shape[0]) if osym is not None else nout)
        prod = ctypes.c_size_t()
        _check(load_library().modem_rx_process(self._h, _ptr(iq), n, _ptr(oiq), _ptr(osym), cap,
                                               ctypes.byref(prod), _stream_handle(stream, self.device)),
               "Demodulator.process")
        self._consumed += n
        self.carrier.sample += n                 # = modem_rx_sample(h): one per input sample
        k = prod.value
        return (None if oiq is None else (oiq if int(oiq.shape[0]) == k else oiq[:k])), \
               (None if osym is None else (osym if int(osym.shape[0]) == k else osym[:k]))

    @staticmethod
    def process_batch(rxs, iqs, out_iq=None, out_sym=None, stream=None):
        """`r.process(x)` for every (demodulator, input) pair in order, as one call
        (modem_rx_process_batch): channels of one configuration with device buffers share one
        kernel launch per 8 channels. Returns [(iq, sym), ...] as process does."""
        rxs, iqs = list(rxs), list(iqs)
        if len(rxs) != len(iqs) or len(set(map(id, rxs))) != len(rxs):
            raise ValueError("one input buffer per distinct demodulator")
        n = len(rxs)
        ns = [_check_rx_input(x, r.in_dtype, "Demodulator.process_batch") for r, x in zip(rxs, iqs)]
        nouts = [r.noutputs(k) for r, k in zip(rxs, ns)]
        if out_iq is None:
            out_iq = [_empty_like_input(x, (k, 2), np.float16 if r.out_dtype == DTYPE_F16 else np.float32)
                      for r, x, k in zip(rxs, iqs, nouts)]
        if out_sym is None:
            out_sym = [_empty_like_input(x, (k,), np.uint8) if r._slicer is not None else None
                       for r, x, k in zip(rxs, iqs, nouts)]
        caps = [min(int(a.shape[0]) if a is not None else k, int(b.shape[0]) if b is not None else k)
                for a, b, k in zip(out_iq, out_sym, nouts)]
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        prod = (sz * n)()
        _check(load_library().modem_rx_process_batch(
            (vp * n)(*[r._h.value for r in rxs]), n, (vp * n)(*[_ptr(x) for x in iqs]), (sz * n)(*ns),
            (vp * n)(*[_ptr(a) or None for a in out_iq]), (vp * n)(*[_ptr(b) or None for b in out_sym]),
            (sz * n)(*caps), prod, _stream_handle(stream, rxs[0].device)), "Demodulator.process_batch")
        res = []
        for i, (r, k) in enumerate(zip(rxs, ns)):
            r._consumed += k
            r.carrier.sample = int(load_library().modem_rx_sample(r._h))
            a, b = out_iq[i], out_sym[i]
            res.append((None if a is None else a[: prod[i]], None if b is None else b[: prod[i]]))
        return res

    def flush(self, like=None, stream=None):
        n = len(self.taps) - 1
        nout = self.noutputs(n)
        ref = like if like is not None else np.zeros(1, np.float32)
        npd = np.float16 if self.out_dtype == DTYPE_F16 else np.float32
        oiq = _empty_like_input(ref, (nout, 2), npd)
        osym = _empty_like_input(ref, (nout,), np.uint8) if self._slicer is not None else None
        prod = ctypes.c_size_t()
        _check(load_library().modem_rx_flush(self._h, _ptr(oiq), _ptr(osym), nout, ctypes.byref(prod),
                                             _stream_handle(stream, self.device)), "Demodulator.flush")
        self._consumed += n
        self.carrier.sample = int(load_library().modem_rx_sample(self._h))
        return oiq[: prod.value], (None if osym is None else osym[: prod.value])

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.modem_rx_destroy(self._h)
            self._h = None


# --------------------------------------------------------------------- FIR (B5) ----
LOCK_SAMPLES = 64   # demodulator.rs:5


class Demodulator:
    """Demodulator (demodulator.rs:7-56) with its PLL lock, as the `demodulate` binary drives it
    (demodulate.rs:29-43): `lock_phase(sig)` runs PLL::handle (pll.rs:16-22) over the first 64
    complex samples (host, modem_pll_lock: 64 serial steps of control logic), then `process`
    gives (2*FIR(x.re*cos), 2*FIR(-x.re*sin)) at every further sample on the GPU with the locked
    offset (`phase = carrier.next() + pll.phase_offset`, demodulator.rs:50) — by default with
    MIX_REFERENCE_REAL_EXACT, bit-identical to the reference (exact=False: the fast real mix,
    within 1e-5). `sig`: (n, 2) float32 (re, im) — a CUDA tensor or a numpy array — or, for
    `process`, (n,) int16 real samples."""

    def __init__(self, carrier: Carrier, lowpass: np.ndarray, device: int = 0, exact: bool = True):
        self.carrier, self.lowpass, self.device = carrier, np.ascontiguousarray(lowpass, np.float32), device
        self.exact = exact
        self.phase_offset = 0.0
        self._rx = None

    def lock_phase(self, sig):
        """Consume the first 64 samples of `sig` (demodulator.rs:32-36); returns the rest."""
        head = sig[:LOCK_SAMPLES]
        if int(head.shape[0]) < LOCK_SAMPLES:
            raise ModemPanic(ERR_INVALID_ARG, "lock_phase: called `Option::unwrap()` on a `None` value")
        h = np.ascontiguousarray(head.detach().cpu().numpy() if _is_torch(head) else head, np.float32)
        off = (ctypes.c_float * 1)(self.phase_offset)
        _check(load_library().modem_pll_lock(self.carrier.sample_freq, self.carrier.sample, _fptr(h),
                                             LOCK_SAMPLES, off), "Demodulator.lock_phase")
        self.phase_offset = float(off[0])
        self.carrier.sample += LOCK_SAMPLES
        return sig[LOCK_SAMPLES:]

    def process(self, sig, stream=None):
        """(n, 2) float32 (i, q), one per input sample (Iterator::next, demodulator.rs:44-56)."""
        if self._rx is None:
            i16 = _dtype_name(sig) == "int16"
            if i16 and not self.exact:
                raise ValueError("Demodulator.process: int16 input needs exact=True "
                                 "(MIX_REFERENCE_REAL_EXACT reads i16 samples; the fast real mix does not)")
            self._rx = DemodulatorRx(self.carrier, self.lowpass, decim=1, decim_offset=0,
                                     mix=MIX_REFERENCE_REAL_EXACT if self.exact else MIX_REFERENCE_REAL,
                                     in_dtype=DTYPE_I16 if i16 else DTYPE_F32, device=self.device,
                                     phase_offset=self.phase_offset)
        iq, _ = self._rx.process(sig, want_sym=False, stream=stream)
        return iq


class FIRFilter:
    """FIRFilter (fir.rs:3-35): causal FIR, zero initial history, one output per input."""

    def __init__(self, coefs, device: int = 0):
        self.device = device
        self.coefs = np.ascontiguousarray(coefs, dtype=np.float32)
        if len(self.coefs) == 0:
            raise ModemPanic(ERR_INVALID_ARG, "FIRFilter: attempt to calculate the remainder with a divisor of zero")
        h = ctypes.c_void_p()
        _check(load_library().modem_fir_create(_fptr(self.coefs), len(self.coefs), device, ctypes.byref(h)),
               "FIRFilter")
        self._h = h

    def process(self, x, stream=None):
        n = int(x.shape[0])
        y = _empty_like_input(x, (n,), np.float32)
        _check(load_library().modem_fir_process(self._h, _ptr(x), _ptr(y), n, _stream_handle(stream, self.device)),
               "FIRFilter.process")
        return y

    def add(self, sample: float) -> float:
        return float(self.process(np.array([sample], dtype=np.float32))[0])

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.modem_fir_destroy(self._h)
            self._h = None


class RxBatchPlan:
    """A prepared `DemodulatorRx.process_batch` over fixed buffers (iqs[c] -> out_iq[c],
    out_sym[c]; either output may be None): each `run()` is one modem_rx_process_batch call."""

    def __init__(self, rxs, iqs, out_iq, out_sym):
        self.rxs, self.iqs = list(rxs), list(iqs)
        n = self.n = len(self.rxs)
        out_iq, out_sym = list(out_iq), list(out_sym)
        if len(self.iqs) != n or len(out_iq) != n or len(out_sym) != n or len(set(map(id, self.rxs))) != n:
            raise ValueError("one input and one output set per distinct demodulator")
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        self._ns = [_check_rx_input(x, r.in_dtype, "RxBatchPlan") for r, x in zip(self.rxs, self.iqs)]
        caps = [min(int(a.shape[0]) if a is not None else 1 << 62, int(b.shape[0]) if b is not None else 1 << 62)
                for a, b in zip(out_iq, out_sym)]
        self._hs = (vp * n)(*[r._h.value for r in self.rxs])
        self._ins = (vp * n)(*[_ptr(x) for x in self.iqs])
        self._nsa = (sz * n)(*self._ns)
        self._oiq = (vp * n)(*[_ptr(a) or None for a in out_iq])
        self._osym = (vp * n)(*[_ptr(b) or None for b in out_sym])
        self._caps = (sz * n)(*caps)
        self._prod = (sz * n)()
        self._fn = load_library().modem_rx_process_batch

    def run(self, stream=None):
        """Returns the kept instants produced per channel."""
        _check(self._fn(self._hs, self.n, self._ins, self._nsa, self._oiq, self._osym, self._caps, self._prod,
                        _stream_handle(stream, self.rxs[0].device)), "RxBatchPlan.run")
        L = load_library()
        for r, k in zip(self.rxs, self._ns):
            r._consumed += k
            r.carrier.sample = int(L.modem_rx_sample(r._h))
        return list(self._prod)


class ChainPlan:
    """One period of the sample-buffer loop as one C call (modem_chain_*): `run()` equals
    `tx.process(bits, out=samples)` followed by `rx.process(samples, out_iq=out_iq,
    out_sym=out_sym)` — the DigitalModulator's samples of the bit buffer (modulator.rs:85-100),
    then the Demodulator over them (demodulator.rs:44-56) — with the device buffers checked once
    here instead of on every call. Both handles' Python-side state (carried bits, carrier
    sample, consumed samples) advances as those calls would advance it."""

    def __init__(self, tx: "DigitalModulator", rx: "DemodulatorRx", bits, samples, out_iq=None, out_sym=None):
        self.tx, self.rx = tx, rx
        self.bits, self.samples, self.out_iq, self.out_sym = bits, samples, out_iq, out_sym
        if tx.dtype != rx.in_dtype or tx.out_mode == OUT_REAL:
            raise ValueError("ChainPlan: the RX must read the TX's interleaved samples (one dtype)")
        # the C side sizes every buffer from its first dimension: a buffer of the wrong width
        # would be written past its end on the device
        _check_rx_input(samples, tx.dtype, "ChainPlan samples")
        want_out = _IN_DTYPE_NAME[rx.out_dtype]
        if out_iq is not None and (len(out_iq.shape) != 2 or int(out_iq.shape[1]) != 2
                                   or _dtype_name(out_iq) != want_out):
            raise ValueError(f"ChainPlan: out_iq must be (k, 2) {want_out} (the RX's out_dtype), "
                             f"got {tuple(out_iq.shape)} {_dtype_name(out_iq)}")
        if out_sym is not None and (len(out_sym.shape) != 1 or _dtype_name(out_sym) != "uint8"):
            raise ValueError(f"ChainPlan: out_sym must be (k,) uint8, got {tuple(out_sym.shape)} {_dtype_name(out_sym)}")
        self._nbits = int(bits.numel() if _is_torch(bits) else bits.size)
        caps = [int(x.shape[0]) for x in (out_iq, out_sym) if x is not None]
        h = ctypes.c_void_p()
        _check(load_library().modem_chain_create(tx._h, rx._h, _ptr(bits), self._nbits, _ptr(samples),
                                                 int(samples.shape[0]), _ptr(out_iq) or None, _ptr(out_sym) or None,
                                                 min(caps) if caps else 1 << 62, ctypes.byref(h)), "ChainPlan")
        self._h = h
        self._n, self._k = ctypes.c_size_t(), ctypes.c_size_t()
        self._pn, self._pk = ctypes.byref(self._n), ctypes.byref(self._k)
        self._fn = load_library().modem_chain_run

    def run(self, stream=None):
        """Returns (samples produced, kept instants produced)."""
        _check(self._fn(self._h, self._pn, self._pk, _stream_handle(stream, self.tx.device)), "ChainPlan.run")
        n = self._n.value
        tx, rx = self.tx, self.rx
        tx._ncarry = (tx._ncarry + self._nbits) % tx.bps
        tx.carrier.sample += n
        rx._consumed += n
        rx.carrier.sample += n
        return n, self._k.value

    @property
    def fused(self) -> int:
        """1 or 2: the last run() was one launch (TX and RX of the period fused; 2: with the
        samples handed over in LDS), 0: two launches, -1: no run yet."""
        return int(load_library().modem_chain_fused(self._h))

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.modem_chain_destroy(self._h)
            self._h = None


class ChainBatchPlan:
    """One period of a bank of independent channels as one C call (modem_chain_batch_*): `run()`
    equals `ChainPlan(tx[i], rx[i], bits[i], samples[i], out_iq[i], out_sym[i]).run()` for every
    channel i (the DigitalModulator's samples of each channel's bits, modulator.rs:85-100, then
    that channel's Demodulator over them, demodulator.rs:44-56), run as one TX launch and then one
    RX launch per `group` consecutive channels, with the handles and buffers checked once here.
    Every handle's Python-side state advances as those calls would advance it. Raises ModemError
    (MODEM_ERR_UNSUPPORTED) when the handles do not share one matrix-core configuration per side."""

    def __init__(self, txs, rxs, bits, samples, out_iq, out_sym, group: int = 8):
        self.txs, self.rxs = list(txs), list(rxs)
        self.bits, self.samples, self.out_iq, self.out_sym = list(bits), list(samples), list(out_iq), list(out_sym)
        n = self.n = len(self.txs)
        if not (len(self.rxs) == len(self.bits) == len(self.samples) == len(self.out_iq) == len(self.out_sym) == n):
            raise ValueError("ChainBatchPlan: one modulator, demodulator and buffer set per channel")
        for tx, rx, y, oiq, osym in zip(self.txs, self.rxs, self.samples, self.out_iq, self.out_sym):
            if tx.dtype != rx.in_dtype or tx.out_mode == OUT_REAL:
                raise ValueError("ChainBatchPlan: each RX must read its TX's interleaved samples (one dtype)")
            _check_rx_input(y, tx.dtype, "ChainBatchPlan samples")
            want_out = _IN_DTYPE_NAME[rx.out_dtype]
            if len(oiq.shape) != 2 or int(oiq.shape[1]) != 2 or _dtype_name(oiq) != want_out:
                raise ValueError(f"ChainBatchPlan: out_iq must be (k, 2) {want_out}, got {tuple(oiq.shape)} {_dtype_name(oiq)}")
            if len(osym.shape) != 1 or _dtype_name(osym) != "uint8":
                raise ValueError(f"ChainBatchPlan: out_sym must be (k,) uint8, got {tuple(osym.shape)} {_dtype_name(osym)}")
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        self._nb = [int(b.numel() if _is_torch(b) else b.size) for b in self.bits]
        txh = (vp * n)(*[t._h.value for t in self.txs])
        rxh = (vp * n)(*[r._h.value for r in self.rxs])
        outc = (sz * n)(*[min(int(a.shape[0]), int(b.shape[0])) for a, b in zip(self.out_iq, self.out_sym)])
        h = ctypes.c_void_p()
        _check(load_library().modem_chain_batch_create(
            txh, rxh, n, int(group), (vp * n)(*[_ptr(b) for b in self.bits]), (sz * n)(*self._nb),
            (vp * n)(*[_ptr(y) for y in self.samples]), (sz * n)(*[int(y.shape[0]) for y in self.samples]),
            (vp * n)(*[_ptr(x) for x in self.out_iq]), (vp * n)(*[_ptr(x) for x in self.out_sym]), outc,
            ctypes.byref(h)), "ChainBatchPlan")
        self._h = h
        self._prod, self._kout = (sz * n)(), (sz * n)()
        self._fn = load_library().modem_chain_batch_run

    def run(self, stream=None):
        """Returns (samples produced, kept instants produced) per channel. A launch error part-way
        through a run (ModemError, HIP) leaves some groups' handles advanced: the plan is then
        failed in the library and every later run raises too."""
        _check(self._fn(self._h, self._prod, self._kout, _stream_handle(stream, self.txs[0].device)),
               "ChainBatchPlan.run")
        for tx, rx, k, n in zip(self.txs, self.rxs, self._nb, self._prod):
            tx._ncarry = (tx._ncarry + k) % tx.bps
            tx.carrier.sample += n
            rx._consumed += n
            rx.carrier.sample += n
        return list(self._prod), list(self._kout)

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.modem_chain_batch_destroy(self._h)
            self._h = None


def prng_bits(seed: int, nbits: int, device: int = 0, stream=None):
    """Synthetic bit stream (GLUE): splitmix64, one byte per bit, on the device."""
    import torch
    out = torch.empty(int(nbits), dtype=torch.uint8, device=f"cuda:{device}")
    _check(load_library().modem_prng_bits(int(seed), out.data_ptr() if nbits else None, int(nbits), device,
                                          _stream_handle(stream, device)), "prng_bits")
    return out
