"""oracle/oracle.py — TEST INFRASTRUCTURE ONLY.

ctypes wrapper around oracle/_build/libmodem_oracle.so, the plain-C restatement of
ramtej/rust-modem `src/modem` (see modem_oracle.h for what each function restates and how the
restatement is pinned). Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
import this module, and only as the checker / the timed CPU baseline — never as the product.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import List, Optional, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libmodem_oracle.so")

CHANGED, UNCHANGED, FINISHED = 0, 1, 2
BPSK, QPSK, QAM, BASK, MPSK, APSK, OQPSK, DCQPSK, DMPSK, CPFSK, MSK, MFSK, BFSK = range(1, 14)
SLICER_NEAREST, SLICER_QAM_AXIS = 0, 1
MIX_COMPLEX, MIX_REFERENCE_REAL = 0, 1
OUT_IQ_MIXED, OUT_IQ_BASEBAND, OUT_REAL = 0, 1, 2


class Ring(ctypes.Structure):
    _fields_ = [("start", ctypes.c_uint8), ("end", ctypes.c_uint8),
                ("radius", ctypes.c_float), ("phase", ctypes.c_float)]


class Phasor(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int), ("bits_per_symbol", ctypes.c_size_t),
                ("bits_per_carrier", ctypes.c_size_t), ("amplitude", ctypes.c_float),
                ("phase", ctypes.c_float), ("phase_cos", ctypes.c_float), ("phase_sin", ctypes.c_float),
                ("max_symbol", ctypes.c_float), ("num_symbols", ctypes.c_float), ("shift", ctypes.c_float),
                ("even", ctypes.c_int), ("nrings", ctypes.c_int), ("rings", Ring * 8),
                ("freq", ctypes.c_float), ("samples_per_bit", ctypes.c_size_t),
                ("cur_coef", ctypes.c_float), ("increase_map", ctypes.c_int), ("prev", ctypes.c_uint8)]


class SymbolClock(ctypes.Structure):
    _fields_ = [("samples_per_symbol", ctypes.c_size_t), ("counter", ctypes.c_size_t)]


class BitsSource(ctypes.Structure):
    _fields_ = [("bits", ctypes.c_void_p), ("nbits", ctypes.c_size_t), ("clock", SymbolClock),
                ("bits_per_symbol", ctypes.c_size_t), ("idx", ctypes.c_size_t)]


class AsciiBits(ctypes.Structure):
    _fields_ = [("text", ctypes.c_void_p), ("len", ctypes.c_size_t), ("pos", ctypes.c_size_t),
                ("clock", SymbolClock), ("bits", ctypes.c_uint8 * 8), ("nbits", ctypes.c_size_t),
                ("panicked", ctypes.c_int)]


class Source(ctypes.Structure):
    _fields_ = [("is_ascii", ctypes.c_int), ("bits", BitsSource), ("ascii", AsciiBits)]


class EvenOdd(ctypes.Structure):
    _fields_ = [("data", Source), ("clock", SymbolClock), ("cur", ctypes.c_uint8 * 2)]


class Slicer(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int), ("bps", ctypes.c_size_t), ("lut", ctypes.POINTER(ctypes.c_float)),
                ("bits_per_carrier", ctypes.c_int), ("inv_scale", ctypes.c_float),
                ("max_symbol", ctypes.c_float)]


class IQSample(ctypes.Structure):
    _fields_ = [("carrier", ctypes.c_float), ("i", ctypes.c_float), ("q", ctypes.c_float)]


def build() -> str:
    """Compile the oracle (gcc, -ffp-contract=off) into oracle/_build/."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


_L = None


def lib():
    global _L
    if _L is not None:
        return _L
    if not os.path.exists(LIB):
        build()
    L = ctypes.CDLL(LIB)
    c = ctypes
    f, sz, u8, u64, i, vp = c.c_float, c.c_size_t, c.c_uint8, c.c_uint64, c.c_int, c.c_void_p
    fp = c.POINTER(c.c_float)
    P = c.POINTER
    sig = {
        "or_mod_trig": (f, [f]), "or_bit_to_sign": (f, [u8]), "or_bytes_to_bits": (u8, [vp, sz]),
        "or_max_symbol": (sz, [sz]), "or_freq_ang_freq": (f, [sz]), "or_freq_sample_freq": (f, [sz, sz]),
        "or_rates_samples_per_symbol": (sz, [sz, sz]),
        "or_carrier_phases": (None, [f, u64, sz, fp]),
        "or_symbol_clock_init": (None, [P(SymbolClock), sz]), "or_symbol_clock_next": (i, [P(SymbolClock)]),
        "or_bits_init": (None, [P(BitsSource), vp, sz, sz, sz]),
        "or_bits_next": (i, [P(BitsSource), P(c.c_void_p)]),
        "or_ascii_init": (None, [P(AsciiBits), vp, sz, sz, sz]),
        "or_ascii_read_bits": (i, [P(AsciiBits)]), "or_ascii_next": (i, [P(AsciiBits), P(c.c_void_p)]),
        "or_even_odd_init": (i, [P(EvenOdd), P(Source), sz, sz]),
        "or_even_odd_next": (i, [P(EvenOdd), P(c.c_void_p)]),
        "or_bpsk_new": (i, [P(Phasor), f, f]), "or_qpsk_new": (i, [P(Phasor), f, f]),
        "or_qam_new": (i, [P(Phasor), sz, f, f]), "or_bask_new": (i, [P(Phasor), f]),
        "or_mpsk_new": (i, [P(Phasor), sz, f, f]), "or_apsk_new": (i, [P(Phasor), f, sz, P(Ring), i]),
        "or_oqpsk_new": (i, [P(Phasor), f]), "or_dcqpsk_new": (i, [P(Phasor), f]),
        "or_dmpsk_new": (i, [P(Phasor), sz, f, f, f]),
        "or_cpfsk_new": (i, [P(Phasor), sz, sz, sz, f, sz]), "or_msk_new": (i, [P(Phasor), f, sz]),
        "or_mfsk_new": (i, [P(Phasor), sz, f, f, i]), "or_bfsk_new": (i, [P(Phasor), f, f]),
        "or_phasor_update": (None, [P(Phasor), u64, vp, sz]),
        "or_phasor_i": (f, [P(Phasor), u64, vp, sz]), "or_phasor_q": (f, [P(Phasor), u64, vp, sz]),
        "or_fir_block": (None, [fp, sz, fp, sz, fp]),
        "or_iq_modulate": (None, [P(IQSample), fp, fp]),
        "or_demodulate": (None, [f, u64, f, fp, sz, fp, sz, fp, fp]),
        "or_pll_handle": (None, [vp, f, f, f]),
        "or_prng_bits": (None, [u64, vp, sz]), "or_rrc_taps": (i, [sz, sz, c.c_double, fp]),
        "or_phasor_lut": (i, [P(Phasor), fp]), "or_slice": (u8, [P(Slicer), f, f]),
        "or_tx_chain": (sz, [P(Phasor), vp, sz, sz, fp, sz, f, u64, sz, i, fp]),
        "or_tx_chain_src": (sz, [P(Phasor), vp, sz, sz, fp, sz, f, u64, sz, i, i, fp]),
        "or_rx_chain": (sz, [fp, sz, f, u64, i, fp, sz, sz, sz, P(Slicer), fp, vp, sz]),
        "or_demodulate_front": (sz, [f, fp, sz, fp, sz, fp, sz, fp, fp, fp]),
        "or_modulate_cli": (c.c_long, [c.c_char_p, sz, sz, sz, sz, i, c.c_char_p, sz, fp, sz]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype, fn.argtypes = res, args
    _L = L
    return L


def _fp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _u8(b: Sequence[int]):
    a = np.ascontiguousarray(np.asarray(b, dtype=np.uint8))
    return a, a.ctypes.data_as(ctypes.c_void_p)


# ----------------------------------------------------------------- small helpers ----
def mod_trig(x: float) -> float:
    return lib().or_mod_trig(x)


def bit_to_sign(b: int) -> float:
    return lib().or_bit_to_sign(b)


def bytes_to_bits(b: Sequence[int]) -> int:
    a, p = _u8(b)
    return lib().or_bytes_to_bits(p, len(a))


def max_symbol(bps: int) -> int:
    return lib().or_max_symbol(bps)


def sample_freq(hz: int, sr: int) -> float:
    return lib().or_freq_sample_freq(hz, sr)


def carrier_phases(sf: float, s0: int, n: int) -> np.ndarray:
    out = np.zeros(n, dtype=np.float32)
    lib().or_carrier_phases(sf, s0, n, _fp(out))
    return out


def new_phasor(kind: int, *args) -> Phasor:
    p = Phasor()
    L = lib()
    ctor = {BPSK: L.or_bpsk_new, QPSK: L.or_qpsk_new, QAM: L.or_qam_new, BASK: L.or_bask_new,
            MPSK: L.or_mpsk_new, OQPSK: L.or_oqpsk_new, DCQPSK: L.or_dcqpsk_new, DMPSK: L.or_dmpsk_new,
            CPFSK: L.or_cpfsk_new, MSK: L.or_msk_new, MFSK: L.or_mfsk_new, BFSK: L.or_bfsk_new}
    if kind == APSK:
        amplitude, bps, rings = args
        arr = (Ring * len(rings))(*[Ring(a, b, r, ph) for (a, b, r, ph) in rings])
        rc = L.or_apsk_new(ctypes.byref(p), amplitude, bps, arr, len(rings))
    else:
        rc = ctor[kind](ctypes.byref(p), *args)
    if rc != 0:
        raise AssertionError("reference assert! would panic")
    return p


def phasor_i(p: Phasor, s: int, b: Sequence[int]) -> float:
    a, ptr = _u8(b)
    return lib().or_phasor_i(ctypes.byref(p), s, ptr, len(a))


def phasor_q(p: Phasor, s: int, b: Sequence[int]) -> float:
    a, ptr = _u8(b)
    return lib().or_phasor_q(ctypes.byref(p), s, ptr, len(a))


def phasor_update(p: Phasor, s: int, b: Sequence[int]) -> None:
    a, ptr = _u8(b)
    lib().or_phasor_update(ctypes.byref(p), s, ptr, len(a))


def phasor_lut(p: Phasor) -> np.ndarray:
    out = np.zeros((1 << p.bits_per_symbol, 2), dtype=np.float32)
    assert lib().or_phasor_lut(ctypes.byref(p), _fp(out)) == 0
    return out


def fir_block(coefs: np.ndarray, x: np.ndarray) -> np.ndarray:
    coefs = np.ascontiguousarray(coefs, np.float32)
    x = np.ascontiguousarray(x, np.float32)
    y = np.zeros_like(x)
    lib().or_fir_block(_fp(coefs), len(coefs), _fp(x), len(x), _fp(y))
    return y


def iq_modulate(carrier: float, i: float, q: float) -> Tuple[float, float]:
    s = IQSample(carrier, i, q)
    re, im = ctypes.c_float(), ctypes.c_float()
    lib().or_iq_modulate(ctypes.byref(s), ctypes.byref(re), ctypes.byref(im))
    return re.value, im.value


def demodulate(sf: float, s0: int, phase_offset: float, taps, x_re) -> Tuple[np.ndarray, np.ndarray]:
    taps = np.ascontiguousarray(taps, np.float32)
    x_re = np.ascontiguousarray(x_re, np.float32)
    oi, oq = np.zeros_like(x_re), np.zeros_like(x_re)
    lib().or_demodulate(sf, s0, phase_offset, _fp(taps), len(taps), _fp(x_re), len(x_re), _fp(oi), _fp(oq))
    return oi, oq


def prng_bits(seed: int, nbits: int) -> np.ndarray:
    out = np.zeros(nbits, dtype=np.uint8)
    lib().or_prng_bits(seed, out.ctypes.data_as(ctypes.c_void_p), nbits)
    return out


def rrc_taps(ntaps: int, sps: int, beta: float) -> np.ndarray:
    out = np.zeros(ntaps, dtype=np.float32)
    assert lib().or_rrc_taps(ntaps, sps, beta, _fp(out)) == 0
    return out


def make_slicer(kind: int, bps: int, lut: Optional[np.ndarray] = None, bits_per_carrier: int = 0,
                inv_scale: float = 0.0, max_symbol_: float = 0.0) -> Slicer:
    s = Slicer()
    s.kind, s.bps = kind, bps
    if lut is not None:
        s._lut = np.ascontiguousarray(lut, np.float32).reshape(-1)
        s.lut = _fp(s._lut)
    s.bits_per_carrier, s.inv_scale, s.max_symbol = bits_per_carrier, inv_scale, max_symbol_
    return s


def qam_axis_slicer(bps: int, amplitude: float) -> Slicer:
    cs = bps // 2
    ms = np.float32((1 << cs) - 1)
    scale = np.float32(np.float32(amplitude) / ms) / np.float32(2.0)   # qam.rs:28
    return make_slicer(SLICER_QAM_AXIS, bps, None, cs, float(np.float32(1.0) / scale), float(ms))


def tx_chain(p: Phasor, bits: np.ndarray, sps: int, taps: Optional[np.ndarray], sf: float, s0: int,
             flush_syms: int = 0, out_mode: int = OUT_IQ_MIXED, even_odd: bool = False) -> np.ndarray:
    """or_tx_chain_src: DigitalModulator over Bits (or EvenOddOffset(Bits), data.rs:81-123)."""
    bits = np.ascontiguousarray(bits, np.uint8)
    nsym = len(bits) // p.bits_per_symbol + flush_syms
    per = 1 if out_mode == OUT_REAL else 2
    out = np.zeros(nsym * sps * per + 1, dtype=np.float32)
    t = np.zeros(1, np.float32) if taps is None else np.ascontiguousarray(taps, np.float32)
    n = lib().or_tx_chain_src(ctypes.byref(p), bits.ctypes.data_as(ctypes.c_void_p), len(bits), sps, _fp(t),
                              0 if taps is None else len(t), sf, s0, flush_syms, out_mode, int(even_odd),
                              _fp(out))
    out = out[: n * per]
    return out if per == 1 else out.reshape(n, 2)


def rx_chain(x_iq: np.ndarray, sf: float, s0: int, mix: int, taps: np.ndarray, sps: int, D: int,
             slicer: Optional[Slicer]) -> Tuple[np.ndarray, np.ndarray]:
    x = np.ascontiguousarray(x_iq, np.float32).reshape(-1)
    n = len(x) // 2
    taps = np.ascontiguousarray(taps, np.float32)
    cap = n // sps + 2
    oiq = np.zeros((cap, 2), np.float32)
    osym = np.zeros(cap, np.uint8)
    k = lib().or_rx_chain(_fp(x), n, sf, s0, mix, _fp(taps), len(taps), sps, D,
                          ctypes.byref(slicer) if slicer is not None else None, _fp(oiq),
                          osym.ctypes.data_as(ctypes.c_void_p), cap)
    return oiq[:k], osym[:k]


def modulate_cli(name: str, text: bytes, sr: int = 10000, br: int = 220, cf: int = 1000, pc: int = 0,
                 iq: bool = False) -> Optional[np.ndarray]:
    cap = max(16, len(text) * (sr // max(br, 1) + 1) * 2 + sr)
    out = np.zeros(cap, np.float32)
    n = lib().or_modulate_cli(name.encode(), sr, br, cf, pc, int(iq), text, len(text), _fp(out), cap)
    return None if n < 0 else out[:n]


# -------------------------------------------------- source iterators (data.rs) ----
def symbol_clock_ticks(sps: int, n: int) -> List[bool]:
    c = SymbolClock()
    lib().or_symbol_clock_init(ctypes.byref(c), sps)
    return [bool(lib().or_symbol_clock_next(ctypes.byref(c))) for _ in range(n)]


def _drain(next_fn, obj, bps, n):
    out = []
    for _ in range(n):
        ptr = ctypes.c_void_p()
        u = next_fn(ctypes.byref(obj), ctypes.byref(ptr))
        if u == FINISHED:
            out.append((FINISHED, None))
        else:
            out.append((u, list(ctypes.string_at(ptr.value, bps))))
    return out


def bits_updates(bits: Sequence[int], sps: int, bps: int, n: int):
    a, p = _u8(bits)
    s = BitsSource()
    s._keep = a
    lib().or_bits_init(ctypes.byref(s), p, len(a), sps, bps)
    return _drain(lib().or_bits_next, s, bps, n)


def even_odd_updates(bits: Sequence[int], sps: int, bps: int, n: int):
    a, p = _u8(bits)
    src = Source()
    src.is_ascii = 0
    lib().or_bits_init(ctypes.byref(src.bits), p, len(a), sps, bps)
    e = EvenOdd()
    e._keep = a
    assert lib().or_even_odd_init(ctypes.byref(e), ctypes.byref(src), sps, bps) == 0
    return _drain(lib().or_even_odd_next, e, 2, n)


def ascii_reader(text: bytes, sps: int, bps: int) -> AsciiBits:
    buf = ctypes.create_string_buffer(text, len(text))
    a = AsciiBits()
    a._keep = buf
    lib().or_ascii_init(ctypes.byref(a), ctypes.cast(buf, ctypes.c_void_p), len(text), sps, bps)
    return a


def ascii_updates(text: bytes, sps: int, bps: int, n: int):
    a = ascii_reader(text, sps, bps)
    return _drain(lib().or_ascii_next, a, bps, n)


def demodulate_front(sf: float, x: np.ndarray, hilbert: np.ndarray, lowpass: np.ndarray):
    """or_demodulate_front: (i, q) per sample after the 64-sample PLL lock, and the offset."""
    x = np.ascontiguousarray(x, np.float32)
    h = np.ascontiguousarray(hilbert, np.float32)
    lp = np.ascontiguousarray(lowpass, np.float32)
    n = len(x)
    oi = np.zeros(max(n - 64, 1), np.float32)
    oq = np.zeros(max(n - 64, 1), np.float32)
    off = np.zeros(1, np.float32)
    k = lib().or_demodulate_front(sf, _fp(x), n, _fp(h), len(h), _fp(lp), len(lp), _fp(oi), _fp(oq), _fp(off))
    return oi[:k], oq[:k], float(off[0])
