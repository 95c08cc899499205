"""The reference's own known-answer tests, run against the CPU oracle (CPU only).

Each test restates one `#[cfg(test)]` of ramtej/rust-modem with the same inputs and expected
values; together they pin the oracle's bit→symbol map and symbol timing.
"""
import numpy as np
import pytest

from conftest import PI_4


def test_symbol_clock(o):
    """data.rs:194-209 test_symbol_clock: period 5, the first call ticks."""
    assert o.symbol_clock_ticks(5, 11) == [True, False, False, False, False,
                                           True, False, False, False, False, True]


def test_bits(o):
    """data.rs:211-224 test_bits: [1,0,1,1], sps 3, bps 2."""
    C, U, F = o.CHANGED, o.UNCHANGED, o.FINISHED
    assert o.bits_updates([1, 0, 1, 1], 3, 2, 7) == [
        (C, [1, 0]), (U, [1, 0]), (U, [1, 0]), (C, [1, 1]), (U, [1, 1]), (U, [1, 1]), (F, None)]


def test_evenodd(o):
    """data.rs:226-246 test_evenodd: OQPSK half-symbol Q offset over Bits([1,1,1,0,0,1], 4, 2)."""
    C, U, F = o.CHANGED, o.UNCHANGED, o.FINISHED
    want = [(C, [1, 0]), (U, [1, 0]), (C, [1, 1]), (U, [1, 1]), (C, [1, 1]), (U, [1, 1]),
            (C, [1, 0]), (U, [1, 0]), (C, [0, 0]), (U, [0, 0]), (C, [0, 1]), (U, [0, 1]), (F, None)]
    assert o.even_odd_updates([1, 1, 1, 0, 0, 1], 4, 2, 13) == want


def test_ascii(o):
    """data.rs:248-279 test_ascii, on an in-memory copy of its `ascii.bits` file."""
    text = b"000\n111\n101"
    a = o.ascii_reader(text, 1, 3)
    assert [bool(o.lib().or_ascii_read_bits(__import__("ctypes").byref(a))) for _ in range(4)] == \
        [True, True, True, False]
    C, U, F = o.CHANGED, o.UNCHANGED, o.FINISHED
    assert o.ascii_updates(text, 2, 3, 7) == [
        (C, [0, 0, 0]), (U, [0, 0, 0]), (C, [1, 1, 1]), (U, [1, 1, 1]), (C, [1, 0, 1]), (U, [1, 0, 1]),
        (F, None)]


def test_b2b(o):
    """digital/util.rs:21-25 test_b2b."""
    assert o.bytes_to_bits([0, 0, 0, 1]) == 0b0001
    assert o.bytes_to_bits([0, 1, 0, 1]) == 0b0101


def test_max_symbol(o):
    """digital/util.rs:27-33 test_max_symbol."""
    assert [o.max_symbol(n) for n in (1, 2, 4, 8)] == [0b1, 0b11, 0b1111, 0b11111111]


def test_qam(o):
    """qam.rs:68-84 test_qam: QAM::new(4, 0.0, 6.0), exact levels."""
    q = o.new_phasor(o.QAM, 4, 0.0, 6.0)
    for bits, (i, qq) in {(0, 0, 0, 0): (-3.0, -3.0), (0, 0, 0, 1): (-3.0, -1.0),
                          (1, 0, 1, 1): (1.0, 3.0), (1, 1, 1, 1): (3.0, 3.0)}.items():
        assert o.phasor_i(q, 0, bits) == i
        assert o.phasor_q(q, 0, bits) == qq


def test_mpsk(o):
    """mpsk.rs:49-63 test_mpsk: 4-PSK on the unit circle."""
    p = o.new_phasor(o.MPSK, 2, 0.0, 1.0)
    assert o.phasor_i(p, 0, [0, 0]) == 1.0 and o.phasor_q(p, 0, [0, 0]) == 0.0
    assert abs(o.phasor_i(p, 0, [0, 1])) < 1e-3 and o.phasor_q(p, 0, [0, 1]) == 1.0
    assert o.phasor_i(p, 0, [1, 0]) == -1.0 and abs(o.phasor_q(p, 0, [1, 0])) < 1e-3
    assert abs(o.phasor_i(p, 0, [1, 1])) < 1e-3 and o.phasor_q(p, 0, [1, 1]) == -1.0


def test_dmpsk(o):
    """dmpsk.rs:50-84 test_dmpsk: differential phase walk, tolerance 1e-6."""
    half_pi = float(np.float32(np.float32(np.pi) / np.float32(2.0)))
    d = o.new_phasor(o.DMPSK, 2, 1.0, 0.0, half_pi)
    want = [(1, 0), (1, 0), (0, 1), (0, -1), (-1, 0), (-1, 0), (-1, 0), (0, 1)]
    steps = [None, [0, 0], [0, 1], [1, 0], [1, 1], [0, 0], [0, 0], [1, 1]]
    for b, (wi, wq) in zip(steps, want):
        if b is not None:
            o.phasor_update(d, 123, b)
        assert abs(o.phasor_i(d, 0, []) - wi) < 1e-6
        assert abs(o.phasor_q(d, 0, []) - wq) < 1e-6


# ------------------------------------------------ reference constants ----
def f32hex(x):
    return np.float32(x).view(np.uint32).item()


def test_lut_constants(o):
    """BPSK(π/4) = ±0x3f3504f3 (bpsk.rs:17-31), QPSK amplitude sqrtf(0.5) (qpsk.rs:11-35),
    QAM scale A/ms/2 = 0x3e2aaaab (16) / 0x3d088889 (256) (qam.rs:28); peak level 0.5."""
    lut = o.phasor_lut(o.new_phasor(o.BPSK, PI_4, 1.0))
    assert {f32hex(abs(v)) for v in lut.ravel()} == {0x3f3504f3}
    lut = o.phasor_lut(o.new_phasor(o.QPSK, 0.0, 1.0))
    assert {f32hex(abs(v)) for v in lut.ravel()} == {0x3f3504f3}
    for bps, scale in ((4, 0x3e2aaaab), (8, 0x3d088889)):
        lut = o.phasor_lut(o.new_phasor(o.QAM, bps, 0.0, 1.0))
        s1 = 1 << (bps // 2 - 1)              # pos_symbol(s1) = 2*s1 - ms = +1 -> Q = scale
        assert f32hex(lut[s1, 1]) == scale
        assert np.max(np.abs(lut)) == np.float32(0.5)


def test_carrier_w(o):
    """Freq::new(1, 4).sample_freq() = fl(fl(2·PI)·1)/4 = 0x3fc90fdb (freq.rs:19-26)."""
    assert f32hex(o.sample_freq(1, 4)) == 0x3fc90fdb


def test_qam_assert(o):
    """qam.rs:17 assert!(bits_per_symbol > 1): a 1-bit QAM is a reference panic."""
    with pytest.raises(AssertionError):
        o.new_phasor(o.QAM, 1, 0.0, 1.0)
