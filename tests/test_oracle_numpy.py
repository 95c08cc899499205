"""Independent numpy restatements cross-check the C oracle where no reference test pins it
(FIRFilter, Carrier, IQSample::modulate and Demodulator are untested upstream).

numpy float32 arithmetic rounds every operation and never contracts a*b+c, which is exactly
Rust's f32 semantics, so the integer / f32-op parts (carrier phase, FIR fold, bit packing,
slicer) must agree bit for bit. numpy's own float32 sin/cos are not glibc's `sinf/cosf`
(which the oracle, like Rust on Linux, calls), so results that pass through a sin/cos are
compared to a stated tolerance instead. CPU only, sizes that finish in seconds.
"""
import numpy as np
import pytest

from conftest import CONFIGS, oracle_phasor, oracle_slicer

F = np.float32
TWO_PI = np.uint32(0x40C90FDB).view(np.float32)    # std::f32::consts::PI * 2.0


def np_mod_trig(x):
    """util.rs:3-6: x - TWO_PI * floor(x / TWO_PI), each op rounded to f32."""
    x = np.asarray(x, F)
    return (x - TWO_PI * np.floor(x / TWO_PI)).astype(F)


def np_phases(w, s0, n):
    """carrier.rs:17-26: mod_trig(sample_freq * (s as f32)) for s = s0 .. s0 + n - 1."""
    s = np.arange(s0, s0 + n, dtype=np.uint64).astype(F)   # u64 -> f32 round-to-nearest-even
    return np_mod_trig(F(w) * s)


def np_fir(h, x):
    """fir.rs:18-34: y[n] = fold_{k=0..L-1} (acc + x[n-k] * h[k]) from 0.0, x[<0] = 0."""
    h = np.asarray(h, F)
    x = np.asarray(x, F)
    xp = np.concatenate([np.zeros(len(h) - 1, F), x])
    acc = np.zeros(len(x), F)
    for k in range(len(h)):
        acc = (acc + xp[len(h) - 1 - k: len(h) - 1 - k + len(x)] * h[k]).astype(F)
    return acc


def np_splitmix_bits(seed, nbits):
    """GLUE: splitmix64 words, bit i = (word[i/64] >> (i%64)) & 1."""
    M = (1 << 64) - 1
    st, out = seed, np.zeros(nbits, np.uint8)
    for w0 in range(0, nbits, 64):
        st = (st + 0x9E3779B97F4A7C15) & M
        z = st
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        z ^= z >> 31
        for i in range(min(64, nbits - w0)):
            out[w0 + i] = (z >> i) & 1
    return out


def np_rrc(L, sps, beta):
    """GLUE: root-raised-cosine, centred, unit energy (double), rounded to f32."""
    t = (np.arange(L) - (L - 1) / 2.0) / sps
    h = np.empty(L)
    for i, ti in enumerate(t):
        if ti == 0.0:
            h[i] = 1.0 - beta + 4.0 * beta / np.pi
        elif beta > 0 and abs(abs(4.0 * beta * ti) - 1.0) < 1e-12:
            h[i] = beta / np.sqrt(2.0) * ((1 + 2 / np.pi) * np.sin(np.pi / (4 * beta)) +
                                          (1 - 2 / np.pi) * np.cos(np.pi / (4 * beta)))
        else:
            h[i] = (np.sin(np.pi * ti * (1 - beta)) + 4 * beta * ti * np.cos(np.pi * ti * (1 + beta))) / \
                   (np.pi * ti * (1 - (4 * beta * ti) ** 2))
    return (h / np.sqrt(np.sum(h * h))).astype(F)


# ------------------------------------------------------------------ bit-exact checks ----
@pytest.mark.parametrize("hz,sr", [(1, 4), (1000, 10000)])
@pytest.mark.parametrize("s0", [0, (1 << 24) - 256, (1 << 26) - 256, (1 << 32) - 100, (1 << 40) + 7])
def test_carrier_phase_bit_exact(o, hz, sr, s0):
    """Carrier phase φ[n] bit-exact, including past the f32 precision cliff (§8a a9)."""
    w = o.sample_freq(hz, sr)
    assert np.array_equal(o.carrier_phases(w, s0, 512).view(np.uint32), np_phases(w, s0, 512).view(np.uint32))


def test_mod_trig_bit_exact(o):
    rng = np.random.default_rng(1)
    xs = np.concatenate([rng.uniform(0, 1e8, 2000), rng.uniform(-100, 100, 500), [0.0, TWO_PI, 2 * TWO_PI]]).astype(F)
    got = np.array([o.mod_trig(float(x)) for x in xs], F)
    assert np.array_equal(got.view(np.uint32), np_mod_trig(xs).view(np.uint32))


@pytest.mark.parametrize("L", [1, 2, 33, 129])
def test_fir_fold_bit_exact(o, L):
    """FIRFilter::add over a block equals the sequential fold, bit for bit (release wrap)."""
    rng = np.random.default_rng(L)
    h = rng.standard_normal(L).astype(F)
    x = rng.standard_normal(3000).astype(F)
    assert np.array_equal(o.fir_block(h, x).view(np.uint32), np_fir(h, x).view(np.uint32))


def test_prng_bits(o):
    for seed in (0x5EED0000, 0x5EED0003, 0):
        assert np.array_equal(o.prng_bits(seed, 1000), np_splitmix_bits(seed, 1000))


@pytest.mark.parametrize("L,sps", [(33, 4), (65, 4), (129, 4), (513, 8), (31, 2)])
def test_rrc_taps(o, L, sps):
    got, want = o.rrc_taps(L, sps, 0.35), np_rrc(L, sps, 0.35)
    assert np.max(np.abs(got - want)) <= 2 * np.finfo(F).eps * np.max(np.abs(want))
    assert abs(float(np.sum(got.astype(np.float64) ** 2)) - 1.0) < 1e-6


def np_qam_slice(re, im, bps, amplitude=1.0):
    """GLUE: per-axis round-and-clamp inverse of qam.rs:32-60 (scale = A/ms/2)."""
    cs = bps // 2
    ms = F((1 << cs) - 1)
    scale = F(F(amplitude) / ms) / F(2)
    inv = F(1) / scale
    si = np.fmin(np.fmax(np.rint(((re.astype(F) * inv + ms) * F(0.5)).astype(F)), F(0)), ms).astype(np.int64)
    sq = np.fmin(np.fmax(np.rint(((im.astype(F) * inv + ms) * F(0.5)).astype(F)), F(0)), ms).astype(np.int64)
    return ((si << cs) | sq).astype(np.uint8)


@pytest.mark.parametrize("bps", [4, 8])
def test_qam_slicer_bit_exact(o, bps):
    """The QAM-axis slicer on noisy constellation points (ties and clamps included)."""
    sl = o.qam_axis_slicer(bps, 1.0)
    lut = o.phasor_lut(o.new_phasor(o.QAM, bps, 0.0, 1.0))
    rng = np.random.default_rng(bps)
    idx = rng.integers(0, 1 << bps, 4000)
    pts = lut[idx] + rng.normal(0, 0.05, (4000, 2)).astype(F)
    pts[:8] = [[0.6, -0.6], [-0.6, 0.6], [0, 0], [1e9, -1e9], [0.5, 0.5], [-0.5, -0.5], [1e-30, 0], [np.nan, -np.inf]]
    pts = pts.astype(F)
    got = np.array([o.lib().or_slice(__import__("ctypes").byref(sl), float(a), float(b)) for a, b in pts], np.uint8)
    assert np.array_equal(got, np_qam_slice(pts[:, 0], pts[:, 1], bps))
    assert np.array_equal(np_qam_slice(lut[:, 0], lut[:, 1], bps), np.arange(1 << bps, dtype=np.uint8))


# --------------------------------------------------------- tolerance (sin/cos) checks ----
def np_tx_chain(lut, bits, bps, sps, taps, w, s0):
    """GLUE + modulator.rs: LUT symbols, zero-stuffed, per-rail FIR, mixed onto the carrier."""
    sym = (bits.reshape(-1, bps).astype(np.int64) @ (1 << np.arange(bps)[::-1]))
    n = len(sym) * sps
    xi, xq = np.zeros(n, F), np.zeros(n, F)
    xi[::sps], xq[::sps] = lut[sym, 0], lut[sym, 1]
    yi, yq = np_fir(taps, xi), np_fir(taps, xq)
    ph = np_phases(w, s0, n).astype(np.float64)
    c, s = np.cos(ph), np.sin(ph)
    return np.stack([yi * c - yq * s, yi * s + yq * c], 1)


def np_rx_chain(x, taps, sps, D, w, s0):
    """GLUE: x * e^{-j phase}, per-rail FIR, keep n = D + k*sps."""
    ph = np_phases(w, s0, len(x)).astype(np.float64)
    c, s = np.cos(ph), np.sin(ph)
    zr = (x[:, 0] * c + x[:, 1] * s).astype(F)
    zi = (x[:, 1] * c - x[:, 0] * s).astype(F)
    ri, rq = np_fir(taps, zr), np_fir(taps, zi)
    return np.stack([ri[D::sps], rq[D::sps]], 1)


@pytest.mark.parametrize("cfg", ["c1_bpsk", "c2_qpsk", "c3_qam16"])
@pytest.mark.parametrize("s0", [0, (1 << 24) - 1000])
def test_tx_rx_chain_vs_numpy(o, cfg, s0):
    name, bps, L, sps = CONFIGS[cfg]
    p = oracle_phasor(o, name)
    lut = o.phasor_lut(p)
    taps = o.rrc_taps(L, sps, 0.35)
    w = o.sample_freq(1, 4)
    bits = o.prng_bits(0x5EED0000, 600 * bps)
    y = o.tx_chain(p, bits, sps, taps, w, s0)
    ynp = np_tx_chain(lut, bits, bps, sps, taps, w, s0)
    assert y.shape == ynp.shape
    tol = 1e-5 * float(np.max(np.abs(ynp)))              # sin/cos ulps only here
    assert float(np.max(np.abs(y - ynp))) <= tol
    iq, sym = o.rx_chain(y, w, s0, o.MIX_COMPLEX, taps, sps, L - 1, oracle_slicer(o, name, bps))
    iqnp = np_rx_chain(y, taps, sps, L - 1, w, s0)
    assert iq.shape == iqnp.shape
    assert float(np.max(np.abs(iq - iqnp))) <= 1e-5 * float(np.max(np.abs(iqnp)))
    sent = (bits.reshape(-1, bps).astype(np.int64) @ (1 << np.arange(bps)[::-1])).astype(np.uint8)
    assert np.array_equal(sym, sent[: len(sym)])        # clean loopback: every decision right


def test_reference_demodulator_vs_numpy(o):
    """demodulator.rs:44-56: (2·FIR_I(x·cos φ), 2·FIR_Q(x·(−sin φ))) at every sample."""
    rng = np.random.default_rng(5)
    x = rng.standard_normal(2000).astype(F)
    taps = o.rrc_taps(65, 4, 0.35)
    w = o.sample_freq(1000, 10000)
    oi, oq = o.demodulate(w, 7, 0.0, taps, x)
    ph = np_phases(w, 7, len(x)).astype(np.float64)
    wi = F(2) * np_fir(taps, (x * np.cos(ph)).astype(F))
    wq = F(2) * np_fir(taps, (x * -np.sin(ph)).astype(F))
    assert np.max(np.abs(oi - wi)) <= 1e-5 * np.max(np.abs(wi))
    assert np.max(np.abs(oq - wq)) <= 1e-5 * np.max(np.abs(wq))


def test_iq_modulate(o):
    """modulator.rs:45-48: (i + jq) * e^{j carrier}."""
    rng = np.random.default_rng(3)
    for ph, i, q in rng.uniform(-3, 3, (200, 3)).astype(F):
        re, im = o.iq_modulate(float(ph), float(i), float(q))
        c, s = np.cos(float(ph)), np.sin(float(ph))
        assert abs(re - (i * c - q * s)) <= 4e-7 * (abs(i) + abs(q))
        assert abs(im - (i * s + q * c)) <= 4e-7 * (abs(i) + abs(q))


# ----------------------------------- the product's exact floor(x / 2π) (GPU phase, H1) ----
def test_phase_floor_division_replacement():
    """The HIP kernels replace floor(fl(x / TWO_PI)) by floor(q1), q0 = x*RC, r = fma(-q0, TWO_PI, x),
    q1 = fma(r, RC, q0), RC = fl(1/TWO_PI). Exhaustively verified over every non-negative f32
    when it was designed; here a seeded sample plus the ranges the carrier reaches."""
    RC = np.float32(float.fromhex("0x1.45f306p-3"))
    rng = np.random.default_rng(11)
    x = np.concatenate([rng.uniform(0, 2 ** 30, 1 << 20), np.arange(0, 1 << 16),
                        np.float32(np.pi / 2) * np.arange((1 << 24) - 4096, (1 << 24) + 4096),
                        rng.uniform(0, 1e30, 1 << 16)]).astype(F)
    ld = np.longdouble

    def fma(a, b, c):   # exact a*b + c with one rounding to f32 (x87 64-bit significand)
        return (a.astype(ld) * b.astype(ld) + c.astype(ld)).astype(F)

    q0 = (x * RC).astype(F)
    r = fma(-q0, np.full_like(x, TWO_PI), x)
    q1 = fma(r, np.full_like(x, RC), q0)
    assert np.array_equal(np.floor(q1), np.floor((x / TWO_PI).astype(F)))
