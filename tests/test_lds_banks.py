"""LDS bank model of the RX matched-filter reads (rx_mfma, modem_rx.hip).

MI355X_MICROARCH.md §LDS: a wave64 `ds_read_b128` is serviced in 4 lane groups,
{0-3,12-15,20-27}, {4-11,16-19,28-31} and the same +32, with bank = (byte address / 4) mod 64;
two different addresses on one bank within a group cost an extra cycle. This restates the
kernel's address formulas (A rows: `rxh_pos` padding; B tap tables: `rx_mfma_table_len`
padding and `rx_mfma_table_copies`) and checks every (decimation, k-steps) variant the
library instantiates is conflict-free. The old layout (8 pad halves, tables padded to 16 mod
64) is checked to show the 2-way conflicts the PMC counter measured (144 extra cycles per
wave tile on C3 = 36 reads x 4 groups).
"""

G0 = [*range(0, 4), *range(12, 16), *range(20, 28)]
G1 = [*range(4, 12), *range(16, 20), *range(28, 32)]
GROUPS = [G0, G1, [x + 32 for x in G0], [x + 32 for x in G1]]

VARIANTS = [(2, 2), (2, 3), (2, 5), (2, 8), (4, 3), (4, 4), (4, 6), (4, 8), (8, 5), (8, 6), (8, 9), (8, 20)]


def extra_cycles(addr):
    """Extra LDS cycles of one ds_read_b128 whose lane l reads 16 B at byte addr(l)."""
    tot = 0
    for g in GROUPS:
        banks = {}
        for lane in g:
            a = addr(lane)
            for d in range(4):
                banks.setdefault((a // 4 + d) % 64, set()).add(a)
        tot += max(len(v) for v in banks.values()) - 1
    return tot


def table_copies(dec):
    return 8 // (8 if dec % 8 == 0 else 4 if dec % 4 == 0 else 2 if dec % 2 == 0 else 1)


def table_len(dec, nks, residue):
    n = (32 * nks + 15 * dec + 8 + 7) & ~7
    return n + ((residue(dec) - (n % 64)) % 64 + 64) % 64


def new_residue(dec):          # rx_mfma_table_len (modem_internal.h)
    return 32 if dec % 8 == 4 else 16


def old_residue(dec):
    return 16


def a_cost(dec, nks, pad):
    rw = 16 * dec
    rp = rw + pad
    worst = 0
    for s in range(nks):
        aoff = 32 * s + pad * ((32 * s) // rw)
        worst = max(worst, extra_cycles(lambda l: 2 * ((l & 15) * rp + 8 * (l >> 4) + aoff)))
    return worst


def b_cost(dec, nks, residue):
    nc, tb = table_copies(dec), table_len(dec, nks, residue)
    worst = 0
    for s in range(nks):
        for lo in (0, 1):
            def addr(lane, s=s, lo=lo):
                i, g = lane & 15, lane >> 4
                xb = 8 * g + (15 - i) * dec
                q = xb & 7
                return 2 * ((q // (8 // nc)) * 2 * tb + lo * tb + (xb - q) + 32 * s)
            worst = max(worst, extra_cycles(addr))
    return worst


def test_a_reads_conflict_free():
    for dec, nks in VARIANTS:
        assert a_cost(dec, nks, 16) == 0, (dec, nks)


def test_b_reads_conflict_free():
    for dec, nks in VARIANTS:
        assert b_cost(dec, nks, new_residue) == 0, (dec, nks)


def test_old_layout_matches_measured_conflicts():
    # C3 (decim 4, 6 k-steps): 24 A reads and 12 B reads per wave tile, 4 extra cycles each
    assert a_cost(4, 6, 8) == 4
    assert b_cost(4, 6, old_residue) == 4
    assert 24 * a_cost(4, 6, 8) + 12 * b_cost(4, 6, old_residue) == 144


def swz_pos(e):
    """RxMfma::ppos for decim 4 (4 waves): 16-B chunks XOR-swizzled within groups of 8."""
    return ((((e >> 3) ^ (((e >> 7) & 3) << 1)) << 3) | (e & 7))


def swz8_pos(e):
    """RxMfma::ppos for decim 8 (4 waves): 16-B chunks XOR-swizzled within each 128-sample
    row of 16 chunks by the row's low 3 bits."""
    return ((((e >> 3) ^ (((e >> 7) & 7) << 1)) << 3) | (e & 7))


def test_swizzled_decim8_layout_conflict_free():
    """C5's RX (decim 8, 20 k-steps; two planes for f16 samples, four for f32): the unpadded
    swizzled plane. A reads: lane (i, g) of wave w, k-step s reads 8 halves at sample
    (16 w + i) * 128 + 8 g + 32 s; staging writes: ds_write_b64 of 4 consecutive samples per
    lane, slots 1024 samples apart; the swizzle is a bijection within every row (no LDS
    beyond the unpadded plane) and repeats every 1024 samples (the slot offset)."""
    for w in range(4):
        for s in range(20):
            assert extra_cycles(lambda l: 2 * swz8_pos((16 * w + (l & 15)) * 128 + 8 * (l >> 4) + 32 * s)) == 0
    for u in range(9):
        for g in range(4):
            banks = {}
            for lane in range(16 * g, 16 * g + 16):
                a = 2 * swz8_pos(4 * lane + 1024 * u)
                for d in range(2):
                    banks.setdefault((a // 4 + d) % 32, set()).add(a)
            assert max(len(v) for v in banks.values()) == 1
    for base in range(0, 8192, 128):
        assert sorted(swz8_pos(e) for e in range(base, base + 128)) == list(range(base, base + 128))
    for e in range(0, 4096):
        assert swz8_pos(e + 1024) == swz8_pos(e) + 1024
    # the unswizzled, unpadded decim-8 plane would be 15-way conflicted on every A read
    assert extra_cycles(lambda l: 2 * ((l & 15) * 128 + 8 * (l >> 4))) > 0


def test_swizzled_layout_conflict_free():
    # A reads: lane (i, g) of wave w, k-step s reads 8 halves at sample (16 w + i) * 64 + 8 g + 32 s
    for w in range(4):
        for s in range(8):
            assert extra_cycles(lambda l: 2 * swz_pos((16 * w + (l & 15)) * 64 + 8 * (l >> 4) + 32 * s)) == 0
    # staging writes: ds_write_b64, 4 groups of 16 contiguous lanes, bank = (a / 4) mod 32
    for u in range(5):
        for g in range(4):
            banks = {}
            for lane in range(16 * g, 16 * g + 16):
                a = 2 * (swz_pos(4 * lane) + 1024 * u)
                for d in range(2):
                    banks.setdefault((a // 4 + d) % 32, set()).add(a)
            assert max(len(v) for v in banks.values()) == 1
    # a bijection within every aligned group of 8 chunks (no LDS beyond the unpadded plane)
    for base in range(0, 4096, 64):
        assert sorted(swz_pos(e) for e in range(base, base + 64)) == list(range(base, base + 64))


# ------------------------------------------------------------------------------------------------
# The fused small call's LDS sample window (chain_small, modem_chain.hip): the TX writes every
# emitted sample (8-B float2) at raw_pos(i), the RX stages its quads from it (lane l of a wave reads
# elements q + 4 l + j, j = 0..3, one ds_read_b64 each). ds_read_b64 is serviced as lanes {0-31},
# {32-63} with bank = dword mod 64, i.e. element mod 32; ds_write_b64 as 4 groups of 16 contiguous
# lanes with bank = dword mod 32, i.e. element mod 16 (MI355X_MICROARCH.md §LDS).

def raw_pos(i):                # modem_device.h
    return i ^ ((i >> 5) & 3)


def b64_read_extra(elem):
    tot = 0
    for g in (range(0, 32), range(32, 64)):
        banks = {}
        for lane in g:
            banks.setdefault(elem(lane) % 32, set()).add(elem(lane))
        tot += max(len(v) for v in banks.values()) - 1
    return tot


def b64_write_extra(elem):
    tot = 0
    for g in (range(0, 16), range(16, 32), range(32, 48), range(48, 64)):
        banks = {}
        for lane in g:
            banks.setdefault(elem(lane) % 16, set()).add(elem(lane))
        tot += max(len(v) for v in banks.values()) - 1
    return tot


def test_handoff_window_conflict_free():
    """RX quad reads from the window at every start offset: 3 extra cycles per group and read
    unswizzled (4-way, the 102,400 cycles per C2 launch the PMC counter measured), none with
    raw_pos; the TX's stores (lane l: 64 (l >> 4) + (l & 15) + 16 r from a 16-aligned base) stay
    conflict-free."""
    for q in range(0, 64):
        for j in range(4):
            assert b64_read_extra(lambda l: q + 4 * l + j) == 6          # 2 groups x (4-way - 1)
            assert b64_read_extra(lambda l: raw_pos(q + 4 * l + j)) == 0
    for base in range(0, 1024, 16):
        for r in range(4):
            assert b64_write_extra(lambda l: raw_pos(base + 64 * (l >> 4) + (l & 15) + 16 * r)) == 0
    # the general path's one-sample-per-lane reads (consecutive lanes, consecutive elements) from
    # a 32-aligned start stay conflict-free
    for q in range(0, 1024, 32):
        assert b64_read_extra(lambda l: raw_pos(q + l)) == 0
    # a permutation inside aligned groups of 4: a window of 4 k elements maps onto itself
    assert sorted(raw_pos(i) for i in range(4 * 300)) == list(range(4 * 300))


def test_tx_lut_gather_conflicts_match_pmc():
    """The sps-8 TX's LDS bank conflicts are its symbol-LUT gathers, not the plane copies.

    The fast TX staging looks each symbol up in an LDS copy of the split LUT (tx_mfma, 8 B per
    entry, one ds_read_b64 per lane and staging slot: two groups of 32 lanes, bank = dword mod 64).
    256-QAM's random indices spread 32 lanes over 32 bank pairs, so a read costs the largest
    number of distinct entries on one pair, minus one, per group. Over C5's launch (2^23 symbols,
    8192 tiles of NE = 1024 + 94 window symbols, one lane per symbol) the model gives the
    SQ_LDS_BANK_CONFLICT both C5 TX launches measured (615,682, profiles/r05_c5h_pmc_summary.txt
    and r05_c5_pmc_summary.txt), i.e. ~2.4 K LDS cycles per CU in an 83-104 us launch; 16-QAM's
    16 entries sit on 16 distinct pairs (C3's TX: 0)."""
    import numpy as np
    rng = np.random.default_rng(7)

    def extra(nent, trials):
        tot = 0
        for _ in range(trials):
            e = rng.integers(0, nent, 64)
            for g in (e[:32], e[32:]):
                u = np.unique(g)
                tot += np.bincount((2 * u) % 64, minlength=64).max() - 1
        return tot / trials

    wave_reads = (1024 + 94) / 64 * 8192
    pred = extra(256, 4000) * wave_reads
    assert abs(pred / 615682 - 1) < 0.03, pred
    assert extra(16, 200) == 0
