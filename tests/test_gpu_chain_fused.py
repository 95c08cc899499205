"""The fused chain launch (rust-modem_amd/csrc/modem_chain.hip: one period's TX and RX in one
persistent launch, each workgroup demodulating only samples it modulated itself) against the
two launches (MODEM_CHAIN_FUSED=0 at create time), bit for bit, over several periods of a
continuing stream: the sample buffer, the RX I/Q and the decisions of every period, and the
handles' carrier samples. Cases cover the three filters the fused form is built for (65 taps
and 129 taps at sps 4, 513 taps at sps 8; f32 and f16 samples), both tile sizes (small calls:
one 16x16 sub-tile per wave; at-size calls: four), ragged calls (a bit carry, so the TX
row-block lead and the RX instant lead change from period to period), a constellation scaled
down so that the RX stages at a nonzero exponent, and sizes where the two sides pick
different tile sizes or the calls are at size (then the plan runs the two launches:
fused() == 0). A stream's first period has no fused form (its RX instants start at instant
0, so a tile's window reaches into the next TX tile) and may also run as the two launches. The
decisions of the last period are also checked against the symbols sent (the reference's
loopback, SURVEY §8c: hard decisions bit-exact)."""
import os

import numpy as np
import pytest

from conftest import CONFIGS, sent_symbols

pytestmark = pytest.mark.gpu

SEED = 0x5EED1000


def make_pair(m, o, cfg, dtype, amp):
    name, bps, L, sps = CONFIGS[cfg]
    taps = m.rrc_taps(L, sps, 0.35)
    w = o.sample_freq(1, 4)

    def phasor():
        return {"qpsk": lambda: m.QPSK(0.0, amp), "qam16": lambda: m.QAM(4, 0.0, amp),
                "qam256": lambda: m.QAM(8, 0.0, amp)}[name]()
    tx = m.DigitalModulator(m.Carrier(w, 777), phasor(), sps, taps, dtype=dtype)
    rx = m.DemodulatorRx(m.Carrier(w, 777), taps, decim=sps, decim_offset=L - 1, mix=m.MIX_COMPLEX,
                         slicer=phasor().slicer(), in_dtype=dtype, out_dtype=dtype)
    return tx, rx


# (config, dtype, symbols per period, extra bits (carry), periods, amplitude, fused expected:
# 1 every period after the first, 0 none, None either — a ragged call fuses in the periods whose
# TX and RX leads put every RX window inside its own TX tiles)
CASES = [
    ("c2_qpsk", 0, 3000, 1, 4, 1.0, None),          # small tiles, ragged
    ("c2_qpsk", 0, 1 << 18, 0, 3, 1.0, 1),          # the C2 call
    ("c3_qam16", 0, 5000, 3, 5, 1.0, None),         # small tiles, ragged, row-block lead cycles
    ("c3_qam16", 0, (1 << 18) + 4 * 37, 2, 3, 1.0, None),   # many small tiles, ragged
    ("c3_qam16", 0, 1 << 16, 0, 3, 1.0 / 64, 1),    # RX staged at a nonzero exponent
    ("c5_qam256", 0, 7000, 5, 3, 1.0, None),        # 513 taps sps 8, ragged: at sps 8 the small
                                                    # tiles give m = 2 (a 256-instant RX tile = 2048
                                                    # samples = two 128-symbol TX tiles)
    ("c5_qam256", 0, 1 << 17, 0, 3, 1.0, 1),        # 513 taps sps 8, many tiles
    ("c5_qam256", 1, 1 << 17, 0, 3, 1.0, 1),        # f16 samples
    ("c2_qpsk", 1, 1 << 18, 1, 3, 1.0, None),       # f16 samples, ragged
    ("c3_qam16", 0, 1 << 21, 0, 2, 1.0, 0),         # TX small tiles, RX at-size tiles: two launches
    ("c3_qam16", 0, 1 << 22, 0, 2, 1.0, 0),         # the C3 call: two launches (faster at size)
]


@pytest.mark.parametrize("cfg,dtype,nsym,extra,periods,amp,want", CASES)
def test_fused_chain_equals_two_launches(m, o, torch_cuda, cfg, dtype, nsym, extra, periods, amp, want):
    torch = torch_cuda
    name, bps, L, sps = CONFIGS[cfg]
    nb = nsym * bps + extra
    hb = o.prng_bits(SEED + 900 + nsym % 1000, nb)
    bits = torch.from_numpy(hb).cuda()
    tdt = torch.float16 if dtype else torch.float32
    cap = (nb + bps) // bps * sps
    bufs = []
    for _ in range(2):
        bufs.append((torch.empty((cap, 2), dtype=tdt, device="cuda"),
                     torch.empty((cap // sps + 1, 2), dtype=tdt, device="cuda"),
                     torch.empty(cap // sps + 1, dtype=torch.uint8, device="cuda")))
    (txf, rxf), (txt, rxt) = make_pair(m, o, cfg, dtype, amp), make_pair(m, o, cfg, dtype, amp)
    fused = m.ChainPlan(txf, rxf, bits, *bufs[0])
    os.environ["MODEM_CHAIN_FUSED"] = "0"
    try:
        two = m.ChainPlan(txt, rxt, bits, *bufs[1])
    finally:
        del os.environ["MODEM_CHAIN_FUSED"]
    how = []
    for p in range(periods):
        n1, k1 = fused.run()
        n2, k2 = two.run()
        torch.cuda.synchronize()
        assert (n1, k1) == (n2, k2), p
        how.append(fused.fused)
        assert two.fused == 0, p
        (y1, q1, s1), (y2, q2, s2) = bufs
        assert torch.equal(y1[:n1], y2[:n2]), f"period {p}: samples differ"
        assert torch.equal(q1[:k1], q2[:k2]), f"period {p}: RX I/Q differ"
        assert torch.equal(s1[:k1], s2[:k2]), f"period {p}: decisions differ"
        assert txf.carrier.sample == txt.carrier.sample and rxf.carrier.sample == rxt.carrier.sample
    if want == 1:
        assert all(h >= 1 for h in how[1:]), how
    elif want == 0:
        assert not any(how), how
    if want == 1 and dtype == 0 and sps == 4:   # one RX tile per workgroup: the LDS hand-off form
        assert all(h == 2 for h in how[1:]), how
    print(f"\n[fused] {cfg} dtype {dtype} nsym {nsym}+{extra}b: fused per period {how}")
    # the last period's decisions are the symbols of the continuing stream
    nsym_p = (nb + 0) // bps
    stream = np.concatenate([hb] * periods)
    sent = sent_symbols(stream[: (len(stream) // bps) * bps], bps)
    c_prev = rxf.carrier.sample - 777 - n1                 # samples consumed before the last call
    k0 = max(0, -(-(c_prev - (L - 1)) // sps))             # its first kept instant
    got = bufs[0][2][:k1].cpu().numpy()
    assert nsym_p > 0 and np.array_equal(got, sent[k0: k0 + k1]), "decisions are not the symbols sent"


# the fused forms also exist with one RX output only (RXE_IQ: I/Q, no slicer output; RXE_SYM:
# QAM-axis decisions only): (config, dtype, symbols per period, periods, which output, form
# expected after period 0). QPSK's nearest-point decisions alone have no steady-state epilogue
# (rx_mfma_em: RXE_GEN), so that call takes the two launches.
ONE_OUTPUT_CASES = [
    ("c2_qpsk", 0, 1 << 18, 3, "iq", 2),       # chain_small: the LDS hand-off form
    ("c2_qpsk", 0, 1 << 18, 3, "sym", 0),      # nearest-point decisions only: two launches
    ("c3_qam16", 0, 1 << 16, 3, "iq", 2),
    ("c3_qam16", 0, 1 << 16, 3, "sym", 2),
    ("c5_qam256", 0, 1 << 17, 3, "iq", 1),     # chain_mfma: the drained-stores form
    ("c5_qam256", 0, 1 << 17, 3, "sym", 1),
]


@pytest.mark.parametrize("cfg,dtype,nsym,periods,which,form", ONE_OUTPUT_CASES)
def test_fused_chain_one_output(m, o, torch_cuda, cfg, dtype, nsym, periods, which, form):
    torch = torch_cuda
    name, bps, L, sps = CONFIGS[cfg]
    nb = nsym * bps
    hb = o.prng_bits(SEED + 77 + nsym % 1000, nb)
    bits = torch.from_numpy(hb).cuda()
    tdt = torch.float16 if dtype else torch.float32
    cap = nb // bps * sps
    bufs = []
    for _ in range(2):
        y = torch.empty((cap, 2), dtype=tdt, device="cuda")
        q = torch.empty((cap // sps + 1, 2), dtype=tdt, device="cuda") if which == "iq" else None
        s = torch.empty(cap // sps + 1, dtype=torch.uint8, device="cuda") if which == "sym" else None
        bufs.append((y, q, s))
    (txf, rxf), (txt, rxt) = make_pair(m, o, cfg, dtype, 1.0), make_pair(m, o, cfg, dtype, 1.0)
    fused = m.ChainPlan(txf, rxf, bits, *bufs[0])
    os.environ["MODEM_CHAIN_FUSED"] = "0"
    try:
        two = m.ChainPlan(txt, rxt, bits, *bufs[1])
    finally:
        del os.environ["MODEM_CHAIN_FUSED"]
    how = []
    for p in range(periods):
        n1, k1 = fused.run()
        n2, k2 = two.run()
        torch.cuda.synchronize()
        assert (n1, k1) == (n2, k2), p
        how.append(fused.fused)
        (y1, q1, s1), (y2, q2, s2) = bufs
        assert torch.equal(y1[:n1], y2[:n2]), f"period {p}: samples differ"
        if which == "iq":
            assert torch.equal(q1[:k1], q2[:k2]), f"period {p}: RX I/Q differ"
        else:
            assert torch.equal(s1[:k1], s2[:k2]), f"period {p}: decisions differ"
    assert all(h == form for h in how[1:]), how
    print(f"\n[fused one output] {cfg} {which}: forms {how}")
