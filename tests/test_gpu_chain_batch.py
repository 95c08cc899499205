"""modem_chain_batch_* (ChainBatchPlan): one period of a bank of independent channels — the
DigitalModulator's samples of each channel's bits (modulator.rs:85-100), then that channel's
Demodulator over them (demodulator.rs:44-56) — as one TX launch and one RX launch per group of
channels, with the handles and buffers checked once at create. Checked bit for bit against each
channel's own ChainPlan (the single-channel prepared step) over several periods, ragged groups
included, and for the refusals the create-time checks owe (mixed configurations, a handle twice,
host buffers)."""
import numpy as np
import pytest

from conftest import CONFIGS, product_phasor, sent_symbols

pytestmark = pytest.mark.gpu


def bank(m, torch, name, nch, nsamp, seed0, dtype=0):
    ph_name, bps, L, sps = CONFIGS[name]
    taps = m.rrc_taps(L, sps, 0.35)
    w = m.Freq(1, 4).sample_freq()
    tdt = torch.float16 if dtype else torch.float32
    out = []
    for c in range(nch):
        ph = product_phasor(m, ph_name)
        tx = m.DigitalModulator(m.Carrier(w), ph, sps, taps, dtype=dtype)
        rx = m.DemodulatorRx(m.Carrier(w), taps, decim=sps, decim_offset=L - 1, mix=m.MIX_COMPLEX,
                             slicer=product_phasor(m, ph_name).slicer(), in_dtype=dtype, out_dtype=dtype)
        bits = m.prng_bits(seed0 + c, nsamp // sps * bps)
        y = torch.empty((nsamp, 2), dtype=tdt, device="cuda")
        oiq = torch.empty((nsamp // sps, 2), dtype=tdt, device="cuda")
        osym = torch.empty(nsamp // sps, dtype=torch.uint8, device="cuda")
        out.append(dict(tx=tx, rx=rx, bits=bits, y=y, oiq=oiq, osym=osym))
    return out


@pytest.mark.parametrize("name,nch,group,nsamp,dtype", [("c4_qpsk", 5, 2, 1 << 18, 0),
                                                        ("c4_qpsk", 8, 8, 1 << 20, 0),
                                                        ("c3_qam16", 3, 4, 1 << 20, 0),
                                                        ("c4_qpsk", 4, 3, 1 << 20, 1)])
def test_batch_plan_equals_per_channel_plans(m, torch_cuda, name, nch, group, nsamp, dtype):
    torch = torch_cuda
    a = bank(m, torch, name, nch, nsamp, 0x5EED2000, dtype)
    b = bank(m, torch, name, nch, nsamp, 0x5EED2000, dtype)
    plan = m.ChainBatchPlan([d["tx"] for d in a], [d["rx"] for d in a], [d["bits"] for d in a],
                            [d["y"] for d in a], [d["oiq"] for d in a], [d["osym"] for d in a], group=group)
    singles = [m.ChainPlan(d["tx"], d["rx"], d["bits"], d["y"], d["oiq"], d["osym"]) for d in b]
    _, bps, L, sps = CONFIGS[name]
    for period in range(3):
        n, k = plan.run()
        for c, (sp, da, db) in enumerate(zip(singles, a, b)):
            n1, k1 = sp.run()
            assert (n[c], k[c]) == (n1, k1)
            assert torch.equal(da["y"].view(torch.int16), db["y"].view(torch.int16)), (period, c)
            assert torch.equal(da["oiq"][:k1].view(torch.int16), db["oiq"][:k1].view(torch.int16)), (period, c)
            assert torch.equal(da["osym"][:k1], db["osym"][:k1]), (period, c)
            assert da["tx"].carrier.sample == db["tx"].carrier.sample and da["rx"].carrier.sample == db["rx"].carrier.sample
        if period == 0:
            # the first period's decisions are the symbols sent (after the filter's lag)
            lag = (L - 1) // sps
            for d in a:
                sent = sent_symbols(d["bits"].cpu().numpy(), bps)
                got = d["osym"][: len(sent) - lag].cpu().numpy()
                assert np.array_equal(got, sent[: len(got)])


def test_batch_plan_refusals(m, torch_cuda):
    torch = torch_cuda
    a = bank(m, torch, "c4_qpsk", 2, 1 << 16, 1)
    c3 = bank(m, torch, "c3_qam16", 1, 1 << 16, 9)
    cols = lambda ds: ([d["tx"] for d in ds], [d["rx"] for d in ds], [d["bits"] for d in ds], [d["y"] for d in ds],
                       [d["oiq"] for d in ds], [d["osym"] for d in ds])
    with pytest.raises(m.ModemError) as e:              # two filter configurations in one bank
        m.ChainBatchPlan(*cols(a + c3))
    assert e.value.status == -2                         # MODEM_ERR_UNSUPPORTED
    with pytest.raises(m.ModemPanic):                   # a handle twice
        m.ChainBatchPlan(*cols([a[0], a[0]]))
    with pytest.raises(m.ModemPanic):                   # group outside 1..8
        m.ChainBatchPlan(*cols(a), group=9)
    t, r, bits, y, oiq, osym = cols(a)
    with pytest.raises(m.ModemPanic):                   # host memory
        m.ChainBatchPlan(t, r, [bits[0], bits[1].cpu().numpy()], y, oiq, osym)


def test_batch_plan_one_lane_equals_two_lanes(m, torch_cuda, monkeypatch):
    """MODEM_CHAIN_BATCH_LANES=1 (every launch on the caller's stream) and the default two lanes
    (groups alternating between the caller's stream and the plan's own) give the same samples,
    I/Q and decisions, bit for bit, and both finish on the caller's stream (no explicit sync of
    the plan's stream: torch's stream-ordered reads see the results)."""
    torch = torch_cuda
    outs = []
    for lanes in ("1", "2"):
        monkeypatch.setenv("MODEM_CHAIN_BATCH_LANES", lanes)
        a = bank(m, torch, "c4_qpsk", 6, 1 << 18, 0x5EED3000)
        plan = m.ChainBatchPlan([d["tx"] for d in a], [d["rx"] for d in a], [d["bits"] for d in a],
                                [d["y"] for d in a], [d["oiq"] for d in a], [d["osym"] for d in a], group=2)
        for _ in range(2):
            plan.run()
        s = torch.cuda.current_stream()
        outs.append([torch.cat([d["y"].view(torch.int32).flatten(), d["oiq"].view(torch.int32).flatten(),
                                d["osym"].to(torch.int32)]).clone() for d in a])
        s.synchronize()
    for x, y in zip(*outs):
        assert torch.equal(x, y)
