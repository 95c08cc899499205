#!/usr/bin/env python3
"""bench.py — Msamples/s through the TX+RX chain on MI355X (BASELINE.json `metric`).

A step is one pass of the hot path over one batch: bits (device-resident, one byte per bit)
-> TX kernel (symbol map + 129-tap RRC + carrier mix) -> 2^24 complex f32 samples in HBM
-> RX kernel (conjugate mix + matched filter at the symbol instants + slicer) -> decimated
I/Q + u8 decisions. Workload per GPU is BASELINE config 3 (16-QAM, 129-tap RRC, sps 4,
16 M samples); with --gpus N each rank runs its own independent channel (weak scaling, no
data-path collective — SURVEY.md §8e). `--config c4` is BASELINE config 4 as the one job it
names: 64 QPSK channels of 2^22 samples over the node, 64 / N per GPU (strong scaling), each
step running the rank's channels in groups of 8 (a TX launch, then an RX launch, per group;
consecutive groups alternate between two HIP streams: modem_chain_batch_*).
`value` = samples processed by all ranks / the max over ranks of the timed region. Before the warmup each rank runs --settle-ms (500) of untimed
back-to-back steps: the device clock dips for the first ~100 ms of sustained load, and the
driver's 20-step region (~1.2 ms) would otherwise measure that transient (tools/region_probe.py).

Also reported: the dominant kernel's HBM roofline (algorithmic bytes per launch / its mean
duration from HIP events on the launch stream; peak 8 TB/s), the whole chain's roofline,
and the CPU oracle (the reference loop restated in C) timed on a bounded sample on rank 0.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c4|c5|c5h]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

METRIC = "Msamples/s through TX+RX chain (129-tap RRC, f32 I/Q); % HBM roofline"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
SEED = 0x5EED0000

# name: (phasor, bps, ntaps, sps, samples per channel, channels per GPU, dtype, description)
WORKLOADS = {
    "c3": ("qam16", 4, 129, 4, 1 << 24, 1, 0,
           "c3: 16-QAM, 129-tap RRC TX + matched-filter RX loopback, 2^24 complex f32 samples/GPU"),
    "c2": ("qpsk", 2, 65, 4, 1 << 20, 1, 0, "c2: QPSK, 65-tap RRC, 2^20 complex f32 samples/GPU"),
    "c4": ("qpsk", 2, 65, 4, 1 << 22, 64, 0,
           "c4: 64 independent QPSK channels x 2^22 complex f32 samples over the node (64/N per GPU), 65-tap RRC"),
    "c5": ("qam256", 8, 513, 8, 1 << 26, 1, 0, "c5: 256-QAM, 513-tap RRC, sps 8, 2^26 complex f32 samples/GPU"),
    "c5h": ("qam256", 8, 513, 8, 1 << 26, 1, 1, "c5: 256-QAM, 513-tap RRC, sps 8, 2^26 complex f16 samples/GPU"),
}

# BASELINE config 4 is one fixed job, "64 independent QPSK channels x 4 M samples, sharded 8 per
# GPU across 8 x MI355X": its channel count is the whole node's, and --gpus N gives each rank
# 64 / N of them (strong scaling: the 1-, 2-, 4- and 8-GPU lines time the same 2^28 samples).
# Every other config's count is per GPU (weak scaling).
FIXED_TOTAL = {"c4"}
# channels per TX / RX launch pair of a multi-channel step (the batch entry points take up to 8
# per launch, modem_internal.h kBatchMax); the groups run one after another, TX then RX each
GROUP_DEFAULT = {"c4": 8}


def rank_workload(config, world):
    """The workload tuple one rank runs and the line's scaling: for FIXED_TOTAL configs the
    channel count becomes count / world (it must divide), else it is already per GPU."""
    wl = WORKLOADS[config]
    if config not in FIXED_TOTAL:
        return wl, "weak"
    total = wl[5]
    if world < 1 or total % world:
        raise ValueError(f"config {config}: {total} channels do not split over {world} GPUs")
    return wl[:5] + (total // world,) + wl[6:], "strong"


def algorithmic_bytes(bps, ntaps, sps, nsamp, dtype):
    """bits in + TX write (TX); RX read + decimated I/Q + u8 decision (RX)."""
    S = 4 if dtype == 1 else 8
    nsym = nsamp // sps
    nout = nsym                      # steady state: one kept instant per symbol period
    tx = nsym * bps + nsamp * S
    rx = nsamp * S + nout * (S + 1)
    return tx, rx, nout


def channel_seed(rank, nch, c):
    """Channel c of rank `rank` (nch channels per rank) is global channel rank * nch + c: every
    rank owns distinct channels (no exchange), and a FIXED_TOTAL job's ranks cover exactly its
    channels 0 .. total - 1, whatever the node size."""
    return SEED + rank * nch + c


class GpuRunner:
    """The product path: rust_modem_amd handles on this rank's GPU, buffers resident in HBM."""

    def __init__(self, wl, rank, device, streams=1, batch=False, amplitude=1.0, group=0):
        import torch
        import __graft_entry__ as g
        self.torch = torch
        m = g.package()
        self._m = m
        name, bps, L, sps, nsamp, nch, dtype, _ = wl
        self.bps, self.L, self.sps, self.nsamp, self.nch, self.dtype = bps, L, sps, nsamp, nch, dtype
        torch.cuda.set_device(device)
        self.stream = torch.cuda.current_stream()
        # channels are independent streams of samples: channel c's TX and RX
        # are queued on HIP stream c % streams, so the kernels of different channels overlap
        # (one channel's tail with the next one's head); stream 0 is the current stream
        self.streams = [self.stream] + [torch.cuda.Stream() for _ in range(max(1, streams) - 1)]
        # or all channels through the batch entry points (one TX and one RX launch per step)
        self.batch = batch
        taps = m.rrc_taps(L, sps, 0.35)
        w = m.Freq(1, 4).sample_freq()
        # amplitude != 1 scales the constellation (and with it the RX input and the slicer)
        A = float(amplitude)
        ph = {"qpsk": lambda: m.QPSK(0.0, A), "qam16": lambda: m.QAM(4, 0.0, A),
              "qam256": lambda: m.QAM(8, 0.0, A)}[name]
        self.ch = []
        nbits = nsamp // sps * bps
        for c in range(nch):
            seed = channel_seed(rank, nch, c)
            bits = m.prng_bits(seed, nbits, device=device)
            tx = m.DigitalModulator(m.Carrier(w), ph(), sps, taps, dtype=dtype, device=device)
            rx = m.DemodulatorRx(m.Carrier(w), taps, decim=sps, decim_offset=L - 1, mix=m.MIX_COMPLEX,
                                 slicer=ph().slicer(), in_dtype=dtype, out_dtype=dtype, device=device)
            # every handle of this rank lives on the rank's GPU (ranks that share one GPU in the
            # tests would otherwise hide a handle left on device 0)
            assert tx.device == device and rx.device == device, (tx.device, rx.device, device)
            tdt = torch.float16 if dtype == 1 else torch.float32
            y = torch.empty((nsamp, 2), dtype=tdt, device=f"cuda:{device}")
            nout = rx.noutputs(nsamp)
            oiq = torch.empty((nsamp // sps, 2), dtype=tdt, device=f"cuda:{device}")
            osym = torch.empty(nsamp // sps, dtype=torch.uint8, device=f"cuda:{device}")
            self.ch.append(dict(bits=bits, tx=tx, rx=rx, y=y, oiq=oiq, osym=osym, nout=nout))
        if batch:       # prepared batch calls over the fixed per-channel buffers
            # groups of `group` channels (all of them when 0): the step runs each group's TX
            # launch and then its RX launch, so that a group's samples are re-read while they
            # are still in the Infinity Cache (64 channels x 32 MiB at once would not be)
            g = group if group > 0 else nch
            self.group = min(g, nch)
            self._txp, self._rxp = [], []
            for c0 in range(0, nch, self.group):
                ch = self.ch[c0:c0 + self.group]
                self._txp.append(m.TxBatchPlan([d["tx"] for d in ch], [d["bits"] for d in ch], [d["y"] for d in ch]))
                self._rxp.append(m.RxBatchPlan([d["rx"] for d in ch], [d["y"] for d in ch], [d["oiq"] for d in ch],
                                               [d["osym"] for d in ch]))
            # the step: one prepared C call for every group (modem_chain_batch_*: the handles and
            # buffers checked once, not per call), and the first group's pair alone for the chain leg
            self._cbp = self._cbp0 = None
            if hasattr(m, "ChainBatchPlan") and hasattr(m.load_library(), "modem_chain_batch_run"):
                def plan(chs):
                    return m.ChainBatchPlan([d["tx"] for d in chs], [d["rx"] for d in chs], [d["bits"] for d in chs],
                                            [d["y"] for d in chs], [d["oiq"] for d in chs], [d["osym"] for d in chs],
                                            group=self.group)
                self._cbp = plan(self.ch)
                self._cbp0 = plan(self.ch[:self.group])
            # experiment switch (A/B only): MODEM_BENCH_BATCH=plans runs the per-group TX / RX
            # batch plans instead of the prepared call
            if os.environ.get("MODEM_BENCH_BATCH", "") == "plans":
                self._cbp = None
        # one prepared C call per channel and step (modem_chain_run = modem_tx_process +
        # modem_rx_process on the fixed device buffers): the TX and RX kernels of the step with
        # the buffers checked once, so that the host stays ahead of small steps (C2)
        chain = hasattr(m.load_library(), "modem_chain_run")   # (experiment builds of older sources: no)
        self._plans = None if batch or not chain else [
            m.ChainPlan(d["tx"], d["rx"], d["bits"], d["y"], d["oiq"], d["osym"]) for d in self.ch]
        torch.cuda.synchronize()

    def tx(self, c, stream=None):
        d = self.ch[c]
        d["tx"].process(d["bits"], out=d["y"], stream=stream)

    def rx(self, c, stream=None):
        d = self.ch[c]
        d["rx"].process(d["y"], out_iq=d["oiq"], out_sym=d["osym"], stream=stream)

    def step(self):
        if self.batch:
            if self._cbp is not None:
                self._cbp.run()
                return
            for txp, rxp in zip(self._txp, self._rxp):
                txp.run()
                rxp.run()
            return
        if len(self.streams) == 1 and self._plans:
            for pl in self._plans:
                pl.run()
            return
        if len(self.streams) > 1:
            for st in self.streams[1:]:
                st.wait_stream(self.stream)     # the step starts after what precedes it
        for c in range(self.nch):
            st = self.streams[c % len(self.streams)]
            self.tx(c, st)
            self.rx(c, st)
        for st in self.streams[1:]:
            self.stream.wait_stream(st)         # and ends when every channel has

    def sync(self):
        self.torch.cuda.synchronize()

    def fused(self):
        """The form of the last step (modem_chain_fused): 1 one launch per channel whose RX
        re-reads the sample buffer it wrote (chain_mfma), 2 one launch with the samples handed
        to the RX in LDS (chain_small: the buffer is written, not re-read), 0 two launches."""
        return self._plans[0].fused if self._plans and self._plans[0].fused > 0 else 0

    def two_launch_chain_ms(self, budget_ms=10.0, rounds=5):
        """The canonical two-stage loopback (TX launch, then an RX launch that
        re-reads the sample buffer from memory) for channel 0 when the product step is a fused
        launch: fresh handles of the same configuration and a ChainPlan created with
        MODEM_CHAIN_FUSED=0, over the same buffers, timed as the legs are (median of rounds)."""
        torch, m = self.torch, self._m
        d = self.ch[0]
        old = os.environ.get("MODEM_CHAIN_FUSED")
        os.environ["MODEM_CHAIN_FUSED"] = "0"
        try:
            tx = m.DigitalModulator(m.Carrier(d["tx"].carrier.sample_freq), d["tx"].phasor, self.sps,
                                    d["tx"].taps, dtype=self.dtype, device=d["tx"].device)
            rx = m.DemodulatorRx(m.Carrier(d["rx"].carrier.sample_freq), d["rx"].taps, decim=self.sps,
                                 decim_offset=self.L - 1, mix=m.MIX_COMPLEX, slicer=d["rx"]._slicer,
                                 in_dtype=self.dtype, out_dtype=self.dtype, device=d["rx"].device)
            plan = m.ChainPlan(tx, rx, d["bits"], d["y"], d["oiq"], d["osym"])
        finally:
            if old is None:
                del os.environ["MODEM_CHAIN_FUSED"]
            else:
                os.environ["MODEM_CHAIN_FUSED"] = old
        for _ in range(8):
            plan.run()
        torch.cuda.synchronize()
        assert plan.fused == 0
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(self.stream)
        for _ in range(8):
            plan.run()
        ev[1].record(self.stream)
        torch.cuda.synchronize()
        n = max(200, int(budget_ms / max(ev[0].elapsed_time(ev[1]) / 8, 1e-4)) + 1)
        res = []
        for _ in range(rounds):
            for _ in range(n):          # untimed backlog
                plan.run()
            ev[0].record(self.stream)
            for _ in range(n):
                plan.run()
            ev[1].record(self.stream)
            torch.cuda.synchronize()
            res.append(ev[0].elapsed_time(ev[1]) / n)
        return sorted(res)[rounds // 2]

    def launch_channels(self):
        """Channels one timed TX or RX launch covers (the legs time the first group)."""
        return self.group if self.batch else 1

    def _tx_all(self):
        if self.batch:
            self._txp[0].run()
        else:
            self.tx(0)

    def _step_timed(self):
        if self.batch:
            if self._cbp0 is not None:
                self._cbp0.run()
                return
            self._txp[0].run()
            self._rxp[0].run()
        elif self._plans:
            self._plans[0].run()
        else:
            self.tx(0)
            self.rx(0)

    def _rx_all(self):
        if self.batch:
            self._rxp[0].run()
        else:
            self.rx(0)

    def kernel_times_ms(self, budget_ms=10.0, min_reps=200, rounds=5):
        """Mean device time of one TX launch, one RX launch and one TX+RX pair, from HIP events
        on the launch stream (channel 0's launches, or the first channel group's batch launches). Each leg is timed directly as back-to-back launches between two events: TX
        alone, RX alone (re-reading the sample buffer the last TX wrote, resident in HBM), and
        the chain. The amount of work is a device-time budget, independent of --steps (the
        driver's 20 steps are ~1 ms of C3, while the clock settles over the first few ms of
        back-to-back launches: profiles/r02_wall_probe.txt): per leg and round an untimed
        backlog of >= budget_ms (so that events are never recorded while the device waits for
        the host), then max(min_reps, budget_ms of launches) timed. Rounds are interleaved and
        the medians reported (a single round swings by a few us with the clocks)."""
        torch = self.torch
        legs = (("chain", self._step_timed), ("tx", self._tx_all), ("rx", self._rx_all))
        est = {}
        for name, fn in legs:                  # per-launch estimate, for the budget
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            for _ in range(4):
                fn()
            ev[0].record(self.stream)
            for _ in range(8):
                fn()
            ev[1].record(self.stream)
            torch.cuda.synchronize()
            est[name] = max(ev[0].elapsed_time(ev[1]) / 8, 1e-4)
        res = {"tx": [], "rx": [], "chain": []}
        reps = {}
        for _ in range(rounds):
            for name, fn in legs:
                n_back = max(8, int(budget_ms / est[name]) + 1)
                n = reps[name] = max(min_reps, int(budget_ms / est[name]) + 1)
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                for _ in range(n_back):
                    fn()
                ev[0].record(self.stream)
                for _ in range(n):
                    fn()
                ev[1].record(self.stream)
                torch.cuda.synchronize()
                res[name].append(ev[0].elapsed_time(ev[1]) / n)
        med = {k: sorted(v)[rounds // 2] for k, v in res.items()}
        self.leg_reps = reps
        return med["tx"], med["rx"], med["chain"]

    def sent_symbols(self, c):
        torch = self.torch
        b = self.ch[c]["bits"].view(-1, self.bps).to(torch.int64)
        wts = torch.tensor([1 << (self.bps - 1 - k) for k in range(self.bps)], device=b.device)
        return (b * wts).sum(1).to(torch.uint8)

    def check(self):
        """The decisions of every channel equal the symbols that channel sent (size-independent
        parity property)."""
        torch = self.torch
        for c, d in enumerate(self.ch):
            sent = self.sent_symbols(c)
            # the stream continues across steps; the last RX call of a channel decides symbols
            # k in [j*nsym - (L-1)/sps, ...) of its stream, and symbol k of call j is symbol
            # (k mod nsym) of the (repeated) batch
            nout = d["nout"]
            got = d["osym"][:nout]
            lag = (self.L - 1 + self.sps - 1) // self.sps
            nsym = self.nsamp // self.sps
            idx = (torch.arange(nout, device=got.device) - lag) % nsym
            if not torch.equal(got, sent[idx]):
                return False
        return True

    def gather_ms(self, reps=5):
        """SURVEY.md §8e's final host gather: the D2H copy of this GPU's u8 decisions (every
        channel) into pinned host memory, on the launch stream, timed by HIP events (median of
        `reps`). Returns (ms, bytes)."""
        torch = self.torch
        host = [torch.empty(d["nout"], dtype=torch.uint8, pin_memory=True) for d in self.ch]
        nbytes = sum(d["nout"] for d in self.ch)
        ts = []
        for _ in range(reps):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record(self.stream)
            for h, d in zip(host, self.ch):
                h.copy_(d["osym"][:d["nout"]], non_blocking=True)
            ev[1].record(self.stream)
            torch.cuda.synchronize()
            ts.append(ev[0].elapsed_time(ev[1]))
        self.gathered = host
        return sorted(ts)[reps // 2], nbytes


def _cpu_threads():
    """Host threads for the multi-core leg: the CPUs this process may run on, at most 16 (the
    GPU box's CPU share per GPU; nproc there shows the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_baseline(wl, nsamp_cpu, threads=None):
    """The CPU oracle (the reference loop structure restated in C) on a bounded sample of the
    workload: one thread on `nsamp_cpu` samples, then `threads` threads on independent channels
    (seed + c, as the GPU channels) of nsamp_cpu / 2 samples each, as SURVEY.md §8d asks (the
    ctypes calls release the GIL, so the threads run the C loop in parallel). The reported
    value is the multi-core rate; the single-thread rate is kept beside it."""
    import __graft_entry__ as g
    from concurrent.futures import ThreadPoolExecutor
    o = g.oracle()
    name, bps, L, sps = wl[0], wl[1], wl[2], wl[3]
    taps = o.rrc_taps(L, sps, 0.35)
    w = o.sample_freq(1, 4)

    def chain(seed, nsamp):
        p = {"qpsk": lambda: o.new_phasor(o.QPSK, 0.0, 1.0), "qam16": lambda: o.new_phasor(o.QAM, 4, 0.0, 1.0),
             "qam256": lambda: o.new_phasor(o.QAM, 8, 0.0, 1.0)}[name]()
        sl = o.qam_axis_slicer(bps, 1.0) if name.startswith("qam") else \
            o.make_slicer(o.SLICER_NEAREST, bps, o.phasor_lut(p))
        bits = o.prng_bits(seed, nsamp // sps * bps)
        y = o.tx_chain(p, bits, sps, taps, w, 0)
        o.rx_chain(y, w, 0, o.MIX_COMPLEX, taps, sps, L - 1, sl)
        return len(y)

    t0 = time.perf_counter()
    n1 = chain(SEED, nsamp_cpu)
    dt1 = time.perf_counter() - t0
    T = threads or _cpu_threads()
    per = max(sps, nsamp_cpu // 2 // sps * sps)
    with ThreadPoolExecutor(T) as ex:
        t0 = time.perf_counter()
        nt = sum(ex.map(lambda c: chain(SEED + c, per), range(T)))
        dtT = time.perf_counter() - t0
    return {"value": round(nt / dtT / 1e6, 4), "unit": "Msamples/s", "cores": T, "kind": "port",
            "sample": f"{T} threads x {per} samples ({per // sps} symbols) of the same workload on independent "
                      f"channels, TX+RX oracle loop (per-sample FIRFilter at full rate, glibc sin/cos), "
                      f"{dtT:.1f} s",
            "single_thread": {"value": round(n1 / dt1 / 1e6, 4), "cores": 1,
                              "sample": f"{n1} samples ({n1 // sps} symbols), {dt1:.1f} s"},
            "cpu": _cpu_model()}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def pmc_traffic(config):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (None if absent)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(config)
    except (OSError, ValueError):
        return None


def run(args, runner_factory, dist=None, rank=0, world=1):
    wl, scaling = rank_workload(args.config, world)
    name, bps, L, sps, nsamp, nch, dtype, desc = wl
    r = runner_factory(wl, rank)
    # Clock settling (untimed): back-to-back steps for --settle-ms of wall time before the
    # warmup. The device clock dips for the first ~100+ ms of sustained load: the same C3 chain
    # step takes 60-71 us in 20-step regions there against 58.5-59 once settled, on one box
    # (tools/region_probe.py, profiles/r03_region_probe.txt); the driver's 20-step region
    # (~1.2 ms) otherwise measures where it falls in that transient, not the steady state the
    # metric is about. The timed region below is still exactly --steps full steps.
    if dist is not None:
        dist.barrier()      # the ranks settle together and reach the timing barrier together
    settle = settle_clocks(r, getattr(args, "settle_ms", 0.0))
    for _ in range(args.warmup):
        r.step()
    r.sync()
    if dist is not None:
        dist.barrier()
    r.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        r.step()
    r.sync()
    if dist is not None:
        dist.barrier()
    r.sync()
    dt = time.perf_counter() - t0
    if dist is not None:
        dt = dist.max_over_ranks(dt)
    total = nsamp * nch * args.steps * world
    value = total / dt / 1e6
    ok = r.check()
    g_ms, g_bytes = r.gather_ms()
    if dist is not None:
        ok = dist.max_over_ranks(0.0 if ok else 1.0) == 0.0
        g_ms = dist.max_over_ranks(g_ms)
    t_tx, t_rx, t_chain = r.kernel_times_ms()
    b_tx, b_rx, nout = algorithmic_bytes(bps, L, sps, nsamp, dtype)
    per_launch = r.launch_channels() if hasattr(r, "launch_channels") else 1   # channels one timed launch covers
    b_tx, b_rx, nsamp_launch = b_tx * per_launch, b_rx * per_launch, nsamp * per_launch
    # the step's kernels: one fused launch (small calls, modem_chain.hip) or the TX and RX
    # launches, of which the longer is the dominant kernel
    fused = getattr(r, "fused", lambda: 0)()
    S = 4 if dtype == 1 else 8
    # bytes the step's launches actually move: the LDS hand-off form (fused == 2) writes the
    # sample buffer but hands the samples to the RX in LDS, so it is priced without the re-read
    b_moved = b_tx + b_rx - (nsamp_launch * S if fused == 2 else 0)
    if fused == 2:
        dom = ("chain (fused TX+RX launch, samples handed to the RX in LDS: buffer written, not re-read)",
               t_chain, b_moved, "chain")
    elif fused:
        dom = ("chain (fused TX+RX launch, RX re-reads the sample buffer)", t_chain, b_moved, "chain")
    else:
        dom = ("rx", t_rx, b_rx, "rx") if t_rx >= t_tx else ("tx", t_tx, b_tx, "tx")
    two = None
    if fused and hasattr(r, "two_launch_chain_ms"):
        t_two = r.two_launch_chain_ms()
        g_two = (b_tx + b_rx) / (t_two * 1e-3) / 1e9
        two = {"chain_ms": round(t_two, 5), "achieved": round(g_two, 1), "frac": round(g_two / HBM_PEAK_GBS, 4),
               "device_msamples_per_s": round(nsamp_launch / (t_two * 1e-3) / 1e6, 1),
               "what": "the canonical two-stage loopback (TX launch, RX launch re-reading the sample buffer; "
                       "MODEM_CHAIN_FUSED=0), HIP events, priced at the algorithmic bytes"}
    achieved = dom[2] / (dom[1] * 1e-3) / 1e9
    traffic = pmc_traffic(args.config)
    # PMC bytes of the dominant kernel per launch (profiles/pmc_traffic.json; for a fused chain only
    # when its entry was measured on the same form)
    dom_traffic = traffic.get(dom[3]) if isinstance(traffic, dict) else None
    if dom[3] == "chain" and isinstance(traffic, dict) and traffic.get("chain_form") != fused:
        dom_traffic = None
    if isinstance(traffic, dict) and traffic.get("channels_per_launch", per_launch) != per_launch:
        dom_traffic = None          # measured on another launch size (channel group)
    chain_gbs = b_moved / (t_chain * 1e-3) / 1e9
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "Msamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "settle": settle,
        "ms_per_step": round(dt / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f16" if dtype == 1 else "f32",
        "data": f"synthetic: splitmix64 bits (seed 0x5EED0000 + channel), one byte per bit, device-resident",
        "config": {"workload": desc, "samples_per_gpu_per_step": nsamp * nch, "channels_per_gpu": nch,
                   "channels_total": nch * world, "channels_per_launch": per_launch,
                   "streams_per_gpu": len(getattr(r, "streams", [None])),
                   "channel_batch": bool(getattr(r, "batch", False)),
                   "ntaps": L, "sps": sps, "bits_per_symbol": bps, "rrc_beta": 0.35,
                   "carrier": "Freq::new(1, 4) (fs/4)", "parallelism": f"{world} independent channel set(s), "
                   "one per GPU, no collectives" + (f"; one job of {nch * world} channels, {nch} per GPU"
                                                    if scaling == "strong" else "") + (f" (timing barrier and max over ranks: "
                                                    f"{dist.td.get_backend()})" if dist is not None else "")},
        "roofline": {"bound": "hbm", "kernel": dom[0], "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": dom_traffic,
                     "algorithmic_bytes_per_launch": dom[2], "mean_launch_ms": round(dom[1], 5)},
        "chain_roofline": {"tx_ms": round(t_tx, 5), "rx_ms": round(t_rx, 5), "chain_ms": round(t_chain, 5),
                           "tx_bytes": b_tx, "rx_bytes": b_rx,
                           "bytes_per_sample": round((b_tx + b_rx) / nsamp_launch, 4),
                           "moved_bytes_per_sample": round(b_moved / nsamp_launch, 4),
                           "fused": bool(fused), "fused_form": fused,
                           "two_launch": two,
                           "rx_in_chain_ms": None if fused else round(t_chain - t_tx, 5),
                           "rx_in_chain_frac": None if fused else
                           round(b_rx / ((t_chain - t_tx) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                           "reps_per_leg": getattr(r, "leg_reps", None),
                           "achieved": round(chain_gbs, 1), "frac": round(chain_gbs / HBM_PEAK_GBS, 4),
                           "device_msamples_per_s": round(nsamp_launch / (t_chain * 1e-3) / 1e6, 1)},
        "decisions_match_sent": ok,
        # the host gather of the decisions, timed separately from `value`
        "gather": {"ms": round(g_ms, 5), "bytes_per_gpu": g_bytes,
                   "gb_per_s": round(g_bytes / (g_ms * 1e-3) / 1e9, 2) if g_ms > 0 else None,
                   "what": "D2H of every rank's u8 decisions (all channels) into pinned host memory, "
                           "HIP events on the launch stream, max over ranks; not in the timed region"},
    }
    if args.amplitude != 1.0:
        out["config"]["amplitude"] = args.amplitude
    if rank == 0 and world == 1 and args.config == "c3" and not args.no_out_of_cache:
        del r
        out["roofline_out_of_cache"] = out_of_cache_roofline(runner_factory)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(wl, args.cpu_samples)
    return out


def settle_clocks(r, settle_ms):
    """Back-to-back steps for settle_ms of wall time, untimed, queued in batches of up to ~5 ms
    of device work (the queue drains only between batches; a batch is sized from the previous
    one's rate, so that ranks that start together end within ~5 ms of each other). Returns what
    ran, for the JSON line."""
    if settle_ms <= 0:
        return None
    t0 = time.perf_counter()
    n, batch = 0, 1
    while True:
        tb = time.perf_counter()
        for _ in range(batch):
            r.step()
        r.sync()
        n += batch
        now = time.perf_counter()
        left = settle_ms * 1e-3 - (now - t0)
        if left <= 0:
            break
        per = max((now - tb) / batch, 1e-6)
        batch = max(1, min(int(min(left, 0.005) / per) + 1, 100000))
    return {"ms": round((time.perf_counter() - t0) * 1e3, 1), "steps": n,
            "what": "untimed back-to-back steps before the warmup (device clock settling)"}


def out_of_cache_roofline(runner_factory, config="c5"):
    """The C3 chain's 2^24-sample working set (~180 MB) fits the 256 MiB Infinity Cache, whose
    hits FETCH_SIZE and the roofline count like HBM reads; C5 f32 (512 MiB of samples) does
    not. Its RX launch and chain, timed the same way, give the out-of-cache figure."""
    wl = WORKLOADS[config]
    name, bps, L, sps, nsamp, nch, dtype, desc = wl
    r = runner_factory(wl, 0)
    for _ in range(3):
        r.step()
    r.sync()
    t_tx, t_rx, t_chain = r.kernel_times_ms(10, rounds=3)
    b_tx, b_rx, _ = algorithmic_bytes(bps, L, sps, nsamp, dtype)
    rx_gbs = b_rx / (t_rx * 1e-3) / 1e9
    chain_gbs = (b_tx + b_rx) / (t_chain * 1e-3) / 1e9
    return {"workload": desc, "kernel": "rx", "achieved": round(rx_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(rx_gbs / HBM_PEAK_GBS, 4), "mean_launch_ms": round(t_rx, 5),
            "algorithmic_bytes_per_launch": b_rx, "tx_ms": round(t_tx, 5), "chain_ms": round(t_chain, 5),
            "chain_frac": round(chain_gbs / HBM_PEAK_GBS, 4),
            "chain_msamples_per_s": round(nsamp / (t_chain * 1e-3) / 1e6, 1)}


class _Dist:
    """Timing barrier and max-over-ranks reduction. `device` None: gloo on the host (ranks that
    share a GPU, or CPU tests); else nccl (= RCCL) on this rank's GPU."""

    def __init__(self, td, device):
        self.td, self.device = td, device

    def barrier(self):
        if self.device is not None:
            self.td.barrier(device_ids=[self.device])
        else:
            self.td.barrier()

    def max_over_ranks(self, x):
        import torch
        t = torch.tensor([x], dtype=torch.float64,
                         device=f"cuda:{self.device}" if self.device is not None else "cpu")
        self.td.all_reduce(t, op=self.td.ReduceOp.MAX)
        return float(t.item())


def _parser():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    # GPUs of this node: under a launcher (torch.distributed.run: WORLD_SIZE set) it must equal
    # WORLD_SIZE; without one, N > 1 starts N rank processes itself (one per GPU)
    ap.add_argument("--gpus", type=int, default=1)
    # 2000 steps of C3 are ~120 ms of device time: the timed region's fixed start/stop cost
    # (~0.2 ms: first launch, final sync) stays well under 1 % of it. The warmup is as long:
    # the first few ms of back-to-back launches run slower (clocks settling) — C3 measured
    # 61.0 us/step timed after 50 warmup steps, 58.5 us after 2000 (tools/wall_probe.sh,
    # profiles/r02_wall_probe.txt)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=2000)
    ap.add_argument("--config", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--settle-ms", type=float, default=500.0)
    ap.add_argument("--cpu-samples", type=int, default=1 << 25)   # ~15 s of oracle work
    ap.add_argument("--no-cpu-baseline", action="store_true")
    # HIP streams the channels of a multi-channel config are spread over (0: one per channel,
    # at most 4 = the box's GPU_MAX_HW_QUEUES)
    ap.add_argument("--streams", type=int, default=0)
    # multi-channel configs go through modem_*_process_batch (one launch for all channels of
    # the step) unless --no-batch, which queues per-channel calls on --streams streams
    ap.add_argument("--no-batch", action="store_true")
    # channels per TX / RX launch pair of a batched step (0: the config's default, GROUP_DEFAULT)
    ap.add_argument("--group", type=int, default=0)
    # constellation amplitude (1.0 = BASELINE); e.g. 1/16 puts the RX input below 2^-3
    ap.add_argument("--amplitude", type=float, default=1.0)
    # skip the C5 f32 out-of-Infinity-Cache roofline measured after the C3 line
    ap.add_argument("--no-out-of-cache", action="store_true")
    return ap


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _wait_ranks(procs, timeout_s, poll_s=0.2):
    """Wait for every rank process. A rank that exits non-zero, or the overall timeout, ends the
    rest (terminate, then kill); returns the exit codes (the timeout reports 124 for the ranks
    it ended, as `timeout` does) and the code of the first rank seen failing (None if none)."""
    t0 = time.monotonic()
    rcs = [None] * len(procs)
    failed = timed_out = False
    first_bad = None
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
                if rcs[i] not in (None, 0):
                    failed = True
                    if first_bad is None:
                        first_bad = rcs[i]
        if failed or time.monotonic() - t0 > timeout_s:
            timed_out = not failed
            break
        time.sleep(poll_s)
    if failed or timed_out:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for i, p in enumerate(procs):
            try:
                p.wait(10)
            except Exception:
                p.kill()
                p.wait()
            if rcs[i] is None:
                rcs[i] = 124 if timed_out else p.returncode
    if timed_out:
        first_bad = 124
    return rcs, first_bad


def _spawn(args, argv, timeout_s=1800.0):
    """--gpus N without a launcher: N fresh rank processes (`python bench.py` with RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_* set), started before this process touches the GPU (it
    never does). Rank 0's JSON line is printed and returned; the exit status is the worst of
    the ranks'. All ranks are polled: when one exits non-zero the others are terminated (a rank
    left waiting in a barrier for a dead peer would otherwise hang the bench), and the whole
    run is bounded by `timeout_s`."""
    import subprocess
    import tempfile
    env = dict(os.environ, WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    procs = []
    # rank 0's stdout goes to a file, so that polling never blocks on a full pipe
    out_f = tempfile.TemporaryFile(mode="w+")
    for r in range(args.gpus):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=e,
                                      stdout=out_f if r == 0 else subprocess.DEVNULL, text=True))
    rcs, first_bad = _wait_ranks(procs, timeout_s)
    out_f.seek(0)
    out0 = out_f.read()
    out_f.close()
    line = None
    for ln in (out0 or "").splitlines():
        if ln.startswith("{"):
            line = ln
    if line is not None:
        print(line, flush=True)
    if first_bad is not None:
        raise SystemExit(first_bad)
    bad = [rc for rc in rcs if rc != 0]
    if bad:
        raise SystemExit(bad[0])
    if line is None:
        raise SystemExit(1)
    return json.loads(line)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = _parser().parse_args(argv)
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    try:
        rank_workload(args.config, args.gpus)
    except ValueError as e:               # before any GPU work: a node size the job does not split over
        print(f"bench.py: {e}", file=sys.stderr)
        raise SystemExit(2)
    wenv = os.environ.get("WORLD_SIZE")
    if wenv is None and args.gpus > 1:
        return _spawn(args, argv)
    world = int(wenv or "1")
    if wenv is not None and world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} disagrees with WORLD_SIZE={world} of the launcher",
              file=sys.stderr)
        raise SystemExit(2)
    wl, _ = rank_workload(args.config, world)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    device = local
    if wenv is not None:      # under a launcher (any world size, so one rank exercises RCCL too)
        import torch
        import torch.distributed as td
        ndev = torch.cuda.device_count()
        if ndev < 1:
            raise SystemExit("bench.py: no GPU")
        device = local % ndev
        torch.cuda.set_device(device)
        if world <= ndev:     # one GPU per rank: RCCL for the barrier and the max over ranks
            td.init_process_group("nccl", device_id=torch.device(f"cuda:{device}"))
            dist = _Dist(td, device)
        else:                 # ranks share a GPU (a one-GPU box): RCCL cannot, gloo on the host
            td.init_process_group("gloo")
            dist = _Dist(td, None)
    nch = wl[5]
    nst = args.streams if args.streams > 0 else min(nch, 4)
    batch = nch > 1 and not args.no_batch
    group = args.group if args.group > 0 else GROUP_DEFAULT.get(args.config, 0)
    out = run(args, lambda wl, r: GpuRunner(wl, r, device, 1 if batch else nst, batch, args.amplitude, group),
              dist, rank, world)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.td.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
