"""bench.py's multi-rank harness with world_size 2 over gloo on the CPU.

Channels shard across ranks with no data-path collective: each rank runs its own channel set,
the only communication is the timing barrier and the max-over-ranks reduction. The GPU runner
is replaced by a small CPU runner built on the oracle (test infrastructure), so the test covers
the harness arithmetic and the rank → channel assignment, not the kernels.
"""
import json
import os
import socket
import time

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class CpuRunner:
    """Oracle TX -> RX on a tiny channel per rank (stand-in for bench.GpuRunner)."""

    def __init__(self, wl, rank, o, bench):
        name, bps, L, sps, nsamp, nch, dtype, _ = wl
        self.o, self.rank, self.bps, self.L, self.sps = o, rank, bps, L, sps
        self.p = o.new_phasor(o.QAM, bps, 0.0, 1.0)
        self.taps = o.rrc_taps(L, sps, 0.35)
        self.w = o.sample_freq(1, 4)
        self.seeds = [bench.channel_seed(rank, nch, c) for c in range(nch)]
        self.bits = [o.prng_bits(s, nsamp // sps * bps) for s in self.seeds]
        self.steps = 0

    def step(self):
        o = self.o
        self.out = []
        for b in self.bits:
            y = o.tx_chain(self.p, b, self.sps, self.taps, self.w, 0)
            self.out.append(o.rx_chain(y, self.w, 0, o.MIX_COMPLEX, self.taps, self.sps, self.L - 1,
                                       o.qam_axis_slicer(self.bps, 1.0))[1])
        if self.rank == 1:
            time.sleep(0.05)                 # the slower rank sets the reported time
        self.steps += 1

    def sync(self):
        pass

    def kernel_times_ms(self, *a, **k):
        return 0.01, 0.02, 0.03

    def gather_ms(self):
        # the host gather of every channel's decisions (here already host arrays)
        t0 = time.perf_counter()
        self.gathered = [np.array(x, copy=True) for x in self.out]
        return (time.perf_counter() - t0) * 1e3, sum(len(x) for x in self.out)

    def check(self):
        for b, got in zip(self.bits, self.out):
            sent = b.reshape(-1, self.bps).astype(np.int64) @ (1 << np.arange(self.bps)[::-1])
            if not np.array_equal(got, sent[: len(got)].astype(np.uint8)):
                return False
        return True


def _worker(rank, world, port, outdir, config="tiny"):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch.distributed as td
    import bench
    import oracle as o
    td.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    bench.WORKLOADS["tiny"] = ("qam16", 4, 129, 4, 1 << 12, 2, 0, "tiny: 2 channels x 4096 samples")
    # a fixed job of 4 channels over the node (as config 4's 64): 4 / world per rank
    bench.WORKLOADS["tinyjob"] = ("qam16", 4, 129, 4, 1 << 12, 4, 0, "tinyjob: 4 channels x 4096 samples")
    bench.FIXED_TOTAL.add("tinyjob")
    args = bench.argparse.Namespace(config=config, steps=3, warmup=1, no_cpu_baseline=True, cpu_samples=0,
                                    amplitude=1.0, no_out_of_cache=True, settle_ms=0.0)
    runners = []

    def factory(wl, r):
        runners.append(CpuRunner(wl, r, o, bench))
        return runners[0]

    out = bench.run(args, factory, bench._Dist(td, None), rank, world)
    out["_seeds"] = runners[0].seeds
    with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
        json.dump(out, f)
    td.destroy_process_group()


def test_two_ranks_gloo(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    outs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)]
    for out in outs:
        assert out["n_gpus"] == world and out["scaling"] == "weak"
        assert out["decisions_match_sent"] is True
        assert "cpu_baseline" not in out               # only rank 0 at N = 1 times the CPU
    # both ranks report the same (max-over-ranks) time and the whole-job sample count
    assert outs[0]["ms_per_step"] == outs[1]["ms_per_step"]
    assert outs[0]["ms_per_step"] >= 50.0              # rank 1 sleeps 50 ms per step
    total = (1 << 12) * 2 * 3 * world
    assert abs(outs[0]["value"] - total / (outs[0]["ms_per_step"] * 3 / 1e3) / 1e6) <= 0.02 * outs[0]["value"]
    # ranks own disjoint channels
    assert not set(outs[0]["_seeds"]) & set(outs[1]["_seeds"])
    # the host gather of the decisions, timed apart from `value`, max over ranks
    for out in outs:
        g = out["gather"]
        assert g["bytes_per_gpu"] == 2 * (((1 << 12) - 128) // 4) and g["ms"] >= 0   # L - 1 = 128 samples of lag
    assert outs[0]["gather"]["ms"] == outs[1]["gather"]["ms"]


def test_fixed_job_splits_channels_over_ranks(tmp_path):
    """A FIXED_TOTAL config (config 4: 64 channels over the node) at world size 2: each rank runs
    half of the job's channels, the ranks' seeds are exactly global channels 0 .. total - 1 with
    no overlap, `value` counts the whole job once, and the line says strong scaling."""
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), "tinyjob"), nprocs=world, join=True)
    outs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)]
    import bench
    for out in outs:
        assert out["scaling"] == "strong" and out["decisions_match_sent"] is True
        assert out["config"]["channels_per_gpu"] == 2 and out["config"]["channels_total"] == 4
    seeds = outs[0]["_seeds"] + outs[1]["_seeds"]
    assert sorted(seeds) == [bench.SEED + c for c in range(4)]
    total = (1 << 12) * 4 * 3
    assert abs(outs[0]["value"] - total / (outs[0]["ms_per_step"] * 3 / 1e3) / 1e6) <= 0.02 * outs[0]["value"]


def test_fixed_job_rank_workload():
    """bench.rank_workload: config 4's 64 channels split 64 / 32 / 16 / 8 over 1 / 2 / 4 / 8 GPUs;
    a node size that does not divide the job is refused (bench.py exits 2 before any GPU work);
    the other configs keep their per-GPU count (weak scaling)."""
    import bench
    for n in (1, 2, 4, 8):
        wl, sc = bench.rank_workload("c4", n)
        assert wl[5] == 64 // n and sc == "strong" and wl[4] == 1 << 22
    assert bench.rank_workload("c3", 8) == (bench.WORKLOADS["c3"], "weak")
    with pytest.raises(ValueError):
        bench.rank_workload("c4", 3)
    with pytest.raises(SystemExit) as e:
        bench.main(["--gpus", "3", "--config", "c4"])
    assert e.value.code == 2


def test_gpus_flag_must_match_launcher(monkeypatch):
    """Under a launcher (WORLD_SIZE set) --gpus must equal WORLD_SIZE: bench.py exits 2 before
    touching a GPU instead of timing a different node size than the line reports."""
    import bench
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(SystemExit) as e:
        bench.main(["--gpus", "1"])
    assert e.value.code == 2
    monkeypatch.setenv("WORLD_SIZE", "1")
    with pytest.raises(SystemExit) as e:
        bench.main(["--gpus", "4"])
    assert e.value.code == 2


def test_gpus_flag_spawns_ranks(monkeypatch):
    """Without a launcher, --gpus N starts N rank processes (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_* set, one port for all) and returns rank 0's line; the parent itself never imports
    torch.cuda. The child processes are stubbed here (no GPU on the CPU runner)."""
    import subprocess
    import bench
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    started = []

    class FakePopen:
        def __init__(self, cmd, env, stdout, text):
            started.append((cmd, {k: env[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}))
            self.rank = int(env["RANK"])
            if self.rank == 0:
                stdout.write("log line\n" + json.dumps({"n_gpus": 4, "value": 1.0}) + "\n")
                stdout.flush()

        def poll(self):
            return 0

        def wait(self, timeout=None):
            return 0

    monkeypatch.setattr(subprocess, "Popen", FakePopen)
    out = bench.main(["--gpus", "4", "--config", "c4", "--steps", "3"])
    assert out == {"n_gpus": 4, "value": 1.0}
    assert [e["RANK"] for _, e in started] == ["0", "1", "2", "3"]
    assert all(e["WORLD_SIZE"] == "4" and e["MASTER_ADDR"] == "127.0.0.1" for _, e in started)
    assert len({e["MASTER_PORT"] for _, e in started}) == 1
    assert all(cmd[-6:] == ["--gpus", "4", "--config", "c4", "--steps", "3"] for cmd, _ in started)


def test_cpu_baseline_multicore_leg():
    """bench.cpu_baseline: the single-thread leg plus the threaded leg over independent
    channels (seed + c), bounded sample, with the thread count it used in `cores`."""
    import bench
    out = bench.cpu_baseline(bench.WORKLOADS["c3"], 1 << 14, threads=2)
    assert out["kind"] == "port" and out["unit"] == "Msamples/s"
    assert out["cores"] == 2 and out["value"] > 0
    assert out["single_thread"]["cores"] == 1 and out["single_thread"]["value"] > 0
    assert "2 threads x 8192 samples" in out["sample"]
    assert 1 <= bench._cpu_threads() <= 16


def test_settle_clocks_runs_untimed_steps_for_the_budget():
    """bench.settle_clocks: back-to-back steps until the wall-clock budget is spent, synchronising
    after each batch (the queue drains only between batches), batches sized from the measured
    step rate; 0 ms runs nothing. It happens before the warmup, outside the timed region."""
    import bench

    class R:
        def __init__(self):
            self.steps = self.syncs = 0

        def step(self):
            self.steps += 1
            time.sleep(0.0005)

        def sync(self):
            self.syncs += 1

    r = R()
    assert bench.settle_clocks(r, 0) is None and r.steps == 0
    t0 = time.perf_counter()
    out = bench.settle_clocks(r, 60.0)
    dt = (time.perf_counter() - t0) * 1e3
    assert out["steps"] == r.steps and r.steps >= 20
    assert 60.0 <= out["ms"] <= dt + 1.0 and dt < 60.0 + 20.0     # batches end near the budget
    assert r.syncs < r.steps                                      # steps are queued in batches


def test_spawn_ends_ranks_when_one_fails():
    """bench._wait_ranks polls every rank: a rank that exits non-zero ends the others (a rank
    waiting in a barrier for a dead peer would otherwise hang the bench) and its code is the
    one reported; an overall timeout ends every rank with 124."""
    import subprocess
    import sys
    import bench
    sleeper = [sys.executable, "-c", "import time; time.sleep(60)"]
    procs = [subprocess.Popen(sleeper), subprocess.Popen([sys.executable, "-c", "raise SystemExit(3)"]),
             subprocess.Popen(sleeper)]
    t0 = time.monotonic()
    rcs, first_bad = bench._wait_ranks(procs, timeout_s=50)
    assert time.monotonic() - t0 < 30
    assert first_bad == 3 and rcs[1] == 3
    assert all(p.poll() is not None for p in procs)
    procs = [subprocess.Popen(sleeper) for _ in range(2)]
    t0 = time.monotonic()
    rcs, first_bad = bench._wait_ranks(procs, timeout_s=1.0)
    assert time.monotonic() - t0 < 30
    assert first_bad == 124 and rcs == [124, 124]
    assert all(p.poll() is not None for p in procs)
