"""bench.py's multi-rank path with the real kernels: two ranks (processes) on the
box's GPU, gloo for the timing barrier and the max-over-ranks reduction (RCCL needs one GPU per
rank; the driver's 8-GPU scaling run uses it). Each rank runs its own channel set through the HIP
TX -> RX chain; checks that every rank's decisions equal the symbols it sent, that the ranks
report one (max-over-ranks) time and the whole-job sample count, and that their channel seeds
are disjoint (weak scaling, no data-path collective)."""
import json
import os
import socket

import pytest
import torch.multiprocessing as mp

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, outdir):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as td
    import bench
    td.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    bench.WORKLOADS["small"] = ("qam16", 4, 129, 4, 1 << 18, 2, 0, "small: 2 channels x 2^18 C3 samples")
    args = bench.argparse.Namespace(config="small", steps=20, warmup=3, no_cpu_baseline=True, cpu_samples=0,
                                    amplitude=1.0, no_out_of_cache=True)
    runner = []

    def factory(wl, r):
        runner.append(bench.GpuRunner(wl, r, 0, streams=1, batch=True))
        return runner[0]
    out = bench.run(args, factory, bench._Dist(td, None), rank, world)
    out["_seeds"] = [bench.channel_seed(rank, 2, c) for c in range(2)]
    with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
        json.dump(out, f)
    torch.cuda.synchronize()
    td.destroy_process_group()


def test_two_ranks_real_kernels(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    outs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)]
    for out in outs:
        assert out["n_gpus"] == world and out["scaling"] == "weak"
        assert out["decisions_match_sent"] is True
    assert outs[0]["ms_per_step"] == outs[1]["ms_per_step"]
    total = (1 << 18) * 2 * 20 * world
    assert abs(outs[0]["value"] - total / (outs[0]["ms_per_step"] * 20 / 1e3) / 1e6) <= 0.02 * outs[0]["value"]
    assert not set(outs[0]["_seeds"]) & set(outs[1]["_seeds"])
