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


def test_bench_gpus_flag_two_ranks():
    """`bench.py --gpus 2` without a launcher: two fresh rank processes (here both on the box's
    one GPU, so the timing barrier runs over gloo; one GPU per rank uses RCCL) sharing config 4's
    one 64-channel job, 32 channels each in groups of 8; rank 0's line reports the node size,
    every channel's decisions on both ranks, and the host gather of the decisions timed apart
    from `value`, which counts the job's 64 x 2^22 samples per step."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    out = bench.main(["--gpus", "2", "--config", "c4", "--steps", "10", "--warmup", "3", "--settle-ms", "50",
                      "--no-cpu-baseline"])
    assert out["n_gpus"] == 2 and out["scaling"] == "strong"
    assert out["config"]["channels_per_gpu"] == 32 and out["config"]["channels_total"] == 64
    assert out["config"]["channels_per_launch"] == 8
    assert out["decisions_match_sent"] is True
    g = out["gather"]
    assert g["bytes_per_gpu"] == 32 * ((1 << 22) // 4 - 16) and g["ms"] > 0
    total = (1 << 22) * 64 * 10
    assert abs(out["value"] - total / (out["ms_per_step"] * 10 / 1e3) / 1e6) <= 0.02 * out["value"]


def test_c4_job_one_gpu_groups_of_four():
    """Config 4's whole 64-channel job on one GPU (the N = 1 point of its scaling curve), in
    groups of 4 channels per launch pair: every channel's decisions equal the symbols it sent."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    out = bench.main(["--config", "c4", "--group", "4", "--steps", "5", "--warmup", "2", "--settle-ms", "20",
                      "--no-cpu-baseline"])
    assert out["n_gpus"] == 1 and out["scaling"] == "strong"
    assert out["config"]["channels_per_gpu"] == 64 and out["config"]["channels_per_launch"] == 4
    assert out["decisions_match_sent"] is True
    assert out["gather"]["bytes_per_gpu"] == 64 * ((1 << 22) // 4 - 16)


def test_rccl_branch_under_launcher(tmp_path):
    """The driver's multi-GPU invocation (python -m torch.distributed.run ... bench.py --gpus N)
    with one rank on the box's GPU: bench.py takes its RCCL branch (init_process_group("nccl")
    with the rank's device, the device barrier and the max-over-ranks all_reduce on a GPU
    tensor), the branch every rank of the driver's 8-GPU scaling run takes."""
    import subprocess
    import sys
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--config", "c2", "--steps", "20", "--warmup", "3", "--settle-ms", "0",
           "--no-cpu-baseline", "--no-out-of-cache"]
    r = subprocess.run(cmd, cwd=str(tmp_path), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 1 and out["decisions_match_sent"] is True
    assert "max over ranks: nccl" in out["config"]["parallelism"], out["config"]["parallelism"]
