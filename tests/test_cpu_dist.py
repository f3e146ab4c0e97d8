"""Batch-shard logic of upr/dist.py over a world_size-2 gloo group on CPU."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from upr.dist import shard_bounds, gather_shards, gather_to_rank0


def test_shard_bounds_cover_exactly():
    for total in (1, 7, 32, 256, 257):
        for world in (1, 2, 4, 8):
            spans = [shard_bounds(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    full = torch.arange(total * 6, dtype=torch.float32).reshape(total, 2, 3)
    a, b = shard_bounds(total, world, rank)
    got = gather_shards(full[a:b] * 1.0, total)
    ok = bool(torch.equal(got, full))
    g0 = gather_to_rank0(full[a:b] * 1.0, total)
    ok = ok and (bool(torch.equal(g0, full)) if rank == 0 else g0 is None)
    q.put((rank, ok))
    dist.destroy_process_group()


def test_gloo_gather_world2():
    ctx = mp.get_context("spawn")
    for total in (8, 5):
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_worker, args=(r, 2, port, total, q)) for r in range(2)]
        for p in procs:
            p.start()
        res = [q.get(timeout=120) for _ in procs]
        for p in procs:
            p.join(timeout=60)
        assert sorted(res) == [(0, True), (1, True)]


def _subgroup_worker(rank, world, port, total, q):
    """World 3; the subgroup is global ranks {1, 2}: its group rank 0 is global
    rank 1, so gather_to_rank0(dst=0) must land on global rank 1."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sub = dist.new_group([1, 2])  # every rank takes part in new_group
    ok = True
    if rank in (1, 2):
        full = torch.arange(total * 4, dtype=torch.float32).reshape(total, 4)
        gr = dist.get_rank(sub)
        a, b = shard_bounds(total, 2, gr)
        g0 = gather_to_rank0(full[a:b] * 1.0, total, group=sub, dst=0)
        ok = bool(torch.equal(g0, full)) if rank == 1 else g0 is None
        g1 = gather_to_rank0(full[a:b] * 1.0, total, group=sub, dst=1)
        ok = ok and (bool(torch.equal(g1, full)) if rank == 2 else g1 is None)
        got = gather_shards(full[a:b] * 1.0, total, group=sub)
        ok = ok and bool(torch.equal(got, full))
    q.put((rank, ok))
    dist.destroy_process_group()


def test_gloo_gather_subgroup_world3():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_subgroup_worker, args=(r, 3, port, 5, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert sorted(res) == [(0, True), (1, True), (2, True)]


def _grad_worker(rank, world, port, q):
    from types import SimpleNamespace
    from upr.dist import allreduce_grads
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = torch.arange(10, dtype=torch.float32) * (rank + 1)
    opt = SimpleNamespace(flat=SimpleNamespace(grad=g))
    allreduce_grads(opt)
    # mean over ranks of k * (r + 1) = k * (world + 1) / 2
    want = torch.arange(10, dtype=torch.float32) * (world + 1) / 2
    q.put((rank, bool(torch.allclose(opt.flat.grad, want))))
    dist.destroy_process_group()


def test_gloo_allreduce_grads_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_grad_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert sorted(res) == [(0, True), (1, True)]


def test_bench_gpus2_launches_two_gloo_ranks():
    """`bench.py --gpus 2` run directly is a launcher: it starts torch.distributed.run
    with 2 ranks (here with --dry-run: gloo, CPU step) and rank 0 reports
    n_gpus 2 with the max-over-ranks time; both ranks are distinct processes."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "3",
                        "--warmup", "1"], capture_output=True, text=True, timeout=240, cwd=repo)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 3
    ranks = out["ranks"]
    assert sorted(rk for rk, _ in ranks) == [0, 1]
    assert len({pid for _, pid in ranks}) == 2 and os.getpid() not in {pid for _, pid in ranks}


def _bench_json(args):
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py")] + args, capture_output=True, text=True,
                       timeout=240, cwd=repo)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_gpus2_line_carries_evidence_keys():
    """An N>1 line carries rank 0's parity, the roofline object and the nested
    fp16 object; cpu_baseline and train_amp are N=1 only; --collect rank0 runs
    the gather-to-rank-0 collect through the same timed loop (gloo here)."""
    out = _bench_json(["--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "1", "--collect", "rank0"])
    assert out["n_gpus"] == 2
    for k in ("roofline", "parity", "fp16_preact_aspp", "config"):
        assert k in out, k
    assert "parity" in out["fp16_preact_aspp"]
    assert "cpu_baseline" not in out and "train_amp" not in out
    assert "collect=rank0" in out["config"]["parallelism"]


def test_bench_n1_line_carries_cpu_and_train_keys():
    out = _bench_json(["--dry-run", "--steps", "2", "--warmup", "1"])
    for k in ("roofline", "parity", "cpu_baseline", "fp16_preact_aspp", "train_amp"):
        assert k in out, k
    ci = out["cpu_baseline"]["cpu"]
    assert ci["threads"] >= 1 and "cpu_model" in ci and ci["os_cpu_count"] >= ci["threads"]


def test_bench_config_labels():
    """bench.py names only the configs BASELINE.json defines; every other
    combination is labelled off-config (the dry-run line carries the label)."""
    import importlib.util
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(repo, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    assert b.cfg_label("fp32", "plain", 512, 32) == "configs[1]"
    assert b.cfg_label("fp16", "preact_aspp", 512, 32) == "configs[2]"
    assert b.cfg_label("fp16", "preact_aspp", 1024, 32) == "configs[3]"
    assert b.cfg_label("fp32", "preact_aspp", 1024, 32) == "configs[3]"
    for args in (("fp16", "plain", 512, 32), ("fp32", "preact_aspp", 512, 32), ("fp32", "plain", 512, 8),
                 ("fp16", "preact_aspp", 512, 16), ("fp32", "plain", 1024, 32), ("fp16", "preact_aspp", 256, 32)):
        assert b.cfg_label(*args) == "off-config", args
    out = _bench_json(["--dry-run", "--steps", "1", "--warmup", "0"])
    assert out["config"]["workload"] == "configs[1]"
    assert out["fp16_preact_aspp"]["config"]["workload"] == "configs[2]"
    out = _bench_json(["--dry-run", "--steps", "1", "--warmup", "0", "--precision", "fp16"])
    assert out["config"]["workload"] == "off-config"
    out = _bench_json(["--dry-run", "--steps", "1", "--warmup", "0", "--precision", "fp16", "--variant",
                       "preact_aspp", "--size", "1024"])
    assert out["config"]["workload"] == "configs[3]" and "fp16_preact_aspp" not in out
