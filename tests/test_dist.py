"""Multi-GPU control plane and batch split, exercised with gloo on the CPU
(world_size 2), as SURVEY.md §8e prescribes: contiguous equal-byte shards, no
data-path collective, barrier + max-over-ranks timing only."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from talos_amd.dist import ControlPlane, device_for, shard_by_bytes


def test_shard_equal_records():
    lens = np.full(524288, 16384)
    cuts = [shard_by_bytes(lens, 8, r) for r in range(8)]
    assert cuts[0] == (0, 65536) and cuts[-1] == (458752, 524288)
    assert all(b - a == 65536 for a, b in cuts)


def test_shard_zipf_balanced_and_disjoint():
    from talos_amd.workload import zipf_lengths
    lens = zipf_lengths(100000, seed=3)
    for world in (2, 4, 8):
        cuts = [shard_by_bytes(lens, world, r) for r in range(world)]
        assert cuts[0][0] == 0 and cuts[-1][1] == len(lens)
        assert all(cuts[i][1] == cuts[i + 1][0] for i in range(world - 1))
        per = [int(lens[a:b].sum()) for a, b in cuts]
        assert max(per) - min(per) <= 2 * 16384


def test_device_for_refuses_fewer_gpus(monkeypatch):
    monkeypatch.delenv("TLSGPU_ALLOW_SHARED_GPU", raising=False)
    assert [device_for(r, 8) for r in range(8)] == list(range(8))
    with pytest.raises(RuntimeError):
        device_for(1, 1)           # rank 1 of a 2-GPU run on a 1-GPU box: no silent wrap
    with pytest.raises(RuntimeError):
        device_for(0, 0)
    # sharing only on explicit request (the N-ranks-on-one-GPU rehearsal)
    assert [device_for(r, 1, allow_shared=True) for r in range(4)] == [0, 0, 0, 0]
    monkeypatch.setenv("TLSGPU_ALLOW_SHARED_GPU", "1")
    assert device_for(3, 2) == 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    cp = ControlPlane(world)
    cp.barrier()
    mx = cp.max([1.0 + rank, 10.0 - rank])
    sm = cp.sum([float(rank)])
    lens = np.full(1000, 1400)
    lo, hi = shard_by_bytes(lens, world, rank)
    cp.barrier()
    cp.close()
    q.put((rank, mx, sm, lo, hi))


def test_gloo_world2_control_plane():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert [r[1] for r in res] == [[2.0, 10.0], [2.0, 10.0]]
    assert [r[2] for r in res] == [[1.0], [1.0]]
    assert [(r[3], r[4]) for r in res] == [(0, 500), (500, 1000)]


def test_bench_split_plumbing():
    """bench.py's multi-GPU split choice and group member list (no GPU): N > 1
    ranks or an explicit device list measure the C ABI's tlsgpu_group split."""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "bench", os.path.join(os.path.dirname(os.path.dirname(__file__)), "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert bench.choose_split(None, 1, "") == "ranks"
    assert bench.choose_split(None, 1, "", 1) == "ranks"
    assert bench.choose_split(None, 8, "") == "group"
    assert bench.choose_split(None, 1, "0,0") == "group"
    assert bench.choose_split("ranks", 8, "") == "ranks"
    assert bench.choose_split("group", 1, "") == "group"
    # `python bench.py --gpus 8` with no launcher (world 1) measures 8 GPUs
    assert bench.choose_split(None, 1, "", 8) == "group"
    assert bench.group_devices("", 1, 1) == [0]
    assert bench.group_devices("", 4, 1) == [0, 1, 2, 3]
    assert bench.group_devices("", 1, 8) == list(range(8))
    assert bench.group_devices("", 8, 1) == list(range(8))
    assert bench.group_devices("0,0", 1, 1) == [0, 0]
    with pytest.raises(SystemExit):
        bench.group_devices("-1", 1, 1)
    # fewer visible GPUs than asked for: exit non-zero, never wrap
    bench.check_devices(list(range(8)), 8, False)
    with pytest.raises(SystemExit):
        bench.check_devices(list(range(8)), 1, False)
    with pytest.raises(SystemExit):
        bench.check_devices([0, 1], 1, True)
    bench.check_devices([0, 0], 1, True)      # the explicit one-GPU rehearsal


def test_bench_gpus8_without_launcher_parses_to_group(monkeypatch, capsys):
    """`python bench.py --gpus 8` (the driver's BENCH command shape at N = 8,
    no torch.distributed.run) reaches group_mode over devices 0..7."""
    import importlib.util
    import sys
    spec = importlib.util.spec_from_file_location(
        "bench_g8", os.path.join(os.path.dirname(os.path.dirname(__file__)), "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    seen = {}

    def fake_group_mode(args, world, rank):
        seen.update(world=world, rank=rank,
                    devices=bench.group_devices(args.devices, args.gpus, world))
    monkeypatch.setattr(bench, "group_mode", fake_group_mode)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "20", "--warmup", "5"])
    bench.main()
    assert seen == {"world": 1, "rank": 0, "devices": list(range(8))}
