"""World-size-2 gloo tests of bench.py's multi-process contract (CPU, no GPU).

The hot path does not shard through a collective (attention is per
(batch, head); 8 GPUs = 8 independent replicas), so the only distributed logic is bench.py's:
barrier, local timing, MAX over ranks of the elapsed time, value = world * work / max time,
rank 0 prints. These tests run that exact helper on two gloo ranks, plus the replica rule that
every rank computes the same per-rank workload on its own data (seeded by rank).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        _worker_body(rank, world, port, q)
    except Exception:  # report instead of dying silently
        import traceback
        q.put((rank, "error", traceback.format_exc(), None))


def _worker_body(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    el = 1.0 + rank          # rank 1 is the slow one
    t = torch.tensor([el], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    value = world * 10.0 / t.item()
    # replicas: each rank builds its own synthetic batch (seeded by rank) of the same shape
    qt, kt, vt, _, cq, ck = bench.make_inputs(2, 2, 64, 64, 16, torch.float32, "cpu", seed=rank)
    shapes = torch.tensor(list(qt.shape) + list(kt.shape), dtype=torch.int64)
    gathered = [torch.zeros_like(shapes) for _ in range(world)]
    dist.all_gather(gathered, shapes)
    first = torch.tensor([qt.flatten()[0].item()])
    firsts = [torch.zeros(1) for _ in range(world)]
    dist.all_gather(firsts, first)
    dist.barrier()
    q.put((rank, value, [g.tolist() for g in gathered], [f.item() for f in firsts]))
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_bench_aggregation_two_ranks():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in range(world)]
    res = [r for r in res]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for r in res:
        assert r[1] != "error", r[2]
    res.sort()
    # value = world * work / MAX(elapsed): both ranks agree, and the slow rank sets the time
    assert res[0][1] == res[1][1] == pytest.approx(2 * 10.0 / 2.0)
    # same per-rank workload shape on every rank (weak scaling), different data per rank
    assert res[0][2][0] == res[0][2][1]
    assert res[0][3][0] != res[0][3][1]
