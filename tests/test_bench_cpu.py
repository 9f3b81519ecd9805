"""bench.py's multi-GPU record contract, on the CPU: the default (--config auto)
names ONE workload at every N (cfg2 per GPU, weak scaling), so the driver's
1/2/4/8-GPU curve compares like with like; the N = 2 check runs two gloo ranks
through the same config / sharding / naming code bench.py's ranks run."""
import argparse
import os
import socket

import torch.distributed as dist
import torch.multiprocessing as mp

import bench
from replication_faster_rcnn_amd import dist as fdist
from replication_faster_rcnn_amd import synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _record(world, rank):
    """(config name, workload, global batch, this rank's images) as bench.main builds them."""
    args = argparse.Namespace(config="auto")
    cfg = bench.resolve_config(args, world)
    c = synth.CONFIGS[cfg]
    n_total = c["batch"] * world if cfg != "cfg3" else c["batch"]
    mine = fdist.shard(n_total, rank, world)
    return cfg, bench.workload_name(cfg, c, len(mine), n_total, world, c["C"], False), n_total, list(mine)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rec = _record(world, rank)
    out = [None] * world
    dist.all_gather_object(out, rec)
    if rank == 0:
        q.put(out)
    dist.barrier()
    dist.destroy_process_group()


def test_auto_config_is_one_workload_at_every_n():
    recs = {w: _record(w, 0) for w in (1, 2, 4, 8)}
    assert {r[0] for r in recs.values()} == {"cfg2"}
    assert len({r[1] for r in recs.values()}) == 1          # same workload string
    assert [recs[w][2] for w in (1, 2, 4, 8)] == [8, 16, 32, 64]  # N = 8: configs[2]'s 64 images
    assert recs[8][2] == synth.CONFIGS["cfg3"]["batch"]


def test_two_gloo_ranks_name_the_n1_workload():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = q.get(timeout=120)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    n1 = _record(1, 0)
    assert [o[1] for o in out] == [n1[1], n1[1]]               # both ranks: the N = 1 workload
    assert out[0][3] + out[1][3] == list(range(16))             # 8 images each, every image once
    assert len(out[0][3]) == len(n1[3]) == 8
