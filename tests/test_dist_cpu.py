"""World-size-2 gloo test of the multi-GPU path's sharding + all-gather
(the same helpers bench.py uses over RCCL), with oracle proposals standing in
for the device ones: gathered detections are identical to the unsharded run."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from replication_faster_rcnn_amd import dist as fdist
from replication_faster_rcnn_amd import synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _proposals(img, anchors, post):
    from oracle import ref_numpy as orc
    A = len(anchors)
    rois, idx = orc.propose_one(anchors, synth.rpn_scores(A, 0, img), synth.rpn_deltas(A, 0, img),
                                320, 240, 800, post)
    r = np.zeros((post, 4), np.float32)
    i = np.full(post, -1, np.int32)
    r[:len(rois)] = rois
    i[:len(idx)] = idx
    return r, i, len(rois)


def _worker(rank, world, port, n_total, post, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import ref_numpy as orc
    anchors = orc.generate_anchors(orc.generate_anchor_base(), 16, 20, 15)
    mine = [_proposals(img, anchors, post) for img in fdist.shard(n_total, rank, world)]
    rois = torch.from_numpy(np.stack([m[0] for m in mine])) if mine else torch.zeros((0, post, 4))
    idx = torch.from_numpy(np.stack([m[1] for m in mine])) if mine else torch.zeros((0, post), dtype=torch.int32)
    cnt = torch.tensor([m[2] for m in mine], dtype=torch.int32)
    g = fdist.all_gather_detections(rois, idx, cnt, n_total)
    if rank == 0:
        q.put([t.numpy() for t in g])
    dist.barrier()
    dist.destroy_process_group()


def test_shard_covers_batch():
    for n, w in [(64, 8), (64, 2), (10, 4), (3, 8)]:
        got = [i for r in range(w) for i in fdist.shard(n, r, w)]
        assert got == list(range(n))


@pytest.mark.parametrize("world,n_total", [(2, 4), (4, 8), (4, 10), (4, 3)])
def test_rank_gather_is_p_invariant(world, n_total):
    post = 50
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, post, q)) for r in range(world)]
    for p in procs:
        p.start()
    rois, idx, cnt = q.get(timeout=120)
    assert len(cnt) == n_total  # uneven (3/3/3/1) and empty (1/1/1/0) shards padded, then trimmed
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from oracle import ref_numpy as orc
    anchors = orc.generate_anchors(orc.generate_anchor_base(), 16, 20, 15)
    for img in range(n_total):
        r, i, c = _proposals(img, anchors, post)
        assert cnt[img] == c
        assert np.array_equal(rois[img], r) and np.array_equal(idx[img], i)
