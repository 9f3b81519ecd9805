"""Multi-process HIP path (BASELINE configs[2]): two ranks on
the one GPU of the box, each running the device proposal layer + the head's
RoIPool on its per-image shard of cfg3's 64 images, detections gathered over
gloo (host copies; RCCL needs one GPU per rank, which only the driver's 8-GPU
node has).  The gathered detections and every image's pooled features must be
bit-identical to one process running all 64 images (P-invariance of
nets/rpn.py:131-136 per-image sharding)."""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(images, dev):
    """propose + head RoIPool on `images` (global indices) -> host rois, idx,
    cnt and a sha256 of each image's pooled features + argmax."""
    from bench import make_inputs
    from replication_faster_rcnn_amd import anchors as A, ops
    c, sc, de, x = make_inputs("cfg3", images, dev)
    base = A.generate_anchor_base_device(anchor_scales=c["scales"])
    rois, idx, cnt = ops.propose(sc, de, img_w=c["img_w"], img_h=c["img_h"], pre_nms=c["pre_nms"],
                                 post_nms=c["post_nms"], anchor_base=base, feat_h=c["feat_h"],
                                 feat_w=c["feat_w"])
    N, post = sc.size(0), c["post_nms"]
    inds = torch.arange(N, device=dev, dtype=torch.float32).repeat_interleave(post)
    pooled, am, _ = ops.roi_pool_head(x, rois.view(-1, 4), inds, 7, c["img_h"], c["img_w"],
                                      rois_sorted=True)
    torch.cuda.synchronize()
    hashes = []
    for i in range(N):
        h = hashlib.sha256()
        h.update(pooled[i * post:(i + 1) * post].cpu().numpy().tobytes())
        h.update(am[i * post:(i + 1) * post].cpu().numpy().tobytes())
        hashes.append(h.hexdigest())
    return rois.cpu(), idx.cpu(), cnt.cpu(), hashes


def _worker(rank, world, port, n_total, q):
    import torch.distributed as dist
    from replication_faster_rcnn_amd import dist as fdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    mine = fdist.shard(n_total, rank, world)
    rois, idx, cnt, hashes = _run(mine, dev)
    g = fdist.all_gather_detections(rois, idx, cnt, n_total)
    all_hashes = [None] * world
    dist.all_gather_object(all_hashes, hashes)
    if rank == 0:
        q.put(([t.numpy().copy() for t in g], [h for hs in all_hashes for h in hs]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_two_ranks_match_one_process_cfg3(world):
    import torch.multiprocessing as mp
    n_total = 64
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        (g_rois, g_idx, g_cnt), g_hash = q.get(timeout=110)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    rois, idx, cnt, hashes = _run(range(n_total), torch.device("cuda", 0))
    assert g_cnt.shape == (n_total,) and np.array_equal(g_cnt, cnt.numpy())
    assert np.array_equal(g_idx, idx.numpy())
    assert np.array_equal(g_rois.view(np.int32), rois.numpy().view(np.int32))
    assert g_hash == hashes
    assert (cnt.numpy() > 0).all()
