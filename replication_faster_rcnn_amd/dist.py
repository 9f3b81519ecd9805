"""Per-image data parallelism over GPUs.

Images are independent on this path (nets/rpn.py:131, train.py:71,91, the
RoIPool batch index), so a batch shards per image with no collective in the
data path; each rank seeds its inputs by GLOBAL image index, so results do not
depend on the number of ranks.  The only collective is one all-gather of the
fixed-size (padded) detections at the end of a step -- RCCL over xGMI with the
"nccl" backend on MI355X, gloo on CPU for tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard(n_total: int, rank: int, world: int) -> range:
    """Contiguous block of global image indices owned by `rank`."""
    per = (n_total + world - 1) // world
    lo = min(rank * per, n_total)
    return range(lo, min(lo + per, n_total))


def all_gather_detections(rois: torch.Tensor, idx: torch.Tensor, cnt: torch.Tensor):
    """rois [n,post,4], idx [n,post], cnt [n] per rank (same n on every rank)
    -> the same three tensors for all ranks' images, in rank order.

    One collective per step: each image's detections are packed into one
    int32 row (boxes bit-cast, anchor indices, count; ``post * 5 + 1`` words),
    gathered with a single ``all_gather_into_tensor`` and returned as views of
    the gathered buffer.  Small all-gathers over xGMI are latency-bound, and
    this one sits on the proposal stream, which is the step's critical path --
    three separate gathers cost three latencies."""
    world = dist.get_world_size()
    n, post = idx.shape
    packed = torch.cat([rois.contiguous().view(torch.int32).reshape(n, post * 4),
                        idx.to(torch.int32).reshape(n, post), cnt.to(torch.int32).reshape(n, 1)], 1)
    g = torch.empty((world * n, post * 5 + 1), dtype=torch.int32, device=packed.device)
    dist.all_gather_into_tensor(g, packed)
    rois_all = g[:, : post * 4].view(torch.float32).view(world * n, post, 4)
    idx_all = g[:, post * 4: post * 5]
    cnt_all = g[:, post * 5]
    return rois_all, idx_all, cnt_all
