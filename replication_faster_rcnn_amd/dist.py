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
    -> the same three tensors for all ranks' images, in rank order."""
    world = dist.get_world_size()
    outs = []
    for t in (rois, idx, cnt):
        t = t.contiguous()
        g = torch.empty((world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(g, t)
        outs.append(g)
    return tuple(outs)
