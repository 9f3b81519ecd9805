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
    """Contiguous block of global image indices owned by `rank`: blocks of
    ceil(n_total / world), so only the last ranks can hold fewer (or none)."""
    per = (n_total + world - 1) // world
    lo = min(rank * per, n_total)
    return range(lo, min(lo + per, n_total))


def all_gather_detections(rois: torch.Tensor, idx: torch.Tensor, cnt: torch.Tensor,
                          n_total: int = None):
    """rois [n,post,4], idx [n,post], cnt [n] of this rank's shard (``shard``)
    -> the same three tensors for all ``n_total`` images, in global order.

    One collective per step: each image's detections are packed into one int32
    row (boxes bit-cast, anchor indices, count; ``post * 5 + 1`` words).  Every
    rank contributes ceil(n_total / world) rows -- uneven or empty shards are
    padded with count 0 / index -1 rows -- so a single ``all_gather_into_tensor``
    serves any batch size; since shards are contiguous blocks, the first
    ``n_total`` gathered rows are the images in order.  Results are views of the
    gathered buffer.  Small all-gathers over xGMI are latency-bound and this one
    sits on the proposal stream (the step's critical path): three separate
    gathers would cost three latencies."""
    world = dist.get_world_size()
    n, post = idx.shape[0], idx.shape[1]
    if n_total is None:
        n_total = n * world
    per = (n_total + world - 1) // world
    if n > per:
        raise RuntimeError(f"all_gather_detections: {n} images on this rank > ceil({n_total}/{world})")
    width = post * 5 + 1
    packed = torch.zeros((per, width), dtype=torch.int32, device=idx.device)
    if per > n:
        packed[n:, post * 4: post * 5] = -1
    if n:
        packed[:n, : post * 4] = rois.contiguous().view(torch.int32).reshape(n, post * 4)
        packed[:n, post * 4: post * 5] = idx.to(torch.int32).reshape(n, post)
        packed[:n, post * 5] = cnt.to(torch.int32)
    g = torch.empty((world * per, width), dtype=torch.int32, device=idx.device)
    dist.all_gather_into_tensor(g, packed)
    g = g[:n_total]
    rois_all = g[:, : post * 4].view(torch.float32).view(n_total, post, 4)
    idx_all = g[:, post * 4: post * 5]
    cnt_all = g[:, post * 5]
    return rois_all, idx_all, cnt_all
