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


class DetectionGather:
    """Preallocated all-gather of every rank's padded detections.

    Each rank owns one flat int32 block of ``per = ceil(n_total / world)``
    image slots laid out ``[rois per*post*4 | anchor idx per*post | count
    per]``; :meth:`outputs` hands out contiguous views of this rank's ``n``
    slots, so the proposal layer writes its results straight into the send
    buffer (``ops.propose(..., out=g.outputs())``) and a step issues ONE
    ``all_gather_into_tensor`` with no packing copies and no allocation.
    Unused slots (uneven or empty shards) are padded once here (count 0,
    index -1, zero boxes) and never written again.  Small all-gathers over xGMI
    are latency bound: issue :meth:`gather` on a side stream that waits for
    the proposals, so the RoIPool of the same step does not wait for it."""

    def __init__(self, n_total: int, post: int, device, backend: str = None):
        if not dist.is_initialized():
            raise RuntimeError("DetectionGather: torch.distributed is not initialised")
        self.world = dist.get_world_size()
        self.rank = dist.get_rank()
        self.n_total, self.post = int(n_total), int(post)
        self.per = (self.n_total + self.world - 1) // self.world
        self.n = len(shard(self.n_total, self.rank, self.world))
        self.device = torch.device(device)
        self.backend = backend or dist.get_backend()
        # gloo moves host tensors: ranks sharing a GPU gather through the host
        self.host = self.backend != "nccl" and self.device.type == "cuda"
        per, p = self.per, self.post
        self.width = per * p * 5 + per
        self.flat = torch.zeros(self.width, dtype=torch.int32, device=self.device)
        self.flat[per * p * 4: per * p * 5] = -1
        gdev = "cpu" if self.host else self.device
        # flat: gloo's all_gather_into_tensor wants [world * width], not [world, width]
        self.g_flat = torch.empty(self.world * self.width, dtype=torch.int32, device=gdev)
        self.g = self.g_flat.view(self.world, self.width)
        if self.host:
            self.h_flat = torch.empty(self.width, dtype=torch.int32, pin_memory=True)

    def outputs(self):
        """(rois fp32 [n,post,4], idx int32 [n,post], cnt int32 [n]): views of
        this rank's slots in the send buffer."""
        per, p, n = self.per, self.post, self.n
        f = self.flat
        rois = f[: n * p * 4].view(torch.float32).view(n, p, 4)
        idx = f[per * p * 4: per * p * 4 + n * p].view(n, p)
        cnt = f[per * p * 5: per * p * 5 + n]
        return rois, idx, cnt

    def gather(self):
        """All-gather the send buffers; returns (rois [world,per,post,4] fp32,
        idx [world,per,post], cnt [world,per]) views of the gathered buffer --
        rank r's block holds global images r*per ... (see :meth:`ordered`)."""
        if self.host:
            self.h_flat.copy_(self.flat)  # synchronous: gloo reads the host copy
            dist.all_gather_into_tensor(self.g_flat, self.h_flat)
        else:
            dist.all_gather_into_tensor(self.g_flat, self.flat)
        per, p = self.per, self.post
        g = self.g
        rois = g[:, : per * p * 4].view(torch.float32).unflatten(1, (per, p, 4))
        idx = g[:, per * p * 4: per * p * 5].unflatten(1, (per, p))
        cnt = g[:, per * p * 5:]
        return rois, idx, cnt

    def ordered(self, gathered=None):
        """The gathered detections in global image order, ``n_total`` rows
        (rois [n_total,post,4], idx [n_total,post], cnt [n_total]; copies)."""
        rois, idx, cnt = gathered if gathered is not None else self.gather()
        n = self.n_total
        return (rois.reshape(-1, self.post, 4)[:n], idx.reshape(-1, self.post)[:n],
                cnt.reshape(-1)[:n])


def all_gather_detections(rois: torch.Tensor, idx: torch.Tensor, cnt: torch.Tensor, n_total: int):
    """rois [n,post,4], idx [n,post], cnt [n] of this rank's shard
    (``shard(n_total, rank, world)``) -> the same three tensors for all
    ``n_total`` images, in global order (one collective; see DetectionGather,
    which the bench uses with preallocated buffers)."""
    world = dist.get_world_size()
    n, post = idx.shape[0], idx.shape[1]
    mine = len(shard(n_total, dist.get_rank(), world))
    if n != mine:
        raise RuntimeError(f"all_gather_detections: {n} images on rank {dist.get_rank()}, but "
                           f"shard({n_total}, rank, {world}) holds {mine}")
    dg = DetectionGather(n_total, post, idx.device)
    r, i, c = dg.outputs()
    if n:
        r.copy_(rois)
        i.copy_(idx)
        c.copy_(cnt)
    return dg.ordered()
