"""Probe: where the anchor-target sampler spends its time (GPU box)."""
import time

import numpy as np
import torch

from replication_faster_rcnn_amd import anchors as A, synth, targets
from replication_faster_rcnn_amd.utils import rng_state_to_device

dev = torch.device("cuda")
base = A.generate_anchor_base_device()
an = A.generate_anchors(base, 16, 38, 38).to(dev)
for N in (1, 4, 16):
    gl = [synth.gt_boxes(600, 600, 32, 0, i) for i in range(N)]
    bx = torch.from_numpy(np.stack([b for b, _ in gl])).to(dev)
    lb = torch.from_numpy(np.stack([l for _, l in gl])).to(dev)
    np.random.seed(0)
    rng, _ = rng_state_to_device(dev)
    for sample in (False, True):
        for _ in range(3):
            targets.anchor_targets(bx, lb, an, rng=rng, sample=sample)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            reg, lab = targets.anchor_targets(bx, lb, an, rng=rng, sample=sample)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 10 * 1e6
        _, lab0 = targets.anchor_targets(bx, lb, an, sample=False)
        q = (lab0 == 0).sum(1).tolist()
        p = (lab0 == 1).sum(1).tolist()
        print(f"N={N} sample={sample}: {dt:.0f} us/call; pos {p[:4]} neg {q[:4]}", flush=True)

# timeline of one N=1 call: per 624-word block (s_memrealtime = 100 MHz)
import ctypes
from replication_faster_rcnn_amd import _lib
lib = _lib.load()
lib.frcnn_dbg_samp_probe.restype = ctypes.c_int
gl = [synth.gt_boxes(600, 600, 32, 0, 0)]
bx = torch.from_numpy(np.stack([b for b, _ in gl])).to(dev)
lb = torch.from_numpy(np.stack([l for _, l in gl])).to(dev)
rng, _ = rng_state_to_device(dev)
torch.cuda.synchronize()
lib.frcnn_dbg_samp_probe(1, None, 0)
targets.anchor_targets(bx, lb, an, rng=rng)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (4 * 2048))()
n = lib.frcnn_dbg_samp_probe(0, buf, 4 * 2048)
lib.frcnn_dbg_samp_probe(0, None, 0)
a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 4)[:n].astype(np.int64)
print("blocks", n)
for r in a[:40]:
    print(f"twist {(r[1]-r[0])*10:6d} ns  fixpt {(r[2]-r[1])*10:6d} ns  iters {r[3]}  gap_from_prev", flush=True)
if n > 1:
    print("block period ns:", np.diff(a[:, 0]) * 10)
