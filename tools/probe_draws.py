"""The chip-wide draws (draws.h) at the cfg5 training shape: each op timed with
HIP events for both sampler paths, and the chain's header (calls, chunks,
consumed words, slow walks; with a -DFRCNN_DRAW_PROF build the chain's cycles:
total / waiting for the prefetchers / matched entries / serial walks).

    python tools/probe_draws.py            (FRCNN_LIB_PATH=... for a profiling build)
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import ref_numpy as orc  # noqa: E402  (inputs only)
from replication_faster_rcnn_amd import _lib, synth, targets  # noqa: E402
from replication_faster_rcnn_amd import utils as U  # noqa: E402

HDR = ["nc", "nseg", "nchunks", "nblocks", "p0", "used_chunks", "consumed", "status", "fallbacks",
       "slow", "total_steps"]


def hdr(lib, which, N, n, G, ns, ws):
    buf = (ctypes.c_ubyte * (48 + 64))()
    lib.frcnn_debug_draw_hdr(which, N, n, G, ns, ctypes.c_void_p(ws.data_ptr()), buf)
    ints = np.frombuffer(bytes(buf[:48]), np.int32)
    prof = np.frombuffer(bytes(buf[48:]), np.uint64)
    d = dict(zip(HDR, ints.tolist()))
    d["stalls"], d["spins"] = int(prof[5]), int(prof[4])
    if prof[0]:
        d["cyc"] = {"total": int(prof[0]), "wait": int(prof[1]), "hit": int(prof[2]), "walk": int(prof[3]),
                    "per_chunk": round(int(prof[0]) / max(d["used_chunks"], 1), 1)}
    return d


def main():
    lib = _lib.load()
    dev = torch.device("cuda")
    N, G, img = 16, 32, 600
    anchors = orc.generate_anchors(orc.generate_anchor_base(), 16, 38, 38)
    at = torch.from_numpy(anchors).to(dev)
    bl = [synth.gt_boxes(img, img, G, 0, i) for i in range(N)]
    boxes = torch.from_numpy(np.stack([b for b, _ in bl])).to(dev)
    labels = torch.from_numpy(np.stack([l for _, l in bl])).to(dev)
    rp = np.zeros((N, 600, 4), np.float32)
    cnts = []
    for i in range(N):
        r, _ = orc.propose_one(anchors, synth.rpn_scores(len(anchors), 0, i), synth.rpn_deltas(len(anchors), 0, i),
                               img, img, 12000, 600)
        rp[i, :len(r)] = r
        cnts.append(len(r))
    rp = torch.from_numpy(rp).to(dev)
    cnt = torch.tensor(cnts, dtype=torch.int32, device=dev)
    A = at.size(0)
    for path in ("walk", "chip"):
        _lib.set_path("sampler", path)
        np.random.seed(0)
        rng, _ = U.rng_state_to_device(dev)
        aplan = targets.anchor_targets_prepare(boxes, labels, at)
        pplan = targets.proposal_targets_prepare(rp, cnt, boxes, labels, n_sample=128)
        for it in range(4):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record()
            targets.anchor_targets_draw(aplan, rng=rng)
            e[1].record()
            s_cnt = torch.empty(N, dtype=torch.int32, device=dev)
            targets.proposal_targets_draw(pplan, rng=rng, count=s_cnt)
            e[2].record()
            torch.cuda.synchronize()
            if it:
                line = {"path": path, "at_us": round(e[0].elapsed_time(e[1]) * 1e3, 1),
                        "pt_us": round(e[1].elapsed_time(e[2]) * 1e3, 1)}
                if path == "chip":
                    line["at"] = hdr(lib, 0, N, A, G, 256, aplan.ws)
                    line["pt"] = hdr(lib, 1, N, pplan.Rp, G, 128, pplan.ws)
                print(line, flush=True)


if __name__ == "__main__":
    main()
