"""Timeline probe of the hybrid proposal kernels (cfg2 inputs): per image,
s_memrealtime (100 MHz) at the phase ends of propose_fused_kernel<.,1>
(keys, select, compact, sort, gather, hand-off) and <.,2> (load, sweep, exit);
prints the median phase lengths in us."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import make_inputs  # noqa: E402
from replication_faster_rcnn_amd import _lib, anchors as A, ops, synth  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
    dev = torch.device("cuda", 0)
    c = synth.CONFIGS[cfg]
    c, sc, de, x = make_inputs(cfg, c["batch"], 0, dev)
    base = A.generate_anchor_base_device(anchor_scales=c["scales"])
    lib = _lib.load()
    run = lambda: ops.propose(sc, de, img_w=c["img_w"], img_h=c["img_h"], pre_nms=c["pre_nms"],  # noqa
                              post_nms=c["post_nms"], anchor_base=base, feat_h=c["feat_h"], feat_w=c["feat_w"])
    run()
    torch.cuda.synchronize()
    assert lib.frcnn_dbg_prop_probe(1) == 0
    run()
    torch.cuda.synchronize()
    lib.frcnn_dbg_prop_probe(0)
    buf = (ctypes.c_ulonglong * (64 * 16))()
    assert lib.frcnn_dbg_prop_stamps(buf, 64 * 16) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(64, 16).astype(np.int64)[: sc.size(0)]
    names = ["k1_keys", "k1_select", "k1_compact", "k1_sort", "k1_gather", "k1_handoff"]
    out = {nm: float(np.median(a[:, i + 1] - a[:, i])) / 100 for i, nm in enumerate(names)}
    out["k1_total"] = float(np.median(a[:, 6] - a[:, 0])) / 100
    out["gap_k1_end_to_k3_start"] = float(np.median(a[:, 8] - a[:, 6])) / 100
    out["k3_load"] = float(np.median(a[:, 9] - a[:, 8])) / 100
    out["k3_sweep"] = float(np.median(a[:, 10] - a[:, 9])) / 100
    out["k3_rest"] = float(np.median(a[:, 11] - a[:, 10])) / 100
    print(json.dumps({k: round(v, 2) for k, v in out.items()}, indent=1))


if __name__ == "__main__":
    main()
