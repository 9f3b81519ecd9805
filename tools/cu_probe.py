"""Where do the workgroups of a CU-masked stream run?  Prints, for a few CU
masks (hipExtStreamCreateWithCUMask numbering), the (XCC, SE, SH, CU) of every
workgroup of a probe launch -- used to pick per-XCD-balanced reservations for
the proposal streams (bench.py --prop-cus).

    python tools/cu_probe.py
"""
import ctypes
import os
import sys
from collections import Counter

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replication_faster_rcnn_amd import _lib  # noqa: E402


def probe(stream, nblocks=64, spin=400):
    lib = _lib.load()
    out = torch.zeros(2 * nblocks, dtype=torch.int32, device="cuda")
    _lib.check(lib.frcnn_probe_hw_ids(_lib.ptr(out), nblocks, spin, ctypes.c_void_p(stream.cuda_stream)),
               "probe")
    torch.cuda.synchronize()
    v = out.view(-1, 2).cpu().tolist()
    res = []
    for hw, xcc in v:
        hw &= 0xFFFFFFFF
        res.append((xcc & 0xF, (hw >> 13) & 0x7, (hw >> 12) & 1, (hw >> 8) & 0xF))
    return res


def main():
    n = _lib.cu_count()
    print("CUs", n)
    masks = {
        "all": None,
        "bits 0-7": range(8),
        "bits 0-31": range(32),
        "bits i%8==0": range(0, n, 8),
        "bits i%8==3": range(3, n, 8),
        "bits 0,1,8,9,..(i%8<2)": [i for i in range(n) if i % 8 < 2],
        "bits 32-63": range(32, 64),
        "bits i%32<4": [i for i in range(n) if i % 32 < 4],
    }
    for name, m in masks.items():
        s = _lib.cu_stream(None if m is None else list(m))
        r = probe(s, nblocks=64 if m is None else 2 * len(list(m)))
        xcc = Counter(t[0] for t in r)
        uniq = sorted(set(r))
        print(f"{name:26s} cu_count={_lib.stream_cu_count(s):3d} wgs={len(r)} distinct CUs={len(uniq)} "
              f"per-XCC={dict(sorted(xcc.items()))}")
        print("   first CUs (xcc,se,sh,cu):", uniq[:12])


if __name__ == "__main__":
    main()
