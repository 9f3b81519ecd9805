import sys, os, numpy as np, torch
sys.path.insert(0, os.getcwd())
from replication_faster_rcnn_amd import _lib, ops
from oracle import ref_numpy as orc
DEV = torch.device("cuda", 0)
def rr(r, b, H, W, lo=-3, span=40):
    xy = r.uniform(lo, max(H, W) + 2, (len(b), 2)).astype(np.float32)
    wh = r.uniform(0, span, (len(b), 2)).astype(np.float32)
    return np.concatenate([np.asarray(b, np.float32)[:, None], xy, xy + wh], 1).astype(np.float32)
for case, split in [("a", "1"), ("a", "auto"), ("b", "1")]:
    r = np.random.default_rng(5)
    N, C, H, W = 4, 16, 20, 27
    b = np.sort(r.integers(0, N, 200)) if case == "a" else np.zeros(40, int)
    x = r.standard_normal((N, C, H, W), dtype=np.float32)
    rois = rr(r, b, H, W)
    with _lib.kernel_path("roi_pool_split", split), _lib.kernel_path("roi_pool_fwd", "sort"):
        out, am = ops.roi_pool_with_argmax(torch.from_numpy(x).to(DEV), torch.from_numpy(rois).to(DEV), 7, rois_sorted=True)
    oo, oa = orc.roi_pool_forward(x, rois, 7)
    am = am.cpu().numpy(); out = out.cpu().numpy()
    bad = (am != oa) | (out.view(np.uint32) != oo.view(np.uint32))
    print(case, split, "bad elems", bad.sum(), "of", bad.size)
    if bad.any():
        br = np.nonzero(bad.any(axis=(1, 2, 3)))[0]
        print(" bad rois", len(br), br[:40])
        for i in br[:3]:
            bc = np.nonzero(bad[i].any(axis=(1, 2)))[0]
            print("  roi", i, rois[i], "bad ch", bc, "bins bad", np.nonzero(bad[i, bc[0]].ravel())[0])
            print("   got", am[i, bc[0]].ravel()[:20]); print("   exp", oa[i, bc[0]].ravel()[:20])
