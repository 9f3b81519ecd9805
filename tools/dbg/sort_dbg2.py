import sys, os, numpy as np, torch
sys.path.insert(0, os.getcwd())
from replication_faster_rcnn_amd import _lib, ops
from oracle import ref_numpy as orc
DEV = torch.device("cuda", 0)
def rr(r, b, H, W, lo=-3, span=40):
    xy = r.uniform(lo, max(H, W) + 2, (len(b), 2)).astype(np.float32)
    wh = r.uniform(0, span, (len(b), 2)).astype(np.float32)
    return np.concatenate([np.asarray(b, np.float32)[:, None], xy, xy + wh], 1).astype(np.float32)
for case in ["invalid_ends", "gaps", "cfg4_shape", "ph5"]:
  for split in ["1", "3"]:
    r = np.random.default_rng(sum(map(ord, case)))
    N, C, H, W = 4, 16, 20, 27
    ph = (5, 5) if case == "ph5" else (7, 7)
    if case == "invalid_ends":
        b = np.concatenate([[-1, -1], np.sort(r.integers(0, N, 200)), [N, N, N + 3]])
    elif case == "gaps":
        b = np.sort(np.concatenate([np.zeros(60, int), np.full(90, 3)]))
    elif case == "cfg4_shape":
        N, C, H, W = 1, 16, 50, 84
        b = np.zeros(500, int)
    else:
        b = np.sort(r.integers(0, N, 700))
    x = r.standard_normal((N, C, H, W), dtype=np.float32)
    x[:, :, 2:9, 3:12] = np.round(x[:, :, 2:9, 3:12])
    rois = rr(r, b, H, W)
    res = {}
    for path in ["sort", "wave"]:
        with _lib.kernel_path("roi_pool_split", split), _lib.kernel_path("roi_pool_fwd", path):
            out, am = ops.roi_pool_with_argmax(torch.from_numpy(x).to(DEV), torch.from_numpy(rois).to(DEV), ph, rois_sorted=True)
        res[path] = (out.cpu().numpy(), am.cpu().numpy())
    oo, oa = orc.roi_pool_forward(x, rois, ph)
    lib = _lib.load()
    if hasattr(lib, "frcnn_debug_sort_check"):
        import ctypes
        buf = (ctypes.c_ulonglong * 16)()
        lib.frcnn_debug_sort_check(ctypes.cast(buf, ctypes.c_void_p), 1)
        print(case, split, "dbg", list(buf)[:10])
    valid = (b >= 0) & (b < N)
    for path in res:
        out, am = res[path]
        bad = ((am != oa) | (out.view(np.uint32) != oo.view(np.uint32)))[valid]
        print(case, split, path, "bad elems", bad.sum(), "of", bad.size)
        if bad.any():
            vi = np.nonzero(valid)[0]
            br = vi[np.nonzero(bad.any(axis=(1, 2, 3)))[0]]
            print(" bad rois", len(br), br[:40])
            for i in br[:3]:
                bb = (am[i] != oa[i]) | (out[i].view(np.uint32) != oo[i].view(np.uint32))
                bc = np.nonzero(bb.any(axis=(1, 2)))[0]
                print("  roi", i, rois[i], "bad ch", bc, "bins bad", np.nonzero(bb[bc[0]].ravel())[0])
                print("   got", am[i, bc[0]].ravel()[:25], out[i, bc[0]].ravel()[:6]); print("   exp", oa[i, bc[0]].ravel()[:25], oo[i, bc[0]].ravel()[:6])
