"""CPU-side checks of the drop-in boundary (no compute calls, no GPU)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "frcnn_capi.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(frcnn_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_path():
    syms = declared_symbols()
    for s in ["frcnn_propose", "frcnn_nms", "frcnn_roi_pool_fwd", "frcnn_roi_pool_bwd",
              "frcnn_generate_anchors", "frcnn_anchor_base", "frcnn_reg2bbox"]:
        assert s in syms


def test_library_exports_every_declared_symbol():
    from replication_faster_rcnn_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail("libfrcnn_mi355x.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for s in declared_symbols():
        assert hasattr(lib, s), s
    # the ctypes table covers exactly the header
    assert sorted(_lib.SIGNATURES) == declared_symbols()


def test_loader_fails_loudly_without_gpu():
    import torch
    from replication_faster_rcnn_amd import _lib
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(_lib.FrcnnError):
        _lib.load(require_gpu=True)
    lib = _lib.load(require_gpu=False)
    assert b"gfx950" in lib.frcnn_version()


def test_argument_validation_without_gpu():
    """Shape errors are reported before any HIP call (rc=-1 + message)."""
    from replication_faster_rcnn_amd import _lib
    lib = _lib.load(require_gpu=False)
    rc = lib.frcnn_roi_pool_fwd(None, None, 1, 1, 1, 1, 1, 0, 7, 1.0, 0, None, None, None, 0, None)
    assert rc == -1 and b"output_size" in lib.frcnn_last_error()
    p = _lib.ProposeParams()
    assert lib.frcnn_propose_workspace_size(ctypes.byref(p)) == 0  # N=0 rejected
    p.N, p.A, p.pre_nms, p.post_nms = 2, 21546, 6000, 300
    ws = lib.frcnn_propose_workspace_size(ctypes.byref(p))
    assert ws > 2 * 6000 * 94 * 8  # holds the NMS bitmask
    assert lib.frcnn_nms_workspace_size(0) == 0


def test_set_path_accepts_the_documented_paths_only():
    """frcnn_set_path (host-only, no HIP call): every op / path the header documents is
    accepted, anything else is rejected with rc=-1 and a message naming it."""
    from replication_faster_rcnn_amd import _lib
    lib = _lib.load(require_gpu=False)
    ok = {"roi_pool_fwd": ["auto", "wave", "dense", "generic"],
          "roi_pool_bwd": ["auto", "ring", "plain"],
          "propose": ["auto", "hybrid", "lazy", "wide"],
          "roi_pool_fwd_store": ["auto", "temporal", "nt"],
          "sampler": ["auto", "walk", "chip", "chip_only", "chip_tight"],
          "roi_pool_split": ["auto", "0", "7", "64"],
          "roi_pool_cg": ["auto", "4", "8", "16"]}
    try:
        for op, paths in ok.items():
            for p in paths:
                assert lib.frcnn_set_path(op.encode(), p.encode()) == 0, (op, p)
        for op, p in [("roi_pool_fwd_store", "streaming"), ("roi_pool_split", "65"), ("roi_pool_split", "x"),
                      ("roi_pool_cg", "2"), ("sampler", "tiles"), ("sampler", "chip_wide"), ("roi_pool_fwd", "key"),
                      ("roi_pool_fwd", "pair"), ("roi_pool_bwd", "band"), ("no_such_op", "auto")]:
            assert lib.frcnn_set_path(op.encode(), p.encode()) == -1, (op, p)
            assert p.encode() in lib.frcnn_last_error()
    finally:
        for op in ok:
            lib.frcnn_set_path(op.encode(), b"auto")
