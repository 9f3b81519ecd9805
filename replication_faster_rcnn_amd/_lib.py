"""ctypes binding of the C-ABI library ``libfrcnn_mi355x.so`` (include/frcnn_capi.h).

The library is built in-tree by ``__graft_entry__.build()`` (or ``make -C
replication_faster_rcnn_amd/csrc``).  There is no CPU fallback: if the
library is missing or no GPU is visible, every op raises.

torch is imported before the library is loaded so that the library's
``libamdhip64.so.7`` dependency resolves to the HIP runtime torch already
loaded (same soname): one runtime, one device-pointer space, torch streams
usable directly.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# FRCNN_LIB_PATH: A/B tools may point at another build of the same library
LIB_PATH = os.environ.get("FRCNN_LIB_PATH") or os.path.join(_HERE, "libfrcnn_mi355x.so")

P = ctypes.c_void_p
I32 = ctypes.c_int
I64 = ctypes.c_int64
F32 = ctypes.c_float
F64 = ctypes.c_double
SZ = ctypes.c_size_t


class ProposeParams(ctypes.Structure):
    """frcnn_propose_params (include/frcnn_capi.h)."""

    _fields_ = [("N", I32), ("A", I32), ("K", I32), ("feat_h", I32), ("feat_w", I32),
                ("feat_stride", I32), ("img_h", F32), ("img_w", F32), ("min_size", F32),
                ("pre_nms", I32), ("post_nms", I32), ("iou_threshold", F64)]


# name -> (restype, argtypes); must match include/frcnn_capi.h exactly
SIGNATURES = {
    "frcnn_version": (ctypes.c_char_p, []),
    "frcnn_last_error": (ctypes.c_char_p, []),
    "frcnn_device_cu_count": (I32, [P]),
    "frcnn_set_path": (I32, [ctypes.c_char_p, ctypes.c_char_p]),
    "frcnn_roi_pool_fwd_kernel": (I32, [I64, I32, I32, I32, I32, I32, I32, I32, I32, P, ctypes.c_char_p, SZ]),
    "frcnn_roi_pool_bwd_kernel": (I32, [I64, I32, I32, I32, I32, I32, I32, ctypes.c_char_p, SZ]),
    "frcnn_stream_create": (I32, [P, I32, P]),
    "frcnn_stream_destroy": (I32, [P]),
    "frcnn_stream_cu_count": (I32, [P, P]),
    "frcnn_probe_hw_ids": (I32, [P, I32, I32, P]),
    "frcnn_anchor_base": (I32, [P, I32, P, I32, F64, P, P]),
    "frcnn_generate_anchors": (I32, [P, I32, I32, I32, I32, P, P]),
    "frcnn_reg2bbox": (I32, [P, P, I64, P, P]),
    "frcnn_rpn_head_epilogue": (I32, [P, P, I32, I32, I32, I32, P, P, P, P]),
    "frcnn_propose_workspace_size":(SZ, [ctypes.POINTER(ProposeParams)]),
    "frcnn_propose": (I32, [ctypes.POINTER(ProposeParams), P, P, P, P, P, P, P, P, SZ, P]),
    "frcnn_nms_workspace_size": (SZ, [I64]),
    "frcnn_nms": (I32, [P, P, I64, F64, P, P, P, SZ, P]),
    "frcnn_roi_transform": (I32, [P, P, I64, F32, F32, I32, I32, P, P]),
    "frcnn_roi_pool_fwd_workspace_size": (SZ, [I64, I32, I32]),
    "frcnn_roi_pool_fwd": (I32, [P, P, I64, I32, I32, I32, I32, I32, I32, F32, I32, P, P, P, SZ, P]),
    "frcnn_roi_pool_fwd_head": (I32, [P, P, P, I64, I32, I32, I32, I32, I32, I32, F32, F32, F32, I32,
                                      P, P, P, P, SZ, P]),
    "frcnn_roi_pool_bwd_workspace_size": (SZ, [I64, I32, I32, I32]),
    "frcnn_roi_pool_bwd": (I32, [P, P, P, I64, I32, I32, I32, I32, I32, I32, F32, P, P, SZ, P]),
    "frcnn_bbox_iou": (I32, [P, I32, I64, P, I32, I64, P, P]),
    "frcnn_bbox2reg": (I32, [P, I32, P, I32, I64, P, P]),
    "frcnn_anchor_target_workspace_size": (SZ, [I32, I32, I32]),
    "frcnn_anchor_target": (I32, [I32, I32, I32, P, P, P, I32, F64, F64, F64, P, P, P, P, P, P,
                                  SZ, P]),
    "frcnn_anchor_target_prepare": (I32, [I32, I32, I32, P, P, P, F64, F64, P, SZ, P]),
    "frcnn_anchor_target_sample": (I32, [I32, I32, I32, P, I32, F64, P, P, P, P, P, P, SZ, P]),
    "frcnn_proposal_target_workspace_size": (SZ, [I32, I32, I32, I32]),
    "frcnn_proposal_target": (I32, [I32, I32, P, P, I32, P, P, I32, F64, F64, F64, F64, P, P, P,
                                    P, P, P, P, P, SZ, P]),
    "frcnn_anchor_target_draw": (I32, [I32, I32, I32, I32, F64, P, P, SZ, P]),
    "frcnn_anchor_target_finish": (I32, [I32, I32, I32, P, P, P, P, P, P, SZ, P]),
    "frcnn_proposal_target_draw": (I32, [I32, I32, I32, I32, F64, P, P, P, SZ, P]),
    "frcnn_proposal_target_finish": (I32, [I32, I32, I32, I32, P, P, P, P, P, P, P, SZ, P]),
    "frcnn_proposal_target_prepare": (I32, [I32, I32, P, P, I32, P, P, I32, F64, F64, F64, P, SZ, P]),
    "frcnn_proposal_target_sample": (I32, [I32, I32, I32, I32, F64, P, P, P, P, P, P, P, P, SZ, P]),
    "frcnn_anchor_target_draw_status": (I32, [I32, I32, I32, P, SZ, P]),
    "frcnn_proposal_target_draw_status": (I32, [I32, I32, I32, I32, P, SZ, P]),
    "frcnn_target_draws": (I32, [I32, I32, I32, I32, F64, P, SZ, I32, I32, I32, F64, P, SZ, P, P, P]),
}

# diagnostic entry points of instrumented builds only (not in include/frcnn_capi.h)
DEBUG_SIGNATURES = {
    "frcnn_debug_sampler_prof": (I32, [P, I32]),  # -DFRCNN_SAMPLER_PROF (tools/probe_sampler.py)
}

_lib = None
_gpu_checked = False


class FrcnnError(RuntimeError):
    pass


def load(require_gpu: bool = True):
    """Load the library (raises FrcnnError if it was not built).  With
    ``require_gpu`` also insist that a HIP device is visible."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FrcnnError(f"HIP library not built: {LIB_PATH} missing "
                             "(run __graft_entry__.build() or make -C replication_faster_rcnn_amd/csrc)")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("FRCNN_LIB_PATH") and not hasattr(lib, name):
                continue  # an older build under A/B: bind what it exports
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        for name, (res, args) in DEBUG_SIGNATURES.items():
            if hasattr(lib, name):
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
        _lib = lib
    global _gpu_checked
    if require_gpu and not _gpu_checked:
        if not torch.cuda.is_available():
            raise FrcnnError("replication_faster_rcnn_amd needs an MI355X (no HIP device visible); "
                             "there is no CPU fallback")
        _gpu_checked = True
    return _lib


def check(rc: int, what: str):
    if rc != 0:
        msg = _lib.frcnn_last_error().decode()
        raise FrcnnError(f"{what} failed (rc={rc}): {msg}")


_raw_stream = torch._C._cuda_getCurrentRawStream  # hipStream_t of the current torch stream (int)
_cur_device = torch._C._cuda_getDevice


def stream_ptr(device=None) -> int:
    """hipStream_t (as an int, for c_void_p arguments) of torch's current
    stream on `device` (default: the current device).  The raw torch._C
    getters are used on the issue path: torch.cuda.current_stream() builds a
    Stream object (~2.5 us per call)."""
    if device is None:
        return _raw_stream(_cur_device())
    if isinstance(device, int):
        return _raw_stream(device)
    d = torch.device(device)
    return _raw_stream(d.index if d.index is not None else _cur_device())


def ptr(t):
    """Device address of a tensor (int) or None (NULL) for c_void_p arguments."""
    return t.data_ptr() if t is not None else None


def device():
    """The device the HIP path runs on (current CUDA/HIP device)."""
    return torch.device("cuda", torch.cuda.current_device())


def workspace(nbytes: int, dev) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=dev)


_ws_cache = {}


def cached_workspace(tag: str, nbytes: int, dev) -> torch.Tensor:
    """Grow-only scratch buffer per (op, device, current stream): the C-ABI's
    workspaces are stream-ordered scratch, so one buffer per stream serves every
    call on that stream (no allocation on the issue path).  Allocated while the
    stream is current, so the caching allocator orders its reuse on that stream."""
    di = dev.index if isinstance(dev, torch.device) and dev.index is not None else _cur_device()
    key = (tag, di, _raw_stream(di))
    ws = _ws_cache.get(key)
    if ws is None or ws.numel() < nbytes:
        ws = torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=torch.device("cuda", di))
        _ws_cache[key] = ws
    return ws


def cu_count() -> int:
    lib = load()
    n = ctypes.c_int(0)
    check(lib.frcnn_device_cu_count(ctypes.byref(n)), "device_cu_count")
    return int(n.value)


def cu_stream(cu_mask=None) -> torch.cuda.ExternalStream:
    """A torch stream on the CUs listed in ``cu_mask`` (iterable of CU indices,
    hipExtStreamCreateWithCUMask numbering; None = every CU).  The HIP stream
    lives as long as the process (frcnn_stream_destroy is left to the caller
    via ``stream.frcnn_handle``)."""
    lib = load()
    h = ctypes.c_void_p(0)
    if cu_mask is None:
        check(lib.frcnn_stream_create(None, 0, ctypes.byref(h)), "stream_create")
    else:
        n = cu_count()
        words = (ctypes.c_uint32 * ((n + 31) // 32))()
        for c in cu_mask:
            if not 0 <= int(c) < n:
                raise ValueError(f"CU {c} out of range [0, {n})")
            words[int(c) // 32] |= 1 << (int(c) % 32)
        check(lib.frcnn_stream_create(words, len(words), ctypes.byref(h)), "stream_create")
    s = torch.cuda.ExternalStream(h.value, device=device())
    s.frcnn_handle = h.value
    return s


def stream_cu_count(stream) -> int:
    lib = load()
    n = ctypes.c_int(0)
    check(lib.frcnn_stream_cu_count(ctypes.c_void_p(stream.cuda_stream), ctypes.byref(n)),
          "stream_cu_count")
    return int(n.value)


def roi_pool_fwd_kernel(R, N, C, H, W, PH=7, PW=7, rois_sorted=True, head=True, stream=None) -> str:
    """frcnn_roi_pool_fwd_kernel: the template name of the RoIPool forward kernel
    a call of this shape launches on `stream` (default: the current stream)."""
    lib = load()
    s = stream if stream is not None else torch.cuda.current_stream()
    buf = ctypes.create_string_buffer(128)
    check(lib.frcnn_roi_pool_fwd_kernel(int(R), int(N), int(C), int(H), int(W), int(PH), int(PW),
                                        int(bool(rois_sorted)), int(bool(head)),
                                        ctypes.c_void_p(s.cuda_stream), buf, 128), "roi_pool_fwd_kernel")
    return buf.value.decode()


def roi_pool_bwd_kernel(R, N, C, H, W, PH=7, PW=7) -> str:
    """frcnn_roi_pool_bwd_kernel: the template name of the RoIPool backward kernel
    a call of this shape launches."""
    lib = load()
    buf = ctypes.create_string_buffer(128)
    check(lib.frcnn_roi_pool_bwd_kernel(int(R), int(N), int(C), int(H), int(W), int(PH), int(PW), buf, 128),
          "roi_pool_bwd_kernel")
    return buf.value.decode()


def set_path(op: str, path) -> None:
    """frcnn_set_path: select a kernel path ("auto" restores the default)."""
    lib = load(require_gpu=False)
    check(lib.frcnn_set_path(op.encode(), str(path).encode()), f"set_path({op}, {path})")


@contextlib.contextmanager
def kernel_path(op: str, path):
    """Run a block with one op's kernel path forced (tests / A-B tools)."""
    set_path(op, path)
    try:
        yield
    finally:
        set_path(op, "auto")
