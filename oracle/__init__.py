"""ORACLE -- test infrastructure only.

CPU restatement of the reference's region-proposal + RoI hot path, used as
the checker for the HIP path.  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import anything from here; the
product package ``replication_faster_rcnn_amd`` never does.

* ``oracle.ref_numpy`` -- numpy restatement of ``utils/anchors.py``,
  ``utils/utils.py``, ``nets/rpn.py:47-79`` and ``nets/heads.py:42-48``.
* ``oracle.tv_ops`` (``tv_ops.c``) -- plain-C restatement of torchvision's CPU
  ``nms`` / ``roi_pool`` / ``_roi_pool_backward`` (third-party, not vendored in
  the reference, not installed here: "parity unpinned" against torchvision
  itself; pinned against the golden fixtures that the genuine reference
  Python produced with this restatement standing in for torchvision).
"""
