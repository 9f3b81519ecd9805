"""Golden-generation stand-in for torchvision (absent from this image).

Only ``ops.nms`` and ``ops.roi_pool.roi_pool`` exist, and they delegate to the
oracle's C restatement of torchvision's CPU kernels.  Used ONLY by
tests/golden/make_golden.py so that the genuine reference modules
(utils/utils.py, nets/rpn.py, nets/heads.py) import and run; it is not part of
the product and is never on sys.path otherwise.
"""
