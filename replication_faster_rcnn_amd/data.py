"""Ground-truth data contract of the reference loader (utils/data_loader.py),
SURVEY.md §8(f) row 4.

The target creators (``targets``) and the training step consume gt exactly as
``voc_data`` produces it: ``box`` f64 [32, 4] in ``[ymin, xmin, ymax, xmax]``
order (row = height axis, the reference's "x"), rounded with ``np.around``,
rescaled to ``new_size``, every negative entry set to -1; ``label`` f64 [32]
with -1 for padding, difficult objects and unparsable objects.  Valid gt rows
are ``label != -1`` (train.py:74-76).

Host-side by nature (XML text, a few dozen numbers per image): this module is
the format, not a kernel.  Image decoding / resize / normalisation
(skimage, torchvision.transforms; utils/data_loader.py:37,70-73) are not on the
hot path and those libraries are absent here.
"""
from __future__ import annotations

import xml.etree.ElementTree as ET

import numpy as np

from .utils import PASCAL_VOC_CLASSES, PASCAL_VOC_NUM_CLASSES

CLASS2NUM = dict(zip(PASCAL_VOC_CLASSES, range(PASCAL_VOC_NUM_CLASSES)))


def _etree_to_dict(el):
    """ElementTree -> the nested dict xmltodict.parse builds for a VOC
    annotation: leaves are text, a tag seen once is a dict, repeated tags a list."""
    children = list(el)
    if not children:
        return el.text
    out = {}
    for ch in children:
        v = _etree_to_dict(ch)
        if ch.tag in out:
            if not isinstance(out[ch.tag], list):
                out[ch.tag] = [out[ch.tag]]
            out[ch.tag].append(v)
        else:
            out[ch.tag] = v
    return out


def parse_voc_annotation(xml_text: str) -> dict:
    """xmltodict.parse(...) of a VOC annotation file (utils/data_loader.py:92)."""
    root = ET.fromstring(xml_text)
    return {root.tag: _etree_to_dict(root)}


def get_labels(doc: dict, difficult: bool = False, n_obj: int = 32, class2num=CLASS2NUM):
    """utils/data_loader.py:81-117 ``voc_data._get_labels`` on a parsed annotation.

    Kept as the reference behaves, quirks included (they decide which gt boxes
    the target creators see):
    * a single ``<object>`` parses to a dict, and the reference iterates its
      KEYS, so every row it touches becomes -1 (no valid gt for that image);
    * an unknown class name, a missing/unparsable bndbox or (with
      ``difficult=False``) a missing ``difficult`` tag marks the row -1;
    * boxes are ``np.around``-ed (half to even) AFTER parsing, -1 rows included.
    Returns (labels f64 [n_obj], boxes f64 [n_obj, 4]).
    """
    labels = -1 * np.ones(n_obj)
    boxes = -1 * np.ones([n_obj, 4])
    objects = doc["annotation"]["object"]
    for obj_ind, obj in enumerate(objects):
        if obj_ind >= n_obj:
            break
        try:
            labels[obj_ind] = class2num[obj["name"]]
            bb = obj["bndbox"]
            boxes[obj_ind, :] = np.array([float(bb["ymin"]), float(bb["xmin"]),
                                          float(bb["ymax"]), float(bb["xmax"])])
            if not difficult and obj["difficult"] == "1":
                labels[obj_ind] = -1
        except Exception:  # the reference's bare except (utils/data_loader.py:112)
            labels[obj_ind] = -1
            boxes[obj_ind, :] = [-1, -1, -1, -1]
    return np.array(labels), np.around(boxes)


def rescale_boxes(box: np.ndarray, image_hw, new_size=(600, 600)) -> np.ndarray:
    """utils/data_loader.py:63-70: rows (cols 0,2) by image height, cols 1,3 by
    width, in f64 (divide, then multiply); negative entries -> -1.  Returns a
    new array (the reference edits in place)."""
    b = np.array(box, dtype=np.float64, copy=True)
    new_h, new_w = new_size
    b[:, [0, 2]] = b[:, [0, 2]] / image_hw[0] * new_h
    b[:, [1, 3]] = b[:, [1, 3]] / image_hw[1] * new_w
    b[b < 0] = -1
    return b


def load_targets(xml_text: str, image_hw, new_size=(600, 600), difficult=False, n_obj=32):
    """One ``voc_data.__getitem__``'s (box, label) pair (image handling aside)."""
    label, box = get_labels(parse_voc_annotation(xml_text), difficult=difficult, n_obj=n_obj)
    return rescale_boxes(box, image_hw, new_size), label


def collate_targets(samples):
    """DataLoader default collate of the (box, label) pairs -> the batch
    tensors train.py:59-76 indexes: box [N, 32, 4] f64, label [N, 32] f64."""
    import torch
    boxes = torch.from_numpy(np.stack([s[0] for s in samples]))
    labels = torch.from_numpy(np.stack([s[1] for s in samples]))
    return boxes, labels
