"""Golden fixture of the ground-truth data contract
from the GENUINE reference loader utils/data_loader.py.

Run in the build container only (it needs /root/reference):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_data.py

utils/data_loader.py imports skimage, torchvision.transforms and xmltodict at
module top; none is installed here, so tests/golden/_datastub stands in:
skimage returns arrays of registered shapes (only the image SHAPE enters the
box rescale), the transforms pass images through (image normalisation is not
part of the contract), and xmltodict.parse is a restatement of its published
behaviour (version unpinned: the reference pins none).  So ``voc_data``'s
own code -- the ImageSets list, _get_labels with its quirks (single-object
dict iteration, unknown class, missing bndbox / difficult, the bare except,
np.around) and __getitem__'s rescale / negative-to--1 -- is pinned by the
genuine reference; the XML-to-dict step is the restatement.

Writes tests/golden/data_loader.npz: the annotation XML texts, image shapes,
and the (box, label) every sample of the dataset yields.
"""
from __future__ import annotations

import os
import sys
import tempfile

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))  # the repo: _tvstub's ops use the oracle
sys.path.insert(0, os.path.join(HERE, "_datastub"))
sys.path.insert(0, REF)

import numpy as np  # noqa: E402
from skimage import io as stub_io  # noqa: E402

from utils import data_loader as ref_dl  # noqa: E402  (reference utils/data_loader.py)

assert ref_dl.__file__.startswith(REF), ref_dl.__file__
CLASSES = list(ref_dl.PASCAL_VOC_CLASSES)


def obj(name, ymin, xmin, ymax, xmax, difficult="0", bndbox=True, pose=True):
    bb = (f"<bndbox><xmin>{xmin}</xmin><ymin>{ymin}</ymin><xmax>{xmax}</xmax>"
          f"<ymax>{ymax}</ymax></bndbox>") if bndbox else ""
    dif = f"<difficult>{difficult}</difficult>" if difficult is not None else ""
    ps = "<pose>Unspecified</pose><truncated>0</truncated>" if pose else ""
    return f"<object><name>{name}</name>{ps}{dif}{bb}</object>"


def doc(fname, objs, h, w):
    return (f"<annotation><folder>VOC2012</folder><filename>{fname}</filename>"
            f"<size><width>{w}</width><height>{h}</height><depth>3</depth></size>"
            f"<segmented>0</segmented>{''.join(objs)}</annotation>")


def cases():
    r = np.random.default_rng(2024)
    out = []
    # hand-made quirks
    out.append(([obj("dog", 10.5, 20.4, 100.5, 200.6), obj("person", 1, 2, 3, 4, difficult="1"),
                 obj("unicorn", 5, 6, 7, 8), obj("car", 0, 0, 0, 0, bndbox=False),
                 obj("cat", 11.5, 12.5, 13.5, 14.5, difficult=None), obj("tvmonitor", 7, 8, 9, 10)],
                (375, 500)))
    out.append(([obj("bird", 48, 30, 201, 333)], (333, 500)))               # one object: a dict
    out.append(([obj("bus", 0.5, 1.5, 2.5, 3.5), obj("cow", 2.5, 3.5, 4.5, 5.5)], (480, 640)))
    out.append(([obj(CLASSES[i % 20], i, 2 * i, i + 30, 2 * i + 40) for i in range(40)], (500, 486)))
    out.append(([obj("horse", -3, -5, 50, 60), obj("sheep", 10, 20, 5, 8)], (281, 500)))
    # random VOC-like annotations
    for k in range(24):
        h, w = int(r.integers(200, 501)), int(r.integers(200, 501))
        objs = []
        for _ in range(int(r.integers(2, 12))):
            y = np.sort(r.uniform(0, h, 2))
            x = np.sort(r.uniform(0, w, 2))
            dif = "1" if r.random() < 0.15 else "0"
            name = CLASSES[int(r.integers(0, 20))] if r.random() > 0.05 else "background"
            fmt = (lambda v: f"{v:.1f}") if r.random() < 0.5 else (lambda v: str(int(round(v))))
            objs.append(obj(name, fmt(y[0]), fmt(x[0]), fmt(y[1]), fmt(x[1]), difficult=dif))
        out.append((objs, (h, w)))
    return out


def main():
    cs = cases()
    with tempfile.TemporaryDirectory() as root:
        for d in ("ImageSets/Main", "Annotations", "JPEGImages"):
            os.makedirs(os.path.join(root, d))
        names, xmls, shapes = [], [], []
        for i, (objs, (h, w)) in enumerate(cs):
            n = f"2012_{i:06d}"
            x = doc(n + ".jpg", objs, h, w)
            open(os.path.join(root, "Annotations", n + ".xml"), "w").write(x)
            stub_io.SHAPES[n + ".jpg"] = (h, w, 3)
            names.append(n)
            xmls.append(x)
            shapes.append((h, w))
        open(os.path.join(root, "ImageSets/Main/aeroplane_train.txt"), "w").write(
            "".join(f"{n} {1 if i % 2 else -1}\n" for i, n in enumerate(names)))
        res = {}
        for difficult in (False, True):
            ds = ref_dl.voc_data(root, "train", difficult=difficult, new_size=(600, 600))
            boxes, labels = [], []
            for i in range(len(ds)):
                s = ds[i]
                boxes.append(np.asarray(s["box"], np.float64))
                labels.append(np.asarray(s["label"], np.float64))
            tag = "difficult" if difficult else "default"
            res[f"box_{tag}"] = np.stack(boxes)
            res[f"label_{tag}"] = np.stack(labels)
    np.savez_compressed(os.path.join(HERE, "data_loader.npz"), xml=np.array(xmls), hw=np.array(shapes),
                        **res)
    print("wrote data_loader.npz:", len(xmls), "annotations")


if __name__ == "__main__":
    main()
