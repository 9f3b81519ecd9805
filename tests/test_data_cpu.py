"""Ground-truth data contract (utils/data_loader.py:63-117) -- host code, CPU.

The hand-derived cases below follow utils/data_loader.py line by line; the
golden test at the end pins the contract to the GENUINE loader, run by
tests/golden/make_golden_data.py with skimage / torchvision.transforms /
xmltodict (absent here) stood in for -- the XML-to-dict step is a
restatement of xmltodict.parse (version unpinned), everything voc_data does
with the parsed document is the reference's own code.
"""
import numpy as np

from replication_faster_rcnn_amd import data


def _obj(name, ymin, xmin, ymax, xmax, difficult="0", bndbox=True):
    bb = (f"<bndbox><xmin>{xmin}</xmin><ymin>{ymin}</ymin><xmax>{xmax}</xmax>"
          f"<ymax>{ymax}</ymax></bndbox>") if bndbox else ""
    dif = f"<difficult>{difficult}</difficult>" if difficult is not None else ""
    return f"<object><name>{name}</name><pose>Left</pose>{dif}{bb}</object>"


def _xml(objs):
    return ("<annotation><folder>VOC2012</folder><filename>x.jpg</filename>"
            + "".join(objs) + "</annotation>")


def test_get_labels_rows_and_quirks():
    xml = _xml([
        _obj("dog", 10.5, 20.4, 100.5, 200.6),          # np.around: half to even
        _obj("person", 1, 2, 3, 4, difficult="1"),      # difficult -> label -1, box kept
        _obj("unicorn", 5, 6, 7, 8),                    # unknown class -> row -1
        _obj("car", 0, 0, 0, 0, bndbox=False),          # no bndbox -> row -1
        _obj("cat", 11.5, 12.5, 13.5, 14.5, difficult=None),  # no <difficult> -> row -1
        _obj("tvmonitor", 7, 8, 9, 10),
    ])
    label, box = data.get_labels(data.parse_voc_annotation(xml))
    assert label.dtype == np.float64 and label.shape == (32,) and box.shape == (32, 4)
    assert label[:6].tolist() == [12, -1, -1, -1, -1, 20]
    assert box[0].tolist() == [10.0, 20.0, 100.0, 201.0]       # [ymin, xmin, ymax, xmax]
    assert box[1].tolist() == [1, 2, 3, 4]
    assert (box[2:5] == -1).all() and box[5].tolist() == [7, 8, 9, 10]
    assert (label[6:] == -1).all() and (box[6:] == -1).all()
    # difficult=True keeps the difficult object
    label_d, _ = data.get_labels(data.parse_voc_annotation(xml), difficult=True)
    assert label_d[1] == 15


def test_single_object_iterates_keys():
    """One <object> parses to a dict; the reference iterates its keys, so the
    image ends up with no valid gt (utils/data_loader.py:97-113)."""
    label, box = data.get_labels(data.parse_voc_annotation(_xml([_obj("dog", 1, 2, 3, 4)])))
    assert (label == -1).all() and (box == -1).all()


def test_truncates_at_n_obj():
    xml = _xml([_obj("bird", i, i, i + 10, i + 10) for i in range(40)])
    label, box = data.get_labels(data.parse_voc_annotation(xml))
    assert (label == 3).all() and box[31].tolist() == [31, 31, 41, 41]


def test_rescale_and_collate():
    xml = _xml([_obj("dog", 50, 100, 150, 300), _obj("cat", 0, 0, 375, 500)])
    box, label = data.load_targets(xml, (375, 500), new_size=(600, 600))
    np.testing.assert_array_equal(box[0], [50 / 375 * 600, 100 / 500 * 600,
                                           150 / 375 * 600, 300 / 500 * 600])
    assert box[1].tolist() == [0.0, 0.0, 600.0, 600.0]
    assert (box[2:] == -1).all()  # padding rescaled negative -> -1
    b, lab = data.collate_targets([(box, label), (box, label)])
    assert tuple(b.shape) == (2, 32, 4) and tuple(lab.shape) == (2, 32)
    assert ((lab[0] != -1).sum()) == 2


def test_load_targets_vs_genuine_loader_golden():
    """tests/golden/data_loader.npz: (box, label) of every sample of the GENUINE
    utils/data_loader.py voc_data (tests/golden/make_golden_data.py, skimage /
    transforms / xmltodict stood in for -- the XML-to-dict step is a restatement
    of xmltodict.parse, version unpinned) over 29 annotations: single object,
    > 32 objects, difficult / unknown class / missing bndbox / missing
    difficult, fractional and negative coordinates, both ``difficult`` modes.
    Bit-exact (f64)."""
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "data_loader.npz"))
    for tag, dif in (("default", False), ("difficult", True)):
        for i, (xml, hw) in enumerate(zip(g["xml"], g["hw"])):
            box, label = data.load_targets(str(xml), tuple(int(v) for v in hw), new_size=(600, 600),
                                           difficult=dif)
            assert np.array_equal(label, g[f"label_{tag}"][i]), (tag, i)
            assert np.array_equal(box.view(np.uint64), g[f"box_{tag}"][i].view(np.uint64)), (tag, i)
