"""Golden-generation stand-in for xmltodict (absent from this image; the
reference pins no version).  Restates the published behaviour of
``xmltodict.parse`` with its defaults, for the element-only documents of VOC
annotations: an element with children becomes a dict (insertion order), a
repeated child tag a list, a leaf its text (None when empty), attributes
``@name`` keys.  Used ONLY by tests/golden/make_golden_data.py so that the
genuine utils/data_loader.py runs; never on sys.path otherwise."""
import xml.etree.ElementTree as _ET


def _conv(el):
    d = {"@" + k: v for k, v in el.attrib.items()}
    kids = list(el)
    if not kids:
        if not d:
            return el.text
        if el.text and el.text.strip():
            d["#text"] = el.text
        return d
    for ch in kids:
        v = _conv(ch)
        if ch.tag in d:
            if not isinstance(d[ch.tag], list):
                d[ch.tag] = [d[ch.tag]]
            d[ch.tag].append(v)
        else:
            d[ch.tag] = v
    return d


def parse(text):
    root = _ET.fromstring(text)
    return {root.tag: _conv(root)}
