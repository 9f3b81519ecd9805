"""skimage.io stand-in: imread -> zeros of the shape registered in SHAPES."""
import os

import numpy as np

SHAPES = {}


def imread(name):
    return np.zeros(SHAPES[os.path.basename(name)], np.uint8)
