"""skimage.transform stand-in: resize -> zeros of the requested shape."""
import numpy as np


def resize(image, shape):
    return np.zeros(tuple(shape) + tuple(image.shape[2:]), np.float64)
