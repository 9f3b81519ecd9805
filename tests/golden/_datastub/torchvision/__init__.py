"""torchvision stand-in for the data-loader golden: ``transforms`` (image
normalisation, not checked) here, and ``ops`` from tests/golden/_tvstub
(utils/utils.py, which the loader imports for the class table, imports it).
Used ONLY by tests/golden/make_golden_data.py."""
import os as _os

__path__.append(_os.path.join(_os.path.dirname(_os.path.dirname(_os.path.dirname(__file__))),
                              "_tvstub", "torchvision"))
