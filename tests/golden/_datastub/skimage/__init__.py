"""Golden-generation stand-in for scikit-image (absent from this image): the
data-loader golden needs only image SHAPES (utils/data_loader.py:63-70), so
``io.imread`` returns zeros of the shape registered for the file name and
``transform.resize`` zeros of the requested shape.  Used ONLY by
tests/golden/make_golden_data.py."""
