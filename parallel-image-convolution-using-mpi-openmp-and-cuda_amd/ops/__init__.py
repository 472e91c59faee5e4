"""Stencil operators: native HIP/CPU dispatch and the NumPy oracle."""
from .stencil import Engine, convolve, image_geometry  # noqa: F401
from .reference import numpy_convolve, numpy_step  # noqa: F401
