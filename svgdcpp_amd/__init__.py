"""svgdcpp_amd -- MI355X-native SVGD inner step behind the SVGDCpp plugin API.

The compute path is the HIP library ``libsvgdcpp_amd.so`` (kernels for gfx950
+ C ABI, include/svgdcpp_amd/svgd_capi.h).  This package is the Python host
mirror of the reference API (see api.py) plus the ctypes binding (_capi.py).
Importing the API does not touch the GPU; creating an SVGD/Context does.
"""
from . import _capi
from .api import (SVGD, AdaGrad, Adam, Context, DeviceError, DimensionMismatchException,
                  GaussianRBFKernel, GaussianSum, Kernel, Model, MultivariateNormal, Optimizer,
                  RMSProp, SVGDOptions, UnsetException)

__all__ = [
    "SVGD", "SVGDOptions", "Context", "Model", "MultivariateNormal", "GaussianSum", "Kernel",
    "GaussianRBFKernel", "Optimizer", "Adam", "AdaGrad", "RMSProp", "DimensionMismatchException",
    "UnsetException", "DeviceError", "lib",
]


def lib():
    """The loaded C-ABI library (raises ImportError if it was not built)."""
    return _capi.lib()
