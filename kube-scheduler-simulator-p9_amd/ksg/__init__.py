"""MI355X scheduling-cycle engine: Python binding of the C ABI in include/ksg.h.

The product path is libksg.so (HIP kernels + C++ host layer).  This package only
loads it through ctypes; there is no CPU fallback — importing `Scheduler` on a
machine without the built library raises immediately.
"""
from .engine import KsgError, Scheduler, PodResult, lib_path, load_library  # noqa: F401
from . import generator  # noqa: F401

PLUGINS = ["NodeResourcesFit", "NodeResourcesBalancedAllocation", "TaintToleration",
           "NodeAffinity", "PodTopologySpread", "InterPodAffinity"]
