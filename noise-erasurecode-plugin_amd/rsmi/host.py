"""Loader of the C++ host layer (noise-erasurecode-plugin_amd/host/: the
ShardPlugin mirror of main.go, the infectious-style FEC, the
erasurecode.Shard codec, the C++ config-1 timing harness), built into
lib/_rsmi_host*.so by csrc/Makefile.

The module must be the in-tree build next to lib/librsmi.so (it links that
engine through its rpath): a _rsmi_host found anywhere else on sys.path would
be another build of the mirror, so it is refused.  Raises ImportError if the
module was not built."""
import importlib
import os
import sys

_LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib")
if _LIB not in sys.path:
    sys.path.insert(0, _LIB)

_mod = importlib.import_module("_rsmi_host")
if os.path.dirname(os.path.abspath(_mod.__file__)) != _LIB:
    raise ImportError(f"_rsmi_host loaded from {_mod.__file__}, not the in-tree build in {_LIB}")

__all__ = [name for name in vars(_mod) if not name.startswith("_")]
globals().update({name: getattr(_mod, name) for name in __all__})
