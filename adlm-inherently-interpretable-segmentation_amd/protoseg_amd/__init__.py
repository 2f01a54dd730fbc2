"""protoseg_amd — the ProtoSeg prototype layer and prototype push on MI355X (gfx950).

Host-side mirror of the reference's PPNet / push interface over ``libprotoseg_hip.so``
(C ABI in include/protoseg_hip.h). Importing this package does not touch the GPU; the
first kernel call loads the library and fails loudly if it (or a ROCm device) is missing.
"""
from ._lib import LIB_PATH, ProtosegError, version  # noqa: F401

__all__ = ["LIB_PATH", "ProtosegError", "version"]
