"""hydra_amd -- MI355X-native (gfx950) bucket-reduction hot path of hydra/Gloo.

The product is libhydra_hip.so (C-ABI, include/hydra_hip.h): a hand-written CDNA4 streaming
chunk-sum behind Gloo's reduce-function plug-point, its host-staged form, and the RCCL/xGMI ring.
This package is the thin Python face used by tests and bench.py.  See DESIGN.md.
"""
from ._lib import HydraError, build, lib  # noqa: F401

__all__ = ["HydraError", "build", "lib"]
