"""abd_amd -- MI355X-native poisoned-audio training hot path.

Drop-in accelerated replacements for quantum-bitss/Audio-Backdoor-Attack's per-batch
pipeline (trigger injection -> MFCC -> smallcnn forward/backward -> Adam -> ASR/acc
bookkeeping).  Compute runs in libabd.so (hand-written gfx950 HIP kernels behind a
C ABI, include/abd.h); this package is the Python host side that mirrors the
reference's interfaces.  Import it as ``import abd_amd`` (see abd_amd.py at the repo
root).
"""
from . import _lib  # noqa: F401
from ._lib import AbdError, load_library  # noqa: F401

__all__ = ["AbdError", "load_library", "features", "models", "training", "triggers", "pipeline", "flowmur"]


def __getattr__(name):
    import importlib
    if name in ("features", "models", "training", "triggers", "pipeline", "parallel_dp", "flowmur"):
        return importlib.import_module(f"{__name__}.{name}")
    raise AttributeError(name)
