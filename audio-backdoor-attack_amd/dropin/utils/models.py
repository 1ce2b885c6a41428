"""Drop-in for utils/models.py.

``smallcnn`` (utils/models.py:17-65, the BASELINE model) runs on libabd.  The other backbones
(largecnn, smalllstm, lstmwithattention, RNN, ResNet -- out of scope) are the
reference's own classes, loaded from the checkout behind this package; the accelerated
``train()`` / ``test()`` refuse them with an AbdError rather than silently running PyTorch.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _root  # noqa: F401,E402
from abd_amd.models import smallcnn  # noqa: F401,E402

from . import reference_module  # noqa: E402

_OTHERS = ("largecnn", "smalllstm", "lstmwithattention", "RNN", "ResNet", "ResidualBlock")


def _missing(name):
    def make(*a, **k):
        raise NotImplementedError(f"{name}: no reference utils/models.py on sys.path to take it from "
                                  "(abd_amd accelerates smallcnn only)")
    return make


def __getattr__(name):
    """The other backbones resolve lazily (PEP 562): importing this module for smallcnn does not
    execute the reference's utils/models.py; the first access to one of them does, once."""
    if name not in _OTHERS:
        raise AttributeError(f"module {__name__!r} has no attribute {name!r}")
    ref = reference_module("models")
    obj = getattr(ref, name) if ref is not None and hasattr(ref, name) else _missing(name)
    globals()[name] = obj
    return obj


def __dir__():
    return sorted(set(globals()) | set(_OTHERS))
