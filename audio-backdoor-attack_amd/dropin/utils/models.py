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
_ref = reference_module("models")


def _missing(name):
    def make(*a, **k):
        raise NotImplementedError(f"{name}: no reference utils/models.py on sys.path to take it from "
                                  "(abd_amd accelerates smallcnn only)")
    return make


for _n in _OTHERS:
    globals()[_n] = getattr(_ref, _n) if _ref is not None and hasattr(_ref, _n) else _missing(_n)
