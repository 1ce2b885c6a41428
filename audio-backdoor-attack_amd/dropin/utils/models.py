"""Drop-in for utils/models.py: smallcnn runs on libabd; the other backbones are out of scope."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _root  # noqa: F401,E402
from abd_amd.models import smallcnn  # noqa: F401,E402


def _unsupported(name):
    def make(*a, **k):
        raise NotImplementedError(f"{name} is not accelerated by abd_amd (only smallcnn, the BASELINE model)")
    return make


largecnn = _unsupported("largecnn")
smalllstm = _unsupported("smalllstm")
lstmwithattention = _unsupported("lstmwithattention")
RNN = _unsupported("RNN")
ResNet = _unsupported("ResNet")
ResidualBlock = _unsupported("ResidualBlock")
