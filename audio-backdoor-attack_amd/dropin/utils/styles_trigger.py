"""Drop-in for utils/styles_trigger.py: the pedalboard boards run as libabd kernels (csrc/effects.hip);
PitchShift (styles 0 and 3) runs as the board's phase-vocoder pitch stage."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _root  # noqa: F401,E402
from abd_amd.triggers import get_boards, poison_style  # noqa: F401,E402
