"""Drop-in for utils/styles_trigger.py: pedalboard effects are not accelerated yet (§8f item 4)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _root  # noqa: F401,E402
from abd_amd.triggers import get_boards, poison_style  # noqa: F401,E402
