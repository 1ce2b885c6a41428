"""Drop-in for utils/badnet_trigger.py."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _root  # noqa: F401,E402
from abd_amd.triggers import generate_trigger, add_trigger_to_mfcc  # noqa: F401,E402
