"""Drop-in for utils/ultra_trigger.py."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _root  # noqa: F401,E402
from abd_amd.triggers import GenerateTrigger, TriggerInfeasible  # noqa: F401,E402
