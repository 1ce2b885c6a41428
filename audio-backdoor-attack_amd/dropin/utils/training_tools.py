"""Drop-in for utils/training_tools.py (fused device train/test steps)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _root  # noqa: F401,E402
from abd_amd.training import train, test, clean_train, clean_test, EarlyStoppingModel  # noqa: F401,E402
