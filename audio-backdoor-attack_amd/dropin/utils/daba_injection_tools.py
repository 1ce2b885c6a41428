"""Drop-in for utils/daba_injection_tools.py: DABA poisoning with batched device selection/injection."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _root  # noqa: F401,E402
from abd_amd.features import librosa_MFCC  # noqa: F401,E402
from abd_amd.daba import load_victim_model, my_custom_random, daba_poison_data  # noqa: F401,E402
