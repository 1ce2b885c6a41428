"""Drop-in for utils/flowmur_generate_trigger.py: SNR mix, MFCC, its backward and the trigger
optimisation loop run in libabd (abd_amd.flowmur)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _root  # noqa: F401,E402
from abd_amd.triggers import deploy_trigger_to_waveform  # noqa: F401,E402
from abd_amd.flowmur import generate_trigger, pretrain_model  # noqa: F401,E402
