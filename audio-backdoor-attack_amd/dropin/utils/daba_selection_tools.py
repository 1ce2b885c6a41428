"""Drop-in for utils/daba_selection_tools.py: librosa MFCC and the pydub int16 overlay on the device."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _root  # noqa: F401,E402
from abd_amd.features import librosa_MFCC  # noqa: F401,E402
from abd_amd.io import read_wav_int16, write_wav_int16  # noqa: E402
from abd_amd import triggers as _t  # noqa: E402


def single_trigger_injection_db(org_wav_path, trigger_wav_path, output_path, po_db):
    """pydub song1.overlay(song2 + (po_db - song2.dBFS)) -> 16-bit wav (daba_selection_tools.py:24-39)."""
    host, sr = read_wav_int16(org_wav_path)
    trig, _ = read_wav_int16(trigger_wav_path)
    out = _t.single_trigger_injection_db(host, trig, po_db)
    write_wav_int16(output_path, out, sr)
    return out, output_path


def gen_trigger_variants_db(poison_num):
    import random
    random.seed(35)
    v = [0, -5, -10, -15, -20, -25, -30, -35, -40]
    return [v[i % len(v)] for i in random.sample(range(0, poison_num), poison_num)]
