"""Drop-in for utils/daba_selection_tools.py: librosa MFCC, the pydub int16 overlay and the
trigger / host selection (batched per-utterance forwards) on the device."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _root  # noqa: F401,E402
from abd_amd.features import librosa_MFCC  # noqa: F401,E402
from abd_amd.io import read_wav_int16, write_wav_int16  # noqa: E402
from abd_amd import triggers as _t  # noqa: E402
from abd_amd.daba import (get_filenames, calc_ent, cross_entropy, one_sotamax_entropy,  # noqa: F401,E402
                          Cer_sotamax_entropy, Cer_triggers_selection, Inf_cross_entropy, Inf_hosts_selection,
                          trigger_selection_hosts_selection, gen_trigger_variants_db)


def single_trigger_injection_db(org_wav_path, trigger_wav_path, output_path, po_db):
    """pydub song1.overlay(song2 + (po_db - song2.dBFS)) -> 16-bit wav (daba_selection_tools.py:24-39)."""
    host, sr = read_wav_int16(org_wav_path)
    trig, _ = read_wav_int16(trigger_wav_path)
    out = _t.single_trigger_injection_db(host, trig, po_db)
    write_wav_int16(output_path, out, sr)
    return out, output_path
