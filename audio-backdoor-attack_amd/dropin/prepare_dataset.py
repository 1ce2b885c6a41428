"""Drop-in for the reference's prepare_dataset.py: MFCC on the MI355X + the dataset plumbing.

Put ``audio-backdoor-attack_amd/dropin`` ahead of the reference checkout on
``sys.path``; the attack scripts then import this module unchanged.
"""
import os

import numpy as np
import torch

import _root  # noqa: F401
from abd_amd import resident as _resident
from abd_amd.features import MFCC, resample  # noqa: F401  (prepare_dataset.py:35-47, :60)
from abd_amd.io import read_wav, LABEL_SETS, train_test_split_35

__all__ = ["MFCC", "BDDataset", "prepare_clean_dataset", "load_clean_data"]


class BDDataset(_resident.BDDataset):
    """Dict samples {'mfcc', 'label', 'poison_indicator'} (prepare_dataset.py:13-33).  Loaders over it
    feed training.train() / test() from HBM-resident copies (abd_amd/resident.py)."""


def prepare_clean_dataset(data_path, directory_name, labels, waveform_to_consider, n_mfcc, n_fft, hop_length,
                          sr=16000, save=True):
    """Load wavs (int16/32768), resample to sr on the device (prepare_dataset.py:60), keep clips >= sr
    samples, batched MFCC on the device, 80/20 split (seed 35)."""
    waves, labs = [], []
    for li, label in enumerate(labels):
        d = os.path.join(data_path, label)
        for name in os.listdir(d):
            if not name.endswith(".wav"):
                continue
            w, rate = read_wav(os.path.join(d, name))
            if rate != sr:  # only ultrasonic changes rate (16 kHz -> 44.1 kHz)
                w = resample(torch.from_numpy(w), rate, sr).numpy()
            if w.shape[0] >= waveform_to_consider:
                # prepare_dataset.py:61-63: `waveform[:waveform_to_consider]` slices the CHANNEL dim of
                # the (1, L) tensor, so every kept clip is kept whole; clips of different lengths make
                # the reference's np.array() fail, and np.stack fails here the same way
                waves.append(w[None, :])
                labs.append(li)
    waves = np.stack(waves).astype(np.float32)
    dev = torch.device("cuda", torch.cuda.current_device())
    mf = MFCC(torch.tensor(waves, device=dev), sr, n_mfcc, n_fft, hop_length).transpose(2, 3).cpu().numpy()
    tr, te = train_test_split_35(len(waves))
    out = (waves[tr], waves[te], mf[tr], mf[te], np.array(labs)[tr], np.array(labs)[te])
    if save:
        path = directory_name + "/clean/"
        os.makedirs(path, exist_ok=True)
        for n, a in zip(("clean_train_wav", "clean_test_wav", "clean_train_mfcc", "clean_test_mfcc",
                         "clean_train_label", "clean_test_label"), out):
            np.save(path + n, a)
    return out


def load_clean_data(args, load=False):
    """prepare_dataset.py:86-112: label set by --dataset, .npy cache under record/<result>/<dataset>/clean/."""
    data_path, labels = LABEL_SETS[args.dataset]
    directory_name = "record/" + args.result + "/" + args.dataset
    if load:
        path = directory_name + "/clean/"
        return tuple(np.load(path + n + ".npy") for n in ("clean_train_wav", "clean_test_wav", "clean_train_mfcc",
                                                          "clean_test_mfcc", "clean_train_label",
                                                          "clean_test_label"))
    return prepare_clean_dataset(data_path, directory_name, labels, args.sample_rate, args.n_mfcc, args.n_fft,
                                 args.hop_length, sr=args.sample_rate, save=True)
