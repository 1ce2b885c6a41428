"""Small host I/O helpers: 16-bit PCM wav via the stdlib, label sets, the 80/20 split."""
from __future__ import annotations

import wave

import numpy as np

# prepare_dataset.py:86-97 / daba.py:42-51 label lists and data roots
LABEL_SETS = {
    "SCDv1-10": ("./data/SpeechCommands/speech_commands_v0.01",
                 ["yes", "no", "up", "down", "left", "right", "on", "off", "stop", "go"]),
    "SCDv1-30": ("./data/SpeechCommands/speech_commands_v0.01",
                 ["bed", "bird", "cat", "dog", "down", "eight", "five", "four", "go", "happy", "house", "left",
                  "marvin", "nine", "no", "off", "on", "one", "right", "seven", "sheila", "six", "stop", "three",
                  "tree", "two", "up", "wow", "yes", "zero"]),
    "SCDv2-10": ("./data/SpeechCommands/speech_commands_v0.02",
                 ["zero", "one", "two", "three", "four", "five", "six", "seven", "eight", "nine"]),
    "SCDv2-26": ("./data/speech_commands_v0.02",
                 ["zero", "backward", "bed", "bird", "cat", "dog", "down", "follow", "forward", "go", "happy",
                  "house", "learn", "left", "marvin", "no", "off", "on", "right", "sheila", "stop", "tree", "up",
                  "visual", "wow", "yes"]),
    # BASELINE configs[1] names a 35-class Speech Commands v2 set that the reference lacks:
    # the full v0.02 vocabulary (SURVEY.md §0 discrepancy 1)
    "SCDv2-35": ("./data/SpeechCommands/speech_commands_v0.02",
                 ["backward", "bed", "bird", "cat", "dog", "down", "eight", "five", "follow", "forward", "four",
                  "go", "happy", "house", "learn", "left", "marvin", "nine", "no", "off", "on", "one", "right",
                  "seven", "sheila", "six", "stop", "three", "tree", "two", "up", "visual", "wow", "yes", "zero"]),
}


def read_wav_int16(path):
    with wave.open(path) as w:
        if w.getsampwidth() != 2:
            raise ValueError(f"{path}: only 16-bit PCM is supported")
        a = np.frombuffer(w.readframes(w.getnframes()), dtype=np.int16)
        if w.getnchannels() > 1:
            a = a.reshape(-1, w.getnchannels())[:, 0]
        return a.copy(), w.getframerate()


def read_wav(path):
    """torchaudio.load normalisation: int16 / 32768 (pinned by test.ipynb cell 12)."""
    a, sr = read_wav_int16(path)
    return a.astype(np.float32) / 32768.0, sr


def write_wav_int16(path, samples, sr):
    with wave.open(path, "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(int(sr))
        w.writeframes(np.asarray(samples, dtype=np.int16).tobytes())


def train_test_split_35(n, test_size=0.2):
    """sklearn train_test_split(..., test_size=0.2, random_state=35) index split (prepare_dataset.py:66)."""
    from sklearn.model_selection import train_test_split
    idx = np.arange(n)
    tr, te = train_test_split(idx, test_size=test_size, random_state=35)
    return tr, te
