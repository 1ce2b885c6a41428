"""GPU: JingleBack style boards (pedalboard chains, libabd style board) vs oracle/effects.py."""
import numpy as np
import pytest
import torch

import abd_amd
from abd_amd import triggers as T
from abd_amd._lib import AbdError
from oracle import effects as oe

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    abd_amd.load_library()
    return torch.device("cuda", 0)


def clips(n=6, L=16000, seed=0):
    r = np.random.default_rng(seed)
    t = np.arange(L) / 16000
    x = 0.3 * np.sin(2 * np.pi * r.uniform(100, 3000, (n, 1)) * t) + r.normal(0, 0.05, (n, L))
    x[1] *= 4.0           # drive the ladder saturation into its clamp
    x[2, 8000:] = 0.0
    return np.clip(x, -1, 1).astype(np.float32)


def rel(a, b):
    return np.abs(a - b).max() / np.abs(b).max()


def test_style5_board_matches_oracle(dev):
    x = clips()
    board = T.get_boards()[5]
    y = T.poison_style(x[:, None], board, 16000)            # (n, 1, L) numpy like the reference call
    assert y.shape == (6, 1, 16000) and y.dtype == np.float32
    ref = oe.style5(x)
    assert rel(y[:, 0], ref) < 1e-4, rel(y[:, 0], ref)


def test_single_effects_match_oracle(dev):
    x = clips(4, 4003, seed=1)
    xd = torch.tensor(x, device=dev)
    for fx, ref in ((T.Distortion(30), oe.style1(x)),
                    (T.LadderFilter(mode=T.LadderFilter.Mode.LPF24, cutoff_hz=700, resonance=0.4, drive=2.0),
                     oe.ladder(x.astype(np.float64), 16000, mode=3, cutoff_hz=700, resonance=0.4, drive=2.0)),
                    (T.Phaser(rate_hz=3.0, depth=0.8, centre_frequency_hz=900, feedback=0.3, mix=0.7),
                     oe.phaser(x.astype(np.float64), 16000, 3.0, 0.8, 900, 0.3, 0.7))):
        y = T.Pedalboard([fx]).apply_device(xd, 16000).cpu().numpy()
        assert rel(y, ref) < 1e-4, (fx, rel(y, ref))


def test_fast_path_matches_generic_chain(dev, monkeypatch):
    """The compile-time chain kernel (ladder and phaser pipelined) == the runtime-dispatch kernel."""
    x = torch.tensor(clips(70, 5001, seed=3), device=dev)
    boards = [T.get_boards()[5], T.get_boards()[1],
              T.Pedalboard([T.Gain(-3), T.Distortion(10), T.Phaser(rate_hz=2, feedback=0.5)]),
              T.Pedalboard([T.Phaser(), T.Gain(6)])]            # non-canonical order: generic either way
    fast = [b.apply_device(x, 16000) for b in boards]
    monkeypatch.setenv("ABD_FX_GENERIC", "1")
    slow = [b.apply_device(x, 16000) for b in boards]
    for f, s in zip(fast, slow):
        assert float((f - s).abs().max()) <= 1e-6 * float(s.abs().max())


def test_gathered_rows_and_unsupported_styles(dev):
    x = torch.tensor(clips(8, 16000, seed=2), device=dev)
    board = T.get_boards()[5]
    rows = torch.tensor([5, 0, 5], dtype=torch.int32, device=dev)
    y = board.apply_device(x, 16000, rows=rows)
    full = board.apply_device(x, 16000)
    assert torch.equal(y[0], full[5]) and torch.equal(y[1], full[0]) and torch.equal(y[2], full[5])
    for s in (0, 3):   # PitchShift (Rubber Band)
        with pytest.raises(AbdError, match="not accelerated"):
            T.poison_style(x[:1].cpu().numpy(), T.get_boards()[s])


@pytest.mark.parametrize("style", [2, 4])
def test_chorus_reverb_styles_match_oracle(dev, style):
    x = clips(5, 16000, seed=4)
    y = T.poison_style(x[:, None], T.get_boards()[style], 16000)[:, 0]
    ref = oe.style2(x) if style == 2 else oe.style4(x)
    assert rel(y, ref) < 1e-4, rel(y, ref)
    # the reverb tail really is there (wet energy after the input stops)
    if style == 4:
        assert np.abs(y[2, 12000:]).max() > 1e-3
