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


def test_gathered_rows_and_unsupported_chains(dev):
    x = torch.tensor(clips(8, 16000, seed=2), device=dev)
    for board in (T.get_boards()[5], T.get_boards()[3]):
        rows = torch.tensor([5, 0, 5], dtype=torch.int32, device=dev)
        y = board.apply_device(x, 16000, rows=rows)
        full = board.apply_device(x, 16000)
        assert torch.equal(y[0], full[5]) and torch.equal(y[1], full[0]) and torch.equal(y[2], full[5])
    for bad in (T.Pedalboard([T.Gain(3), T.PitchShift(5)]),                 # PitchShift opens a board only
                T.Pedalboard([T.LadderFilter(), T.Chorus()])):               # a stateful effect before Chorus
        with pytest.raises(AbdError):
            bad.apply_device(x, 16000)


def pitch_clips(n, L, sr, seed):
    """tones + a noise floor (no exact silence: the phase vocoder's phases of vanishing bins are
    rounding noise in any precision, and they persist into later frames)."""
    r = np.random.default_rng(seed)
    t = np.arange(L) / sr
    x = sum(a * np.sin(2 * np.pi * f * t + ph) for a, f, ph in
            zip(r.uniform(0.05, 0.3, (3, n, 1)), r.uniform(80, 0.2 * sr, (3, n, 1)), r.uniform(0, 6, (3, n, 1))))
    x = x + r.normal(0, 0.02, (n, L))
    return np.clip(x, -1, 1).astype(np.float32)


def device_pitch(board, x, sr):
    """Run a board through the C ABI with a test-owned workspace and return (output, the pitch
    stage's synthesized spectra Y (B, T, K) complex).  Y sits at workspace offset 0 ([clip][frame]
    [bin] float2), written by the phase recursion and only read afterwards."""
    from abd_amd import _lib as L
    xd = torch.tensor(x, device=dev_of())
    B, n = xd.shape
    h = board._plan(sr, n, xd.device)
    need = L.lib().abd_style_board_workspace_bytes(h, B)
    ws = torch.zeros(need, dtype=torch.uint8, device=xd.device)
    out = torch.empty_like(xd)
    L.check(L.lib().abd_style_board_apply(h, xd.data_ptr(), xd.stride(0), None, B, n, out.data_ptr(), out.stride(0),
                                          ws.data_ptr(), need, L.stream_ptr(xd.device)), "abd_style_board_apply")
    torch.cuda.synchronize()
    r, N, Hs = oe.pitch_params(sr, board.plugins[0].semitones)
    Ls, Tf, ia = oe.pitch_frames(n, r, Hs)
    K = N // 2 + 1
    y = ws[:B * Tf * K * 8].view(torch.float32).cpu().numpy().reshape(B, Tf, K, 2)
    return out.cpu().numpy(), y[..., 0] + 1j * y[..., 1]


def dev_of():
    return torch.device("cuda", torch.cuda.current_device())


@pytest.mark.parametrize("sr,L,semi", [(16000, 16000, 10.0), (16000, 5001, -7.0), (44100, 22050, 10.0)])
def test_pitch_shift_matches_oracle(dev, sr, L, semi):
    """The pitch stage (phase vocoder + resample, N = 1024 below 32 kHz, 2048 above) vs
    oracle/effects.py's float64 restatement: every sample within 1e-4 of the output's max, after
    replaying the device's phase-wrap decisions at genuine near-ties (dphi within rounding of +-pi:
    any precision may wrap either way there; oracle/effects.pitch_shift, ``replay``).
    (Rubber Band itself is absent: parity unpinned against pedalboard.)"""
    x = pitch_clips(4, L, sr, seed=int(sr + L))
    y, Y = device_pitch(T.Pedalboard([T.PitchShift(semi)]), x, sr)
    y2 = T.Pedalboard([T.PitchShift(semi)]).apply_device(torch.tensor(x, device=dev), sr).cpu().numpy()
    assert np.array_equal(y, y2)                                   # deterministic, workspace-independent
    ref, nrep = oe.pitch_shift(x, sr, semi, replay=Y)
    print(f"sr={sr} L={L} semi={semi}: {nrep} replayed wrap decisions of {Y.size}, rel err {rel(y, ref):.2e}")
    assert y.shape == x.shape
    assert nrep <= 1e-3 * Y.size
    assert rel(y, ref) < 1e-4, rel(y, ref)


def test_pitch_styles_0_and_3(dev):
    """styles 0 and 3 end to end (utils/styles_trigger.py:12-34): the tone moves by 10 semitones,
    style 3's Distortion -> Chorus chain runs on the shifted clip (Chorus delays ITS input)."""
    sr, L = 16000, 16000
    x = pitch_clips(3, L, sr, seed=7)
    t = np.arange(L) / sr
    x[0] = (0.3 * np.sin(2 * np.pi * 440.0 * t) + 0.01 * np.random.default_rng(1).normal(size=L)).astype(np.float32)
    y0 = T.poison_style(x[:, None], T.get_boards()[0], sr)[:, 0]
    yd, Y = device_pitch(T.get_boards()[0], x, sr)
    assert np.array_equal(y0, yd)
    ref0, _ = oe.pitch_shift(x, sr, 10.0, replay=Y)
    assert rel(y0, ref0) < 1e-4
    seg = y0[0, 2000:14000] * np.hanning(12000)
    peak = np.argmax(np.abs(np.fft.rfft(seg))) * sr / 12000
    assert abs(peak - 440.0 * 2 ** (10 / 12)) < 2.0, peak
    y3 = T.poison_style(x[:, None], T.get_boards()[3], sr)[:, 0]
    # the chain alone on the device's own shifted clips, then the whole board against the oracle
    # (same replayed pitch stage).  Tolerance: the chorus (depth 5: a 1-58 ms swept delay) reads a
    # hard-clipped signal (tanh x 10) whose slope reaches ~2 per sample, so a 1-ulp difference of
    # the float32 delay table (sin of the LFO phase on the host vs numpy) moves an output by ~1e-4
    chain = oe.chorus(np.tanh(y0.astype(np.float64) * oe.db_to_gain(20.0)), sr, 1.0, 5.0, 8.0, 0.0, 0.5)
    assert rel(y3, chain) < 1e-3, rel(y3, chain)
    ref3 = oe.style3(x, sr, shifted=ref0)
    assert rel(y3, ref3) < 2e-3, rel(y3, ref3)


@pytest.mark.parametrize("style", [2, 4])
def test_chorus_reverb_styles_match_oracle(dev, style):
    x = clips(5, 16000, seed=4)
    y = T.poison_style(x[:, None], T.get_boards()[style], 16000)[:, 0]
    ref = oe.style2(x) if style == 2 else oe.style4(x)
    assert rel(y, ref) < 1e-4, rel(y, ref)
    # the reverb tail really is there (wet energy after the input stops)
    if style == 4:
        assert np.abs(y[2, 12000:]).max() > 1e-3
