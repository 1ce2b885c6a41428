"""GPU parity of the persistent STFT kernels at the bench's sizes.

``stft_mel_fast_kernel`` is persistent: min(items, resident) blocks pull work items (frame pairs)
from 8 atomic queues, steal from the others, hand the next item over through LDS and reuse their
LDS buffers across items.  At B <= 32 every block runs one item, so only these sizes -- and the
capped grids (ABD_STFT_MAX_BLOCKS), where each block walks hundreds of items -- compare the
loop-carried path with the oracle.  Every utterance and every frame is checked against the float64
oracle (prepare_dataset.py:35-47 restated) at 1e-4 of the utterance's max |MFCC|.

The last test runs abd::mfcc on two streams at once with different inputs (ops are
re-entrant): each call takes its own workspace from the caching allocator on its stream.
"""
import numpy as np
import pytest
import torch

import abd_amd
from abd_amd import features as F
from abd_amd import synth
from abd_amd import _lib as L
from abd_amd.pipeline import ultrasonic_trigger
from oracle import mfcc as om

pytestmark = pytest.mark.gpu

RTOL = 1e-4   # fp32 device vs float64 oracle, relative to the utterance's max |MFCC|


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    abd_amd.load_library()
    return torch.device("cuda", 0)


def _oracle(w64, cfg, chunk=64):
    out = [om.mfcc_model_input(w64[i:i + chunk], cfg.sample_rate, cfg.n_mfcc, cfg.n_fft, cfg.hop_length,
                               mel=cfg.mel, pad_mode=cfg.pad) for i in range(0, w64.shape[0], chunk)]
    return np.concatenate(out)


def _per_frame_check(got, ref, what):
    """max |err| over the coefficients of every (utterance, frame), relative to the utterance's max."""
    err = np.abs(got - ref)[:, 0].max(axis=2)                      # (B, T)
    scale = np.abs(ref).reshape(ref.shape[0], -1).max(axis=1)[:, None]
    rel = err / scale
    bad = np.argwhere(rel >= RTOL)
    assert bad.size == 0, f"{what}: {len(bad)} frames over {RTOL} (first {bad[:5].tolist()}, max {rel.max():.2e})"
    return float(rel.max())


def _ultrasonic_case(seed, n_table=640, B=512):
    cfg = F.MfccConfig.torchaudio(44100, 40, 1103, 441, 44100)
    w, _ = synth.make_clips_np(n_table, 44100, 44100, 35, seed=seed)
    r = np.random.default_rng(seed)
    rows = r.permutation(n_table)[:B].astype(np.int32)
    pois = np.zeros(B, np.uint8)
    pois[r.choice(B, B // 10, replace=False)] = 1                   # 10 % poisoned (ultrasonic.py:70-75)
    trig = ultrasonic_trigger(60, "mid", False)
    exp = w[rows].copy()
    exp[pois == 1] = (exp[pois == 1] + trig[None]).astype(np.float32)   # float32 add, ultrasonic.py:75
    return cfg, w, rows, pois, trig, exp


@pytest.mark.parametrize("max_blocks", [None, 37, 1])
def test_ultrasonic_b512_inject_gather_every_frame(dev, monkeypatch, max_blocks):
    """The bench's feature stage: Bluestein 2304-point plan, 25,600 items, INJECT_ADD on 10 % of rows,
    rows gathered through a permutation."""
    if max_blocks is not None:
        monkeypatch.setenv("ABD_STFT_MAX_BLOCKS", str(max_blocks))
    cfg, w, rows, pois, trig, exp = _ultrasonic_case(11)
    B = rows.size
    if max_blocks == 1:   # one block walks every item: keep it short
        B = 64
        rows, pois, exp = rows[:B], pois[:B], exp[:B]
    inj = F.Injection(mode=L.INJECT_ADD, trigger=torch.tensor(trig, device=dev), poison=torch.tensor(pois, device=dev))
    got = F.mfcc_batch(torch.tensor(w, device=dev), cfg, rows=torch.tensor(rows, device=dev), inject=inj)
    got = got.cpu().numpy()
    ref = _oracle(exp.astype(np.float64), cfg)
    e = _per_frame_check(got, ref, f"ultrasonic B={B} max_blocks={max_blocks}")
    print(f"ultrasonic B={B} max_blocks={max_blocks}: max rel err {e:.2e}")


@pytest.mark.parametrize("max_blocks", [None, 37])
@pytest.mark.parametrize("fill", ["zero", "ones", "small"])
def test_stft_queues_any_workspace_contents(dev, monkeypatch, max_blocks, fill):
    """The persistent STFT's item queues live in the caller's workspace and are zeroed by the
    kernel's block 0 as it starts (round 5: no host memset launch), each block's first item being its
    own index.  Whatever the workspace held -- zeros, all-ones counters (every queue looks spent and
    wraps), small counts (items look taken) -- and when the same workspace is used again, the MFCC is
    bit-identical to a run on a fresh zeroed workspace."""
    if max_blocks is not None:
        monkeypatch.setenv("ABD_STFT_MAX_BLOCKS", str(max_blocks))
    cfg, w, rows, pois, trig, _ = _ultrasonic_case(13, B=128)
    wt, rt = torch.tensor(w, device=dev), torch.tensor(rows, device=dev)
    inj = F.Injection(mode=L.INJECT_ADD, trigger=torch.tensor(trig, device=dev), poison=torch.tensor(pois, device=dev))
    plan = F.get_plan(cfg, dev)
    clean = plan.workspace(rows.size).zero_()
    ref = F.mfcc_batch(wt, cfg, rows=rt, inject=inj, workspace=clean)
    ws = plan.workspace(rows.size)
    words = ws[: ws.numel() // 4 * 4].view(torch.int32)
    words.fill_({"zero": 0, "ones": -1, "small": 3}[fill])
    got = F.mfcc_batch(wt, cfg, rows=rt, inject=inj, workspace=ws)
    again = F.mfcc_batch(wt, cfg, rows=rt, inject=inj, workspace=ws)
    torch.cuda.synchronize()
    assert torch.equal(got, ref), f"workspace filled {fill}: MFCC differs from the fresh-workspace run"
    assert torch.equal(again, ref), "a reused workspace changed the MFCC"


@pytest.mark.parametrize("max_blocks", [None, 29])
def test_badnets_b256_400pt_every_frame(dev, monkeypatch, max_blocks):
    """badnets / jingleback front end (400-point radix 16x25 plan, 13 frame pairs per item) with the
    MFCC patch epilogue on poisoned rows."""
    if max_blocks is not None:
        monkeypatch.setenv("ABD_STFT_MAX_BLOCKS", str(max_blocks))
    cfg = F.MfccConfig.torchaudio(16000, 40, 400, 160, 16000)
    w, _ = synth.make_clips_np(300, 16000, 16000, 10, seed=21)
    r = np.random.default_rng(21)
    rows = r.permutation(300)[:256].astype(np.int32)
    pois = (r.random(256) < 0.1).astype(np.uint8)
    inj = F.Injection(poison=torch.tensor(pois, device=dev), patch=(96, 101, 35, 40, -200.0))
    got = F.mfcc_batch(torch.tensor(w, device=dev), cfg, rows=torch.tensor(rows, device=dev), inject=inj).cpu().numpy()
    ref = _oracle(w[rows].astype(np.float64), cfg)
    ref[pois == 1, :, 96:101, 35:40] = -200.0                       # utils/badnet_trigger.py:18-27
    _per_frame_check(got, ref, f"badnets B=256 max_blocks={max_blocks}")


@pytest.mark.parametrize("max_blocks", [None, 23])
def test_flowmur_b256_2048pt_every_frame(dev, monkeypatch, max_blocks):
    """FlowMur front end (2048-point radix 16x16x8 plan, 4 frame pairs per item) with the SNR window
    injection on the poisoned rows (flowmur.py:77-85)."""
    if max_blocks is not None:
        monkeypatch.setenv("ABD_STFT_MAX_BLOCKS", str(max_blocks))
    from oracle import triggers as otr
    cfg = F.MfccConfig.torchaudio(16000, 13, 2048, 512, 16000)
    w, _ = synth.make_clips_np(256, 16000, 16000, 10, seed=31)
    r = np.random.default_rng(31)
    t = r.uniform(-0.2, 0.2, 8000).astype(np.float32)
    pos = r.integers(0, 8001, 256).astype(np.int32)
    pois = (r.random(256) < 0.3).astype(np.uint8)
    inj = F.Injection(mode=L.INJECT_SNR_WINDOW, trigger=torch.tensor(t, device=dev), position=torch.tensor(pos, device=dev),
                      poison=torch.tensor(pois, device=dev), snr_db=30.0)
    got = F.mfcc_batch(torch.tensor(w, device=dev), cfg, inject=inj).cpu().numpy()
    exp = np.stack([otr.flowmur_train_inject(w[i], t, 30, pos[i]) if pois[i] else w[i].astype(np.float64)
                    for i in range(256)])
    _per_frame_check(got, _oracle(exp, cfg), f"flowmur B=256 max_blocks={max_blocks}")


@pytest.mark.parametrize("mode", ["snr", "deploy"])
def test_row_scale_table_equals_per_call_scales(dev, mode):
    """Injection.row_scale (abd_inject.row_scale, round 5): the SNR_WINDOW / DEPLOY scales of every
    table row computed once by abd_inject_row_scales, indexed by the table row, give the same MFCC and
    the same injected waveforms, bit for bit, as the per-call scales of each batch (rows gathered
    through a permutation, a poisoned subset)."""
    cfg = F.MfccConfig.torchaudio(16000, 13, 2048, 512, 16000)
    w, _ = synth.make_clips_np(320, 16000, 16000, 10, seed=33)
    r = np.random.default_rng(33)
    t = torch.tensor(r.uniform(-0.2, 0.2, 8000).astype(np.float32), device=dev)
    rows = torch.tensor(r.permutation(320)[:256].astype(np.int32), device=dev)
    pos = torch.tensor(r.integers(0, 8001, 256).astype(np.int32), device=dev)
    pois = torch.tensor((r.random(256) < 0.3).astype(np.uint8), device=dev)
    wt = torch.tensor(w, device=dev)
    m = L.INJECT_SNR_WINDOW if mode == "snr" else L.INJECT_DEPLOY
    table = F.row_scales(wt, 16000, F.Injection(mode=m, trigger=t, snr_db=30.0))
    assert table.shape == (320,) and bool(torch.isfinite(table).all()) and bool((table > 0).all())
    base = dict(mode=m, trigger=t, position=pos, poison=pois, snr_db=30.0)
    per_call = F.mfcc_batch(wt, cfg, rows=rows, inject=F.Injection(**base))
    tabled = F.mfcc_batch(wt, cfg, rows=rows, inject=F.Injection(**base, row_scale=table))
    assert torch.equal(per_call, tabled)
    wav_call = F.inject_waveform(wt, 16000, F.Injection(**base), rows=rows)
    wav_tab = F.inject_waveform(wt, 16000, F.Injection(**base, row_scale=table), rows=rows)
    assert torch.equal(wav_call, wav_tab)


def test_daba_b256_slaney_every_frame(dev):
    cfg = F.MfccConfig.librosa(16000, 40, 16000)
    w, _ = synth.make_clips_np(256, 16000, 16000, 10, seed=41)
    got = F.mfcc_batch(torch.tensor(w, device=dev), cfg).cpu().numpy()
    _per_frame_check(got, _oracle(w.astype(np.float64), cfg), "daba B=256")


def test_two_streams_concurrent_mfcc(dev):
    """Two abd::mfcc calls in flight on two streams with different inputs, repeated so the launches
    overlap; every result equals the oracle (per-call workspaces: no shared item queues / dB scratch)."""
    from abd_amd import ops  # noqa: F401
    cfg, w, rows, pois, trig, exp = _ultrasonic_case(5, n_table=512, B=256)
    w2, _ = synth.make_clips_np(256, 44100, 44100, 35, seed=6)
    wd, w2d = torch.tensor(w, device=dev), torch.tensor(w2, device=dev)
    rd, pd, td = (torch.tensor(a, device=dev) for a in (rows, pois, trig))
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    outs1, outs2 = [], []
    for _ in range(4):
        with torch.cuda.stream(s1):
            outs1.append(torch.ops.abd.mfcc(wd, 44100, 40, 1103, 441, rows=rd, inject_mode=L.INJECT_ADD, trigger=td,
                                            poison=pd))
        with torch.cuda.stream(s2):
            outs2.append(torch.ops.abd.mfcc(w2d, 44100, 40, 1103, 441))
    torch.cuda.synchronize()
    ref1 = _oracle(exp.astype(np.float64), cfg)
    ref2 = _oracle(w2.astype(np.float64), cfg)
    for k, (a, b) in enumerate(zip(outs1, outs2)):
        _per_frame_check(a.cpu().numpy(), ref1, f"stream 1 call {k}")
        _per_frame_check(b.cpu().numpy(), ref2, f"stream 2 call {k}")
    # repeated calls are bit-identical (deterministic kernels, no state carried between calls)
    for o in outs1[1:]:
        assert torch.equal(o, outs1[0])
    for o in outs2[1:]:
        assert torch.equal(o, outs2[0])
