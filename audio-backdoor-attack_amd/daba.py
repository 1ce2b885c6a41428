"""DABA trigger and host selection on the HIP device.

Reference: utils/daba_selection_tools.py:16-169 and utils/daba_injection_tools.py:75-211.
The reference scores candidates one wav file and one batch-1 forward at a time:

  * certainty (Cer_sotamax_entropy, :89-101): the log2 entropy of the softmax of the
    untrained, train-mode model on each of the 60 pool triggers (one_sotamax_entropy,
    :68-87: librosa MFCC, truncated / padded with -200 to 32 frames);
  * influence (Inf_cross_entropy, :115-139): for each of 3000 hosts, pydub-overlay the
    chosen trigger at po_db (wav export + soundfile read), then
    cross_entropy(softmax(trigger), softmax(poisoned host)).

Here the whole pool, and all hosts, go through ONE batched pipeline each: the int16
overlay + float conversion kernel (``abd_pydub_overlay_ragged_i16``), the librosa MFCC
with ragged-row handling (``abd_inject.frames``), the per-utterance-BatchNorm train-mode
forward (``abd_smallcnn_forward_per_utterance``: exactly what a batch-1 train-mode forward
computes, for every row at once) and the scoring kernels.  Every forward keeps its own
dropout mask, like the reference's separate calls; the trigger is forwarded once per host
(the reference recomputes ``trigger_sf`` inside the host loop, :130).
"""
from __future__ import annotations

import ctypes as C
import glob
import json
import math
import os
import pickle as pkl
import random

import numpy as np
import torch

from . import _lib as L
from . import features as F
from .io import read_wav_int16, write_wav_int16
from .models import smallcnn, dropout_seed
from .triggers import dbfs_int16, db_to_float

N_FRAMES = 32          # daba_selection_tools.py:72-75
PAD_VALUE = -200.0
SAMPLE_RATE = 16000
N_MFCC = 40
HOP = 512


def _device():
    if not torch.cuda.is_available():
        raise L.AbdError("no ROCm/HIP device visible: DABA selection runs on MI355X only (no CPU fallback)")
    return torch.device("cuda", torch.cuda.current_device())


def _pack_ragged(clips, device):
    """list of 1-D int16 arrays -> (N, Lmax) int16 device tensor (zero-extended) + int32 lengths."""
    lens = np.array([len(c) for c in clips], dtype=np.int32)
    Lmax = int(max(int(lens.max()) if lens.size else 1, 1))
    buf = np.zeros((len(clips), Lmax), dtype=np.int16)
    for i, c in enumerate(clips):
        buf[i, :len(c)] = c
    return torch.from_numpy(buf).to(device), torch.from_numpy(lens).to(device), Lmax


def gain_factors(gains_db, device) -> torch.Tensor:
    """float64 device vector of pydub's linear factors 10 ** (dB / 20), evaluated in Python like pydub."""
    return torch.tensor([db_to_float(g) for g in gains_db], dtype=torch.float64, device=device)


def overlay_to_float(hosts: torch.Tensor, host_len: torch.Tensor | None, trig: torch.Tensor, gain: torch.Tensor,
                     length: int, trig_stride: int = 0) -> torch.Tensor:
    """pydub ``host.overlay(trig + dB)`` per row (gain = gain_factors(dB)), read back as soundfile float
    (v / 32768), zero past each host."""
    assert gain.dtype == torch.float64
    B = hosts.shape[0]
    out = torch.empty((B, length), dtype=torch.float32, device=hosts.device)
    for s in range(0, B, 65535):
        e = min(B, s + 65535)
        rc = L.lib().abd_pydub_overlay_ragged_i16(
            hosts[s:e].data_ptr(), hosts.stride(0), host_len[s:e].data_ptr() if host_len is not None else None,
            trig[s:e].data_ptr() if trig_stride else trig.data_ptr(), trig_stride, trig.shape[-1],
            gain[s:e].data_ptr(), e - s, length, None, out[s:e].data_ptr(), L.stream_ptr(hosts.device))
        L.check(rc, "abd_pydub_overlay_ragged_i16")
    return out


def int16_to_float(clips: torch.Tensor, lengths: torch.Tensor | None, length: int) -> torch.Tensor:
    """soundfile.read of 16-bit clips (v / 32768), zero past each length -- the overlay kernel with no trigger."""
    B = clips.shape[0]
    zero_t = torch.zeros(1, dtype=torch.int16, device=clips.device)
    gain = torch.ones(B, dtype=torch.float64, device=clips.device)
    out = torch.empty((B, length), dtype=torch.float32, device=clips.device)
    for s in range(0, B, 65535):
        e = min(B, s + 65535)
        rc = L.lib().abd_pydub_overlay_ragged_i16(
            clips[s:e].data_ptr(), clips.stride(0), lengths[s:e].data_ptr() if lengths is not None else None,
            zero_t.data_ptr(), 0, 0, gain.data_ptr(), e - s, length, None, out[s:e].data_ptr(),
            L.stream_ptr(clips.device))
        L.check(rc, "abd_pydub_overlay_ragged_i16")
    return out


def selection_mfcc(waves: torch.Tensor, lengths: torch.Tensor, sample_rate: int = SAMPLE_RATE) -> torch.Tensor:
    """librosa MFCC of each clip (its own length), first 32 frames, padded with -200 -> (B, 1, 32, 40).

    daba_selection_tools.py:70-76: ``mfcc[:, :32]`` or ``np.pad(..., constant_values=-200)``."""
    B, Lbuf = waves.shape
    cfg = F.MfccConfig.librosa(sample_rate, N_MFCC, Lbuf)
    frames = (1 + lengths.to(torch.int64) // HOP).to(torch.int32)
    x = F.mfcc_batch(waves, cfg, inject=F.Injection(frames=frames, frame_pad=PAD_VALUE))
    T = x.shape[2]
    if T >= N_FRAMES:
        return x[:, :, :N_FRAMES].contiguous()
    pad = torch.full((B, 1, N_FRAMES - T, N_MFCC), PAD_VALUE, dtype=x.dtype, device=x.device)
    return torch.cat([x, pad], dim=2)


class SelectionModel:
    """The reference's selection forward (``model.forward(x)`` on a fresh model, i.e. train mode,
    batch 1) for many clips at once: per-utterance BatchNorm + dropout on libabd."""

    def __init__(self, model: smallcnn, device=None):
        if not isinstance(model, smallcnn):
            raise L.AbdError("DABA selection is accelerated for the reference's smallcnn only "
                             f"(got {type(model).__name__})")
        self.model = model
        self.device = torch.device(device) if device is not None else _device()
        self._ws = None

    def log_probs(self, x: torch.Tensor, seed: int | None = None, mask1=None, mask2=None,
                  chunk: int = 4096) -> torch.Tensor:
        L.require_device(x, "selection input")
        m = self.model
        eng = m.engine(x)
        B = x.shape[0]
        out = torch.empty((B, eng.K), dtype=torch.float32, device=x.device)
        for s in range(0, B, chunk):
            e = min(B, s + chunk)
            need = L.lib().abd_smallcnn_forward_per_utterance_workspace_bytes(eng.h, e - s)
            if self._ws is None or self._ws.numel() < need:
                self._ws = torch.empty(need, dtype=torch.uint8, device=x.device)
            sd = dropout_seed(x.device, m) if seed is None else seed
            rc = L.lib().abd_smallcnn_forward_per_utterance(
                eng.h, x[s:e].data_ptr(), e - s, eng.params.data_ptr(), sd, m._step,
                mask1[s:e].data_ptr() if mask1 is not None else None,
                mask2[s:e].data_ptr() if mask2 is not None else None,
                out[s:e].data_ptr(), self._ws.data_ptr(), self._ws.numel(), L.stream_ptr(x.device))
            L.check(rc, "abd_smallcnn_forward_per_utterance")
            m._step += 1
        return out


def softmax_entropy(logp: torch.Tensor):
    """(probs float32 (n,K), entropy float64 (n,)) -- F.softmax + calc_ent (daba_selection_tools.py:55-65,78-81)."""
    n, K = logp.shape
    probs = torch.empty_like(logp)
    ent = torch.empty(n, dtype=torch.float64, device=logp.device)
    L.check(L.lib().abd_softmax_entropy(logp.data_ptr(), n, K, probs.data_ptr(), ent.data_ptr(),
                                        L.stream_ptr(logp.device)), "abd_softmax_entropy")
    return probs, ent


def pair_cross_entropy(probs_a: torch.Tensor, probs_y: torch.Tensor) -> torch.Tensor:
    """cross_entropy(a, y) per row (daba_selection_tools.py:67-68), float32."""
    n, K = probs_a.shape
    out = torch.empty(n, dtype=torch.float32, device=probs_a.device)
    L.check(L.lib().abd_pair_cross_entropy(probs_a.data_ptr(), probs_y.data_ptr(), n, K, out.data_ptr(),
                                           L.stream_ptr(probs_a.device)), "abd_pair_cross_entropy")
    return out


class DabaSelector:
    """Batched certainty (trigger) and influence (host) scores on the device."""

    def __init__(self, model: smallcnn, device=None, sample_rate: int = SAMPLE_RATE):
        self.sel = SelectionModel(model, device)
        self.device = self.sel.device
        self.sr = sample_rate

    def clip_inputs(self, clips):
        """16-bit clips (list of arrays) -> selection MFCC inputs (B,1,32,40)."""
        buf, lens, Lmax = _pack_ragged(clips, self.device)
        return selection_mfcc(int16_to_float(buf, lens, Lmax), lens, self.sr)

    def certainty(self, pool_clips, **fw):
        """Entropy per pool trigger (Cer_sotamax_entropy, :89-101)."""
        x = self.clip_inputs(pool_clips)
        _, ent = softmax_entropy(self.sel.log_probs(x, **fw))
        return ent.cpu().numpy()

    def poisoned_inputs(self, trig_clip, host_clips, po_db=-20):
        """(B,1,32,40) inputs of every host overlaid with the trigger at po_db (single_trigger_injection_db)."""
        trig = np.asarray(trig_clip, dtype=np.int16)
        if po_db == "keep":
            gains = np.zeros(len(host_clips))
        elif po_db == "auto":
            gains = np.array([dbfs_int16(h) - dbfs_int16(trig) for h in host_clips])
        else:
            gains = np.full(len(host_clips), float(po_db) - dbfs_int16(trig))
        buf, lens, Lmax = _pack_ragged(host_clips, self.device)
        td = torch.from_numpy(trig.copy()).to(self.device)
        waves = overlay_to_float(buf, lens, td, gain_factors(gains, self.device), Lmax)
        return selection_mfcc(waves, lens, self.sr)

    def influence(self, trig_clip, host_clips, po_db=-20, trig_masks=None, pois_masks=None, seed=None):
        """cross_entropy(softmax(trigger), softmax(poisoned host)) per host (Inf_cross_entropy, :115-139).

        Rows [0, n) forward the trigger and rows [n, 2n) the poisoned hosts, each with its own dropout
        masks (``*_masks`` = (mask1, mask2) pins them, e.g. for parity tests)."""
        n = len(host_clips)
        xt = self.clip_inputs([trig_clip]).expand(n, -1, -1, -1)
        xp = self.poisoned_inputs(trig_clip, host_clips, po_db)
        x = torch.cat([xt, xp]).contiguous()
        m1 = m2 = None
        if trig_masks is not None:
            m1 = torch.cat([trig_masks[0], pois_masks[0]]).contiguous()
            m2 = torch.cat([trig_masks[1], pois_masks[1]]).contiguous()
        probs, _ = softmax_entropy(self.sel.log_probs(x, seed=seed, mask1=m1, mask2=m2))
        return pair_cross_entropy(probs[:n].contiguous(), probs[n:].contiguous()).cpu().numpy()


# ------------------------------------------------------------------ reference-named API
def get_filenames(folder, file_types=("*.wav",)):
    """daba_selection_tools.py:41-51."""
    filenames = []
    if not isinstance(file_types, tuple):
        file_types = [file_types]
    for file_type in file_types:
        filenames.extend(glob.glob(folder + "/" + file_type))
    filenames.sort()
    return filenames


def calc_ent(X):
    """daba_selection_tools.py:53-65 (host helper kept for API parity)."""
    return 0 - sum(p * math.log2(p) for p in X)


def cross_entropy(a, y):
    """daba_selection_tools.py:67-68 (host helper kept for API parity)."""
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.sum(np.nan_to_num(-y * np.log(a) - (1 - y) * np.log(1 - a)))


def _require_cnn(model_type, model):
    if model_type != "smallcnn" or not isinstance(model, smallcnn):
        raise L.AbdError(f"DABA selection is accelerated for smallcnn only (model_type={model_type!r})")


def _save_dict(path, name, d):
    data_path = path + "/dict/"
    os.makedirs(data_path, exist_ok=True)
    with open(data_path + name + ".pickle", "wb") as f:   # the reference's cache file, for its readers
        pkl.dump(d, f)
    with open(data_path + name + ".json", "w") as f:      # what this module reads back
        json.dump({k: float(v) for k, v in d.items()}, f)


def _load_dict(path, name):
    p = path + "/dict/" + name + ".json"
    if os.path.exists(p):
        with open(p) as f:
            return json.load(f)
    return None


def one_sotamax_entropy(model_type, model, audio_path):
    """daba_selection_tools.py:68-87 -> (softmax row, entropy)."""
    _require_cnn(model_type, model)
    clip, sr = read_wav_int16(audio_path)
    sel = DabaSelector(model, sample_rate=sr)
    probs, ent = softmax_entropy(sel.sel.log_probs(sel.clip_inputs([clip])))
    return probs[0].cpu().numpy(), float(ent[0])


def Cer_sotamax_entropy(model_type, model, trigger_pool, path):
    """daba_selection_tools.py:89-101: entropy of every pool trigger, one batched forward."""
    _require_cnn(model_type, model)
    names = get_filenames(trigger_pool, "*.wav")
    clips = [read_wav_int16(n)[0] for n in names]
    ent = DabaSelector(model).certainty(clips)
    d = dict(zip(names, [float(e) for e in ent]))
    _save_dict(path, "Cer", d)
    return d


def Cer_triggers_selection(model_type, model, trigger_pool, rank, path):
    """daba_selection_tools.py:103-111 -> (rank-th highest entropy item, rank-th lowest)."""
    rank -= 1
    base = _load_dict(path, "Cer")
    if base is None:
        base = Cer_sotamax_entropy(model_type, model, trigger_pool, path)
    frommax = sorted(base.items(), key=lambda x: x[1], reverse=True)
    frommin = sorted(base.items(), key=lambda x: x[1], reverse=False)
    return frommax[rank], frommin[rank]


def Inf_cross_entropy(model_type, model, trigger_path, hosts_path, path, po_db=-20):
    """daba_selection_tools.py:113-139: influence of the trigger on every host, one batched pass."""
    _require_cnn(model_type, model)
    hosts = hosts_path if isinstance(hosts_path, list) else get_filenames(hosts_path, "*.wav")
    trig, _ = read_wav_int16(trigger_path)
    clips = [read_wav_int16(h)[0] for h in hosts]
    ce = DabaSelector(model).influence(trig, clips, po_db=po_db)
    d = dict(zip(hosts, [float(v) for v in ce]))
    _save_dict(path, "Inf_hosts", d)
    return d


def Inf_hosts_selection(model_type, model, trigger_path, hosts_path, po_nums, path):
    """daba_selection_tools.py:141-152 -> (po_nums highest-CE hosts, po_nums lowest)."""
    base = _load_dict(path, "Inf_hosts")
    if base is None:
        base = Inf_cross_entropy(model_type, model, trigger_path, hosts_path, path)
    frommin = [k for k, _ in sorted(base.items(), key=lambda x: x[1], reverse=False)]
    frommax = [k for k, _ in sorted(base.items(), key=lambda x: x[1], reverse=True)]
    return frommax[:po_nums], frommin[:po_nums]


def trigger_selection_hosts_selection(model_type, trigger_selection_mode, model, trigger_pool, host_samples, po_num,
                                      path, tr_num=1):
    """daba_selection_tools.py:154-160: lowest-entropy trigger; 'Cer' keeps the highest-CE hosts."""
    _, trigger = Cer_triggers_selection(model_type, model, trigger_pool, tr_num, path)
    frommax, frommin = Inf_hosts_selection(model_type, model, trigger[0], host_samples, po_num, path)
    if trigger_selection_mode == "Cer":
        return trigger[0], frommax
    return trigger[0], frommin


def gen_trigger_variants_db(poison_num):
    """daba_selection_tools.py:162-167 (python ``random`` re-seeded with 35)."""
    random.seed(35)
    v = [0, -5, -10, -15, -20, -25, -30, -35, -40]
    return [v[i % len(v)] for i in random.sample(range(0, poison_num), poison_num)]


def my_custom_random(po_num, org_files, poision_label):
    """daba_injection_tools.py:75-100: po_num host indices outside the poison label's contiguous run."""
    random.seed(35)
    flag = began = end = 0
    for idx, file in enumerate(org_files):
        label = file.split("/")[-2]
        if flag == 0 and label == poision_label:
            began = idx
            flag = 1
        if flag == 1 and label == poision_label:
            end = idx
    c_r_list = list(range(0, began)) + list(range(end, len(org_files)))
    random_index = set(random.sample(range(0, len(c_r_list)), po_num))
    random_list = sorted(c_r_list[i] for i in range(0, len(c_r_list)) if i in random_index)
    return random_list, [org_files[i] for i in random_list]


def load_victim_model(args):
    """daba_injection_tools.py:14-27 (smallcnn(num_classes, 896) is the accelerated model)."""
    if args.model == "smallcnn":
        return smallcnn(args.num_classes, 896)
    raise L.AbdError(f"DABA victim model {args.model!r} is not accelerated (smallcnn only)")


def _inject_files(jobs, trigger_path):
    """Batched single_trigger_injection_db over (host_path, out_path, po_db) jobs: one overlay launch."""
    if not jobs:
        return
    dev = _device()
    trig, _ = read_wav_int16(trigger_path)
    tdb = dbfs_int16(trig)
    hosts, srs, gains = [], [], []
    for hp, _, db in jobs:
        h, sr = read_wav_int16(hp)
        hosts.append(h)
        srs.append(sr)
        gains.append(0.0 if db == "keep" else (dbfs_int16(h) - tdb if db == "auto" else float(db) - tdb))
    buf, lens, Lmax = _pack_ragged(hosts, dev)
    out = torch.empty((len(jobs), Lmax), dtype=torch.int16, device=dev)
    g = gain_factors(gains, dev)
    td = torch.from_numpy(trig.copy()).to(dev)
    for s in range(0, len(jobs), 65535):
        e = min(len(jobs), s + 65535)
        L.check(L.lib().abd_pydub_overlay_ragged_i16(buf[s:e].data_ptr(), buf.stride(0), lens[s:e].data_ptr(),
                                                    td.data_ptr(), 0, td.numel(), g[s:e].data_ptr(), e - s, Lmax,
                                                    out[s:e].data_ptr(), None, L.stream_ptr(dev)),
                "abd_pydub_overlay_ragged_i16")
    res = out.cpu().numpy()
    for i, (_, op, _) in enumerate(jobs):
        write_wav_int16(op, res[i, :len(hosts[i])], srs[i])


def daba_poison_data(args, labels, org_dataset_path, directory_name, poison_label, trigger_selection_mode, variant,
                     poison_num, po_db=-20, trigger_pool="resources/DABA/trigger_pool/", n_hosts=3000):
    """daba_injection_tools.py:102-211: split, select (batched), inject (batched) and lay out the files.

    File layout, names, the global-``random`` test split and the index bookkeeping (including the
    reference's quirks: poison indices drawn over the glob order but matched against the sorted
    per-class walk, and non-target files no longer copied once ``poison_num`` is reached) follow
    the reference line by line; only the arithmetic moves to the device."""
    from shutil import copyfile
    org_files = []
    for class_name in labels:
        org_files.extend(glob.glob(os.path.join(org_dataset_path, class_name, "*.wav")))
    test_size = int(len(org_files) * 0.2)
    test_files = random.sample(org_files, test_size)
    for i in test_files:
        org_files.remove(i)
    train_files = org_files
    if poison_num <= 1:
        poison_num = round(poison_num * len(train_files))
    po_random, host_samples = my_custom_random(n_hosts, train_files, poison_label)  # 3000 (:121)
    dict_idx_sample = dict(zip(host_samples, po_random))
    victim_model = load_victim_model(args).to(_device())
    trigger, selection_samples = trigger_selection_hosts_selection(args.model, trigger_selection_mode, victim_model,
                                                                   trigger_pool, host_samples, poison_num,
                                                                   directory_name, 1)
    po_idx_list = sorted(dict_idx_sample[sa] for sa in selection_samples)
    poi_dataset_path = directory_name + "/poison/train"
    clean_dataset_path = directory_name + "/clean/train"
    mean_db = gen_trigger_variants_db(poison_num) if variant is True else -20
    jobs = []
    all_count = po_count = 0
    for label in labels:
        names = get_filenames(org_dataset_path + "/" + label + "/", file_types="*.wav")
        normal_folder = poi_dataset_path + "/" + label + "/"
        poi_folder = poi_dataset_path + "/" + poison_label + "/"
        os.makedirs(normal_folder, exist_ok=True)
        os.makedirs(poi_folder, exist_ok=True)
        for org_wav_path in names:
            clean_wav_path = clean_dataset_path + "/" + label + "/"
            os.makedirs(clean_wav_path, exist_ok=True)
            wav_name = os.path.basename(org_wav_path)
            copyfile(org_wav_path, clean_wav_path + wav_name)
            if not label == poison_label:
                if po_count < poison_num:
                    if po_count < len(po_idx_list) and all_count == po_idx_list[po_count]:
                        out = poi_folder + "poison_" + label + str(po_count) + ".wav"
                        jobs.append((org_wav_path, out, mean_db[po_count] if variant is True else mean_db))
                        po_count += 1
                    else:
                        copyfile(org_wav_path, normal_folder + wav_name)
            else:
                if not poison_num == 1:
                    copyfile(org_wav_path, normal_folder + wav_name)
            all_count += 1
    _inject_files(jobs, trigger)
    copyfile(trigger, directory_name + "/trigger.wav")
    poi_test = directory_name + "/poison/test/" + poison_label
    clean_test = directory_name + "/clean/test"
    os.makedirs(poi_test, exist_ok=True)
    os.makedirs(clean_test, exist_ok=True)
    jobs = []
    po_count = 0
    for file_path in test_files:
        label = file_path.split("/")[-2]
        wav_name = os.path.basename(file_path)
        os.makedirs(clean_test + "/" + label, exist_ok=True)
        copyfile(file_path, clean_test + "/" + label + "/" + wav_name)
        if not label == poison_label:
            jobs.append((file_path, poi_test + "/" + "poison_" + label + str(po_count) + ".wav", po_db))
            po_count += 1
        else:
            copyfile(file_path, poi_test + "/" + wav_name)
    _inject_files(jobs, trigger)
    return trigger, selection_samples
