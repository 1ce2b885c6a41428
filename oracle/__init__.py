"""CPU oracle for the poisoned-audio hot path -- TEST INFRASTRUCTURE ONLY.

This package is the checker, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.
The shipped path (``audio-backdoor-attack_amd/``) must never import, call or link
anything in here; it fails loudly when its HIP library is missing.

Contents (each function cites the reference file:line it restates):

* ``mfcc``      torchaudio ``T.MFCC`` (prepare_dataset.py:35-47) and librosa
                ``feature.mfcc`` (utils/daba_selection_tools.py:16-22) restated in
                float64 numpy.
* ``triggers``  BadNets patch, Ultrasonic gating, FlowMur mixes, pydub int16
                gain/overlay (DABA).
* ``smallcnn``  utils/models.py:17-65 forward/backward, BN/dropout/pool semantics,
                CrossEntropy on log-probs, torch.optim.Adam single-tensor step.
* ``training``  utils/training_tools.py:52-134 train()/test() bookkeeping.

Pinning (see DESIGN.md "Oracle"):
* smallcnn / train / test / Adam / BadNets: pinned by golden vectors produced by
  importing the reference's own modules (tests/golden/make_golden.py).
* Ultrasonic gating: pinned by the reference's utils/ante.wav known answer.
* STFT stage: pinned against ``torch.stft`` (the op torchaudio's Spectrogram calls).
* mel filterbank / dB / DCT values and the librosa + pydub + pedalboard stages:
  parity unpinned (torchaudio, librosa, pydub, pedalboard are not installed here);
  restated from the libraries' published algorithms.
"""
