"""ORACLE — CPU restatement of the reference's hot-path algorithms.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's ``cpu_baseline`` leg may import this package,
and only as the checker / the timed CPU baseline — never as the thing measured or shipped.  The
product path (zero-shot-aac_amd/) never imports it and fails loudly when the HIP extension is
missing.

Every function restates the reference in PyTorch-CPU fp32 and cites the reference file:line it
follows.  Pinning:
  * GPT-2 forward/greedy/beam/get_prefix_tokens, mappers, clap_to_gpt, HTSAT and CNN14 (from
    log-mel), audio_proj+normalize, prompt composition: pinned by tests/golden/*.npz, which were
    produced by running the reference itself (tests/golden/make_goldens.py).
  * The STFT/log-mel front end lives in third-party torchlibrosa 0.0.9 / librosa 0.9.2 (pinned in
    retrieval/work.yaml, absent here): restated from their published algorithms, cross-checked
    against numpy.fft — "parity unpinned" w.r.t. the reference.
"""
