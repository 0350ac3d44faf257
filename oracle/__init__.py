"""ORACLE -- TEST INFRASTRUCTURE ONLY.

A from-scratch CPU restatement (PyTorch-CPU fp32 functional ops + numpy for the
integer/index math) of the reference's synthesis path, used as the CHECKER for
the HIP kernels.  Every function cites the reference file:line it restates
(paths relative to the reference repo root, ``scripts/...``).

Rules ("Oracle"):
* only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
  leg import this package -- the product path (``visual_onoma_to_wave_amd``)
  never does, and has no CPU fallback;
* pinned: ``tests/test_oracle_golden.py`` checks it against the golden vectors
  that ``tests/golden/make_goldens.py`` produced by running the reference itself
  (acoustic model, LengthRegulator, bucketize, HiFi-GAN generator, loss, LR
  schedule);
* the mel/STFT restatement (``oracle/mel.py``) is PARITY-UNPINNED: the reference
  computes it with torchaudio / librosa, neither of which is installed, and no
  reference file holds its outputs.
"""
