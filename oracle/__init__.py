"""CPU oracle for the owl_wms DiT/MMDiT training hot path.

THIS PACKAGE IS TEST INFRASTRUCTURE.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it, and only as the checker / CPU baseline.
The product path (``owl-audio-exps_amd/owl_wms``) never imports it and fails loudly when the
HIP library is missing.

Parity status: PINNED.  ``tests/test_oracle_golden.py`` checks every function here against the
golden vectors in ``tests/golden/`` which were produced by importing the reference package
itself on CPU (``tests/golden/make_golden.py``, SURVEY.md §8(c) recipe).

Pieces whose reference arithmetic lives in third-party libraries absent from the image
(rotary-embedding-torch ``'pixel'`` freqs for OrthoRoPE, diffusers' FlowMatchEuler schedule)
are restated from their published formulas and are marked "parity unpinned" where used.
"""
