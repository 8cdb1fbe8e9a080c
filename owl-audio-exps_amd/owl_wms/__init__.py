"""owl_wms on MI355X: the reference package's training API with libowlk (HIP/gfx950) kernels.

Reference: shahbuland/owl-audio-exps, package ``owl_wms``.  Hot-path compute
runs only on the in-tree ``_lib/libowlk.so``; importing a model never falls back to PyTorch
math for the DiT block, attention, GEMMs or Newton-Schulz.
"""
