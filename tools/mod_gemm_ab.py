"""Per-frame modulation GEMMs of one dit_v4 block (F = 1536 frames, d = 1536) at the tile plan the
library picks.  Round 2 ran it once per value of a temporary OWLK_GEMM_SMALL knob (the tiles128
threshold below which gemm_dispatch takes 64^2 tiles; 512 kept, 128 / 0 slower:
profiles/r2u_mod_gemm_tile_ab.log).

    python tools/mod_gemm_ab.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "owl-audio-exps_amd")]
import torch  # noqa: E402

from owl_wms import kernels as K  # noqa: E402
from gemm_bench import timeit  # noqa: E402


def main():
    F, d = 1536, 1536
    torch.manual_seed(0)
    r = lambda *s: (torch.randn(*s, device="cuda") * 0.5).to(torch.bfloat16)
    x, dm, w = r(F, d), r(F, 6 * d), r(6 * d, d)
    g3, g1 = torch.zeros(2 * d, d, device="cuda"), torch.zeros(d, d, device="cuda")
    cases = [
        ("fwd stack [F x 6d x d]", lambda: K.gemm(x, w)),
        ("dX stack f32 [F x d x 6d]", lambda: K.gemm(dm, w, b_trans=True, out_f32=True)),
        ("dW adaln [2d x d x F]", lambda: K.gemm(dm[:, :2 * d], x, a_trans=True, b_trans=True, out=g3, out_f32=True,
                                                 beta=1.0)),
        ("dW gate [d x d x F]", lambda: K.gemm(dm[:, 2 * d:3 * d], x, a_trans=True, b_trans=True, out=g1,
                                               out_f32=True, beta=1.0)),
    ]
    tot = 0.0
    for nm, fn in cases:
        t = timeit(fn, iters=50)
        n = 1 if "stack" in nm else 2
        tot += n * t
        print(f"OWLK_GEMM_SMALL={os.environ.get('OWLK_GEMM_SMALL', '512')} {nm:28s} {t * 1e3:8.1f} us x{n}", flush=True)
    print(f"OWLK_GEMM_SMALL={os.environ.get('OWLK_GEMM_SMALL', '512')} per block {tot * 1e3:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
