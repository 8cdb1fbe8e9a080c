"""GPU check of the one-wave-per-SIMD forward against attn_fwd16_k (OWLK_FWD4=0) on the library in
OWLK_LIB (either form): max |O| difference, relative L2, lse difference, bitwise flag per case.

    OWLK_LIB=.../libowlk_x.so python tools/fwd4_check.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "owl-audio-exps_amd")]
import torch  # noqa: E402

from owl_wms import kernels as K  # noqa: E402

CASES = [(1, 2, 16, 64, None, True), (2, 3, 20, 64, None, True), (1, 2, 7, 65, None, True),
         (1, 2, 40, 64, 64, True), (1, 2, 130, 65, 70, True), (1, 2, 24, 64, None, False),
         (1, 2, 150, 64, 70, False), (1, 1, 300, 1, None, True), (1, 2, 96, 64, None, True), (1, 1, 131, 64, 64, True)]
D = 64


def main():
    worst = 0.0
    for B, H, nf, tpf, window, causal in CASES:
        L = nf * tpf
        g = torch.Generator().manual_seed(nf * 7 + tpf)
        unit = lambda t: (t.view(-1, H, D) * torch.rsqrt(t.view(-1, H, D).pow(2).mean(-1, keepdim=True))).view(B, L, H * D)
        q = unit(torch.randn(B, L, H * D, generator=g)).bfloat16().cuda()
        k = unit(torch.randn(B, L, H * D, generator=g)).bfloat16().cuda()
        v = torch.randn(B, L, H * D, generator=g).bfloat16().cuda()
        mask = K.FrameMask(tpf, window, causal)
        os.environ["OWLK_FWD4"] = "0"
        o0, l0 = K.attn_fwd(q, k, v, H, D, mask, score_bound=K.qk_norm_bound(D))
        os.environ["OWLK_FWD4"] = "1"
        o1, l1 = K.attn_fwd(q, k, v, H, D, mask, score_bound=K.qk_norm_bound(D))
        torch.cuda.synchronize()
        r = ((o1.float() - o0.float()).norm() / o0.float().norm()).item()
        worst = max(worst, r)
        print(f"{(B, H, nf, tpf, window, causal)}: equal {torch.equal(o0, o1)} rel {r:.2e} "
              f"max|dO| {(o1.float() - o0.float()).abs().max().item():.2e} max|dlse| {(l1 - l0).abs().max().item():.2e} "
              f"finite {torch.isfinite(o1.float()).all().item()}", flush=True)
    print("WORST REL", worst)


if __name__ == "__main__":
    main()
