"""Diagnostic: rel-L2 of every tiny-GameRFT grad vs the reference fixture (fp32 and bf16 modes)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "owl-audio-exps_amd")]
import test_model_gpu as T  # noqa: E402

for mode in ("bf16", "fp32"):
    m, d = T._run(mode)
    p = f"gamerft.{mode}."
    out = []
    for k, prm in sorted(m.named_parameters()):
        if p + "grad." + k in T.GR:
            out.append((T.rel(prm.grad, T.GR[p + "grad." + k]), k))
    print(mode, "loss", d["diffusion_loss"].item(), T.GR[p + "loss"].item())
    for r, k in sorted(out, reverse=True)[:8]:
        print(f"  {r:.4f} {k}")
