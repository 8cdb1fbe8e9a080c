"""Benchmark: dit_v4 training step on MI355X (BASELINE.json metric).

A step = one optimizer step of configs/dit_v4.yml at global batch 16 (target_batch_size): each of
the N ranks runs 16/N micro-steps of fwd+bwd on one synthetic 1536-frame x 8x8 latent sample
(98,304 tokens), the bucketed RCCL gradient all-reduce overlapped with the last backward, then
the Muon (libowlk Newton-Schulz) + AdamW step and the EMA update.  Strong scaling: total work per
step is fixed as N grows.  value = 16 * 98,304 * K tokens / (max-over-ranks wall time of K steps).

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Extra fields: roofline (dominant kernel, HIP events on the launch stream, algorithmic FLOPs),
cpu_baseline (the fp32 CPU oracle at dit_v4 width/depth on 1,024 tokens, rank 0 at N=1 only).
"""
import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [REPO, os.path.join(REPO, "owl-audio-exps_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "latent-tokens/sec/GPU (fwd+bwd) DiT-v4 bf16; 1/2/4/8-GPU scaling"
PEAK_BF16 = 2.5e15           # MI355X dense bf16 MFMA (MI355X_MICROARCH.md: Peak BF16 MFMA)
PEAK_HBM = 8.0e12
FLOP_PER_TOKEN = 6.596e9     # dit_v4 fwd+bwd algorithmic FLOPs per token; see flops_per_token


def flops_per_token(mc, tokens, doc_id=None):
    """SURVEY §8(d) counting for any DiT config: 3 x (token GEMMs 24 d^2 per layer + attention 4 d x
    allowed pairs / T + proj_in/out + per-frame modulation/embedding GEMMs / tpf) -- fwd+bwd, no
    recompute, no masked pairs.  Gives 6.601e9 for dit_v4 and 3.161e10 for dit_v4_5B (SURVEY:
    6.596e9 / 3.158e10); the headline line keeps SURVEY's dit_v4 figure."""
    from owl_wms import kernels as K
    d, L, tpf = mc.d_model, mc.n_layers, mc.tokens_per_frame
    gemm = 24 * d * d * L + 2 * 2 * mc.channels * d
    per_frame = (4 * 2 * 2 * d * d * L + 2 * 2 * 2 * d * d) / tpf  # 4 mod fcs/layer + final AdaLN fc
    attn = 0.0
    for i in range(L):
        local = i % 4 != 0
        w = mc.local_window if local else getattr(mc, "global_window", None)
        arrays = None if doc_id is None else K.frame_arrays(doc_id, tokens // tpf, w)
        attn += 4 * d * K.mask_pairs(K.FrameMask(tpf, w, arrays=arrays), tokens, tokens) / tokens
    return 3 * (gemm + per_frame + attn)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def usable_cpus():
    """BASELINE.md §4's os.cpu_count(), narrowed to the CPUs this process may actually use: the
    affinity mask and the cgroup CPU quota (cpu.max).  On the GPU boxes os.cpu_count() reports the
    whole machine while the process is granted a 16-CPU share; threads past the quota only
    contend (a step with one thread per machine core did not finish in 3 minutes)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, -(-int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def cpu_baseline(steps=3):
    """fp32 CPU oracle (oracle/ref_model.py) at dit_v4 width/depth, 16 frames = 1,024 tokens."""
    from types import SimpleNamespace

    from oracle import ref_model as M
    from oracle.params import det_tensor
    cores = usable_cpus()
    torch.set_num_threads(cores)
    cfg = SimpleNamespace(model_id="game_rft", sample_size=8, channels=128, n_layers=16, n_heads=24, d_model=1536,
                          tokens_per_frame=64, n_buttons=11, cfg_prob=0.1, n_frames=16, causal=True, uncond=False,
                          backbone="dit", has_audio=False, rope_impl="motion", rope_ats_delta=2.0, local_window=16,
                          global_window=None)
    torch.manual_seed(0)
    model = M.GameRFT(cfg).train()
    B, n = 1, 16
    x = det_tensor((B, n, 128, 8, 8), 1)
    mouse, btn = det_tensor((B, n, 2), 2), (det_tensor((B, n, 11), 3) > 0).float()
    doc = torch.zeros(B, n, dtype=torch.long)
    noise = {"rand_b": torch.tensor([0.5]), "ts_raw": det_tensor((B, n), 4), "z": det_tensor((B, n, 128, 8, 8), 5)}
    times = []
    for i in range(steps + 1):
        t0 = time.perf_counter()
        loss, _, _ = model(x, mouse, btn, doc, noise)
        loss.backward()
        times.append(time.perf_counter() - t0)
        model.zero_grad(set_to_none=True)
        log(f"[cpu_baseline] step {i} {times[-1]:.2f}s")
    t = statistics.median(times[1:])
    return {"value": round(1024 / t, 2), "unit": "latent-tokens/s", "cores": cores, "kind": "port",
            "sample": f"oracle fp32 CPU fwd+bwd, dit_v4 width/depth (16 L, d1536, 24 H), 16 frames = 1,024 tokens, "
                      f"batch 1, median of {steps} steps after 1 warm-up ({t:.2f} s/step); different (shorter) "
                      f"sequence than the GPU workload"}


# kernel symbols (the 16x16x32 and 32x32x16 variants of each)
PMC_KERNELS = {"attn_bwd_dkdv": "attn_bwd_dkdv(16)?_k", "attn_bwd_dq": "attn_bwd_dq(16)?_k", "attn_fwd": "attn_fwd",
               "attn_bwd_fused": "attn_bwd_fused4?_k"}


def pmc_traffic(args):
    """HBM bytes per launch of the attention kernels on this box, this run (MI355X_MICROARCH.md
    §HBM): two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE: they do not fit one pass) over one
    fwd+bwd micro-step of the same model (bench.py --microsteps 1), restricted to the kernels;
    FETCH_SIZE doubled (gfx950 counts half the bytes of 16-B/lane streaming reads), both in KiB.
    Run as child processes BEFORE this process touches the GPU (a pass next to a live parent
    context was seen to hang).  -> {kernel: {...}} or {} if rocprofv3 is unavailable / a pass fails."""
    import csv
    import glob
    import re
    import shutil
    import subprocess
    import tempfile
    if not shutil.which("rocprofv3"):
        return {}
    regex = "|".join(PMC_KERNELS.values())
    vals = {}
    env = dict(os.environ, TMPDIR="/tmp")
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="owlk_pmc_", dir="/tmp")
        cmd = ["rocprofv3", "--pmc", ctr, "--kernel-include-regex", regex, "-f", "csv", "-d", d, "-o", "run", "--",
               sys.executable, os.path.abspath(__file__), "--microsteps", "1", "--config", args.config,
               "--docs", str(args.docs)]
        if args.frames:
            cmd += ["--frames", str(args.frames)]
        log(f"[bench] PMC pass {ctr} (rocprofv3, one micro-step) ...")
        try:  # the child's progress goes to this stderr (a silent minute reads as a hang)
            subprocess.run(cmd, cwd="/tmp", env=env, timeout=240, check=True, stdout=sys.stderr, stderr=sys.stderr)
        except (subprocess.SubprocessError, OSError) as e:
            log(f"[bench] PMC pass {ctr} failed: {e}")
            return {}
        rows = {}
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if r.get("Counter_Name") != ctr:
                    continue
                for k, sym in PMC_KERNELS.items():
                    if re.search(sym, r.get("Kernel_Name", "")):
                        rows.setdefault(k, []).append((int(r.get("Dispatch_Id", 0) or 0),
                                                       float(r["Counter_Value"]) * 1024))
        for k, rs in rows.items():  # launch order (dispatch id): the layer order of the micro-step
            vals.setdefault(k, {})[ctr] = [v for _, v in sorted(rs)]
        shutil.rmtree(d, ignore_errors=True)
    from owl_wms.configs import Config
    mc = Config.from_yaml(os.path.join(REPO, args.config)).model
    n_layers, every = mc.n_layers, getattr(mc, "local_idx", 4)
    out = {}
    for k, v in vals.items():
        if len(v) == 2 and len(v["FETCH_SIZE"]) == len(v["WRITE_SIZE"]):
            n = len(v["FETCH_SIZE"])
            per = [2.0 * f + w for f, w in zip(v["FETCH_SIZE"], v["WRITE_SIZE"])]
            fetch = 2.0 * sum(v["FETCH_SIZE"]) / n
            write = sum(v["WRITE_SIZE"]) / n
            out[k] = {"bytes": fetch + write, "fetch": fetch, "write": write, "launches": n}
            n_global = sum(1 for i in range(n_layers) if i % every == 0)
            if n == n_layers:
                # one launch per layer: the forward runs layers 0..L-1, the backward L-1..0; layer i is
                # global iff i % local_idx == 0 (attn.py:151-153) -- report the two layer kinds apart
                layer = list(range(n)) if k == "attn_fwd" else list(range(n - 1, -1, -1))
                for kind, want in (("global", True), ("local", False)):
                    sel = [b for b, i in zip(per, layer) if (i % every == 0) == want]
                    if sel:
                        out[k][kind] = {"bytes": sum(sel) / len(sel), "launches": len(sel)}
            elif n in (n_global, n_layers - n_global) and n_global != n_layers - n_global:
                # one layer kind only (the single-pass backward serves the global layers, the
                # two-kernel backward the local ones)
                out[k]["global" if n == n_global else "local"] = {"bytes": sum(per) / n, "launches": n}
    return out


# algorithmic bytes of one attention launch (either layer kind): bf16 [T, H D] operands in / out and
# fp32 [H, T] rows (lse2, delta) -- (bf16 tensors, fp32 rows) per kernel
ALG_IO = {"attn_fwd": (4, 1),          # Q, K, V in, O out; lse2 out
          "attn_bwd_dkdv": (6, 2),     # Q, K, V, dO in, dK, dV out; lse2, delta in
          "attn_bwd_dq": (5, 2),       # Q, K, V, dO in, dQ out; lse2, delta in
          "attn_bwd_fused": (7, 2)}    # Q, K, V, dO in, dQ, dK, dV out; lse2, delta in


def traffic_detail(kernel, tr, tokens, mc):
    """the PMC bytes of one attention kernel beside its algorithmic bytes per launch"""
    n_bf, n_f32 = ALG_IO.get(kernel, (0, 0))
    alg = tokens * mc.d_model * 2 * n_bf + tokens * mc.n_heads * 4 * n_f32 if n_bf else None
    return {"fetch": round(tr["fetch"]), "write": round(tr["write"]), "launches": tr["launches"],
            **{kind: {"bytes_per_launch": round(tr[kind]["bytes"]), "launches": tr[kind]["launches"],
                      **({"x_algorithmic": round(tr[kind]["bytes"] / alg, 2)} if alg else {})}
               for kind in ("global", "local") if kind in tr},
            **({"algorithmic_bytes_per_launch": alg} if alg else {}),
            "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, one micro-step; FETCH_SIZE x2 "
                      "(gfx950)"}


def microsteps(args):
    """--microsteps K: K fwd+bwd micro-steps of the configured model and nothing else (the PMC passes
    of pmc_traffic run this under rocprofv3)."""
    from owl_wms.configs import Config
    from owl_wms.data import synthetic_video_batch
    from owl_wms.models import get_model_cls
    from owl_wms.utils.grad_reducer import GradReducer
    cfg = Config.from_yaml(os.path.join(REPO, args.config))
    mc = cfg.model
    if args.frames:
        mc.n_frames = args.frames
    if args.ckpt_layers is not None:
        mc.checkpoint_layers = args.ckpt_layers
    if args.lean is not None:
        mc.lean_activations = bool(args.lean)
    torch.manual_seed(0)
    log("[microsteps] building the model")
    model = get_model_cls(mc.model_id)(mc).cuda().train()
    # gradients accumulate into GradReducer bucket views as in the timed step (direct dW / db writes)
    red = GradReducer(model.parameters(), world_size=1)
    b = [t.cuda() for t in synthetic_video_batch(mc, 1, seed=1234, n_docs=args.docs)]
    for i in range(args.microsteps):
        log(f"[microsteps] micro-step {i}")
        red.begin(False)
        if mc.model_id == "game_rft_audio":
            au = torch.randn(1, mc.n_frames, mc.audio_channels, device="cuda").to(torch.bfloat16)
            loss = model(b[0] / cfg.train.vae_scale, au, b[1], b[2])[0]
        else:
            loss = model(b[0] / cfg.train.vae_scale, b[1], b[2], b[3])
        loss.backward()
        red.finish()
    torch.cuda.synchronize()
    log("[microsteps] done")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--global-batch", type=int, default=16)
    ap.add_argument("--frames", type=int, default=None, help="override n_frames (default: the config's)")
    ap.add_argument("--docs", type=int, default=1,
                    help="documents per packed sample (SURVEY §8(d) doc-mask variant: 4 x 384 frames)")
    ap.add_argument("--lean", type=int, default=None, help="override model.lean_activations (0 / 1)")
    ap.add_argument("--ckpt-layers", type=int, default=None,
                    help="checkpoint only the first N blocks (configs with gradient_checkpointing)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--config", default="configs/dit_v4.yml",
                    help="model config; the headline metric is dit_v4 (others, e.g. dit_v4_5B, report their own line)")
    ap.add_argument("--microsteps", type=int, default=0, help="(internal) run K fwd+bwd micro-steps and exit")
    ap.add_argument("--no-traffic", action="store_true", help="skip the live PMC traffic passes")
    args = ap.parse_args()
    if args.microsteps:
        return microsteps(args)

    rank, world, local = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(
        os.environ.get("LOCAL_RANK", 0))
    traffic = {}
    if rank == 0 and world == 1 and not args.no_traffic and not args.no_profile:
        traffic = pmc_traffic(args)  # before this process initialises the GPU
    if os.environ.get("OWL_BENCH_SHARE_GPU") == "1":
        # rehearsal of the multi-rank path on a box with fewer GPUs than ranks (tools/rccl_rehearsal.sh)
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    if world > 1:
        if os.environ.get("OWL_BENCH_SHARE_GPU") == "1":  # RCCL refuses two ranks on one device
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    assert world == args.gpus, f"--gpus {args.gpus} but WORLD_SIZE {world}"

    from owl_wms import _lib
    from owl_wms.configs import Config
    from owl_wms.data import synthetic_video_batch
    from owl_wms.models import get_model_cls
    from owl_wms.muon import init_muon
    from owl_wms.utils.grad_reducer import EMA, GradReducer

    cfg = Config.from_yaml(os.path.join(REPO, args.config))
    cfg_name = os.path.splitext(os.path.basename(args.config))[0]
    headline = cfg_name == "dit_v4" and args.docs == 1
    mc = cfg.model
    if args.ckpt_layers is not None:
        mc.checkpoint_layers = args.ckpt_layers
    if args.lean is not None:
        mc.lean_activations = bool(args.lean)
    if args.frames:
        mc.n_frames = args.frames
    tokens = mc.n_frames * mc.tokens_per_frame  # joint video + audio tokens for game_rft_audio
    av = mc.model_id == "game_rft_audio"
    accum = max(1, args.global_batch // world)
    torch.manual_seed(0)
    model = get_model_cls(mc.model_id)(mc).cuda().train()
    docs_fl = None if args.docs == 1 else (torch.arange(mc.n_frames) * args.docs // mc.n_frames)[None]
    fpt = flops_per_token(mc, tokens, docs_fl)  # doc-masked pairs counted exactly for --docs > 1
    n_params = sum(p.numel() for p in model.parameters())
    if world > 1:
        with torch.no_grad():
            for p in model.parameters():
                dist.broadcast(p, 0)
    opt = init_muon(model, rank=rank, world_size=world, **cfg.train.opt_kwargs)
    ema = EMA(model, beta=0.999)
    red = GradReducer(model.parameters(), world_size=world)
    batches = []
    for i in range(2):
        b = [t.cuda() for t in synthetic_video_batch(mc, 1, seed=1234 + rank * 97 + i, n_docs=args.docs)]
        if av:
            g = torch.Generator().manual_seed(4321 + rank * 97 + i)
            b.append(torch.randn(1, mc.n_frames, mc.audio_channels, generator=g).to(torch.bfloat16).cuda())
        batches.append(b)
    vae_scale = cfg.train.vae_scale

    def micro(i, sync):
        vid, mouse, btn, doc = batches[i % 2][:4]
        red.begin(sync)
        if av:
            loss = model(vid / vae_scale, batches[i % 2][4], mouse, btn)[0] / accum
        else:
            loss = model(vid / vae_scale, mouse, btn, doc) / accum
        loss.backward()
        red.finish()
        return loss

    def step():
        for i in range(accum):
            micro(i, i == accum - 1)
        opt.step()
        red.zero_grad()
        ema.update()

    for w in range(args.warmup):
        t0 = time.time()
        step()
        torch.cuda.synchronize()
        log(f"[bench] warmup {w} {time.time() - t0:.2f}s")

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        step()
        if rank == 0:
            log(f"[bench] step {s} issued at {time.perf_counter() - t0:.2f}s")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    ms_per_step = elapsed / args.steps * 1e3
    total_tokens = args.global_batch * tokens * args.steps
    value = total_tokens / elapsed

    # ---- roofline of the dominant kernel: one extra micro-step with HIP events around every launch
    roof, kernels = None, None
    if not args.no_profile:
        torch.cuda.synchronize()
        _lib.profile_begin()
        micro(0, False)
        prof = _lib.profile_end()
        red.zero_grad()
        kernels = sorted(prof.items(), key=lambda kv: -kv[1][1])
        tot_ms = sum(v[1] for v in prof.values())
        # group launches by kernel symbol (rocprof granularity): strip the shape suffix
        sym = {}
        for k, (n, ms, fl) in prof.items():
            s = k.split("[")[0] if k.startswith("gemm") else k.split("[")[0]
            a = sym.setdefault(s, [0, 0.0, 0.0])
            a[0] += n
            a[1] += ms
            a[2] += fl
        dom, (n, ms, fl) = max(sym.items(), key=lambda kv: kv[1][1])
        achieved = fl / (ms / 1e3) if ms > 0 else 0.0
        roof = {"kernel": dom, "bound": "mfma", "achieved": round(achieved / 1e12, 1), "peak": PEAK_BF16 / 1e12,
                "unit": "TFLOP/s", "frac": round(achieved / PEAK_BF16, 4), "traffic": None,
                "launches_per_microstep": n, "avg_launch_ms": round(ms / n, 4),
                "share_of_microstep_kernel_time": round(ms / tot_ms, 3)}
        # HBM bytes per launch of the same kernel, measured in this run on this box (PMC passes in
        # child processes over one micro-step of the same model, pmc_traffic)
        if traffic.get(dom):
            tr = traffic[dom]
            if tr:
                roof["traffic"] = round(tr["bytes"])
                roof["traffic_unit"] = "bytes/launch (HBM, PMC, this run)"
                roof["traffic_detail"] = traffic_detail(dom, tr, tokens, mc)
        # the other attention kernels' traffic, same passes
        if traffic:
            roof["traffic_by_kernel"] = {k: traffic_detail(k, tr, tokens, mc) for k, tr in traffic.items() if tr}
        if rank == 0:
            log("[bench] per-kernel time in one micro-step (ms):")
            for k, (n, ms_, fl_) in kernels[:40]:
                log(f"  {k:60s} n={n:3d} {ms_:9.3f} ms  {fl_ / max(ms_, 1e-9) / 1e9:8.1f} TF/s")
            log(f"  total kernel time {tot_ms:.1f} ms")
    log(f"[bench] peak HBM allocated {torch.cuda.max_memory_allocated() / 2**30:.1f} GiB")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and headline:
        cpu = cpu_baseline()

    if rank == 0:
        metric = METRIC if headline else f"latent-tokens/sec/GPU (fwd+bwd) {cfg_name} bf16"
        out = {"metric": metric, "value": round(value, 1), "unit": "latent-tokens/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 1),
               "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "bf16",
               "data": f"synthetic (random latents of the {cfg_name} shape, random-init weights)",
               "config": {"workload": f"{args.config} training step: global batch {args.global_batch} x "
                                      f"{mc.n_frames} frames x 8x8 latents ({tokens} tokens/sample), fwd+bwd + "
                                      f"{'RCCL grad all-reduce + ' if world > 1 else ''}Muon/AdamW step + EMA",
                          "model": f"{cfg_name} ({mc.n_layers} L, d{mc.d_model}, {mc.n_heads} H, "
                                   f"{n_params / 1e6:.1f}M params)", "global_batch": args.global_batch,
                          "seq_len": tokens, "parallelism": f"dp{world}",
                          **({"docs_per_sample": args.docs} if args.docs > 1 else {})},
               "tokens_per_s_per_gpu": round(value / world, 1),
               "value_is": "whole-job latent tokens/s over all ranks (the driver's bench contract: total "
                           "tokens / max-over-ranks time); the per-GPU figure is tokens_per_s_per_gpu",
               "step_mfma_frac": round(value * (FLOP_PER_TOKEN if headline else fpt) / world / PEAK_BF16, 4),
               "roofline": roof, "cpu_baseline": cpu}
        if kernels:  # the micro-step's largest kernel families by time (same HIP-event pass as roofline)
            out["kernel_rates"] = {k: {"launches": n_, "avg_ms": round(ms_ / n_, 3),
                                       "tflops": round(fl_ / max(ms_, 1e-9) / 1e9, 1),
                                       "frac": round(fl_ / max(ms_, 1e-9) * 1e3 / PEAK_BF16, 4)}
                                   for k, (n_, ms_, fl_) in kernels[:8] if fl_ > 0}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
