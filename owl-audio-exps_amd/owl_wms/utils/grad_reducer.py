"""Data-parallel gradient all-reduce for MI355X (replaces DDP's reducer, rft_trainer.py:95-96).

* Gradients live as views into flat fp32 bucket buffers (p.grad is set once and accumulated
  in place by autograd), so a ready bucket is all-reduced with no flatten/copy.
* Buckets follow reverse parameter order (the order backward produces them) and are sized for
  xGMI rings (default 256 MB: 11 buckets for dit_v4's 2.82 GB of fp32 grads).
* A post-accumulate-grad hook (or ``grad_ready`` from the fused backward, which writes dW / db
  straight into the bucket views with beta = 1) counts ready parameters; on the LAST micro-step of an
  accumulation window a full bucket is launched immediately with ``async_op=True``: RCCL runs
  it on its own HIP stream (ordered after the producing kernels by RCCL's stream wait) while the
  backward of earlier layers continues on the compute stream.  Earlier micro-steps do not
  communicate (equal to the reference's per-micro-step all-reduce up to fp32 summation order).
* ``finish()`` waits for every launched bucket and averages (ReduceOp.AVG when available).
* The persistent single-pass attention backward holds every CU for its whole launch, so a bucket
  issued beside it would wait for its end.  On the synchronising micro-step over RCCL
  the reducer asks libowlk, from its first bucket launch on, to leave ``reserve_cus`` CUs free
  (``owlk_set_cu_reserve``; default 32 = four per XCD, env ``OWL_RCCL_RESERVE_CUS``) and restores the
  full grid in ``finish()``.
"""
import os

import torch
import torch.distributed as dist


class GradReducer:
    def __init__(self, params, bucket_mb=256, world_size=None, process_group=None, reserve_cus=None):
        self.params = [p for p in params if p.requires_grad]
        self.pg = process_group
        self.ws = world_size if world_size is not None else (dist.get_world_size() if dist.is_initialized() else 1)
        cap = bucket_mb * (1 << 20) // 4
        self.buckets = []  # list of (flat buffer, [params])
        # parameters tagged _owl_grad_stack = (group, index) get their views back to back in index
        # order, in one bucket (the DiT block's four modulation weights: one [6d, d] weight-gradient GEMM)
        stacks = {}
        for p in self.params:
            tag = getattr(p, "_owl_grad_stack", None)
            if tag is not None:
                stacks.setdefault(tag[0], []).append((tag[1], p))
        placed = set()
        cur, cur_n = [], 0
        for p in reversed(self.params):
            if id(p) in placed:
                continue
            tag = getattr(p, "_owl_grad_stack", None)
            unit = [q for _, q in sorted(stacks[tag[0]], key=lambda t: t[0])] if tag is not None else [p]
            n = sum(q.numel() for q in unit)
            if cur and cur_n + n > cap:
                self.buckets.append(cur)
                cur, cur_n = [], 0
            cur.extend(unit)
            cur_n += n
            placed.update(id(q) for q in unit)
        if cur:
            self.buckets.append(cur)
        self.flat = []
        self.bucket_of = {}
        for bi, plist in enumerate(self.buckets):
            n = sum(p.numel() for p in plist)
            buf = torch.zeros(n, device=plist[0].device, dtype=torch.float32)
            self.flat.append(buf)
            off = 0
            for p in plist:
                self.bucket_of[p] = bi
                p._owl_grad_view = buf[off:off + p.numel()].view_as(p)
                off += p.numel()
        for p in self.params:
            p._owl_reducer = self  # the fused backward reports direct bucket writes (nn/fused.py grad_done)
        self.sync = False
        nccl = self.ws > 1 and dist.is_initialized() and dist.get_backend(self.pg) == "nccl"
        self.op = dist.ReduceOp.AVG if nccl else dist.ReduceOp.SUM  # RCCL averages in-collective
        if reserve_cus is None:
            reserve_cus = int(os.environ.get("OWL_RCCL_RESERVE_CUS", "32"))
        self.reserve_cus = reserve_cus if nccl else 0  # gloo collectives run on the host
        self._reserved = False
        self.pending = [0] * len(self.buckets)
        self.works = []
        self.ready = set()
        self.hooks = [p.register_post_accumulate_grad_hook(self._hook) for p in self.params]
        self.zero_grad()

    def zero_grad(self):
        for buf in self.flat:
            buf.zero_()
        for p in self.params:
            p.grad = p._owl_grad_view

    def begin(self, sync):
        """Call before each micro-step's backward; sync=True on the last micro-step of the window."""
        self.sync = sync and self.ws > 1
        self.pending = [len(b) for b in self.buckets]
        self.works = []
        self.ready = set()
        for p in self.params:  # autograd may have replaced grad if someone set it to None
            if p.grad is None or p.grad.data_ptr() != p._owl_grad_view.data_ptr():
                if p.grad is not None:
                    p._owl_grad_view.copy_(p.grad)
                p.grad = p._owl_grad_view

    def grad_ready(self, p):
        """p's gradient for this micro-step is complete in its bucket view (a direct write by the
        fused backward).  The direct writes assume one use of p per forward: a second write on the
        synchronising micro-step would land in a bucket whose async all-reduce may already run."""
        if self.sync and p in self.ready:
            raise RuntimeError("GradReducer: a parameter's gradient was written twice in the synchronising "
                               "micro-step (parameter used twice per forward?); its bucket may already be "
                               "in flight")
        self._hook(p)

    def _hook(self, p):
        if not self.sync or p in self.ready:
            return
        self.ready.add(p)
        bi = self.bucket_of[p]
        self.pending[bi] -= 1
        if self.pending[bi] == 0:
            self._launch(bi)

    def _launch(self, bi):
        if self.reserve_cus > 0 and not self._reserved:  # backward launches from here on leave CUs free
            self._reserve(self.reserve_cus)
        self.works.append((dist.all_reduce(self.flat[bi], op=self.op, group=self.pg, async_op=True), bi, self.op))

    def finish(self):
        if not self.sync:
            return
        launched = {bi for _, bi, _ in self.works}
        for bi in range(len(self.buckets)):  # params that received no grad this step
            if bi not in launched:
                self._launch(bi)
        for w, bi, op in self.works:
            w.wait()
            if op == dist.ReduceOp.SUM:
                self.flat[bi].div_(self.ws)
        self.works = []
        self.sync = False
        if self._reserved:
            self._reserve(0)

    def _reserve(self, cus):
        from .. import _lib
        _lib.call("owlk_set_cu_reserve", cus)
        self._reserved = cus > 0


class EMA:
    """ema_pytorch.EMA(model, beta, update_after_step=0, update_every=1) restated (rft_trainer.py:105;
    the library is absent offline: parity unpinned, restated from its published algorithm).

    ``ema_model`` is a frozen deep copy of the model (what the reference samples with,
    rft_trainer.py:244); ``update()``: step s = self.step, then self.step += 1; skip unless
    s % update_every == 0; copy the weights while s <= update_after_step; on the first update
    after that copy them again and set ``initted``; then lerp every parameter toward the online
    weights by 1 - decay, decay = clamp(1 - (1 + e / inv_gamma)^-power, 0, beta) with
    e = max((s + 1) - update_after_step - 1, 0) (the counter is read after its increment; decay 0
    at e = 0).  The lerp is one libowlk
    multi-tensor pass (owlk_ema).  state_dict: 'initted', 'step' and 'ema_model.<param>' keys, the
    ema_pytorch layout (so a reference checkpoint's 'ema' entry loads after prefix stripping)."""

    def __init__(self, model, beta=0.999, update_after_step=0, update_every=1, inv_gamma=1.0, power=2 / 3):
        import copy
        self.online = [model]  # not a submodule (ema_pytorch keeps it in a list too)
        self.beta, self.after, self.every, self.inv_gamma, self.power = beta, update_after_step, update_every, inv_gamma, power
        self.ema_model = copy.deepcopy(model)
        self.ema_model.requires_grad_(False)
        self.params = [p for p in model.parameters()]
        self.shadow = [p for p in self.ema_model.parameters()]
        self.step, self.initted = 0, False

    @property
    def model(self):
        return self.online[0]

    def _copy(self):
        with torch.no_grad():
            for s, p in zip(self.shadow, self.params):
                s.copy_(p.detach())

    def get_current_decay(self):
        epoch = max(self.step - self.after - 1, 0)  # ema_pytorch reads the already-advanced step
        if epoch <= 0:
            return 0.0
        return max(0.0, min(self.beta, 1 - (1 + epoch / self.inv_gamma) ** -self.power))

    @torch.no_grad()
    def update(self):
        step = self.step
        self.step += 1
        if step % self.every != 0:
            return
        if step <= self.after:
            self._copy()
            return
        if not self.initted:
            self._copy()
            self.initted = True
        from .. import kernels as K
        K.ema_lerp(self.shadow, [p.detach() for p in self.params], 1.0 - self.get_current_decay())

    def state_dict(self):
        d = {"initted": torch.tensor(self.initted), "step": torch.tensor(self.step)}
        for k, v in self.ema_model.state_dict().items():
            d["ema_model." + k] = v
        return d

    def load_state_dict(self, d, strict=True):
        sd = {k[len("ema_model."):]: v for k, v in d.items() if k.startswith("ema_model.")}
        self.ema_model.load_state_dict(sd, strict=strict)
        self.initted = bool(d.get("initted", torch.tensor(True)))
        self.step = int(d.get("step", torch.tensor(0)))
