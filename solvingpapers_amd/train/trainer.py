"""Generic training loop shared by every model family.

What the reference spreads over per-notebook loops (gpt/gpt-jax.ipynb:791-802,
gemma/gemma.ipynb:540-560, deepseekv3/deepseekv3.ipynb:2320-2470, ViT/AE/VAE/KD epochs):
step loop, periodic held-out loss, LR warmup + cosine (deepseekv3.ipynb:1976-1986),
grad-norm clipping, gradient accumulation, checkpoint/resume — plus what it lacks
(SURVEY §5): JSONL metrics, NaN/Inf guard (skip the update, abort after N in a row),
RNG + step + data-cursor in checkpoints, auto-resume from ``latest`` (pairs with
``torchrun --max-restarts``), CUDA-event step timing and optional torch.profiler trace.

Parameters live in one FlatParams buffer; data parallelism (RCCL buckets overlapped
with backward, optional ZeRO-1) and the fused flat optimizers come from
parallel/data_parallel.py and train/optim.py. The model must implement
``forward(x, y) -> scalar loss`` (all models in solvingpapers_amd.models do).
"""
from __future__ import annotations

import json
import math
import os
import time
from dataclasses import asdict, dataclass, field
from typing import Callable, Iterable, Optional

import torch
import torch.distributed as dist

from ..parallel.data_parallel import DataParallel
from ..utils.flat import FlatParams
from ..utils.prof import annotate
from . import checkpoint as ckpt
from .optim import FlatAdamW, FlatSGD, cosine_lr


@dataclass
class TrainConfig:
    steps: int = 1000
    grad_accum: int = 1
    # models with forward_pair (DeepSeek-V3, Gemma): micro-batches run in layer-interleaved pairs so
    # each expert-parallel all-to-all / sequence-parallel TP boundary overlaps the other
    # micro-batch's compute (even grad_accum only)
    pair_microbatches: bool = True
    optimizer: str = "adamw"            # adamw | adam | sgd
    lr: float = 3e-4
    min_lr: Optional[float] = None       # None -> constant LR
    warmup: int = 0
    betas: tuple = (0.9, 0.95)
    eps: float = 1e-8
    weight_decay: float = 0.1
    clip: Optional[float] = 1.0
    eval_every: int = 0
    eval_iters: int = 10
    ckpt_dir: Optional[str] = None
    ckpt_every: int = 0
    keep: int = 2
    resume: str = "auto"                 # "auto" (latest if present) | "never" | <path>
    log_path: Optional[str] = None       # JSONL metrics
    log_every: int = 1
    # device values (loss, grad norm, skip flag, step time) are read back in batches of
    # ``sync_every`` steps: one host sync per batch instead of one per step (GPU only)
    sync_every: int = 16
    max_bad_steps: int = 3               # consecutive non-finite grad norms before abort
    zero1: bool = False
    opt_overlap: bool = False
    tokens_per_sample: int = 0           # for tok/s (0 -> x.numel())
    # MFU in the metrics record: model FLOPs per token (0 -> model.flops_per_token(seq_len) when the
    # model has it) against this per-GPU peak (MI355X dense bf16)
    flops_per_token: float = 0.0
    peak_flops: float = 2.5e15
    profile_steps: tuple = ()            # (start, stop) -> torch.profiler trace into ckpt_dir/log dir
    grad_dtype: Optional[torch.dtype] = None
    param_dtype: Optional[torch.dtype] = None


class NonFiniteLoss(RuntimeError):
    pass


class Trainer:
    def __init__(self, model, cfg: TrainConfig, train_batch: Callable[[int], tuple],
                 eval_batch: Optional[Callable[[int], tuple]] = None, dp_group=None, ep_group=None,
                 expert_dp_group=None, hooks: Iterable[Callable] = (), tp_group=None, groups=None):
        """``groups`` (parallel/groups.py ProcessGroups) sets dp/tp/ep/expert-dp groups at once:
        dense gradients are averaged over ``dp_group``, expert gradients summed over
        ``expert_dp_group`` (then / dp), the grad norm reduced over TP and EP as needed."""
        self.model, self.cfg = model, cfg
        self.train_batch, self.eval_batch = train_batch, eval_batch
        self.groups = groups
        if groups is not None:
            dp_group, tp_group = groups.dp_group, groups.tp_group
            ep_group, expert_dp_group = groups.ep_group, groups.expert_dp_group
        self.rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
        self.world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        if self.groups is not None:
            # an explicit layout: dp_group None means dp == 1 (e.g. tp == world), NOT the world
            # group -- a DataParallel there would broadcast rank 0's TP shards to every rank and
            # average the gradients of different shards
            self.dp_size = self.groups.dp
            use_dp = self.groups.dp > 1
        else:
            self.dp_size = (dist.get_world_size(dp_group) if dp_group is not None else self.world) \
                if self.world > 1 else 1
            use_dp = self.world > 1
        pgroups = model.param_groups() if hasattr(model, "param_groups") else None
        self.flat = FlatParams(model, groups=pgroups, align=64 * max(1, self.world),
                               grad_dtype=cfg.grad_dtype, param_dtype=cfg.param_dtype)
        self.dp = DataParallel(model, self.flat, group=dp_group, zero1=cfg.zero1,
                               expert_dp_group=expert_dp_group) if use_dp else None
        if self.dp is not None:
            # before the optimizer is built: FlatOptimizer copies its fp32 master from the
            # params at construction, so a later broadcast would be undone by the first step
            self.dp.broadcast_params()
        shard = (self.dp.shard_ranges(), dp_group) if (self.dp and cfg.zero1) else None
        if cfg.optimizer in ("adamw", "adam"):
            self.opt = FlatAdamW(self.flat, lr=cfg.lr, betas=cfg.betas, eps=cfg.eps, weight_decay=cfg.weight_decay,
                                 max_grad_norm=cfg.clip, adam_l2=cfg.optimizer == "adam", shard=shard,
                                 ep_group=ep_group, tp_group=tp_group)
        elif cfg.optimizer == "sgd":
            self.opt = FlatSGD(self.flat, lr=cfg.lr, weight_decay=cfg.weight_decay, max_grad_norm=cfg.clip,
                               shard=shard, ep_group=ep_group, tp_group=tp_group)
        else:
            raise ValueError(cfg.optimizer)
        for m in getattr(model, "moe_layers", lambda: [])():
            m.balance_group = dp_group
        # overlapped optimizer: a model that waits for each bucket's update before reading it
        # (param_wait_cb: LLaMA3, Gemma, DeepSeek-V3) overlaps it with its next forward; any other model
        # waits for the whole update right after the step (train_step), never reading stale weights
        self._overlap_waits = bool(cfg.opt_overlap and hasattr(model, "param_wait_cb"))
        if self._overlap_waits:
            model.param_wait_cb = self.flat.group_waiter(pgroups) if pgroups else self.flat.wait_bucket
        self.step = 0
        self.tokens_seen = 0     # cumulative training tokens over all DP ranks (the reference logs "tokens")
        self.bad_steps = 0
        self.history = []
        self.hooks = list(hooks)
        self._pending = []      # per-step device values awaiting one batched host read
        self._last_seq = 0
        self._log = None
        if cfg.log_path and self.rank == 0:
            os.makedirs(os.path.dirname(os.path.abspath(cfg.log_path)), exist_ok=True)
            self._log = open(cfg.log_path, "a")

    # ------------------------------------------------------------------ utils
    def _flops_per_token(self, seq):
        if self.cfg.flops_per_token:
            return self.cfg.flops_per_token
        f = getattr(self.model, "flops_per_token", None)
        if f is None or not seq:
            return 0.0
        try:
            return float(f(seq))
        except TypeError:
            return 0.0

    def lr_at(self, step):
        c = self.cfg
        if c.min_lr is None:
            return c.lr * min(1.0, (step + 1) / (c.warmup + 1)) if c.warmup else c.lr
        return cosine_lr(step, c.lr, c.warmup, c.steps, c.min_lr)

    def buffers(self):
        fin = getattr(self.model, "finish_pending_updates", None)
        if fin is not None:
            fin()                             # in-flight routing-bias updates land first
        return {n: b for n, b in self.model.named_buffers() if n.endswith("routing_bias")}

    def log(self, rec):
        self.history.append(rec)
        if self._log is not None:
            self._log.write(json.dumps(rec) + "\n")
            self._log.flush()
        for h in self.hooks:
            h(rec)

    # -------------------------------------------------------------- checkpoint
    def save(self, loss=None):
        if not self.cfg.ckpt_dir:
            return None
        self.flat.wait_all()
        # saved step = index of the last completed step; resume continues at step + 1
        extra = {"loss": loss, "tokens": self.tokens_seen, "config": {k: str(v) for k, v in asdict(self.cfg).items()}}
        if self.groups is not None:
            extra["layout"] = self.groups.layout()
        return ckpt.save(self.cfg.ckpt_dir, self.step - 1, self.flat, self.opt, self.buffers(), extra=extra,
                         keep=self.cfg.keep)

    def maybe_resume(self):
        r = self.cfg.resume
        if r == "never":
            return False
        path = ckpt.latest(self.cfg.ckpt_dir) if (r == "auto" and self.cfg.ckpt_dir) else (None if r == "auto" else r)
        if not path:
            return False
        info = ckpt.load(path, self.flat, self.opt, self.buffers())
        saved = info["extra"].get("layout") if isinstance(info.get("extra"), dict) else None
        if self.groups is not None and saved is not None and saved != self.groups.layout():
            raise RuntimeError(f"checkpoint layout {saved} != running layout {self.groups.layout()}")
        self.step = info["step"] + 1
        if isinstance(info.get("extra"), dict):
            self.tokens_seen = int(info["extra"].get("tokens") or 0)
        return True

    # ------------------------------------------------------------------ eval
    @torch.no_grad()
    def evaluate(self, iters=None):
        """Mean held-out loss (gpt-jax.ipynb:542-552, gemma.ipynb:522-538, deepseekv3.ipynb:2098-2125)."""
        if self.eval_batch is None:
            return None
        self.flat.wait_all()
        fin = getattr(self.model, "finish_pending_updates", None)
        if fin is not None:
            fin()
        was = self.model.training
        self.model.eval()
        tot = 0.0
        n = iters or self.cfg.eval_iters
        for i in range(n):
            x, y = self.eval_batch(i)
            tot += float(self.model(x, y))
        self.model.train(was)
        v = torch.tensor([tot / n], dtype=torch.float64)
        if self.world > 1 and dist.get_backend() == "gloo":
            dist.all_reduce(v)
            v /= self.world
        elif self.world > 1:
            v = v.to(self.flat.device)
            dist.all_reduce(v)
            v = v.cpu() / self.world
        return float(v)

    # ------------------------------------------------------------------ train
    def train_step(self, step):
        """One optimizer step over ``grad_accum`` micro-batches. Returns (loss, ntok, ok) as
        DEVICE tensors (no host sync): ``ok`` is False when the global grad norm was not
        finite and the update was skipped on every rank (FlatOptimizer.clip_coef)."""
        c = self.cfg
        self.opt.zero_grad()
        tot = None
        ntok = 0
        # pair only where the model overlaps something across the two (EP exchanges, TP chunk
        # pipeline): a pair otherwise just doubles the live activations
        pair = (c.pair_microbatches and c.grad_accum % 2 == 0 and hasattr(self.model, "forward_pair")
                and self.model.training and bool(getattr(self.model, "pair_overlaps", lambda: False)()))
        n = 2 if pair else 1
        for mi in range(0, c.grad_accum, n):
            xs = [self.train_batch(step * c.grad_accum + mi + j) for j in range(n)]
            for x, _ in xs:
                ntok += c.tokens_per_sample * x.shape[0] if c.tokens_per_sample else x.numel()
                self._last_seq = x.shape[1] if x.dim() > 1 else 1
            last = mi + n == c.grad_accum
            ctx = self.dp.no_sync() if (self.dp is not None and not last) else _null()
            with ctx:
                with annotate("forward"):
                    loss = self.model.forward_pair(*xs[0], *xs[1]) if pair else self.model(*xs[0])
                with annotate("backward"):
                    (loss / c.grad_accum).backward()
            tot = loss.detach() if tot is None else tot + loss.detach()
        if self.dp is not None:
            with annotate("grad_sync"):
                self.dp.finish_grad_sync()
        sync_sp = getattr(self.model, "sync_sequence_parallel_grads", None)
        if sync_sp is not None:
            sync_sp()
        from ..ops.moe import _WEIGHT_EPOCH
        epoch = _WEIGHT_EPOCH[0]
        with annotate("optimizer"):
            self.opt.step(lr=self.lr_at(step), overlap=c.opt_overlap)
        if c.opt_overlap and (not self._overlap_waits or (self.dp is not None and c.zero1)):
            # models without per-bucket waits, and ZeRO-1: gather_params() below clones this rank's
            # shard on the main stream, so the side-stream update of that shard must be complete
            self.flat.wait_all()
        # cached W^T / fp8 weight images are keyed on this epoch (ops/linear.py CONTRACT)
        assert _WEIGHT_EPOCH[0] != epoch, "optimizer step did not invalidate the cached weight images"
        if self.dp is not None:
            self.dp.gather_params()
        ok = self.opt.last_step_ok()
        return tot / c.grad_accum, ntok, ok

    def _flush(self):
        """Read back the pending steps' device values with one sync, log them, and apply
        the consecutive-bad-step abort."""
        if not self._pending:
            return
        dev = self.flat.device
        if dev.type == "cuda":
            self._pending[-1]["ev"].synchronize()
        for r in self._pending:
            ok = bool(r["ok"]) if r["ok"] is not None else True
            if ok:
                self.bad_steps = 0
            else:
                self.bad_steps += 1
            if r["log"]:
                if dev.type == "cuda" and r["ev0"] is not None:
                    dt = r["ev0"].elapsed_time(r["ev"]) / 1e3
                else:
                    dt = r["dt"]
                gn = r["gn"]
                tps = r["ntok"] * self.dp_size / max(dt, 1e-9)
                rec = {"step": r["step"], "loss": float(r["loss"]) if ok else float("nan"), "lr": r["lr"],
                       "ok": ok, "dt": dt, "tok_per_s": tps, "tokens": r["tokens"],
                       "grad_norm": float(gn) if gn is not None else None}
                fpt = self._flops_per_token(r["seq"])
                if fpt:
                    # per-GPU model FLOP/s over the peak; tok/s is over the DP ranks, each of which
                    # holds 1/(tp*ep...) of the model work for its tokens: divide by the world size
                    rec["mfu"] = tps * fpt / max(1, self.world) / self.cfg.peak_flops
                if dev.type == "cuda":
                    rec["mem_gb"] = torch.cuda.max_memory_allocated(dev) / 1e9
                self.log(rec)
            if self.bad_steps >= self.cfg.max_bad_steps:
                self._pending.clear()
                raise NonFiniteLoss(f"{self.bad_steps} consecutive non-finite gradient norms at step {r['step']}")
        self._pending.clear()

    def fit(self):
        c = self.cfg
        self.model.train()
        self.maybe_resume()
        prof = None
        dev = self.flat.device
        cuda = dev.type == "cuda"
        flush_every = max(1, c.sync_every) if cuda else 1
        while self.step < c.steps:
            s = self.step
            _maybe_inject_fault(s, self.rank)  # test hook: no-op unless SPA_FAULT_STEP is set
            if c.profile_steps and s == c.profile_steps[0]:
                prof = _start_profiler(c)
            ev0 = None
            if cuda:
                ev0 = torch.cuda.Event(enable_timing=True)
                ev0.record()
            t0 = time.perf_counter()
            loss, ntok, ok = self.train_step(s)
            ev = None
            if cuda:
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
            if prof is not None and s + 1 >= c.profile_steps[1]:
                prof.stop()
                prof = None
            gn = self.opt.last_grad_norm
            self.tokens_seen += ntok * self.dp_size
            self._pending.append({"step": s, "loss": loss, "ok": ok, "gn": gn, "lr": self.lr_at(s), "ntok": ntok,
                                  "tokens": self.tokens_seen, "seq": self._last_seq,
                                  "ev0": ev0, "ev": ev, "dt": time.perf_counter() - t0,
                                  "log": s % c.log_every == 0 or s == c.steps - 1})
            evals = c.eval_every and ((s % c.eval_every == 0 and s) or s == c.steps - 1)
            self.step += 1
            ckpt_now = c.ckpt_every and self.step % c.ckpt_every == 0
            if len(self._pending) >= flush_every or evals or ckpt_now or self.step >= c.steps:
                self._flush()
            if evals:
                v = self.evaluate()
                if v is not None:
                    self.log({"step": s, "val_loss": v})
            if ckpt_now:
                self.save(float(loss))
        self._flush()
        self.flat.wait_all()
        if c.ckpt_dir and c.ckpt_every:
            self.save()
        return self.history


def _maybe_inject_fault(step: int, rank: int):
    """Fault injection for the elastic-restart test (SURVEY §5 'Failure detection'):
    ``SPA_FAULT_STEP=s`` (+ ``SPA_FAULT_RANK=r``, default 0) makes rank r die abruptly --
    ``os._exit``, no cleanup, no checkpoint -- when it reaches step s. With
    ``SPA_FAULT_MARKER=<file>`` it fires once (the marker survives the restart), so a run
    under ``torchrun --max-restarts`` crashes, restarts and auto-resumes."""
    at = os.environ.get("SPA_FAULT_STEP")
    if at is None or int(at) != step or int(os.environ.get("SPA_FAULT_RANK", "0")) != rank:
        return
    marker = os.environ.get("SPA_FAULT_MARKER")
    if marker:
        if os.path.exists(marker):
            return
        with open(marker, "w") as f:
            f.write(f"rank {rank} killed at step {step}\n")
    os._exit(17)


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _start_profiler(c: TrainConfig):
    from torch.profiler import ProfilerActivity, profile
    out = os.path.join(c.ckpt_dir or ".", "trace")
    os.makedirs(out, exist_ok=True)
    acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if torch.cuda.is_available() else [])
    p = profile(activities=acts, on_trace_ready=torch.profiler.tensorboard_trace_handler(out))
    p.start()
    return p
