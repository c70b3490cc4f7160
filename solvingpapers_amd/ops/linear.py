"""Linear layer whose weight gradient is written straight into ``main_grad``.

Plain projections are library GEMMs (hipBLASLt through torch.mm); what this
adds is gradient-accumulation fusion: dW = dY^T X is computed directly into
the flat gradient buffer (``torch.mm(out=)`` / ``addmm_``), so backward makes
no per-parameter grad allocation and no extra accumulate pass.
"""
from __future__ import annotations

import os
import weakref

import torch

from ..utils.grad import commit
from . import _ext
from .layout import bias_grad, wgrad

# decode-time products with <= 4 token rows go to the GEMV kernel; SPA_GEMV=0 -> torch.mm
GEMV = os.environ.get("SPA_GEMV", "1") != "0"
GEMV_MAX_ROWS = 4

# dX = dY W runs as the NT product dY (W^T)^T on a transposed copy of W (K-contiguous, like the
# forward's operands) rebuilt once per optimizer step: hipBLASLt at LLaMA3-8B shapes, ABBA-timed
# (profiles/r2_dgrad_layouts.txt): qkv 0.336 -> 0.296 ms, o 0.217 -> 0.205, gate/up 1.365 -> 1.251,
# down 0.717 -> 0.601, LM head 6.07 -> 5.25, against one transpose per weight per step (≈ 6 ms for
# all of LLaMA3-8B with layout.hip's kernel). SPA_DGRAD_WT=0 keeps the NN product.
DGRAD_WT = os.environ.get("SPA_DGRAD_WT", "1") != "0"
# weights below SPA_DGRAD_WT_MIN elements keep NN (ViT-B/16's 0.6-2.4M-element weights gain too:
# 6,115 -> 6,180 img/s ABBA, profiles/r2_vit_dgrad_abba.txt)
DGRAD_WT_MIN_NUMEL = int(os.environ.get("SPA_DGRAD_WT_MIN", str(1 << 18)))
# id(w) -> (validity key, W^T, weakref(w)); entries leave with their tensor (weakref.finalize).
# Not a WeakKeyDictionary: its lookups compare tensor keys with ==, which is elementwise.
#
# CONTRACT (also for the fp8 weight images of ops/moe.py): a cached image is reused while
#   (a) the global weight epoch (ops.moe.bump_weight_epoch) and (b) the tensor's own _version
# are unchanged. Every in-framework writer of parameters bumps the epoch: the fused optimizers
# (train/optim.py _run), checkpoint.load, DataParallel.broadcast_params / gather_params
# (ZeRO-1). (b) catches torch in-place ops ON THE PARAMETER TENSOR ITSELF, but NOT writes
# through the FlatParams buffer (utils/flat.py attaches params as views with ``p.data = view``,
# so each keeps its own version counter) nor raw kernels. Any other code that rewrites weights
# (e.g. a custom optimizer, ``flat.param.copy_``) must call ``invalidate_weight_caches()``
# before the next backward, or dX silently uses the stale W^T. Trainer checks the epoch moved
# after each optimizer step (train/trainer.py). While a HIP graph is captured the cache is
# bypassed: the transpose is recorded into the graph, so replays rebuild it from the live W.
_WT_CACHE: dict = {}


def invalidate_weight_caches():
    """Mark every cached weight image (W^T, fp8) stale; call after writing weights by hand."""
    from .moe import bump_weight_epoch
    bump_weight_epoch()


def transposed_weight(w: torch.Tensor):
    """Contiguous W^T for the dgrad product, or None where it does not apply. Valid while the
    optimizer's weight epoch (bumped by every fused optimizer step) and the tensor's version
    counter (bumped by any torch in-place update) are unchanged -- see CONTRACT above."""
    if not (DGRAD_WT and w.is_cuda and w.dtype == torch.bfloat16 and w.dim() == 2 and w.is_contiguous()
            and w.numel() >= DGRAD_WT_MIN_NUMEL and w.shape[0] % 8 == 0 and w.shape[1] % 8 == 0
            and w.data_ptr() % 16 == 0):
        return None
    from .layout import transpose2d
    from .moe import _WEIGHT_EPOCH
    if torch.cuda.is_current_stream_capturing():
        # never hand an eager image to a graph (replays would not refresh it) and never keep a
        # capture-time tensor in the global cache
        with torch.no_grad():
            return transpose2d(w)
    key = (_WEIGHT_EPOCH[0], w._version, w.data_ptr())
    hit = _WT_CACHE.get(id(w))
    if hit is not None and hit[2]() is not w:
        hit = None                               # defensive: never another tensor's entry
    if hit is not None and hit[0] == key:
        return hit[1]
    with torch.no_grad():
        wt = transpose2d(w)
    if hit is None:
        weakref.finalize(w, _WT_CACHE.pop, id(w), None)
    _WT_CACHE[id(w)] = (key, wt, weakref.ref(w))
    return wt


def dgrad(dy2: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """dX = dY W for dY [T, N], W [N, K] (NT form on the cached W^T where it applies)."""
    wt = transposed_weight(w)
    return torch.mm(dy2, w) if wt is None else torch.mm(dy2, wt.t())


def _commit_bias(b, s):
    """Commit the fp32 column sum ``s`` as the gradient of bias ``b`` (flat buffer or .grad)."""
    def _b(out, acc):
        if out is None:
            return s.to(b.dtype)
        if acc:
            out.add_(s.to(out.dtype))
        else:
            out.copy_(s)
    return commit(b, _b)


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        ctx.w, ctx.b = w, b
        ctx.save_for_backward(x)
        x2 = x.reshape(-1, x.shape[-1])
        if b is not None:
            y = torch.addmm(b, x2, w.t())
        else:
            y = torch.mm(x2, w.t())
        # _unsafe_view: the output is a fresh tensor, not an autograd view, so
        # downstream in-place kernels (packed RoPE) may modify it
        return torch.ops.aten._unsafe_view(y, (*x.shape[:-1], w.shape[0]))

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        w, b = ctx.w, ctx.b
        dy2 = dy.reshape(-1, dy.shape[-1])
        x2 = x.reshape(-1, x.shape[-1])
        dx = dgrad(dy2, w).view(x.shape) if ctx.needs_input_grad[0] else None
        gw = gb = None
        if ctx.needs_input_grad[1]:
            def _w(out, acc):
                return wgrad(dy2, x2, out, acc)
            gw = commit(w, _w)
        if b is not None and ctx.needs_input_grad[2]:
            gb = _commit_bias(b, bias_grad(dy2))
        return dx, gw, gb


class _LinearActFn(torch.autograd.Function):
    """y = act(x W^T + b) (ViT / GPT MLP fc1 + GELU). Forward: library GEMM with the bias
    epilogue, then the activation kernel; the pre-activation u is kept for backward. Backward:
    ONE pass over (dY, u) writes dU = dY act'(u) and its column sums -- the bias gradient --
    (activation.hip act_bwd_colsum), instead of an activation-backward pass and a second read of
    dU for the bias; then dX = dU W and dW = dU^T X as in :class:`_LinearFn`."""

    @staticmethod
    def forward(ctx, x, w, b, kind, alpha):
        x2 = x.reshape(-1, x.shape[-1])
        u = torch.addmm(b, x2, w.t())
        y = _ext.ops().act_fwd(u, kind, alpha)
        ctx.save_for_backward(x, u)
        ctx.w, ctx.b, ctx.kind, ctx.alpha = w, b, kind, alpha
        return torch.ops.aten._unsafe_view(y, (*x.shape[:-1], w.shape[0]))

    @staticmethod
    def backward(ctx, dy):
        x, u = ctx.saved_tensors
        w, b = ctx.w, ctx.b
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        x2 = x.reshape(-1, x.shape[-1])
        gb = None
        if ctx.needs_input_grad[2]:
            du, s = _ext.ops().act_bwd_colsum(dy2, u, ctx.kind, ctx.alpha)
            gb = _commit_bias(b, s)
        else:
            du = _ext.ops().act_bwd(dy2, u, ctx.kind, ctx.alpha)
        dx = dgrad(du, w).view(x.shape) if ctx.needs_input_grad[0] else None
        gw = None
        if ctx.needs_input_grad[1]:
            def _w(out, acc):
                return wgrad(du, x2, out, acc)
            gw = commit(w, _w)
        return dx, gw, gb, None, None


class _LinearGluFn(torch.autograd.Function):
    """glu(x W^T) for a row-stacked [gate ; up] weight (LLaMA's w13, llama3/LLaMA-jax.ipynb:854-855).
    Forward: one GEMM + the GLU kernel, as glu(linear(x, W)). Backward: the GLU backward also writes
    the transposed gradient (activation.hip glu_bwd_t), so dW = dH^T X runs in hipBLASLt's fastest
    form -- both operands token-contiguous -- without the separate transpose pass the plain path
    spends on X (or dH); dX = dH W as in :class:`_LinearFn`."""

    @staticmethod
    def forward(ctx, x, w, kind):
        x2 = x.reshape(-1, x.shape[-1])
        h = torch.mm(x2, w.t())
        f = _ext.ops().glu_fwd(h, kind)
        ctx.save_for_backward(x, h)
        ctx.w, ctx.kind = w, kind
        return torch.ops.aten._unsafe_view(f, (*x.shape[:-1], w.shape[0] // 2))

    @staticmethod
    def backward(ctx, df):
        x, h = ctx.saved_tensors
        w = ctx.w
        x2 = x.reshape(-1, x.shape[-1])
        dh, dht = _ext.ops().glu_bwd_t(df.reshape(-1, df.shape[-1]), h, ctx.kind)
        dx = dgrad(dh, w).view(x.shape) if ctx.needs_input_grad[0] else None
        gw = None
        if ctx.needs_input_grad[1]:
            gw = commit(w, lambda out, acc: wgrad(dh, x2, out, acc, dyt=dht))
        return dx, gw, None


def linear_glu(x, w, kind="silu"):
    """glu(linear(x, w), kind) -- on the GPU (bf16, many tokens, widths % 8; SPA_GLU_T=0, read per
    call, keeps the plain composition) through :class:`_LinearGluFn`."""
    from .activation import glu
    from .reference import ACT_KINDS
    if _glu_t_mode() >= 1 and _glu_t_ok(x, w):
        return _LinearGluFn.apply(x, w, ACT_KINDS[kind])
    return glu(linear(x, w), kind)


class _SwiGluMLPFn(torch.autograd.Function):
    """w2(glu(x W13^T)) -- LLaMA's feed-forward (llama3/LLaMA-jax.ipynb:854-855) with both weight
    gradients in hipBLASLt's both-token-contiguous form: the GLU forward also writes y^T (kept for
    the backward instead of y) and the GLU backward writes dH^T (activation.hip glu_fwd_t /
    glu_bwd_t); only dY of the down projection is transposed by a separate pass."""

    @staticmethod
    def forward(ctx, x, w13, w2, kind):
        x2 = x.reshape(-1, x.shape[-1])
        h = torch.mm(x2, w13.t())
        f, ft = _ext.ops().glu_fwd_t(h, kind)
        y = torch.mm(f, w2.t())
        ctx.save_for_backward(x, h, ft)
        ctx.w13, ctx.w2, ctx.kind = w13, w2, kind
        return torch.ops.aten._unsafe_view(y, (*x.shape[:-1], w2.shape[0]))

    @staticmethod
    def backward(ctx, dy):
        from .layout import transpose2d
        x, h, ft = ctx.saved_tensors
        w13, w2 = ctx.w13, ctx.w2
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        x2 = x.reshape(-1, x.shape[-1])
        need = ctx.needs_input_grad
        dx = gw13 = gw2 = None
        if need[2]:
            dyt = transpose2d(dy2)
            gw2 = commit(w2, lambda out, acc: wgrad(dy2, ft.t(), out, acc, x2t=ft, dyt=dyt))
        dh, dht = _ext.ops().glu_bwd_t(dgrad(dy2, w2), h, ctx.kind)
        if need[0]:
            dx = dgrad(dh, w13).view(x.shape)
        if need[1]:
            gw13 = commit(w13, lambda out, acc: wgrad(dh, x2, out, acc, dyt=dht))
        return dx, gw13, gw2, None


def _glu_t_mode() -> int:
    """SPA_GLU_T (read per call): 0 plain glu(linear(..)), 1 linear_glu only, 2 (default) swiglu_mlp."""
    return int(os.environ.get("SPA_GLU_T", "2"))


def _glu_t_ok(x, w) -> bool:
    T = x.numel() // x.shape[-1] if x.shape[-1] else 0
    return (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and w.dim() == 2
            and w.shape[0] % 16 == 0 and x.shape[-1] % 8 == 0 and T >= 2048 and T % 8 == 0
            and not torch.cuda.is_current_stream_capturing())


def swiglu_mlp(x, w13, w2, kind="silu"):
    """linear(glu(linear(x, w13), kind), w2) with the transposed-operand weight gradients of
    :class:`_SwiGluMLPFn` where it applies (else linear_glu / the plain composition)."""
    if _glu_t_mode() >= 2 and _glu_t_ok(x, w13) and w2.dtype == torch.bfloat16 and w2.dim() == 2:
        from .reference import ACT_KINDS
        return _SwiGluMLPFn.apply(x, w13, w2, ACT_KINDS[kind])
    return linear(linear_glu(x, w13, kind), w2)


def linear_act(x, w, b, kind="gelu", alpha=None):
    """act(linear(x, w, b)) with the activation backward and the bias gradient fused into one
    pass on the GPU (bf16, bias present, widths % 8); elsewhere the two ops in sequence."""
    from .activation import act
    from .reference import ACT_KINDS
    if (b is not None and x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and w.shape[0] % 8 == 0 and x.shape[-1] % 8 == 0 and x.numel() > 0):
        if alpha is None:
            alpha = 0.01 if kind == "leaky_relu" else (1.0 if kind == "elu" else 0.0)
        return _LinearActFn.apply(x, w, b, ACT_KINDS[kind], float(alpha))
    return act(linear(x, w, b), kind, alpha)


def mlp(x, w1, b1, w2, b2, kind="gelu", alpha=None):
    """fc2(act(fc1(x))): hipBLASLt GEMMs with the activation backward and fc1's bias gradient fused
    (linear_act). GEMM epilogues on the 8-phase kernel were measured 2.8 % slower at ViT-B widths
    (fc1 at 630-770 TF vs hipBLASLt's ~1 PF at K = 768, profiles/r3_vit_mlp_epilogue_ab.txt) and
    were removed in round 4."""
    return linear(linear_act(x, w1, b1, kind, alpha), w2, b2)


def _gemv_ok(x, w, b) -> bool:
    """Decode-shaped inference product (<= GEMV_MAX_ROWS token rows, no autograd): routed to
    the weight-streaming GEMV kernel (csrc/kernels/gemv.hip) instead of a library GEMM."""
    if not (GEMV and b is None and x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16):
        return False
    if torch.is_grad_enabled() and (x.requires_grad or w.requires_grad):
        return False
    K = x.shape[-1]
    rows = x.numel() // K if K else 0
    return (1 <= rows <= GEMV_MAX_ROWS and K % 8 == 0 and w.dim() == 2 and w.stride(1) == 1
            and w.stride(0) % 8 == 0 and w.data_ptr() % 16 == 0 and x.stride(-1) == 1
            and x.data_ptr() % 16 == 0)


class _LinearFP8Fn(torch.autograd.Function):
    """fp8 Linear for the dense projections of the DeepSeek-V3 recipe (arXiv 2412.19437 sec. 3.3):
    forward and dX are e4m3 GEMMs on hipBLASLt (torch._scaled_mm, row-wise fp32 scales: one per
    token row of X / dY, one per output channel of W for the forward and per input channel for
    dX); dW runs in fp8 too (dims % 128) on the block-scaled Wgrad kernel with 128 x 1 token
    tiles (ops/moe.py FP8_WGRAD), else bf16 through the fused-accumulation path. Weight images (W and W^T, e4m3 +
    scales) are quantized once per optimizer step (ops/moe.py weight cache). Measured on MI355X
    (tools/probe_scaled_mm.py): 1.7-2.7 PF vs 0.9-1.5 PF bf16 at V3 projection shapes. The
    routed experts use the 1 x 128 / 128 x 128 block-scaled grouped kernel instead."""

    @staticmethod
    def forward(ctx, x, w, b):
        from .moe import quant_rows_fp8, quant_weight_fp8_rows
        ctx.w, ctx.b = w, b
        ctx.save_for_backward(x)
        x2 = x.reshape(-1, x.shape[-1])
        xq, sx = quant_rows_fp8(x2)
        wq, sw, _, _ = quant_weight_fp8_rows(w)
        y = torch._scaled_mm(xq, wq.t(), sx[:, None], sw[None, :], bias=b, out_dtype=x.dtype)
        return torch.ops.aten._unsafe_view(y, (*x.shape[:-1], w.shape[0]))

    @staticmethod
    def backward(ctx, dy):
        from .moe import quant_rows_fp8, quant_weight_fp8_rows
        (x,) = ctx.saved_tensors
        w, b = ctx.w, ctx.b
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        x2 = x.reshape(-1, x.shape[-1])
        dx = None
        if ctx.needs_input_grad[0]:
            dq, sd = quant_rows_fp8(dy2)
            _, _, wtq, swt = quant_weight_fp8_rows(w)
            dx = torch._scaled_mm(dq, wtq.t(), sd[:, None], swt[None, :], out_dtype=dy.dtype).view(x.shape)
        gw = gb = None
        if ctx.needs_input_grad[1] and _dense_wgrad_fp8_ok(dy2, x2, w):
            gw = _dense_wgrad_fp8(w, dy2, x2)
        elif ctx.needs_input_grad[1]:
            def _w(out, acc):
                return wgrad(dy2, x2, out, acc)
            gw = commit(w, _w)
        if b is not None and ctx.needs_input_grad[2]:
            gb = _commit_bias(b, bias_grad(dy2))
        return dx, gw, gb


def _dense_wgrad_fp8_ok(dy2, x2, w):
    from .moe import FP8_WGRAD
    return (FP8_WGRAD and dy2.is_cuda and w.dim() == 2 and w.shape[0] % 128 == 0 and w.shape[1] % 128 == 0
            and dy2.shape[0] > 0)


def _dense_wgrad_fp8(w, dy2, x2):
    """fp8 dW = dY^T X of an fp8 Linear on the block-scaled Wgrad kernel (one group): dY and X
    quantized in 128 x 1 token tiles (transposed images), as the routed experts' dW."""
    from .moe import commit_weight_grad_fp8, padded_offsets, quant_t_fp8_seg
    T = dy2.shape[0]
    off = _one_group(T, dy2.device)
    poff, ld = padded_offsets(off), (T + 127) // 128 * 128
    aq, sa = quant_t_fp8_seg(dy2, off, poff, ld)
    bq, sb = quant_t_fp8_seg(x2, off, poff, ld)
    return commit_weight_grad_fp8(w, aq, sa, bq, sb, poff)


_GROUP1: dict = {}


def _one_group(rows, device):
    """device offsets [0, rows] for the grouped kernels, cached (no per-call H2D copy)."""
    key = (rows, str(device))
    t = _GROUP1.get(key)
    if t is None:
        t = torch.tensor([0, rows], dtype=torch.int32, device=device)
        if len(_GROUP1) > 512:
            _GROUP1.clear()
        _GROUP1[key] = t
    return t


def _fp8_ok(x, w) -> bool:
    K = x.shape[-1]
    return (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and w.dim() == 2
            and w.shape[0] % 16 == 0 and K % 16 == 0 and x.numel() > 0 and (x.numel() // K) % 16 == 0)


def linear(x, w, b=None, fp8=False):
    """y = x w^T (+ b). ``fp8``: e4m3 forward / dX on hipBLASLt with row-wise scales (dims
    multiples of 16; else bf16)."""
    if fp8 and _fp8_ok(x, w) and not _gemv_ok(x, w, b):
        return _LinearFP8Fn.apply(x, w, b)
    if _gemv_ok(x, w, b):
        x2 = x.reshape(-1, x.shape[-1])
        if x2.stride(0) % 8:
            x2 = x2.contiguous()
        return _ext.ops().gemv(x2, w).view(*x.shape[:-1], w.shape[0])
    return _LinearFn.apply(x, w, b)


# (id(w) for w in ws) -> (W view, main_grad view, weakrefs, data pointers): the joint views of
# row-stacked weights that FlatParams placed back to back (linear_rows)
_JOINT: dict = {}


def _joint_views(ws):
    """([sum N, K] weight view, matching main_grad view) spanning the row-stacked weights ``ws``
    when they and their main_grad views are contiguous and back to back in memory (FlatParams
    lays a module's parameters out in registration order), else None. Cached per weight tuple;
    re-validated by data pointers each call."""
    w0 = ws[0]
    mgs = [getattr(w, "main_grad", None) for w in ws]
    if any(m is None for m in mgs):
        return None
    ptrs = tuple(w.data_ptr() for w in ws) + tuple(m.data_ptr() for m in mgs)
    key = tuple(id(w) for w in ws)
    hit = _JOINT.get(key)
    if hit is not None and hit[3] == ptrs and all(r() is w for r, w in zip(hit[2], ws)):
        return hit[0], hit[1]
    K = w0.shape[1]
    rows, off_w, off_g = 0, 0, 0
    for w, m in zip(ws, mgs):
        if (w.dim() != 2 or w.shape[1] != K or w.dtype != w0.dtype or not w.is_contiguous()
                or not m.is_contiguous() or m.dtype != mgs[0].dtype or m.shape != w.shape):
            return None
        if w.data_ptr() != w0.data_ptr() + off_w or m.data_ptr() != mgs[0].data_ptr() + off_g:
            return None
        off_w += w.numel() * w.element_size()
        off_g += m.numel() * m.element_size()
        rows += w.shape[0]
    wd, md = w0.detach(), mgs[0]
    if wd.storage_offset() + rows * K > wd.untyped_storage().nbytes() // wd.element_size():
        return None
    W = wd.as_strided((rows, K), (K, 1), wd.storage_offset())
    MG = md.as_strided((rows, K), (K, 1), md.storage_offset())
    if hit is None:
        weakref.finalize(w0, _JOINT.pop, key, None)
    _JOINT[key] = (W, MG, tuple(weakref.ref(w) for w in ws), ptrs)
    return W, MG


class _LinearRowsFn(torch.autograd.Function):
    """y = x W^T with W the joint view of row-stacked weights: one GEMM forward, one dX GEMM and
    one dW GEMM into the joint main_grad view backward (no concatenation, no dX sum)."""

    @staticmethod
    def forward(ctx, x, W, MG, *ws):
        ctx.W, ctx.MG, ctx.ws = W, MG, ws
        ctx.save_for_backward(x)
        x2 = x.reshape(-1, x.shape[-1])
        return torch.ops.aten._unsafe_view(torch.mm(x2, W.t()), (*x.shape[:-1], W.shape[0]))

    @staticmethod
    def backward(ctx, dy):
        from ..utils.grad import _Gen
        (x,) = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        x2 = x.reshape(-1, x.shape[-1])
        dx = dgrad(dy2, ctx.W).view(x.shape) if ctx.needs_input_grad[0] else None
        if any(ctx.needs_input_grad[3:]):
            acc = getattr(ctx.ws[0], "_spa_gen", -1) == _Gen.value
            assert all((getattr(w, "_spa_gen", -1) == _Gen.value) == acc for w in ctx.ws), \
                "linear_rows: weights committed apart within one iteration"
            wgrad(dy2, x2, ctx.MG, acc)
            for w in ctx.ws:
                w._spa_gen = _Gen.value
        return (dx, None, None) + (None,) * len(ctx.ws)


def linear_rows(x, ws):
    """x [.., K] times the row-stacked weights ``ws`` ([N_i, K] each) -> [.., sum N_i]: ONE GEMM
    per pass when the weights sit back to back in a FlatParams buffer (Gemma's q and MQA K/V
    projections), else the concatenation of separate products."""
    jv = _joint_views(ws)
    if jv is not None and not _gemv_ok(x, jv[0], None):
        return _LinearRowsFn.apply(x, jv[0], jv[1], *ws)
    return torch.cat([linear(x, w) for w in ws], dim=-1)


class Linear(torch.nn.Module):
    """nn.Linear-compatible (weight [out, in]) module using :func:`linear`."""

    def __init__(self, in_features, out_features, bias=True, device=None, dtype=None):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.weight = torch.nn.Parameter(torch.empty(out_features, in_features, device=device, dtype=dtype))
        self.bias = torch.nn.Parameter(torch.empty(out_features, device=device, dtype=dtype)) if bias else None
        self.reset_parameters()

    def reset_parameters(self):
        torch.nn.init.kaiming_uniform_(self.weight, a=5 ** 0.5)
        if self.bias is not None:
            bound = 1 / self.in_features ** 0.5
            torch.nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, x):
        return linear(x, self.weight, self.bias)

    def extra_repr(self):
        return f"in_features={self.in_features}, out_features={self.out_features}, bias={self.bias is not None}"
