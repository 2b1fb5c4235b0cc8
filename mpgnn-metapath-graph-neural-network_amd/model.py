"""Drop-in for the reference ``model.py`` MPGNN wrappers (model.py:132-149, 179-228).

The wrappers stay plain PyTorch (ReLU, Dropout, Linear, LogSoftmax) as in the reference; the
relational layers are the gfx950 ones, and the Linear layers' weight gradient is reduced in
node slices (``linear``: same forward, same parameters, blocked summation order). Module/parameter names, their
order and a seeded initialisation are identical to the reference, so ``state_dict``s load
either way. ``MPNet`` (model.py:153-176) is not provided: it calls its convs with 4 arguments
where CustomRGCNConv.forward needs 5 (mp_rgcn_layer.py:158) and cannot run in the reference.
The score-function classes (model.py:26-125: InputLayer, OutputLayer, Score) are the GPU ones of
``score`` (segment-argmax kernels), re-exported here under the reference's names.
"""
from __future__ import annotations

import ctypes
import os
import weakref

import torch
import torch.nn as nn
import torch.nn.functional as F

from .mp_rgcn_layer import CustomRGCNConv
from .functional import GradStash
from .nn import RGCNConv
from .score import InputLayer, OutputLayer, Score  # noqa: F401  (model.py:26-125)

__all__ = ["Net", "MPNetm", "linear", "InputLayer", "OutputLayer", "Score"]


_WGRAD_WS: dict = {}  # (N, F, O) -> mpgnn_linear_wgrad_workspace_bytes


class _SplitKLinear(torch.autograd.Function):
    """``F.linear`` whose weight gradient is reduced in slices over the node dimension.

    The wrappers' Linear layers see every node as a row (N = 14,541 at C3, 2 M at C5) but have
    few outputs (2 classes, 64 hidden): ``grad_weight = grad_outᵀ @ x`` is then a [O × F] GEMM
    with K = N, which the BLAS library tiles into a handful of long serial-K workgroups (66 µs
    for O = 2 at C3, 6 % of the epoch). Here K is cut into slices of ≤ 1024 rows: one batched
    GEMM over the slices + a sum over them — the same products in fp32, summed in a different
    (blocked) order; for F ≤ 256 and O ≤ 32·256/F the C ABI's ``mpgnn_linear_wgrad`` does it in
    two launches, bias gradient included. Forward and grad_input are exactly the autograd ones
    (``F.linear``, ``mm``)."""

    @staticmethod
    def forward(ctx, x, weight, bias, relu=False):
        ctx.has_bias = bias is not None
        ctx.relu = relu
        # x a ReLU output internal to Net.forward: its ReLU backward fused into grad_input
        ctx.x_src = weakref.ref(x) if getattr(x, "_mpgnn_relu_internal", False) else None
        out = _head_fwd(x, weight, bias, relu)
        if out is None:  # other shapes: the library GEMM
            out = F.linear(x, weight, bias)
            if relu:
                out = torch.relu(out)
        ctx.save_for_backward(x, weight, out if relu else None)
        return out

    @staticmethod
    def backward(ctx, g):
        x, weight, out = ctx.saved_tensors
        gx = gw = gb = None
        g = g.contiguous()
        from .functional import premasked
        if ctx.relu and not premasked(g, out):  # ReLU fused into the forward: threshold_backward, one launch
            from . import _lib
            from .functional import _stream
            masked = torch.empty_like(out)
            _lib.check(_lib.lib.mpgnn_relu_bwd(g.data_ptr(), out.data_ptr(), g.numel(), masked.data_ptr(), _stream(g)),
                       "mpgnn_relu_bwd")
            g = masked
        if ctx.needs_input_grad[0]:
            from .functional import _mask_source, mark_premasked
            src = _mask_source(ctx)
            gx = _head_dgrad(g, weight, x if src is not None else None)
            if gx is None:
                gx = g.mm(weight)
            elif src is not None:
                mark_premasked(gx, src)
        f, o = x.shape[1], g.shape[1]
        # the HIP pair is scalar-FMA work (N·F·O): for the heads with few outputs (O ≤ 32·256/F:
        # Net.lin, MPNetm.fc2) it beats the library's serial-K GEMM; F = O = 128 (MPNetm.fc1 of
        # one metapath) runs on the bf16-split matrix cores behind the same entry point; other
        # wide heads take the batched GEMM
        small = o <= 32 * (256 // max(f, 1)) or (f == 128 and o == 128)
        if ctx.needs_input_grad[1] and f <= 256 and small and x.dtype == g.dtype == torch.float32:
            # one HIP kernel pair (row-sliced partials + ordered slice sum, bias in the same pass)
            # instead of pad + batched GEMM + two reductions (~8 launches)
            from . import _lib
            from .functional import _stream, _workspace
            xc, gc = x.contiguous(), g.contiguous()
            key = (xc.shape[0], f, o)
            nb = _WGRAD_WS.get(key)
            if nb is None:  # the size depends on the shape only: asked once per shape
                nbytes = ctypes.c_int64()
                _lib.check(_lib.lib.mpgnn_linear_wgrad_workspace_bytes(xc.shape[0], f, o, ctypes.byref(nbytes)),
                           "mpgnn_linear_wgrad_workspace_bytes")
                nb = _WGRAD_WS[key] = int(nbytes.value)
            ws = _workspace(nb, x.device)
            gw = torch.empty(o, f, dtype=torch.float32, device=x.device)
            want_b = ctx.has_bias and ctx.needs_input_grad[2]
            gb = torch.empty(o, dtype=torch.float32, device=x.device) if want_b else None
            _lib.check(_lib.lib.mpgnn_linear_wgrad(xc.data_ptr(), gc.data_ptr(), xc.shape[0], f, o, gw.data_ptr(),
                                                   gb.data_ptr() if want_b else None, ws.data_ptr(), _stream(x)),
                       "mpgnn_linear_wgrad")
            return gx, gw, gb, None
        if ctx.needs_input_grad[1]:
            n = x.shape[0]
            slices = max(1, min(256, (n + 1023) // 1024))
            if slices == 1:
                gw = g.t().mm(x)
            else:
                rows = (n + slices - 1) // slices
                pad = rows * slices - n
                gp = F.pad(g, (0, 0, 0, pad)) if pad else g
                xp = F.pad(x, (0, 0, 0, pad)) if pad else x
                gw = torch.bmm(gp.view(slices, rows, -1).transpose(1, 2), xp.view(slices, rows, -1)).sum(0)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            gb = g.sum(0)
        return gx, gw, gb, None


def _aligned(*ts) -> bool:
    return all(t is None or (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and t.data_ptr() % 16 == 0)
               for t in ts)


def _head_fwd(x, weight, bias, relu):
    """act(x @ weightᵀ + bias) through the C ABI's mpgnn_linear_fwd: F = O = 128 (MPNetm.fc1 of a
    128-wide metapath, model.py:224; the bf16-split GEMM + one bias/ReLU pass) and the narrow
    heads O <= 8, F <= 256 (Net.lin model.py:147, MPNetm.fc2 :226; one wave per row, float64
    sums, one rounding): cheap launches where torch's addmm costs ~25 µs of host time (the eager
    C3 mode-SINGLE epoch is host-bound). None: shape or layout not covered."""
    o_ok = (x.dim() == 2 and weight.dim() == 2 and weight.shape[1] == x.shape[1]
            and ((x.shape[1] == 128 and weight.shape[0] == 128) or (weight.shape[0] <= 8 and x.shape[1] <= 256
                                                                   and x.shape[1] % 4 == 0)))
    if (not o_ok or (bias is not None and tuple(bias.shape) != (weight.shape[0],))
            or not _aligned(x, weight, bias)):
        return None  # (a shape mismatch is left to F.linear, which raises as the reference does)
    from . import _lib
    from .functional import _stream
    n, f = x.shape
    o = weight.shape[0]
    out = torch.empty(n, o, dtype=torch.float32, device=x.device)
    st = _lib.lib.mpgnn_linear_fwd(x.data_ptr(), n, f, weight.data_ptr(), o, bias.data_ptr() if bias is not None else None,
                                   _lib.ACT_RELU if relu else _lib.ACT_NONE, out.data_ptr(), _stream(x))
    if st == _lib.MPGNN_ERR_UNSUPPORTED:
        return None
    _lib.check(st, "mpgnn_linear_fwd")
    return out


def _head_dgrad(g, weight, relu_in=None):
    """grad_out @ weight through mpgnn_linear_dgrad (F = O = 128, or O <= 8), else None; with
    ``relu_in`` (the head's input, a ReLU output) mpgnn_linear_dgrad_relu_in: that ReLU's backward
    applied in the same launch."""
    if g.dim() != 2 or weight.dim() != 2 or g.shape[1] != weight.shape[0] or not _aligned(g, weight, relu_in):
        return None
    from . import _lib
    from .functional import _stream
    n, o = g.shape
    f = weight.shape[1]
    gx = torch.empty(n, f, dtype=torch.float32, device=g.device)
    if relu_in is not None:
        st = _lib.lib.mpgnn_linear_dgrad_relu_in(g.data_ptr(), n, o, weight.data_ptr(), f, relu_in.data_ptr(),
                                                 gx.data_ptr(), _stream(g))
    else:
        st = _lib.lib.mpgnn_linear_dgrad(g.data_ptr(), n, o, weight.data_ptr(), f, gx.data_ptr(), _stream(g))
    if st == _lib.MPGNN_ERR_UNSUPPORTED:
        return None
    _lib.check(st, "mpgnn_linear_dgrad")
    return gx


class _HeadLogSoftmax(torch.autograd.Function):
    """``F.log_softmax(layer(x), dim=1)`` for a narrow head (O <= 8 outputs, F <= 256: Net.lin,
    model.py:147-148): the forward ONE launch (mpgnn_linear_fwd with MPGNN_ACT_LOG_SOFTMAX: the
    float64-summed dots, then log_softmax over the row's outputs), the backward one pass
    (mpgnn_linear_logsoftmax_bwd: log_softmax's backward, grad_input — with the ReLU backward of
    an internal input fused, as _SplitKLinear — and the row-sliced weight / bias partials) + the
    ordered partial sum: 2 + 2 launches where the separate ops take 2 + 4."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        from . import _lib
        from .functional import _stream
        ctx.x_src = weakref.ref(x) if getattr(x, "_mpgnn_relu_internal", False) else None
        n, f = x.shape
        o = weight.shape[0]
        out = torch.empty(n, o, dtype=torch.float32, device=x.device)
        _lib.check(_lib.lib.mpgnn_linear_fwd(x.data_ptr(), n, f, weight.data_ptr(), o,
                                             bias.data_ptr() if bias is not None else None, _lib.ACT_LOG_SOFTMAX,
                                             out.data_ptr(), _stream(x)), "mpgnn_linear_fwd (log_softmax)")
        ctx.has_bias = bias is not None
        ctx.save_for_backward(x, weight, out)
        return out

    @staticmethod
    def backward(ctx, g):
        from . import _lib
        from .functional import _mask_source, _stream, _workspace, mark_premasked
        x, weight, logp = ctx.saved_tensors
        g = g.contiguous()
        n, f = x.shape
        o = weight.shape[0]
        src = _mask_source(ctx) if ctx.needs_input_grad[0] else None
        gx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        gw = torch.empty(o, f, dtype=torch.float32, device=x.device)
        gb = torch.empty(o, dtype=torch.float32, device=x.device) if ctx.has_bias else None
        key = ("lsm", n, f, o)
        nb = _WGRAD_WS.get(key)
        if nb is None:
            nbytes = ctypes.c_int64()
            _lib.check(_lib.lib.mpgnn_linear_logsoftmax_bwd_workspace_bytes(n, f, o, ctypes.byref(nbytes)),
                       "mpgnn_linear_logsoftmax_bwd_workspace_bytes")
            nb = _WGRAD_WS[key] = int(nbytes.value)
        ws = _workspace(nb, x.device)
        _lib.check(_lib.lib.mpgnn_linear_logsoftmax_bwd(g.data_ptr(), logp.data_ptr(), x.data_ptr(), n, f, o,
                                                        weight.data_ptr(), x.data_ptr() if src is not None else None,
                                                        gx.data_ptr() if gx is not None else None, gw.data_ptr(),
                                                        gb.data_ptr() if gb is not None else None, ws.data_ptr(),
                                                        _stream(x)), "mpgnn_linear_logsoftmax_bwd")
        if src is not None:
            mark_premasked(gx, src)
        return gx, gw if ctx.needs_input_grad[1] else None, gb if ctx.needs_input_grad[2] else None


class _DropoutRelu(torch.autograd.Function):
    """``F.dropout(x, p, training=True)`` of a ReLU output internal to MPNetm.forward (model.py:
    211-215): the forward is torch's own fused dropout (``torch.native_dropout``: the kernel and
    random stream F.dropout uses on the GPU), the backward ONE launch (mpgnn_dropout_relu_bwd:
    dropout's masked scale with the ReLU backward of x's layer applied, which then skips its own
    launch) instead of two."""

    @staticmethod
    def forward(ctx, x, p):
        out, mask = torch.native_dropout(x, p, True)
        ctx.scale = 1.0 / (1.0 - p)
        ctx.x_src = weakref.ref(x)
        ctx.save_for_backward(mask, x)
        return out

    @staticmethod
    def backward(ctx, g):
        from . import _lib
        from .functional import _mask_source, _stream, mark_premasked
        mask, x = ctx.saved_tensors
        g = g.contiguous()
        src = _mask_source(ctx)
        gx = torch.empty_like(g)
        _lib.check(_lib.lib.mpgnn_dropout_relu_bwd(g.data_ptr(), mask.data_ptr(),
                                                   x.data_ptr() if src is not None else None, ctx.scale, g.numel(),
                                                   gx.data_ptr(), _stream(g)), "mpgnn_dropout_relu_bwd")
        if src is not None:
            mark_premasked(gx, src)
        return gx, None


def dropout_after_relu(module: torch.nn.Dropout, x: torch.Tensor, internal: bool) -> torch.Tensor:
    """``module(x)`` for x = F.relu(conv(...)): _DropoutRelu when x is internal (training, CUDA,
    0 < p < 1, contiguous fp32), else the module itself."""
    if (internal and module.training and not module.inplace and 0.0 < module.p < 1.0 and x.is_cuda
            and x.dtype == torch.float32 and x.is_contiguous() and x.numel() > 0):
        x._mpgnn_relu_internal = True
        return _DropoutRelu.apply(x, float(module.p))
    return module(x)


def head_log_softmax(layer: torch.nn.Linear, x: torch.Tensor) -> torch.Tensor:
    """``F.log_softmax(layer(x), dim=1)`` (Net's output, model.py:147-148): _HeadLogSoftmax for
    fp32 CUDA inputs with O <= 8, F <= 256 (F % 4 == 0, 16-byte aligned), else the two ops."""
    w, b = layer.weight, layer.bias
    if (_HEAD_FUSE and x.dim() == 2 and x.is_cuda and x.is_contiguous() and w.dim() == 2 and w.shape[1] == x.shape[1]
            and w.shape[0] <= 8 and x.shape[1] <= 256 and x.shape[1] % 4 == 0 and w.is_contiguous()
            and (b is None or tuple(b.shape) == (w.shape[0],)) and _aligned(x, w, b)):
        return _HeadLogSoftmax.apply(x, w, b)
    return F.log_softmax(linear(layer, x), dim=1)


def linear(layer: torch.nn.Linear, x: torch.Tensor, activation=None) -> torch.Tensor:
    """``layer(x)`` (``F.relu(layer(x))`` with ``activation='relu'``) with the heads' HIP forward /
    input gradient where covered and the split-K weight gradient above (same parameters)."""
    if activation not in (None, "relu"):
        raise ValueError(f"activation must be None or 'relu', got {activation!r}")
    if x.dim() != 2 or not x.is_cuda:
        out = layer(x)
        return torch.relu(out) if activation == "relu" else out
    return _SplitKLinear.apply(x, layer.weight, layer.bias, activation == "relu")


class _FastTrainToggle:
    """``train(mode)`` / ``eval()`` as nn.Module's (every submodule's ``training`` flag set), as a
    flat loop over ``modules()`` instead of the recursive ``named_children`` + ``__setattr__``
    walk: the reference's loops toggle the model twice per epoch (main.py:1058,1086), which for
    the small-graph epochs (C3 mode SINGLE, ~1 ms, host-bound) cost ~0.1 ms. Falls back to
    nn.Module.train when a submodule overrides ``train``."""

    def train(self, mode: bool = True):
        if not isinstance(mode, bool):
            raise ValueError("training mode is expected to be boolean")
        mods = list(self.modules())
        if any(type(m).train is not torch.nn.Module.train for m in mods if m is not self):
            return torch.nn.Module.train(self, mode)
        for m in mods:
            m.__dict__["training"] = mode
        return self


# MPGNN_GRAD_STASH=0: Net's shared conv2 gradients summed by autograd (A/B switch; same values)
_GRAD_STASH = os.environ.get("MPGNN_GRAD_STASH", "1") != "0"
# MPGNN_RELU_FUSE=0: each of Net's ReLU backwards a launch of its own (A/B switch; same values)
_RELU_FUSE = os.environ.get("MPGNN_RELU_FUSE", "1") != "0"
# MPGNN_HEAD_FUSE=0: Net's head as F.linear + F.log_softmax (A/B switch; rounding-level differences)
_HEAD_FUSE = os.environ.get("MPGNN_HEAD_FUSE", "1") != "0"


def _hooked(*mods) -> bool:
    """A forward hook (sees the activations) or a module backward hook (sees their gradients) on
    any of mods, or a global one: Net's activations are then observable, not internal."""
    from torch.nn.modules import module as _m
    glob = (_m._global_forward_hooks, getattr(_m, "_global_backward_hooks", None),
            getattr(_m, "_global_backward_pre_hooks", None))
    if any(g for g in glob):
        return True
    return any(m._forward_hooks or getattr(m, "_backward_hooks", None) or getattr(m, "_backward_pre_hooks", None)
               for m in mods)


class Net(_FastTrainToggle, torch.nn.Module):
    """RGCN baseline (model.py:132-149): conv1, then the SAME conv2 for layers 1..L-1."""

    def __init__(self, input_dim, hidden_dim, num_rel, output_dim, ll_output_dim, metapath_length):
        super().__init__()
        self.metapath_length = metapath_length
        self.conv1 = RGCNConv(input_dim, hidden_dim, num_rel, flow="target_to_source")
        self.conv2 = RGCNConv(hidden_dim, output_dim, num_rel, flow="target_to_source")
        self.LinearLayer = torch.nn.Linear(output_dim, ll_output_dim)

    def forward(self, x, edge_index, edge_type, *, shard=None, group=None, shard_side="gathered"):
        last = self.metapath_length - 1
        stash = None
        if last >= 2 and _GRAD_STASH and shard is None and group is None and x.is_cuda and torch.is_grad_enabled() and \
                all(p.requires_grad for p in (self.conv2.weight, self.conv2.root, self.conv2.bias)):
            # conv2's gradients over its uses summed inside the backward kernels (GradStash)
            stash = GradStash()
        # the activations between the layers (and into the head) are internal: nothing outside this
        # forward can observe them or their gradients unless a module hook hands them out — then each
        # ReLU's backward stays a launch of its own instead of being fused into the consumer's
        # input-gradient kernel (functional.premasked)
        internal = shard is None and group is None and x.is_cuda and torch.is_grad_enabled() and _RELU_FUSE and \
            not _hooked(self.conv1, self.conv2, self.LinearLayer)
        for layer_index in range(0, self.metapath_length):
            conv = self.conv1 if layer_index == 0 else self.conv2
            kw = {}
            if stash is not None and layer_index >= 1:
                kw["_grad_stash"] = (stash, "first" if layer_index == last else "final" if layer_index == 1 else "mid")
            # F.relu(conv(...)) of model.py:144,146, fused into the layer's combine kernel
            x = conv(x, edge_index, edge_type, shard=shard, group=group, activation="relu", shard_side=shard_side,
                     **kw)
            if internal:
                x._mpgnn_relu_internal = True
        return head_log_softmax(self.LinearLayer, x)  # F.log_softmax(self.LinearLayer(x), dim=1)


class MPNetm(_FastTrainToggle, torch.nn.Module):
    """Multi-metapath MPGNN (model.py:179-228): one CustomRGCNConv chain per metapath, layer l
    of metapath i aggregates over relation metapaths[i][l]; ReLU + Dropout(0.6) after each
    layer; concatenation; fc1 + ReLU; fc2; LogSoftmax."""

    def __init__(self, input_dim, hidden_dim, num_rel, output_dim, ll_output_dim, n_metapaths, metapaths):
        super().__init__()
        self.n_metapaths = n_metapaths
        self.metapaths = metapaths
        self.input_dim = input_dim
        self.hidden_dim = hidden_dim
        self.layers_list = torch.nn.ModuleList()
        for i in range(0, len(metapaths)):
            convs = torch.nn.ModuleList()
            convs.append(CustomRGCNConv(self.input_dim, self.hidden_dim, 1, flow="target_to_source"))
            for _ in range(0, len(metapaths[i]) - 1):
                convs.append(CustomRGCNConv(self.hidden_dim, self.hidden_dim, 1, flow="target_to_source"))
            self.layers_list.append(convs)
        self.fc1 = torch.nn.Linear(self.hidden_dim * len(metapaths), self.hidden_dim)
        self.fc2 = torch.nn.Linear(self.hidden_dim, ll_output_dim)
        self.log_softmax = torch.nn.LogSoftmax(dim=1)
        self.dropout = nn.Dropout(0.6)
        self.dropout2 = nn.Dropout(0.6)

    def forward(self, x, edge_index, edge_type):
        # the ReLU outputs (after each conv and fc1) are internal to this forward unless a module
        # hook observes them: their ReLU backwards then fuse into the consumer's backward (the
        # dropout's, the head's; functional.premasked)
        internal = x.is_cuda and torch.is_grad_enabled() and _RELU_FUSE and not _hooked(
            self.fc1, self.fc2, self.log_softmax, self.dropout, self.dropout2,
            *(c for convs in self.layers_list for c in convs))
        embeddings = []
        for i in range(0, len(self.metapaths)):
            for layer_index in range(0, len(self.metapaths[i])):
                conv = self.layers_list[i][layer_index]
                rel = self.metapaths[i][layer_index]
                # F.relu(conv(...)) of model.py:211,214, fused into the layer's output kernel
                if layer_index == 0:
                    h = conv(layer_index, rel, x, edge_index, edge_type, activation="relu")
                    h = dropout_after_relu(self.dropout, h, internal)
                else:
                    h = conv(layer_index, rel, h, edge_index, edge_type, activation="relu")
                    h = dropout_after_relu(self.dropout2, h, internal)
            embeddings.append(h)
        # torch.cat of ONE embedding (a single metapath) is a copy of it: skipped, same values
        concatenated_embedding = embeddings[0] if len(embeddings) == 1 else torch.cat(embeddings, dim=1)
        h = linear(self.fc1, concatenated_embedding, activation="relu")  # F.relu(fc1(.)), model.py:225
        if _hooked(self.fc2, self.log_softmax):
            return self.log_softmax(linear(self.fc2, h))
        if internal:
            h._mpgnn_relu_internal = True
        return head_log_softmax(self.fc2, h)  # self.log_softmax(self.fc2(h)), model.py:226-227
