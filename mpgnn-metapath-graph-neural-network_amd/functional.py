"""Autograd functions over the HIP kernels (C ABI calls on torch's current HIP stream).

``rgcn_conv``  — one relational conv layer, forward + backward:
    out = Σ_r mean_r(x) @ W_r + x @ root + bias
  mode SINGLE: CustomRGCNConv (mp_rgcn_layer.py:225-246, 260-271), W 2-D, one relation.
  mode ALL:    PyG RGCNConv loop (≙ mp_rgcn_layer.py:249-258), W [R, F_in, F_out].
  Backward replaces the autograd graph the reference builds implicitly (main.py:1078):
  MmBackward (dW, droot, dh = dout·Wᵀ), DivBackward (/count), ScatterAddBackward (gather),
  IndexSelectBackward (index_add_ into node_2) — SURVEY §3 CS-4.

``segment_means`` — the mean aggregation alone (bit-exact vs PyG propagate, no grad).

With ``group`` set (dst-range sharding) the partial outputs of the ranks are
summed by an all-reduce (RCCL over xGMI for the "nccl" backend); grad_x of a node_2 shard is
all-gathered from the owners of the rows, the parameter gradients are all-reduced as one bucket
(by ``distributed.ShardGradReducer`` behind the earlier layers' backward, for nn.RGCNConv).
"""
from __future__ import annotations

import ctypes

import weakref

import torch
import torch.distributed as dist

from ._lib import ACT_NONE, ACT_RELU, MODE_ALL, MODE_SINGLE, MPGNN_ERR_UNSUPPORTED, check, lib
from .plan import GraphPlan

__all__ = ["rgcn_conv", "segment_means", "MODE_SINGLE", "MODE_ALL"]


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _stream_of(device: torch.device) -> int:
    """Raw handle of torch's current stream on ``device`` (the C accessor: ~0.2 µs against ~5 µs
    for ``torch.cuda.current_stream(...).cuda_stream``, which builds a Stream object — this runs
    a few times per layer call, so it shows in the host-bound small-graph epochs)."""
    if _raw_stream is not None:
        return _raw_stream(device.index if device.index is not None else torch.cuda.current_device())
    return torch.cuda.current_stream(device).cuda_stream


def _stream(t: torch.Tensor) -> int:
    return _stream_of(t.device)


def _dev(t: torch.Tensor, name: str) -> torch.Tensor:
    if not t.is_cuda:
        raise RuntimeError(
            f"mpgnn_amd: `{name}` is on {t.device}; the relational aggregation runs only as HIP "
            "kernels on a ROCm GPU (there is no CPU fallback). Move the model and data to 'cuda'.")
    if t.dtype != torch.float32:
        raise TypeError(f"mpgnn_amd: `{name}` must be float32 (the reference computes in fp32), got {t.dtype}")
    t = t.contiguous()
    if t.data_ptr() % 16:
        t = t.clone()
    return t


def _ptr(t):
    return None if t is None else t.data_ptr()


# Workspace per (device, stream): calls on one stream run in stream order, so one growing
# buffer serves them all (and keeps a fixed address for HIP-graph capture). Entry: [buffer,
# captured] — ``captured`` once a kernel using the buffer was recorded into a HIP graph.
_WS: dict = {}
# Buffers outgrown after (or while) a HIP graph captured them: the graph's kernels read and
# write them at every replay, so they must outlive the graph — they are kept per stream key
# until ``release_workspaces`` drops that key (the loops do when their graph is gone).
# A buffer no graph ever captured is dropped at once when outgrown.
_RETIRED: dict = {}


def _workspace(nbytes: int, device: torch.device) -> torch.Tensor:
    key = (device.index, _stream_of(device))
    ent = _WS.get(key)
    capturing = torch.cuda.is_current_stream_capturing()
    if ent is None or ent[0].numel() < nbytes:
        # drop the smaller buffer first when no graph holds it: the caching allocator hands its
        # block back in stream order, so the peak is the new size, not old + new
        old = _WS.pop(key, None)
        if old is not None and (old[1] or capturing):
            _RETIRED.setdefault(key, []).append(old[0])
        del ent, old
        ent = [torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=device), False]
        _WS[key] = ent
    if capturing:
        ent[1] = True
    return ent[0]


def release_workspaces(stream=None) -> None:
    """Drop the cached scratch buffers — every one, or those of one ``torch.cuda.Stream`` —
    once no HIP graph that captured them will be replayed again; the next call allocates anew.
    The caller orders later work after the graph's last replay (the loops make the released
    stream wait for the current one)."""
    if stream is None:
        _WS.clear()
        _RETIRED.clear()
        return
    for key in [k for k in _WS if k[1] == stream.cuda_stream]:
        del _WS[key]
    for key in [k for k in _RETIRED if k[1] == stream.cuda_stream]:
        del _RETIRED[key]


def workspace_bytes_cached() -> int:
    """Bytes held by the scratch-buffer cache (live and retired), for leak checks."""
    return sum(e[0].numel() for e in _WS.values()) + sum(t.numel() for ts in _RETIRED.values() for t in ts)


def _forward(x, weight, root, bias, plan: GraphPlan, mode: int, relation: int, num_relations: int,
             row_lo: int, row_hi: int, group, need_h: bool, act: int = ACT_NONE):
    x = _dev(x, "x")
    weight = _dev(weight, "weight")
    root = _dev(root, "root") if root is not None else None
    bias = _dev(bias, "bias") if bias is not None else None
    plan.to_device(x.device)
    N, f_in = x.shape
    f_out = weight.shape[-1]
    if N != plan.num_nodes:
        raise ValueError(f"x has {N} rows, the graph plan was built for {plan.num_nodes} nodes")
    if weight.shape[-2] != f_in:
        raise RuntimeError(f"mat1 and mat2 shapes cannot be multiplied ({N}x{f_in} and "
                           f"{weight.shape[-2]}x{f_out})")
    ws = _workspace(plan.workspace_bytes(mode, relation, num_relations, f_in, f_out, row_lo, row_hi,
                                         forward_only=True), x.device)
    out = torch.empty(N, f_out, dtype=torch.float32, device=x.device)
    # multi-edge segment means, kept for grad_weight (dW_r = Σ h_segᵀ dout[node_1]; the
    # single-edge segments' means are rows of x, which backward has anyway)
    h_save = torch.empty(plan.hsave_rows(mode, relation, num_relations), f_in, dtype=torch.float32,
                         device=x.device) if need_h else None
    if act != ACT_NONE:  # fused activation: unsharded layers only (see rgcn_conv)
        check(lib.mpgnn_rgcn_fwd_act(plan.handle, mode, int(relation), int(num_relations), x.data_ptr(), f_in,
                                     weight.data_ptr(), _ptr(root), _ptr(bias), f_out, out.data_ptr(),
                                     _ptr(h_save), ws.data_ptr(), act, _stream(x)), "mpgnn_rgcn_fwd_act")
    else:
        check(lib.mpgnn_rgcn_fwd(plan.handle, mode, int(relation), int(num_relations), x.data_ptr(), f_in,
                                 weight.data_ptr(), _ptr(root), _ptr(bias), f_out, row_lo, row_hi,
                                 out.data_ptr(), _ptr(h_save), ws.data_ptr(), _stream(x)),
              "mpgnn_rgcn_fwd")
    if group is not None:
        dist.all_reduce(out, group=group)
    return out, x, weight, root, h_save


class GradStash:
    """Parameter gradients of a layer applied several times in one forward (Net's conv2 for
    layers 1..L-1, model.py:144-146), summed inside the backward kernels instead of by autograd's
    gradient accumulation (one [R, F, F] add per extra use). Each use carries a role: ``"first"``
    (the LAST use in forward order, whose backward runs first: fresh gradients, kept here),
    ``"mid"`` (added to them) and ``"final"`` (the first use: added, then handed to autograd);
    the other uses hand autograd no parameter gradient. The sums are autograd's: dst + new,
    in backward order."""
    __slots__ = ("bufs",)

    def __init__(self):
        self.bufs = None


class _RGCNConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, root, bias, plan: GraphPlan, mode: int, relation: int,
                num_relations: int, row_lo: int, row_hi: int, group, act: int, params_reduced: bool,
                stash=None):
        # x is a ReLU output internal to Net.forward (_relu_internal): the backward fuses that
        # ReLU's backward into grad_x (mpgnn_rgcn_bwd_relu_in) and the producing layer skips its own
        ctx.x_src = weakref.ref(x) if getattr(x, "_mpgnn_relu_internal", False) else None
        out, x, weight, root, h_save = _forward(x, weight, root, bias, plan, mode, relation, num_relations,
                                                row_lo, row_hi, group, ctx.needs_input_grad[1], act)
        ctx.plan = plan
        ctx.mode, ctx.relation, ctx.num_relations = mode, relation, num_relations
        ctx.rows = (row_lo, row_hi)
        ctx.group = group
        ctx.params_reduced = params_reduced
        ctx.has_root, ctx.has_bias = root is not None, bias is not None
        ctx.act = act
        ctx.stash = stash
        ctx.save_for_backward(x, weight, root, h_save, out if act == ACT_RELU else None)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        x, weight, root, h_save, act_out = ctx.saved_tensors
        plan = ctx.plan
        grad_out = grad_out.contiguous()
        if ctx.act == ACT_RELU and not premasked(grad_out, act_out):
            # ReLU backward (threshold_backward): pass where the output > 0, one launch
            masked = torch.empty_like(act_out)
            check(lib.mpgnn_relu_bwd(grad_out.data_ptr(), act_out.data_ptr(), grad_out.numel(), masked.data_ptr(),
                                     _stream(x)), "mpgnn_relu_bwd")
            grad_out = masked
        if grad_out.data_ptr() % 16:
            grad_out = grad_out.clone()
        N, f_in = x.shape
        f_out = weight.shape[-1]
        nx, nw, nr, nb = ctx.needs_input_grad[:4]
        gx = torch.empty_like(x) if nx else None
        mask_src = _mask_source(ctx) if nx and ctx.group is None else None
        if ctx.stash is not None and ctx.group is None and nw and nr and nb and root is not None and ctx.has_bias:
            return _shared_backward(ctx, plan, x, weight, root, h_save, grad_out, gx, mask_src)
        want = [nw, nr and root is not None, nb and ctx.has_bias]
        shapes = [weight.shape, root.shape if root is not None else None, (f_out,)]
        flat = None
        if ctx.group is not None and not ctx.params_reduced and any(want):
            # direct functional caller with a group: dW / droot / dbias written into ONE flat
            # buffer, reduced by one all-reduce (nn.RGCNConv hands this to ShardGradReducer)
            sizes = [int(torch.Size(s).numel()) if w else 0 for w, s in zip(want, shapes)]
            flat = torch.empty(sum(sizes), dtype=torch.float32, device=x.device)
            offs = [0, sizes[0], sizes[0] + sizes[1]]
            gw, gr, gb = (flat[o:o + n].view(s) if w else None for w, s, o, n in zip(want, shapes, offs, sizes))
        else:
            gw, gr, gb = (torch.empty(s, dtype=torch.float32, device=x.device) if w else None
                          for w, s in zip(want, shapes))
        ws = _workspace(plan.workspace_bytes(ctx.mode, ctx.relation, ctx.num_relations, f_in, f_out,
                                             *ctx.rows), x.device)
        args = (plan.handle, ctx.mode, int(ctx.relation), int(ctx.num_relations), x.data_ptr(), f_in,
                weight.data_ptr(), _ptr(root), f_out, _ptr(h_save), grad_out.data_ptr(), ctx.rows[0], ctx.rows[1],
                _ptr(gx), _ptr(gw), _ptr(gr), _ptr(gb), ws.data_ptr(), _stream(x))
        if mask_src is not None:
            check(lib.mpgnn_rgcn_bwd_relu_in(*args, 0), "mpgnn_rgcn_bwd_relu_in")
            mark_premasked(gx, mask_src)
        else:
            check(lib.mpgnn_rgcn_bwd(*args), "mpgnn_rgcn_bwd")
        if ctx.group is not None:
            if gx is not None:
                if plan.shard_side == "gathered":
                    # non-zero only on this rank's node_2 rows: all-gather them (half the bytes)
                    from .distributed import gather_owned_rows
                    gx = gather_owned_rows(gx, plan.shard, ctx.group)
                else:  # node_1 shards gather from every row: partial sums everywhere
                    dist.all_reduce(gx, group=ctx.group)
            if flat is not None:
                dist.all_reduce(flat, group=ctx.group)
        return gx, gw, gr, gb, None, None, None, None, None, None, None, None, None, None


def _mask_source(ctx):
    """The layer input whose producing ReLU the backward may fuse into grad_x: a tensor Net.forward
    tagged internal, that nothing else observes (no tensor hook, no retain_grad)."""
    src = ctx.x_src() if getattr(ctx, "x_src", None) is not None else None
    if src is None or src.retains_grad or getattr(src, "_backward_hooks", None):
        return None
    return src


def mark_premasked(g: torch.Tensor, src: torch.Tensor) -> None:
    """g is the gradient w.r.t. ReLU output src with that ReLU's backward already applied."""
    g._mpgnn_premasked = (src.data_ptr(), src._version, g._version)


def premasked(grad_out: torch.Tensor, act_out: torch.Tensor) -> bool:
    """grad_out came unchanged from a consumer that applied act_out's ReLU backward (the token
    names act_out's storage and version and grad_out's own version: a gradient summed in place
    with another consumer's afterwards no longer matches)."""
    tok = getattr(grad_out, "_mpgnn_premasked", None)
    return tok is not None and tok == (act_out.data_ptr(), act_out._version, grad_out._version)


def _shared_backward(ctx, plan, x, weight, root, h_save, grad_out, gx, mask_src=None):
    """_RGCNConvFn.backward of one use of a shared layer (GradStash)."""
    stash, role = ctx.stash
    N, f_in = x.shape
    f_out = weight.shape[-1]
    ws = _workspace(plan.workspace_bytes(ctx.mode, ctx.relation, ctx.num_relations, f_in, f_out, *ctx.rows), x.device)
    args_head = (plan.handle, ctx.mode, int(ctx.relation), int(ctx.num_relations), x.data_ptr(), f_in,
                 weight.data_ptr(), root.data_ptr(), f_out, _ptr(h_save), grad_out.data_ptr(), ctx.rows[0],
                 ctx.rows[1], _ptr(gx))
    def bwd(bufs, acc):
        tail = (*(b.data_ptr() for b in bufs), ws.data_ptr(), _stream(x))
        if mask_src is not None:
            return lib.mpgnn_rgcn_bwd_relu_in(*args_head, *tail, 1 if acc else 0)
        return (lib.mpgnn_rgcn_bwd_accumulate if acc else lib.mpgnn_rgcn_bwd)(*args_head, *tail)

    if role == "first" or stash.bufs is None:
        bufs = tuple(torch.empty(sh, dtype=torch.float32, device=x.device) for sh in (weight.shape, root.shape, (f_out,)))
        check(bwd(bufs, False), "mpgnn_rgcn_bwd")
        stash.bufs = bufs
    else:
        bufs = stash.bufs
        st = bwd(bufs, True)
        if st == MPGNN_ERR_UNSUPPORTED:  # other widths / modes: fresh gradients, then autograd's add
            new = tuple(torch.empty_like(b) for b in bufs)
            check(bwd(new, False), "mpgnn_rgcn_bwd")
            for b, n in zip(bufs, new):
                b.add_(n)
        else:
            check(st, "mpgnn_rgcn_bwd_accumulate")
    if mask_src is not None and gx is not None:
        mark_premasked(gx, mask_src)
    none = (None,) * 10
    if role == "final":
        stash.bufs = None
        return (gx,) + bufs + none
    return (gx, None, None, None) + none


def rgcn_conv(x: torch.Tensor, weight: torch.Tensor, root, bias, plan: GraphPlan, mode: int,
              relation: int = -1, num_relations: int = 0, row_range=None, group=None,
              activation=None, params_reduced: bool = False, grad_stash=None) -> torch.Tensor:
    """One relational conv layer on the GPU (see module docstring).

    ``activation='relu'`` returns ``F.relu(layer(x))`` (model.py:144,146): fused into the
    combine epilogue when the layer is unsharded, applied after the all-reduce otherwise.
    ``params_reduced``: with a ``group``, the caller reduces the parameter gradients itself
    (``distributed.ShardGradReducer``); otherwise the backward all-reduces them (one bucket).
    ``grad_stash``: ``(GradStash, role)`` for a layer applied several times (see GradStash)."""
    if activation not in (None, "relu"):
        raise ValueError(f"activation must be None or 'relu', got {activation!r}")
    lo, hi = row_range if row_range is not None else (0, plan.num_nodes)
    fuse = activation == "relu" and group is None and plan.shard == (0, plan.num_nodes) \
        and (lo, hi) == (0, plan.num_nodes)
    act = ACT_RELU if fuse else ACT_NONE
    if not torch.is_grad_enabled() or not (x.requires_grad or weight.requires_grad or
                                           (root is not None and root.requires_grad) or
                                           (bias is not None and bias.requires_grad)):
        # inference: no autograd node, no saved means
        out = _forward(x, weight, root, bias, plan, int(mode), int(relation), int(num_relations),
                       int(lo), int(hi), group, False, act)[0]
    else:
        out = _RGCNConvFn.apply(x, weight, root, bias, plan, int(mode), int(relation),
                                int(num_relations), int(lo), int(hi), group, act, bool(params_reduced),
                                grad_stash if group is None else None)
    if activation == "relu" and not fuse:
        out = torch.relu(out)
    return out


class _SegmentMeansFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, plan: GraphPlan, mode: int, relation: int, num_relations: int):
        b, e = plan.select(mode, relation, num_relations)
        h = torch.empty(e - b, x.shape[1], dtype=torch.float32, device=x.device)
        check(lib.mpgnn_rel_mean_fwd(plan.handle, int(mode), int(relation), int(num_relations), x.data_ptr(),
                                     x.shape[1], h.data_ptr(), _stream(x)), "mpgnn_rel_mean_fwd")
        ctx.plan, ctx.mode, ctx.relation, ctx.num_relations = plan, mode, relation, num_relations
        ctx.shape = x.shape
        return h

    @staticmethod
    def backward(ctx, dh):
        plan = ctx.plan
        dh = dh.contiguous()
        F = ctx.shape[1]
        dx = torch.empty(ctx.shape, dtype=torch.float32, device=dh.device)
        nbytes = ctypes.c_int64()
        check(lib.mpgnn_rel_mean_bwd_workspace_bytes(plan.handle, int(ctx.mode), int(ctx.relation),
                                                     int(ctx.num_relations), F, ctypes.byref(nbytes)),
              "mpgnn_rel_mean_bwd_workspace_bytes")
        ws = _workspace(int(nbytes.value), dh.device)
        check(lib.mpgnn_rel_mean_bwd(plan.handle, int(ctx.mode), int(ctx.relation), int(ctx.num_relations),
                                     dh.data_ptr(), F, dx.data_ptr(), ws.data_ptr(), _stream(dh)),
              "mpgnn_rel_mean_bwd")
        return dx, None, None, None, None


def segment_means(x: torch.Tensor, plan: GraphPlan, mode: int, relation: int = -1,
                  num_relations: int = 0) -> torch.Tensor:
    """Segment means [S_sel, F] in relation-major segment order (PyG propagate's mean, bit-exact),
    differentiable: the backward scatters dh / count to the gathered rows (mpgnn_rel_mean_bwd)."""
    x = _dev(x, "x")
    plan.to_device(x.device)
    return _SegmentMeansFn.apply(x, plan, int(mode), int(relation), int(num_relations))
