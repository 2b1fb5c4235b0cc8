"""Loss weights and scores of the reference training loop, computed next to the logits.

The reference scores every epoch with scikit-learn on Python lists
(``f1_score(torch.argmax(pred[idx], 1).tolist(), y.tolist(), average='macro')``,
main.py:1094-1098, main_rgcn.py:409-415), which copies every prediction to the host. Here the
per-class confusion counts are reduced on the device and only those counts (3 × classes
int64) cross to the host, where the F-score is finished with the same float64 arithmetic and
the same numpy reduction scikit-learn 1.7 uses (``precision_recall_fscore_support``:
``f = 2·tp / (true_sum + pred_sum)`` over the sorted union of labels, then ``np.average``).
Results are identical to scikit-learn's (tests/test_loop.py).
"""
from __future__ import annotations

import weakref

import numpy as np
import torch

__all__ = ["f1_macro", "f1_macro_many", "confusion_counts_many", "confusion_counts_rows", "f1_from_counts",
           "class_weight_balanced", "class_weight_tensor", "nll_loss_rows"]


def _count(v: torch.Tensor, bins: int) -> torch.Tensor:
    """bincount of values in [0, bins) (integer scatter-add: exact, and no host read of the
    maximum — torch.bincount's size query — so it can run inside a HIP-graph capture)."""
    out = torch.zeros(bins, dtype=torch.int64, device=v.device)
    return out.scatter_add_(0, v, torch.ones_like(v))


def _confusion_counts(pred: torch.Tensor, y: torch.Tensor, num_classes: int) -> torch.Tensor:
    """[3, C] int64: (count of each label in pred, in y, agreeing positions per label). Labels
    outside [0, C) fall in an overflow bin (nll_loss rejects them before this runs)."""
    pred = pred.reshape(-1).to(torch.int64)
    y = y.reshape(-1).to(device=pred.device, dtype=torch.int64)
    c = num_classes
    over = torch.full_like(y, c)
    pred_c = torch.where((pred >= 0) & (pred < c), pred, over)
    y_c = torch.where((y >= 0) & (y < c), y, over)
    hit = torch.where(pred_c == y_c, y_c, over)  # misses → overflow bin
    return torch.stack([_count(pred_c, c + 1)[:c], _count(y_c, c + 1)[:c], _count(hit, c + 1)[:c]])


def _finish(counts: np.ndarray) -> float:
    pred_sum, true_sum, tp = (counts[0].astype(np.int64), counts[1].astype(np.int64),
                              counts[2].astype(np.int64))
    labels = (pred_sum + true_sum) > 0  # sklearn: unique_labels(y_true, y_pred), sorted
    denom = true_sum[labels].astype(np.float64) + pred_sum[labels].astype(np.float64)
    f = 2.0 * tp[labels].astype(np.float64) / denom
    return float(np.average(f))


def f1_macro_many(pairs: list[tuple[torch.Tensor, torch.Tensor]], num_classes: int) -> list[float]:
    """Macro F1 of several (predictions, labels) pairs with ONE device→host copy.
    Labels must lie in [0, num_classes) (the logits' width; nll_loss enforces it)."""
    if not pairs:
        return []
    counts = torch.stack([_confusion_counts(p, y, num_classes) for p, y in pairs]).cpu().numpy()
    return [_finish(c) for c in counts]


def confusion_counts_many(pairs: list[tuple[torch.Tensor, torch.Tensor]], num_classes: int) -> torch.Tensor:
    """[len(pairs), 3, C] int64 confusion counts, left on the device (no host sync); finish
    with ``f1_from_counts``."""
    return torch.stack([_confusion_counts(p, y, num_classes) for p, y in pairs])


_ROWS_OK: list = []  # (weakref(idx), idx._version, rows) of row lists found in range


def _rows_valid(idx: torch.Tensor, rows: int) -> bool:
    """Every entry of ``idx`` in [0, rows), checked once per list object and version (a list with
    an out-of-range row goes to torch's ops, whose ``scores[idx]`` raises like the reference's
    ``pred[idx]``). Not checked during a capture (no host read): the torch path runs instead."""
    for ri, vi, r in _ROWS_OK:
        if ri() is idx and vi == idx._version and r == rows:
            return True
    if idx.is_cuda and torch.cuda.is_current_stream_capturing():
        return False
    ok = idx.numel() == 0 or bool(((idx >= 0) & (idx < rows)).all().item())
    if ok:
        _ROWS_OK.insert(0, (weakref.ref(idx), idx._version, rows))
        del _ROWS_OK[16:]
    return ok


def confusion_counts_rows(scores: torch.Tensor, lists) -> torch.Tensor:
    """``confusion_counts_many([(torch.argmax(scores[idx], 1), y) for idx, y in lists], C)`` with
    C = scores.shape[1]: [len(lists), 3, C] int64 on the device. On the GPU (float32 scores,
    1-D integer row indices, up to 4 lists) ONE kernel (``mpgnn_confusion_counts``: argmax of
    each listed row + LDS histograms) instead of ~20 torch ops per list; same counts."""
    lists = list(lists)
    ok = (scores.is_cuda and scores.dim() == 2 and scores.dtype == torch.float32 and 0 < len(lists) <= 4
          and 1 <= scores.shape[1] <= 4096  # the kernel's LDS histograms (mpgnn_confusion_counts)
          and all(torch.is_tensor(i) and i.dim() == 1 and i.dtype in (torch.int64, torch.int32) and
                  torch.is_tensor(y) and y.numel() == i.numel() and not y.is_floating_point()
                  for i, y in lists)
          and all(_rows_valid(i, scores.shape[0]) for i, _ in lists))
    if not ok:
        return confusion_counts_many([(torch.argmax(scores[i], 1), y) for i, y in lists], _num_cols(scores))
    import ctypes
    from . import _lib
    from .functional import _stream
    dev = scores.device
    sc = scores.contiguous()
    c = sc.shape[1]
    idx = [i.to(device=dev, dtype=torch.int64).contiguous() for i, _ in lists]
    lab = [y.to(device=dev, dtype=torch.int64).reshape(-1).contiguous() for _, y in lists]
    n = len(lists)
    out = torch.empty(n, 3, c, dtype=torch.int64, device=dev)
    p_idx = (ctypes.c_void_p * n)(*[t.data_ptr() for t in idx])
    p_lab = (ctypes.c_void_p * n)(*[t.data_ptr() for t in lab])
    p_n = (ctypes.c_int64 * n)(*[t.numel() for t in idx])
    _lib.check(_lib.lib.mpgnn_confusion_counts(sc.data_ptr(), sc.shape[0], c, n, p_idx, p_lab, p_n, out.data_ptr(),
                                               _stream(sc)), "mpgnn_confusion_counts")
    return out


# (weakref to the row list, its _version, rows) -> (row_ptr, row_perm): the list grouped by row
# (int32 CSR on the list's device), made once per list outside captures
_ROW_CSR: list = []
# MPGNN_NLL_DENSE=0: the zero fill + scatter backward (A/B switch; same values)
_NLL_DENSE = __import__("os").environ.get("MPGNN_NLL_DENSE", "1") != "0"


def _rows_csr(idx: torch.Tensor, rows: int):
    for ri, vi, n, csr in _ROW_CSR:
        if ri() is idx and vi == idx._version and n == rows:
            return csr
    if not _NLL_DENSE or torch.cuda.is_current_stream_capturing() or idx.numel() == 0 or idx.numel() >= 2 ** 31 or \
            rows >= 2 ** 31:
        return None
    perm = torch.argsort(idx, stable=True)
    ptr = torch.searchsorted(idx[perm], torch.arange(rows + 1, device=idx.device))
    csr = (ptr.to(torch.int32).contiguous(), perm.to(torch.int32).contiguous())
    _ROW_CSR.insert(0, (weakref.ref(idx), idx._version, rows, csr))
    del _ROW_CSR[_NLL_OK_MAX:]
    return csr


class _NllRows(torch.autograd.Function):
    """mpgnn_nll_rows_fwd / _bwd: the loss in one launch, its input gradient in one launch that
    writes it whole from the list grouped by row (mpgnn_nll_rows_bwd_dense; without the grouping,
    inside a capture that did not see the list before: a zero fill + one scatter launch) — torch:
    index_select, nll_loss and their backward, 7 launches."""

    @staticmethod
    def forward(ctx, logp, idx, target, weight=None):
        from . import _lib
        from .functional import _stream
        loss = torch.empty((), dtype=torch.float32, device=logp.device)
        tw = torch.empty((), dtype=torch.float32, device=logp.device)
        wp = weight.data_ptr() if weight is not None else None
        _lib.check(_lib.lib.mpgnn_nll_rows_fwd_weighted(logp.data_ptr(), logp.shape[0], logp.shape[1], idx.data_ptr(),
                                                        target.data_ptr(), idx.numel(), -100, wp, loss.data_ptr(),
                                                        tw.data_ptr(), _stream(logp)), "mpgnn_nll_rows_fwd")
        ctx.lists = (idx, target, tw, weight)
        ctx.shape = tuple(logp.shape)
        ctx.csr = _rows_csr(idx, logp.shape[0])
        return loss

    @staticmethod
    def backward(ctx, g):
        from . import _lib
        from .functional import _stream
        idx, target, tw, weight = ctx.lists
        wp = weight.data_ptr() if weight is not None else None
        g = g.contiguous()
        if ctx.csr is not None:
            grad = torch.empty(ctx.shape, dtype=torch.float32, device=g.device)
            ptr, perm = ctx.csr
            _lib.check(_lib.lib.mpgnn_nll_rows_bwd_dense(g.data_ptr(), tw.data_ptr(), ctx.shape[0], ctx.shape[1],
                                                         ptr.data_ptr(), perm.data_ptr(), target.data_ptr(), -100, wp,
                                                         grad.data_ptr(), _stream(grad)), "mpgnn_nll_rows_bwd_dense")
            return grad, None, None, None
        grad = torch.zeros(ctx.shape, dtype=torch.float32, device=g.device)
        _lib.check(_lib.lib.mpgnn_nll_rows_bwd_weighted(g.data_ptr(), tw.data_ptr(), ctx.shape[0], ctx.shape[1],
                                                        idx.data_ptr(), target.data_ptr(), idx.numel(), -100, wp,
                                                        grad.data_ptr(), _stream(grad)), "mpgnn_nll_rows_bwd")
        return grad, None, None, None


# the (row list, target list) pairs last checked in range, by OBJECT (weakrefs) and _version, with
# the matrix size: the loops pass the same train / val / test lists every epoch, so the one host
# read of the check happens once per list (and never inside a HIP-graph capture)
_NLL_OK: list = []
_NLL_OK_MAX = 4


def _nll_lists_valid(idx: torch.Tensor, target: torch.Tensor, rows: int, c: int) -> bool:
    for ri, vi, rt, vt, shape in _NLL_OK:
        if ri() is idx and vi == idx._version and rt() is target and vt == target._version and shape == (rows, c):
            return True
    if torch.cuda.is_current_stream_capturing():
        return False
    ok = bool((((target == -100) | ((target >= 0) & (target < c))).all() &
               ((idx >= 0) & (idx < rows)).all()).item())
    if ok:
        _NLL_OK.insert(0, (weakref.ref(idx), idx._version, weakref.ref(target), target._version, (rows, c)))
        del _NLL_OK[_NLL_OK_MAX:]
    return ok


def nll_loss_rows(logp: torch.Tensor, idx, target: torch.Tensor, weight=None) -> torch.Tensor:
    """``F.nll_loss(logp[idx].squeeze(-1), target, weight=weight)`` — the loops' losses (main.py:1065,
    1088, 1106, main_rgcn.py:402, 422 unweighted; main_rgcn.py:376-380's training step with the
    balanced class weights); mean over the listed rows, ignore_index -100. On the GPU
    (float32 [rows, C >= 2] log-probabilities, 1-D int64 row and target lists on the same device,
    lists checked in range once) ``mpgnn_nll_rows_fwd`` / ``_bwd``: the same loss up to the
    summation order (a few ulp), the same input gradient bit for bit (tests/test_loop.py).
    Anything else — and lists with an out-of-range entry, so torch raises its own error — runs
    torch's ops."""
    fast = (logp.is_cuda and logp.dim() == 2 and logp.dtype == torch.float32 and logp.shape[1] >= 2
            and torch.is_tensor(idx) and idx.dim() == 1 and idx.dtype == torch.int64 and idx.device == logp.device
            and torch.is_tensor(target) and target.dim() == 1 and target.dtype == torch.int64
            and target.device == logp.device and target.numel() == idx.numel()
            and (weight is None or (torch.is_tensor(weight) and weight.dtype == torch.float32
                                    and weight.device == logp.device and tuple(weight.shape) == (logp.shape[1],)))
            and _nll_lists_valid(idx, target, logp.shape[0], logp.shape[1]))
    if fast:
        return _NllRows.apply(logp.contiguous(), idx.contiguous(), target.contiguous(),
                              weight.contiguous() if weight is not None else None)
    rows = logp.index_select(0, idx.to(logp.device)) if torch.is_tensor(idx) and idx.dim() == 1 and idx.dtype in (
        torch.int64, torch.int32) else logp[idx]
    return torch.nn.functional.nll_loss(rows.squeeze(-1), target, weight=weight)


def _num_cols(t: torch.Tensor) -> int:
    return int(t.shape[1]) if t.dim() > 1 else 1


def f1_from_counts(counts) -> list[float]:
    """Macro F1 of each [3, C] count block (a device tensor is copied to the host here)."""
    c = counts.cpu().numpy() if torch.is_tensor(counts) else np.asarray(counts)
    return [_finish(x) for x in c]


def f1_macro(pred: torch.Tensor, y: torch.Tensor, num_classes: int) -> float:
    """``sklearn.metrics.f1_score(pred, y, average='macro')`` (symmetric in its arguments)."""
    return f1_macro_many([(pred, y)], num_classes)[0]


# one entry: (weakref to the label tensor, its _version, the weights). Keyed on the tensor
# OBJECT (a weakref that dies with it), not its address: a new label tensor landing at a
# freed address must not hit a stale entry.
_CW_LAST: list = [None, -1, None]


_CWT_LAST: list = [None, -1, None, None]


def class_weight_tensor(y: torch.Tensor, device) -> torch.Tensor:
    """``torch.tensor(class_weight_balanced(y), dtype=float)`` on ``device`` (main_rgcn.py:376-379),
    cached for the same label tensor (object and version): the per-epoch host-to-device copy of
    the reference (a blocking copy) happens once."""
    ref, ver, dev, t = _CWT_LAST
    if ref is not None and ref() is y and ver == y._version and dev == str(device):
        return t
    t = torch.tensor(class_weight_balanced(y), dtype=torch.float, device=device)
    _CWT_LAST[:] = [weakref.ref(y), y._version, str(device), t]
    return t


def class_weight_balanced(y: torch.Tensor) -> np.ndarray:
    """``class_weight.compute_class_weight('balanced', classes=np.unique(y), y=y)``
    (main_rgcn.py:378): n_samples / (n_classes · bincount) over the classes present.
    The loops recompute it every epoch on an unchanged label tensor; the answer is cached for
    that same tensor object (and version) so the labels cross to the host once."""
    ref, ver, w = _CW_LAST
    if ref is not None and ref() is y and ver == y._version:
        return w.copy()
    yn = y.detach().cpu().numpy().reshape(-1)
    classes, counts = np.unique(yn, return_counts=True)
    w = yn.shape[0] / (classes.shape[0] * counts.astype(np.float64))
    _CW_LAST[:] = [weakref.ref(y), y._version, w]
    return w.copy()
