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
           "class_weight_balanced", "class_weight_tensor"]


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


def confusion_counts_rows(scores: torch.Tensor, lists) -> torch.Tensor:
    """``confusion_counts_many([(torch.argmax(scores[idx], 1), y) for idx, y in lists], C)`` with
    C = scores.shape[1]: [len(lists), 3, C] int64 on the device. On the GPU (float32 scores,
    1-D integer row indices, up to 4 lists) ONE kernel (``mpgnn_confusion_counts``: argmax of
    each listed row + LDS histograms) instead of ~20 torch ops per list; same counts."""
    lists = list(lists)
    ok = (scores.is_cuda and scores.dim() == 2 and scores.dtype == torch.float32 and 0 < len(lists) <= 4
          and 1 <= scores.shape[1] <= 8192
          and all(torch.is_tensor(i) and i.dim() == 1 and i.dtype in (torch.int64, torch.int32) and
                  torch.is_tensor(y) and y.numel() == i.numel() and not y.is_floating_point()
                  for i, y in lists))
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
