"""Drop-in for the RGCN-baseline training loop of the reference ``main_rgcn.py`` (SURVEY §8a
A11): ``mpgnn_train`` (class-balanced NLL) / ``mpgnn_validation`` / ``mpgnn_test`` /
``mpgnn_parallel_multiple`` (main_rgcn.py:369-472) driving ``Net`` (model.py:132-149) whose
RGCNConv layers run on the gfx950 kernels. The loaders are shared with ``main``
(main_rgcn.py:357-363 ≡ main.py:366-372) except ``get_node_features``, which flips the
one-hot columns here (main_rgcn.py:351) and not in main.py (main.py:353 is commented out).

Same names, arguments, return values and printed lines as the reference; model and data stay
on the GPU and the macro-F1 scores are finished from device-side counts (``metrics``).
``shard``/``group`` (keyword-only, default off) run the dst-range sharded layers (§8e).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from .main import (_adam, _adam_graphable, _epochs, _graphs_enabled, _one_hot_colours, Data,  # noqa: F401
                   get_edge_index_and_type_no_reverse, load_files, load_graph, take_rows)
from .metrics import class_weight_balanced, class_weight_tensor, confusion_counts_rows, f1_from_counts, nll_loss_rows
from .model import Net

__all__ = ["Data", "get_node_features", "mpgnn_train", "mpgnn_validation", "mpgnn_test", "mpgnn_parallel_multiple", "EPOCHS"]

EPOCHS = 999  # ``for epoch in range(1, 1000)`` (main_rgcn.py:457)


def get_node_features(colors):
    """main_rgcn.py:345-353: one-hot columns of the colour frame, float32, columns reversed
    (``np.flip(x, 1)``, main_rgcn.py:351)."""
    return torch.from_numpy(np.flip(_one_hot_colours(colors), 1).copy())


def _forward(model, data):
    kw = getattr(data, "shard_kw", None) or {}
    return model(data.x, data.edge_index, data.edge_type, **kw)


def _train_step(model, optimizer, data):
    """The body of mpgnn_train with the loss left on the device (no host sync)."""
    model.train()
    optimizer.zero_grad()
    out = _forward(model, data)
    weights = class_weight_balanced(data.train_y)
    weights_tensor = class_weight_tensor(data.train_y, out.device)
    # F.nll_loss(out[train_idx], train_y, weight=weights_tensor): one launch each way on the GPU
    loss = nll_loss_rows(out, data.train_idx, data.train_y, weight=weights_tensor)
    loss.backward()
    optimizer.step()
    return loss.detach(), weights


def mpgnn_train(model, optimizer, data):
    """main_rgcn.py:369-393: forward, NLL on train_idx weighted by the balanced class weights
    (main_rgcn.py:376-380), backward, step → (float loss, weights)."""
    loss, weights = _train_step(model, optimizer, data)
    return float(loss), weights


@torch.no_grad()
def _val_counts(model, data):
    """mpgnn_validation's work, kept on the device: (val loss, [2, 3, C] confusion counts of the
    train and validation predictions)."""
    model.eval()
    pred = _forward(model, data)
    loss_val = nll_loss_rows(pred, data.val_idx, data.val_y)
    counts = confusion_counts_rows(pred, [(data.train_idx, data.train_y), (data.val_idx, data.val_y)])
    return loss_val, counts


@torch.no_grad()
def _test_counts(model, data):
    model.eval()
    pred = _forward(model, data)
    loss_test = nll_loss_rows(pred, data.test_idx, data.test_y)
    counts = confusion_counts_rows(pred, [(data.test_idx, data.test_y)])
    return loss_test, counts


@torch.no_grad()
def mpgnn_validation(model, data, class_weight):
    """main_rgcn.py:395-416 → (f1 train, f1 val, f1 val, val loss tensor)."""
    model.eval()
    pred = _forward(model, data)
    loss_val = nll_loss_rows(pred, data.val_idx, data.val_y)
    f1_train, f1_val = f1_from_counts(confusion_counts_rows(pred, [(data.train_idx, data.train_y),
                                                                     (data.val_idx, data.val_y)]))
    return f1_train, f1_val, f1_val, loss_val


@torch.no_grad()
def mpgnn_test(model, data, class_weight):
    """main_rgcn.py:418-432 → (test loss tensor, test macro F1)."""
    model.eval()
    pred = _forward(model, data)
    loss_test = nll_loss_rows(pred, data.test_idx, data.test_y)
    (f1_test,) = f1_from_counts(confusion_counts_rows(pred, [(data.test_idx, data.test_y)]))
    return loss_test, f1_test


def mpgnn_parallel_multiple(data_mpgnn, input_dim, hidden_dim, num_rel, output_dim, ll_output_dim, metapath_length,
                            epochs: int = EPOCHS, verbose: bool = True):
    """main_rgcn.py:452-472: train ``Net`` (L = metapath_length) for 999 epochs with Adam
    (lr 0.01, wd 5e-4), running train / validation / test every epoch and printing every
    10th; returns the test macro F1 of ``best_model`` (the same object as the trained model,
    as in the reference)."""
    model = Net(input_dim, hidden_dim, num_rel, output_dim, ll_output_dim, metapath_length)
    model = model.to(data_mpgnn.x.device)
    use_graph = _graphs_enabled(data_mpgnn)
    optimizer = _adam_graphable(model) if use_graph else _adam(model)
    best_model = model
    class_weight = class_weight_balanced(data_mpgnn.train_y)
    # Every epoch runs what the reference runs (train, validation forward + scores, test forward
    # + score) but leaves the scalars on the device: the host reads them only where the loop
    # prints (every 10th epoch). best_model is the trained model object itself in the
    # reference (main_rgcn.py:465-466 keeps a reference, not a copy), so its per-epoch
    # best-score test changes nothing and needs no host read.
    # (one HIP graph per epoch after three eager ones: main._epochs)
    def epoch_fn():
        loss, _ = _train_step(model, optimizer, data_mpgnn)
        return (loss,) + _val_counts(model, data_mpgnn) + _test_counts(model, data_mpgnn)

    for epoch, (loss, loss_val, vcounts, test_loss, tcounts) in _epochs(epoch_fn, epochs, use_graph):
        if verbose and epoch % 10 == 0:
            train_acc, f1_val_micro = f1_from_counts(vcounts)
            (f1_micro_test,) = f1_from_counts(tcounts)
            print(epoch, "train loss %0.3f" % float(loss), "validation loss %0.3f" % loss_val,
                  "train micro: %0.3f" % train_acc, "validation micro: %0.3f" % f1_val_micro,
                  "test micro: %0.3f" % f1_micro_test)
    test_loss, f1_micro_test = mpgnn_test(best_model, data_mpgnn, class_weight)
    if verbose:
        print("test loss %0.3f" % test_loss, "test micro %0.3f" % f1_micro_test)
    return f1_micro_test
