"""CPU ORACLE for the score function — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, as the checker / the timed CPU baseline. The product path (``mpgnn_amd.score``)
never imports it and has no CPU fallback.

What it restates (pure Python / PyTorch on the CPU, the reference's own control flow):

* ``create_edge_dictionary``  — main.py:387-424 (non-bag branch): {source: [destinations]} over
  the edges of one relation whose source is in ``source_nodes_mask`` (keys in mask order, values
  in edge-file order) and {destination: [labels of its sources]}.
* ``initialize_weights``      — main.py:479-497: weight[dst] = |min(labels) + U(-0.2, 0.2)|
  drawn from Python's ``random`` in destination-dictionary order. The reference starts from
  ``torch.Tensor(N)`` (uninitialised memory) for the other nodes; they are never selected by
  the argmax (only destinations are), and here they are 0.
* ``Score``                   — model.py:26-125: InputLayer (weights [N, 1] parameter),
  OutputLayer with ``LinearLayerAttri = Linear(F, 1, bias=False)``, forward (non-bag branch,
  model.py:74-89): for every source (dictionary order) the FIRST argmax of the destination
  weights (``torch.argmax``: NaN is the maximum), ``max_weights[source] = weights[max_node]``.
* ``train``                   — main.py:641-673 (non-bag): MSE(mean) of the predictions chosen per
  dataset (:653-656), backward, Adam(lr 0.1) step (main.py:521-522), clamp of both parameters
  to [0, 1] (:667-669).
* ``score_relation_parallel`` — main.py:727-760: 100 epochs; returns (relation, loss, dicts).

Pinning: tests/golden/score_synthetic.npz was produced by running the reference's OWN
functions (main.py's create_edge_dictionary / initialize_weights / train / score_relation_parallel
and model.py's Score, through the PyG stand-in of tests/golden/make_golden.py) on the reference's
planted synthetic graph; tests/test_score.py checks this restatement against it.
"""
from __future__ import annotations

import random

import torch
import torch.nn as nn

__all__ = ["masked_edge_index", "create_edge_dictionary", "initialize_weights", "Score", "score_forward",
           "train", "score_relation_parallel", "EPOCHS", "FIRST_MASK_DATASETS"]

EPOCHS = 100  # main.py:755
FIRST_MASK_DATASETS = ("IMDB", "ACM", "DBLP", "fb15k-237")  # main.py:653: labels are per mask position


def masked_edge_index(edge_index, edge_mask):
    """main.py:39-45 (dense branch)."""
    return edge_index[:, edge_mask]


def create_edge_dictionary(edge_index, edge_type, relation, source_nodes_mask, labels, dataset):
    """main.py:387-424, BAGS=False. ``labels`` = data.labels ([N, 1] for 'synthetic', per mask
    position otherwise). Returns (edge_dictionary, destination_dictionary)."""
    ei = masked_edge_index(edge_index, edge_type == relation)
    src_list, dst_list = ei[0].tolist(), ei[1].tolist()
    src_set = set(src_list)
    mask_set = set(source_nodes_mask)
    edge_dictionary = {}
    for index in source_nodes_mask:                        # :396-397 (keys in mask order)
        if index in src_set:
            edge_dictionary[index] = []
    for s, d in zip(src_list, dst_list):                   # :399-401
        if s in mask_set:
            edge_dictionary[s].append(d)
    edge_dictionary = {k: v for k, v in edge_dictionary.items() if v}  # :403-406
    first = {}
    for i, s in enumerate(source_nodes_mask):
        first.setdefault(s, i)                             # list.index = first occurrence
    destination_dictionary = {}
    for s, d in zip(src_list, dst_list):                   # :416-417
        if s in mask_set and d not in destination_dictionary:
            destination_dictionary[d] = []
    for s, d in zip(src_list, dst_list):                   # :418-423
        if s in mask_set:
            lab = labels[s] if dataset == "synthetic" else labels[first[s]]
            destination_dictionary[d].append(lab.item() if torch.is_tensor(lab) else lab)
    return edge_dictionary, destination_dictionary


def initialize_weights(num_nodes, destination_dictionary, rng: random.Random | None = None):
    """main.py:479-497 (start -0.2, end 0.2), Python ``random`` in dictionary order."""
    rng = rng or random
    weights = torch.zeros(num_nodes)
    for key, values in destination_dictionary.items():
        weights[key] = abs(min(values) + rng.uniform(-0.2, 0.2))
    return weights


class Score(nn.Module):
    """model.py:91-125 with InputLayer (:26-34) and OutputLayer (:36-89): parameters
    ``input.weights`` [N, 1] and ``output.LinearLayerAttri.weight`` [1, F] (created in that
    order, the Linear consuming torch's RNG as the reference's does)."""

    def __init__(self, weights, COMPLEX, features_dim):
        super().__init__()
        self.COMPLEX = COMPLEX
        self.features_dim = features_dim
        self.input = nn.Module()
        self.input.weights = nn.Parameter(weights.unsqueeze(-1))
        self.output = nn.Module()
        self.output.LinearLayerAttri = nn.Linear(features_dim, 1, bias=False)

    def forward(self, num_nodes, node_dict):
        return score_forward(self.input.weights, num_nodes, node_dict)


def score_forward(weights, num_nodes, node_dict):
    """model.py:74-89: (max_weights [N, 1], {source: max_node})."""
    max_weights = torch.zeros(num_nodes, 1)
    best = {}
    for source_node in list(node_dict.keys()):
        weights_of_source = weights[node_dict[source_node]].squeeze(-1)
        max_node = node_dict[source_node][torch.argmax(weights_of_source).item()]
        best[source_node] = max_node
        max_weights[source_node] = weights[max_node]
    return max_weights, best


def train(model, optimizer, edge_dictionary, num_nodes, labels, source_nodes_mask, dataset):
    """main.py:641-673, BAGS=False, no frozen weights: one epoch. Returns (loss, {source:
    max_node}, loss_per_node, predictions)."""
    model.train()
    optimizer.zero_grad()
    predictions, best = model(num_nodes, edge_dictionary)
    if dataset in FIRST_MASK_DATASETS:
        predictions, labels = predictions[source_nodes_mask].to(torch.float32), labels.to(torch.float32)
    elif dataset == "synthetic":
        predictions, labels = (predictions[source_nodes_mask].to(torch.float32),
                               labels[source_nodes_mask].to(torch.float32))
    loss = nn.MSELoss(reduction="mean")(predictions, labels)
    loss_per_node = nn.MSELoss(reduction="none")(predictions, labels)
    loss.backward()
    optimizer.step()
    with torch.no_grad():
        model.input.weights[:] = torch.clamp(model.input.weights, min=0.0, max=1.0)
        model.output.LinearLayerAttri.weight[:] = torch.clamp(model.output.LinearLayerAttri.weight, min=0.0, max=1.0)
    return loss, best, loss_per_node, predictions


def score_relation_parallel(edge_index, edge_type, x, labels, relation, source_nodes, dataset,
                            rng: random.Random | None = None, epochs: int = EPOCHS, trace=None):
    """main.py:727-760. ``trace`` (list) receives (loss, {source: max_node}) of every epoch."""
    num_nodes = x.size(0)
    if not source_nodes:
        source_nodes = torch.unique(masked_edge_index(edge_index, edge_type == relation)[0]).tolist()
    ed, dd = create_edge_dictionary(edge_index, edge_type, relation, source_nodes, labels, dataset)
    weights = initialize_weights(num_nodes, dd, rng)
    model = Score(weights, dataset, x.size(1))
    optimizer = torch.optim.Adam(model.parameters(), lr=0.1)
    loss = None
    for _ in range(epochs):
        loss, best, _, _ = train(model, optimizer, ed, num_nodes, labels, source_nodes, dataset)
        if trace is not None:
            trace.append((float(loss.item()), dict(best)))
    return relation, loss.item(), ed, dd, model


# ---------------------------------------------------------------------------------------------
# bag branch (model.py:45-72; main.py:426-438, 543-596, 498-512, 530-543, 641-673, 853-917)
# ---------------------------------------------------------------------------------------------
def create_edge_dictionary_bags(edge_index, edge_type, relation, source_nodes_mask, bags, bag_labels):
    """main.py:387-406 + 426-438 (BAGS=True): the same {source: [destinations]} dictionary, and
    {destination: [labels of every bag holding one of its sources]} — per edge of the relation
    (file order) whose source lies in some bag, the labels of that source's bags (bag order)
    extended onto the destination's list."""
    ei = masked_edge_index(edge_index, edge_type == relation)
    src_list, dst_list = ei[0].tolist(), ei[1].tolist()
    src_set = set(src_list)
    mask_set = set(source_nodes_mask)
    edge_dictionary = {}
    for index in source_nodes_mask:                        # :396-397
        if index in src_set:
            edge_dictionary[index] = []
    for s, d in zip(src_list, dst_list):                   # :399-401
        if s in mask_set:
            edge_dictionary[s].append(d)
    edge_dictionary = {k: v for k, v in edge_dictionary.items() if v}
    tmp = {}                                               # :428-432
    for i, bag in enumerate(bags):
        for node in bag:
            tmp.setdefault(node, []).append(float(bag_labels[i].item()))
    dest = {}                                              # :434-437
    for s, d in zip(src_list, dst_list):
        if s in tmp:
            dest.setdefault(d, []).extend(tmp[s])
    return edge_dictionary, dest


def create_bags(edge_dictionary, destination_dictionary):
    """main.py:545-575: per source, its destinations whose labels are all > 0.9 form one bag
    (label 1); every other destination is a singleton bag (label 0); duplicates removed
    (first kept). Returns (bags, bag_labels [B, 1])."""
    bag, labels = [], []
    for key in edge_dictionary.keys():
        lst = []
        for value in edge_dictionary[key]:
            if min(destination_dictionary[value]) > 0.9:
                lst.append(value)
            elif [value] not in bag:
                bag.append([value])
                labels.append(0)
        if lst:
            bag.append(lst)
            labels.append(1)
    new_bag, new_labels = [], []
    for b, lab in zip(bag, labels):
        if b not in new_bag:
            new_bag.append(b)
            new_labels.append(lab)
    return new_bag, torch.Tensor(new_labels).unsqueeze(-1)


def clean_bags_for_relation_type(bags, bag_labels, edge_dictionary):
    """main.py:577-592: each bag reduced to its nodes that are keys of the edge dictionary;
    emptied bags dropped with their labels."""
    keep, keep_labels = [], []
    for c, b in enumerate(bags):
        tmp = [n for n in b if n in edge_dictionary]
        if tmp:
            keep.append(tmp)
            keep_labels.append(bag_labels[c])
    return keep, torch.Tensor(keep_labels).unsqueeze(-1)


def reinitialize_weights(num_nodes, destination_dictionary, previous_weights, frozen, rng=None):
    """main.py:498-512: frozen destinations keep ``previous_weights``; every other destination
    key gets U(0, 1) from Python's ``random`` in dictionary order; other nodes 0 (uninitialised
    in the reference, never read)."""
    rng = rng or random
    weights = torch.zeros(num_nodes)
    for key in destination_dictionary.keys():
        if key in frozen:
            weights[key] = previous_weights[key]
        else:
            weights[key] = rng.uniform(0., 1.)
    return weights


def retrieve_destinations_low_loss(max_destination_node_dict, loss_per_node):
    """main.py:530-543: destinations of the entries (dict order, i-th entry ↔ loss_per_node[i])
    with loss < 1e-4, first occurrence order."""
    out = []
    for index, (_key, value) in enumerate(max_destination_node_dict.items()):
        if loss_per_node[index] < 0.0001 and value not in out:
            out.append(value)
    return out


def score_forward_bags(weights, lin, bags, node_dict, feat):
    """model.py:45-72 restated with the same tensor operations (so autograd unwinds it as the
    reference's): per bag, per source in the dictionary, ``s = lin(feat[source])``, the first
    argmax of ``weights[dsts] * s``, ``v = weights[max_node] * s``; the bag keeps the first
    source whose v is strictly larger than the running maximum (-10 at the start).
    Returns (max_weights [B, 1], {str(bag): max_node}, {source: v})."""
    max_weights = torch.zeros(len(bags), 1)
    by_bag, by_source = {}, {}
    for i, bag in enumerate(bags):
        cur = -10
        for source_node in bag:
            if source_node in node_dict:
                w_src = weights[node_dict[source_node]].squeeze(-1)
                w_src *= lin(feat[source_node])
                max_node = node_dict[source_node][torch.argmax(w_src).item()]
                by_source[source_node] = weights[max_node] * lin(feat[source_node])
                if by_source[source_node] > cur:
                    cur = by_source[source_node]
                    by_bag[str(bag)] = max_node
                    max_weights[i] = by_source[source_node]
    max_weights.requires_grad_(True)
    return max_weights, by_bag, by_source


def train_bags(model, optimizer, edge_dictionary, bags, bag_labels, feat, frozen, previous_weights, grad_mask):
    """main.py:641-673 with BAGS=True: MSE(mean) of the bag maxima against the bag labels,
    backward, gradient mask when weights are frozen, Adam step, clamps, frozen restore.
    Returns (loss, {source: v}, loss_per_bag, {str(bag): max_node}, predictions)."""
    model.train()
    optimizer.zero_grad()
    pred, by_bag, by_source = score_forward_bags(model.input.weights, model.output.LinearLayerAttri, bags,
                                                 edge_dictionary, feat)
    loss = nn.MSELoss(reduction="mean")(pred, bag_labels)
    loss_per_bag = nn.MSELoss(reduction="none")(pred, bag_labels)
    loss.backward()
    if frozen:
        model.input.weights.grad = model.input.weights.grad * grad_mask
    optimizer.step()
    with torch.no_grad():
        model.input.weights[:] = torch.clamp(model.input.weights, min=0.0, max=1.0)
        model.output.LinearLayerAttri.weight[:] = torch.clamp(model.output.LinearLayerAttri.weight, min=0.0, max=1.0)
        if frozen:
            for idx in range(0, len(model.input.weights[:])):
                if idx in frozen:
                    model.input.weights[:][idx] = previous_weights[idx]
    return loss, by_source, loss_per_bag, by_bag, pred


def score_relation_bags_parallel(edge_index, edge_type, x, bags, bag_labels, relation, features_dim,
                                 rng: random.Random | None = None, epochs: int = 50, trace=None, stop_after=None):
    """main.py:853-917: restarts of 50 epochs until two restarts in a row fail to lower the
    loss; after an improving restart the destinations of the bags with loss < 1e-4 are frozen
    (gradient mask 0) for the next restarts; weights re-drawn per restart. ``trace`` receives
    per epoch (loss, [max node per bag]) and per restart ('restart', loss, frozen list).
    Returns (relation, current_loss, model, predictions_for_each_restart, v); ``stop_after`` ends
    the run after that many train() calls (a prefix of the trajectory, for quick checks) and
    returns None."""
    rng = rng or random
    train_bags._calls = 0
    num_nodes = x.size(0)
    mask = []
    for bag in bags:
        for elm in bag:
            if elm not in mask:
                mask.append(elm)
    ed, dd = create_edge_dictionary_bags(edge_index, edge_type, relation, mask, bags, bag_labels)
    cbags, clabels = clean_bags_for_relation_type(bags, bag_labels, ed)
    weights = initialize_weights(num_nodes, dd, rng)
    grad_mask = torch.ones(len(weights), 1)
    feat = x.type(torch.FloatTensor)
    preds, frozen = {}, []
    v = len(cbags) == 1 or (len(cbags) > 1 and clabels.squeeze().tolist().count(1) == 0)
    rest, current_loss, model = 0, 100, None
    while rest < 2:
        model = Score(weights, "synthetic", features_dim)
        optimizer = torch.optim.Adam(model.parameters(), lr=0.1)
        for _ in range(epochs):
            loss, by_source, loss_per_bag, by_bag, _ = train_bags(model, optimizer, ed, cbags, clabels, feat, frozen,
                                                                  weights, grad_mask)
            if trace is not None:
                trace.append((float(loss.item()), [by_bag.get(str(b)) for b in cbags]))
            calls = getattr(train_bags, "_calls", 0) + 1
            train_bags._calls = calls
            if stop_after is not None and calls >= stop_after:
                train_bags._calls = 0
                return None
        for key, value in by_source.items():
            preds.setdefault(key, []).append(value.item())
        if loss.item() < current_loss:
            frozen = retrieve_destinations_low_loss(by_bag, loss_per_bag)
            current_loss = loss.item()
            rest = 0
        else:
            rest += 1
        for node in frozen:
            grad_mask[node] = 0
        if trace is not None:
            trace.append(("restart", float(loss.item()), list(frozen)))
        weights = reinitialize_weights(num_nodes, dd, model.input.weights.detach()[:, 0], frozen, rng)
    return relation, current_loss, model, preds, v
