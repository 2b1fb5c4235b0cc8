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
