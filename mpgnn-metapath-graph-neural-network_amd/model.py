"""Drop-in for the reference ``model.py`` MPGNN wrappers (model.py:132-149, 179-228).

The wrappers stay plain PyTorch (ReLU, Dropout, Linear, LogSoftmax) exactly as in the
reference; only the relational layers are the gfx950 ones. Module/parameter names, their
order and a seeded initialisation are identical to the reference, so ``state_dict``s load
either way. ``MPNet`` (model.py:153-176) is not provided: it calls its convs with 4 arguments
where CustomRGCNConv.forward needs 5 (mp_rgcn_layer.py:158) and cannot run in the reference.
The score-function classes (model.py:12-125) are outside the hot path.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .mp_rgcn_layer import CustomRGCNConv
from .nn import RGCNConv

__all__ = ["Net", "MPNetm"]


class Net(torch.nn.Module):
    """RGCN baseline (model.py:132-149): conv1, then the SAME conv2 for layers 1..L-1."""

    def __init__(self, input_dim, hidden_dim, num_rel, output_dim, ll_output_dim, metapath_length):
        super().__init__()
        self.metapath_length = metapath_length
        self.conv1 = RGCNConv(input_dim, hidden_dim, num_rel, flow="target_to_source")
        self.conv2 = RGCNConv(hidden_dim, output_dim, num_rel, flow="target_to_source")
        self.LinearLayer = torch.nn.Linear(output_dim, ll_output_dim)

    def forward(self, x, edge_index, edge_type, *, shard=None, group=None):
        for layer_index in range(0, self.metapath_length):
            conv = self.conv1 if layer_index == 0 else self.conv2
            # F.relu(conv(...)) of model.py:144,146, fused into the layer's combine kernel
            x = conv(x, edge_index, edge_type, shard=shard, group=group, activation="relu")
        x = self.LinearLayer(x)
        return F.log_softmax(x, dim=1)


class MPNetm(torch.nn.Module):
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
        embeddings = []
        for i in range(0, len(self.metapaths)):
            for layer_index in range(0, len(self.metapaths[i])):
                conv = self.layers_list[i][layer_index]
                rel = self.metapaths[i][layer_index]
                if layer_index == 0:
                    h = F.relu(conv(layer_index, rel, x, edge_index, edge_type))
                    h = self.dropout(h)
                else:
                    h = F.relu(conv(layer_index, rel, h, edge_index, edge_type))
                    h = self.dropout2(h)
            embeddings.append(h)
        concatenated_embedding = torch.cat(embeddings, dim=1)
        h = F.relu(self.fc1(concatenated_embedding))
        h = self.fc2(h)
        return self.log_softmax(h)
