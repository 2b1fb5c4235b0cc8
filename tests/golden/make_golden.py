#!/usr/bin/env python3
"""Generate the golden vectors under tests/golden/ from the REFERENCE's own code.

Runs only where /root/reference exists (the survey container); the outputs are committed as
data (.npz) and travel to the GPU box — the reference never does.

The reference layer (mp_rgcn_layer.py) and model (model.py) import torch_geometric /
torch_scatter / torch_sparse (requirements.txt:7), which are not installed and cannot be
(no network). A minimal stand-in package tree is written to a temporary directory with:
  * torch_geometric.nn.conv.MessagePassing — PyG 2.3.1 propagate semantics for the one code
    path the reference uses (flow handling, x_j = x.index_select(node_dim, edge_index[j]),
    identity message, aggr='mean' via scatter_add_ / count.clamp(min=1), dim_size = size[i])
  * torch_geometric.nn.inits.glorot / zeros (PyG 2.3.1 formulas)
  * torch_geometric.typing / data / nn.RGCNConv names (RGCNConv raises if instantiated)
  * torch_scatter.scatter / torch_sparse names (only imported, never called on this path)
Everything else — the masking (:29-35,:231), h @ W (:245), squeeze (:246), root (:265),
bias (:268), parameter shapes and glorot init order (:120-155), MPNetm wiring (model.py:179-228)
— is the reference's code, executed as is. The PyG arithmetic itself (third-party) is therefore
restated here, not pinned; it is pinned structurally by the embedding.dat / label.dat KAT.

Outputs (all small):
  kat_synthetic.npz       the two planted synthetic graphs (link/node/label/embedding .dat)
  layer_single.npz        CustomRGCNConv (mode SINGLE) forward + autograd grads, C1 graph
  layer_all.npz           RGCNConv loop (mode ALL) assembled from reference CustomRGCNConv
                          per-relation transforms, forward + grads, C1 graph
  mpnetm_synthetic.npz    MPNetm(2,64,4,64,2,1,[[1,0]]) seed-30 state_dict + eval logits
  score_synthetic.npz     score function, non-bag branch (score_relation_parallel)
  score_bags_synthetic.npz score function, bag branch (score_relation_bags_parallel)

``--only NAME`` runs one generator (e.g. ``--only make_score_bags_golden``).
"""
from __future__ import annotations

import importlib
import os
import sys
import tempfile
import textwrap

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))

STANDIN = {
    "torch_geometric/__init__.py": "from . import nn, data, typing\n",
    "torch_geometric/typing.py": textwrap.dedent("""
        from typing import Optional
        from torch import Tensor
        Adj = Tensor
        OptTensor = Optional[Tensor]
    """),
    "torch_geometric/data/__init__.py": textwrap.dedent("""
        class Data:
            def __init__(self, **kw):
                for k, v in kw.items():
                    setattr(self, k, v)
            def clone(self):
                import copy
                return copy.copy(self)
    """),
    "torch_geometric/nn/__init__.py": textwrap.dedent("""
        from .conv import MessagePassing
        from . import inits
        class RGCNConv:
            def __init__(self, *a, **k):
                raise NotImplementedError('stand-in: PyG RGCNConv is not available')
        __all__ = ['MessagePassing', 'RGCNConv', 'inits']
    """),
    "torch_geometric/nn/inits.py": textwrap.dedent("""
        import math
        import torch
        def glorot(value):
            if isinstance(value, torch.Tensor):
                stdv = math.sqrt(6.0 / (value.size(-2) + value.size(-1)))
                value.data.uniform_(-stdv, stdv)
        def zeros(value):
            if isinstance(value, torch.Tensor):
                value.data.fill_(0.0)
    """),
    "torch_geometric/nn/conv/__init__.py": textwrap.dedent("""
        import torch
        class MessagePassing(torch.nn.Module):
            # PyG 2.3.1 semantics for propagate(edge_index, x=..., size=...) with aggr='mean'
            def __init__(self, aggr='add', flow='source_to_target', node_dim=-2, **kw):
                super().__init__()
                self.aggr = aggr
                self.flow = flow
                self.node_dim = node_dim
            def propagate(self, edge_index, size=None, **kwargs):
                i, j = (1, 0) if self.flow == 'source_to_target' else (0, 1)
                x = kwargs['x']
                x_j = x.index_select(self.node_dim, edge_index[j])
                msg = self.message(x_j)
                index = edge_index[i]
                dim_size = size[i] if size is not None and size[i] is not None else x.size(self.node_dim)
                assert self.aggr == 'mean' and self.node_dim == 0
                count = msg.new_zeros(dim_size)
                count.scatter_add_(0, index, msg.new_ones(msg.size(0)))
                count = count.clamp(min=1)
                out = msg.new_zeros((dim_size,) + tuple(msg.shape[1:]))
                out.scatter_add_(0, index.view(-1, 1).expand_as(msg), msg)
                return out / count.view(-1, 1)
    """),
    "torch_scatter/__init__.py": textwrap.dedent("""
        def scatter(*a, **k):
            raise NotImplementedError('stand-in torch_scatter')
    """),
    "torch_sparse/__init__.py": textwrap.dedent("""
        class SparseTensor:
            pass
        def masked_select_nnz(*a, **k):
            raise NotImplementedError('stand-in torch_sparse')
        def matmul(*a, **k):
            raise NotImplementedError('stand-in torch_sparse')
    """),
}


def import_reference():
    tmp = tempfile.mkdtemp(prefix="pyg_standin_")
    for rel, src in STANDIN.items():
        path = os.path.join(tmp, rel)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            f.write(src)
    sys.path.insert(0, tmp)
    sys.path.insert(0, REF)
    sys.dont_write_bytecode = True
    layer = importlib.import_module("mp_rgcn_layer")
    model = importlib.import_module("model")
    return layer, model


def synthetic_c1(seed=0, N=1000, R=3, dmax=10):
    """C1 graph, mirrors create_graph…:233,245,249 with a seeded PCG64."""
    rng = np.random.Generator(np.random.PCG64(seed))
    deg = rng.integers(1, dmax + 1, size=N)
    n1 = np.repeat(np.arange(N), deg)
    n2 = rng.integers(0, N - 1, size=n1.size)
    n2 = np.where(n2 >= n1, n2 + 1, n2) % N
    rel = rng.integers(0, R, size=n1.size)
    return np.stack([n1, n2]).astype(np.int64), rel.astype(np.int64)


def read_dat(path):
    return np.array([[int(v) for v in line.split()] for line in open(path) if line.strip()], dtype=np.int64)


def make_kat():
    out = {}
    for tag, d in (("L3", "data/synthetic/metapath_length_3/overlap_0rels_0"),
                   ("L4", "data/synthetic/metapath_length_4/overlap_0_rels_0")):
        base = os.path.join(REF, d)
        link = read_dat(os.path.join(base, "link.dat"))          # node_1 rel node_2
        node = read_dat(os.path.join(base, "node.dat"))          # id red blue (one-hot)
        label = read_dat(os.path.join(base, "label.dat"))        # id label
        emb = read_dat(os.path.join(base, "embedding.dat"))      # id e1 e2 (per-hop truth)
        meta = open(os.path.join(base, "metapath.dat")).read().split("\n")
        out[f"{tag}_link"] = link
        out[f"{tag}_node"] = node
        out[f"{tag}_label"] = label
        out[f"{tag}_embedding"] = emb
        out[f"{tag}_metapath_rel"] = np.array([int(v) for v in meta[1].split()], dtype=np.int64)
        out[f"{tag}_metapath_col"] = np.array([int(v) for v in meta[2].split()], dtype=np.int64)
    np.savez_compressed(os.path.join(HERE, "kat_synthetic.npz"), **out)


def grads_of(fn, tensors, gout):
    for t in tensors:
        t.grad = None
    out = fn()
    out.backward(gout)
    return out.detach(), [t.grad.detach().clone() for t in tensors]


def make_layer_goldens(layer):
    ei, et = synthetic_c1()
    edge_index = torch.from_numpy(ei)
    edge_type = torch.from_numpy(et)
    N, R = 1000, 3
    single, allmode = {"edge_index": ei, "edge_type": et}, {"edge_index": ei, "edge_type": et}
    for F_in in (2, 128):
        F_out = 64
        g = torch.Generator().manual_seed(1234 + F_in)
        if F_in == 2:
            x = torch.nn.functional.one_hot(torch.randint(0, 2, (N,), generator=g), 2).float()
        else:
            x = torch.rand(N, F_in, generator=g)
        x.requires_grad_(True)
        gout = torch.randn(N, F_out, generator=g)
        # --- mode SINGLE: reference CustomRGCNConv, one layer per relation -------------
        torch.manual_seed(30)
        conv = layer.CustomRGCNConv(F_in, F_out, 1, flow="target_to_source")
        single[f"F{F_in}_x"] = x.detach().numpy()
        single[f"F{F_in}_gout"] = gout.numpy()
        single[f"F{F_in}_weight"] = conv.weight.detach().numpy().copy()
        single[f"F{F_in}_root"] = conv.root.detach().numpy().copy()
        single[f"F{F_in}_bias"] = conv.bias.detach().numpy().copy()
        for rel in range(R + 1):  # R = relation absent from the graph (empty mask)
            params = [x, conv.weight, conv.root, conv.bias]
            out, grads = grads_of(lambda: conv(0, rel, x, edge_index, edge_type), params, gout)
            single[f"F{F_in}_r{rel}_out"] = out.numpy()
            for name, gr in zip(("dx", "dweight", "droot", "dbias"), grads):
                single[f"F{F_in}_r{rel}_{name}"] = gr.numpy()
            # the mean itself (bit-exact target): h = propagate(masked)
            mask = edge_type == rel
            tmp = layer.masked_edge_index(edge_index, mask)
            single[f"F{F_in}_r{rel}_masked"] = tmp.numpy()
            single[f"F{F_in}_r{rel}_h"] = conv.propagate(tmp, x=x.detach(), size=(N, N)).numpy()
        # --- mode ALL: Σ_r (reference transform of relation r) + x@root + bias ----------
        torch.manual_seed(31)
        W = torch.empty(R, F_in, F_out)
        layer.glorot(W)
        root = torch.empty(F_in, F_out)
        layer.glorot(root)
        bias = (torch.rand(F_out) - 0.5) * 0.1
        W.requires_grad_(True), root.requires_grad_(True), bias.requires_grad_(True)
        c = layer.CustomRGCNConv(F_in, F_out, 1, root_weight=False, bias=False, flow="target_to_source")

        def forward_all():
            # RGCNConv loop ≙ mp_rgcn_layer.py:249-258: out = out + h_r @ W[r]; then root, bias.
            # Each h_r @ W_r is the reference CustomRGCNConv forward (:231-246) with its
            # weight bound to W[r] (functional_call keeps the autograd path to W).
            out = torch.zeros(N, F_out)
            for rel in range(R):
                out = out + torch.func.functional_call(c, {"weight": W[rel]},
                                                       (0, rel, x, edge_index, edge_type))
            out = out + x @ root
            out = out + bias
            return out

        out, grads = grads_of(forward_all, [x, W, root, bias], gout)
        allmode[f"F{F_in}_x"] = x.detach().numpy()
        allmode[f"F{F_in}_gout"] = gout.numpy()
        allmode[f"F{F_in}_weight"] = W.detach().numpy()
        allmode[f"F{F_in}_root"] = root.detach().numpy()
        allmode[f"F{F_in}_bias"] = bias.detach().numpy()
        allmode[f"F{F_in}_out"] = out.numpy()
        for name, gr in zip(("dx", "dweight", "droot", "dbias"), grads):
            allmode[f"F{F_in}_{name}"] = gr.numpy()
    np.savez_compressed(os.path.join(HERE, "layer_single.npz"), **single)
    np.savez_compressed(os.path.join(HERE, "layer_all.npz"), **allmode)


def make_mpnetm_golden(model):
    kat = np.load(os.path.join(HERE, "kat_synthetic.npz"))
    link = kat["L3_link"]
    node = kat["L3_node"]
    edge_index = torch.tensor(np.stack([link[:, 0], link[:, 2]]))
    edge_type = torch.tensor(link[:, 1])
    x = torch.from_numpy(node[:, 1:].astype(np.float32))   # get_node_features, main.py:347-355
    torch.manual_seed(30)                                   # main.py:31
    net = model.MPNetm(2, 64, 4, 64, 2, 1, [[1, 0]])        # model.py:179
    net.eval()
    with torch.no_grad():
        logits = net(x, edge_index, edge_type)
    out = {"logits": logits.numpy(), "x": x.numpy(), "metapath": np.array([1, 0])}
    for k, v in net.state_dict().items():
        out["sd." + k] = v.numpy()
    np.savez_compressed(os.path.join(HERE, "mpnetm_synthetic.npz"), **out)


SCORE_FUNCS = ("masked_edge_index", "create_edge_dictionary", "initialize_weights", "get_model", "get_optimizer",
               "get_loss", "get_loss_per_node", "train", "score_relation_parallel", "create_bags",
               "clean_bags_for_relation_type", "reinitialize_weights", "retrieve_destinations_low_loss",
               "score_relation_bags_parallel")


def reference_main_functions(model):
    """The reference main.py cannot be imported (mpi4py, seaborn, mlxtend, imblearn and utils.py
    are absent), so its score-function definitions are compiled straight from /root/reference/
    main.py (ast: only the named top-level functions, unchanged) into a namespace holding what
    main.py's own imports give them (``from model import *``, random, ...). Nothing of the
    reference is written into this repository; only the outputs below are."""
    import ast
    import random
    src = open(os.path.join(REF, "main.py")).read()
    tree = ast.parse(src)
    keep = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in SCORE_FUNCS]
    assert {n.name for n in keep} == set(SCORE_FUNCS), {n.name for n in keep}
    ns = dict(vars(model))
    ns.update({"random": random, "COMPLEX": "synthetic"})
    exec(compile(ast.Module(body=keep, type_ignores=[]), os.path.join(REF, "main.py"), "exec"), ns)
    return ns


def make_score_golden(model):
    """Score function (model.py:26-125) trained by the reference's own score_relation_parallel
    path (main.py:727-760: create_edge_dictionary :387-438, initialize_weights :479-497, train
    :641-673) on the planted synthetic graph (KAT L3): per epoch the loss and every source's
    argmax destination, plus the final parameters. Two cases:
      rel1_synth   relation 1, dataset 'synthetic' (labels indexed by node), all sources of
                   the relation (the first-iteration mask: sorted unique node_1)
      rel0_mask    relation 0, dataset 'fb15k-237' (labels per mask position), a shuffled mask
                   with one duplicate and nodes without an edge of the relation."""
    import random
    ns = reference_main_functions(model)
    kat = np.load(os.path.join(HERE, "kat_synthetic.npz"))
    link, node, label = kat["L3_link"], kat["L3_node"], kat["L3_label"]
    edge_index = torch.tensor(np.stack([link[:, 0], link[:, 2]]))
    edge_type = torch.tensor(link[:, 1])
    x = torch.from_numpy(node[:, 1:].astype(np.float32))
    N = x.size(0)
    lab = torch.zeros(N, dtype=torch.int64)
    lab[torch.from_numpy(label[:, 0])] = torch.from_numpy(label[:, 1])
    out = {"edge_index": edge_index.numpy(), "edge_type": edge_type.numpy(), "x": x.numpy(), "labels": lab.numpy()}
    epochs = 100
    for tag, rel, dataset in (("rel1_synth", 1, "synthetic"), ("rel0_mask", 0, "fb15k-237")):
        data = model.Data()
        data.x, data.edge_index, data.edge_type, data.num_nodes = x, edge_index, edge_type, N
        if dataset == "synthetic":
            mask = torch.unique(edge_index[0][edge_type == rel]).tolist()
            data.labels = lab.unsqueeze(-1)
        else:
            srcs = torch.unique(edge_index[0][edge_type == rel]).tolist()
            g = np.random.default_rng(7)
            mask = [int(v) for v in g.permutation(srcs)[: len(srcs) // 2]]
            absent = sorted(set(range(N)) - set(srcs))[:5]
            mask = mask[:10] + [absent[0]] + mask[10:] + [mask[3]] + absent[1:]
            data.labels = lab[torch.tensor(mask)].unsqueeze(-1)  # per mask position
        ed, dd = ns["create_edge_dictionary"](data, rel, mask, BAGS=False, dataset=dataset)
        random.seed(1000 + rel)
        weights = ns["initialize_weights"](data, dd, BAGS=False)
        for k in range(N):  # the reference leaves non-destination entries uninitialised
            if k not in dd:
                weights[k] = 0.0
        w0 = weights.clone()
        torch.manual_seed(77)
        mod = ns["get_model"](weights, x.size(1))
        opt = ns["get_optimizer"](mod)
        crit, crit_node = ns["get_loss"](), ns["get_loss_per_node"]()
        losses, argmax = [], []
        keys = list(ed.keys())
        for _ in range(epochs):
            loss, best, _, _, _ = ns["train"](data, ed, mod, opt, crit, mask, crit_node, [], weights, torch.tensor(0),
                                              BAGS=False, bags_to_predict=None, bags_to_predict_labels=None,
                                              dataset=dataset)
            losses.append(loss.item())
            argmax.append([best[k] for k in keys])
        out[f"{tag}_relation"] = np.int64(rel)
        out[f"{tag}_mask"] = np.array(mask, dtype=np.int64)
        out[f"{tag}_mask_labels"] = data.labels.numpy()
        out[f"{tag}_keys"] = np.array(keys, dtype=np.int64)
        out[f"{tag}_key_ptr"] = np.cumsum([0] + [len(ed[k]) for k in keys]).astype(np.int64)
        out[f"{tag}_dst"] = np.array(sum((ed[k] for k in keys), []), dtype=np.int64)
        out[f"{tag}_dd_keys"] = np.array(list(dd.keys()), dtype=np.int64)
        out[f"{tag}_dd_min"] = np.array([min(v) for v in dd.values()], dtype=np.float64)
        out[f"{tag}_dd_len"] = np.array([len(v) for v in dd.values()], dtype=np.int64)
        out[f"{tag}_w0"] = w0.numpy()
        out[f"{tag}_loss"] = np.array(losses)
        out[f"{tag}_argmax"] = np.array(argmax, dtype=np.int32)
        out[f"{tag}_w_final"] = mod.input.weights.detach().numpy()[:, 0]
        out[f"{tag}_lin_final"] = mod.output.LinearLayerAttri.weight.detach().numpy()
        torch.manual_seed(77)
        out[f"{tag}_lin0"] = torch.nn.Linear(x.size(1), 1, bias=False).weight.detach().numpy()
        # the same run through score_relation_parallel itself (its returned loss)
        random.seed(1000 + rel)
        torch.manual_seed(77)
        ret = ns["score_relation_parallel"](data, rel, list(mask) if dataset != "synthetic" else [], x.size(1),
                                            dataset=dataset)
        out[f"{tag}_srp_loss"] = np.float64(ret[1])
    np.savez_compressed(os.path.join(HERE, "score_synthetic.npz"), **out)


def make_score_bags_golden(model):
    """Bag branch of the score function (model.py:45-72) driven by the reference's own
    score_relation_bags_parallel (main.py:853-917: create_edge_dictionary BAGS=True :426-438,
    clean_bags_for_relation_type :577-592, initialize / reinitialize_weights :479-512, train
    BAGS=True :641-673, retrieve_destinations_low_loss :530-543) on the planted synthetic graph
    (KAT L3). The bags come from the reference's create_bags (:545-575) over the dictionaries of
    a first, non-bag scoring of relation 0 (the search's first step, main.py:1309-1380). Every
    train() call of the restarts is recorded (loss, max node per bag, loss per bag), with the
    restart bookkeeping (frozen destinations, the returned current_loss, predictions per source)."""
    import random
    ns = reference_main_functions(model)
    kat = np.load(os.path.join(HERE, "kat_synthetic.npz"))
    link, node, label = kat["L3_link"], kat["L3_node"], kat["L3_label"]
    edge_index = torch.tensor(np.stack([link[:, 0], link[:, 2]]))
    edge_type = torch.tensor(link[:, 1])
    x = torch.from_numpy(node[:, 1:].astype(np.float32))
    N = x.size(0)
    lab = torch.zeros(N, dtype=torch.int64)
    lab[torch.from_numpy(label[:, 0])] = torch.from_numpy(label[:, 1])
    data = model.Data()
    data.x, data.edge_index, data.edge_type, data.num_nodes = x, edge_index, edge_type, N
    data.labels = lab.unsqueeze(-1)
    mask = torch.unique(edge_index[0][edge_type == 0]).tolist()
    ed0, dd0 = ns["create_edge_dictionary"](data, 0, mask, BAGS=False, dataset="synthetic")
    ns["create_bags"](ed0, dd0, data)
    bags, bag_labels = data.bags, data.bag_labels
    out = {"bag_ptr": np.cumsum([0] + [len(b) for b in bags]).astype(np.int64),
           "bag_nodes": np.array(sum(bags, []), dtype=np.int64), "bag_labels": bag_labels.numpy()}
    orig_train = ns["train"]
    for rel in (1, 2, 3, 0):
        calls = []

        def recording_train(*a, **kw):
            res = orig_train(*a, **kw)
            loss, by_source, loss_per_bag, by_bag, pred = res
            cbags = kw["bags_to_predict"]
            calls.append((loss.item(), [by_bag.get(str(b), -1) for b in cbags], loss_per_bag.detach().numpy()[:, 0].copy(),
                          list(a[7])))
            return res
        ns["train"] = recording_train
        random.seed(2000 + rel)
        torch.manual_seed(88)
        r, current_loss, mod, preds, v = ns["score_relation_bags_parallel"](data, rel, x.size(1), dataset="synthetic")
        ns["train"] = orig_train
        tag = f"bags_rel{rel}"
        # the cleaned bags of this relation, as train() received them
        random.seed(2000 + rel)
        mask_b = []
        for bag in bags:
            for elm in bag:
                if elm not in mask_b:
                    mask_b.append(elm)
        edb, ddb = ns["create_edge_dictionary"](data, rel, mask_b, BAGS=True, dataset="synthetic")
        cb, cl = ns["clean_bags_for_relation_type"](data, edb)
        out[f"{tag}_cbag_ptr"] = np.cumsum([0] + [len(b) for b in cb]).astype(np.int64)
        out[f"{tag}_cbag_nodes"] = np.array(sum(cb, []), dtype=np.int64)
        out[f"{tag}_cbag_labels"] = cl.numpy()
        keys = list(edb.keys())
        out[f"{tag}_keys"] = np.array(keys, dtype=np.int64)
        out[f"{tag}_key_ptr"] = np.cumsum([0] + [len(edb[k]) for k in keys]).astype(np.int64)
        out[f"{tag}_dst"] = np.array(sum((edb[k] for k in keys), []), dtype=np.int64)
        out[f"{tag}_dd_keys"] = np.array(list(ddb.keys()), dtype=np.int64)
        out[f"{tag}_dd_min"] = np.array([min(v_) for v_ in ddb.values()], dtype=np.float64)
        out[f"{tag}_dd_len"] = np.array([len(v_) for v_ in ddb.values()], dtype=np.int64)
        out[f"{tag}_loss"] = np.array([c[0] for c in calls])
        out[f"{tag}_bag_argmax"] = np.array([c[1] for c in calls], dtype=np.int32)
        out[f"{tag}_loss_per_bag_last"] = np.array([c[2] for c in calls[49::50]])
        out[f"{tag}_frozen_per_call"] = np.array([len(c[3]) for c in calls], dtype=np.int64)
        out[f"{tag}_current_loss"] = np.float64(current_loss)
        out[f"{tag}_v"] = np.bool_(v)
        pk = list(preds.keys())
        out[f"{tag}_pred_keys"] = np.array(pk, dtype=np.int64)
        out[f"{tag}_pred_vals"] = np.array([preds[k] for k in pk], dtype=np.float64)
        out[f"{tag}_lin_final"] = mod.output.LinearLayerAttri.weight.detach().numpy()
        wf = mod.input.weights.detach().numpy()[:, 0]
        out[f"{tag}_w_final_dd"] = wf[np.array(list(ddb.keys()), dtype=np.int64)]
    np.savez_compressed(os.path.join(HERE, "score_bags_synthetic.npz"), **out)


def make_fb15k_triples():
    """FB15K-237 dev+test triples as entity/relation indices (entities.txt / relations.txt
    order). train.tsv is missing from the reference (.MISSING_LARGE_BLOBS:7); the bench's
    FB15K-shaped graph (mpgnn_amd.data.fb15k237_graph) keeps these 38,000 real triples and
    samples the rest relation-conditionally from them. Written into the package (data, not code)."""
    base = os.path.join(REF, "data/fb15k-237")
    ents = [l.strip() for l in open(os.path.join(base, "entities.txt")) if l.strip()]
    rels = [l.strip() for l in open(os.path.join(base, "relations.txt")) if l.strip()]
    e2i = {e: i for i, e in enumerate(ents)}
    r2i = {r: i for i, r in enumerate(rels)}
    tri = []
    for f in ("dev.tsv", "test.tsv"):
        for line in open(os.path.join(base, f)):
            p = line.rstrip("\n").split("\t")
            if len(p) == 3:
                tri.append((e2i[p[0]], r2i[p[1]], e2i[p[2]]))
    tri = np.array(tri, dtype=np.int32)
    pkg = os.path.join(HERE, "..", "..", "mpgnn-metapath-graph-neural-network_amd", "data")
    os.makedirs(pkg, exist_ok=True)
    np.savez_compressed(os.path.join(pkg, "fb15k237_devtest.npz"), head=tri[:, 0], rel=tri[:, 1],
                        tail=tri[:, 2], num_entities=np.int64(len(ents)), num_relations=np.int64(len(rels)))


def main():
    if not os.path.isdir(REF):
        raise SystemExit("make_golden.py needs /root/reference (survey container only)")
    torch.set_num_threads(1)
    layer, model = import_reference()
    if "--only" in sys.argv:
        name = sys.argv[sys.argv.index("--only") + 1]
        globals()[name](model)
        return
    make_kat()
    make_layer_goldens(layer)
    make_mpnetm_golden(model)
    make_score_golden(model)
    make_score_bags_golden(model)
    make_fb15k_triples()
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)), "bytes")


if __name__ == "__main__":
    main()
