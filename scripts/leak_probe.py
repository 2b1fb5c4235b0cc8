"""Where does memory go between two drop-in loop calls? (diagnostic for the workspace test)"""
import gc
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpgnn_amd  # noqa: E402
from mpgnn_amd import data, main, main_rgcn  # noqa: E402
from mpgnn_amd import functional as fn  # noqa: E402

DEV = torch.device("cuda", 0)
g = data.fb15k237_graph(feat_dim=128, seed=0, recipe="survey")
gen = torch.Generator().manual_seed(1)
y = torch.randint(0, 2, (g.num_nodes,), generator=gen)
perm = torch.randperm(g.num_nodes, generator=gen)
n = g.num_nodes
tr, va, te = perm[: n // 2], perm[n // 2: 3 * n // 4], perm[3 * n // 4:]
d = main.Data(x=g.x, edge_index=g.edge_index, edge_type=g.edge_type, train_idx=tr, train_y=y[tr], val_idx=va,
              val_y=y[va], test_idx=te, test_y=y[te]).to(DEV)
counts = torch.bincount(g.edge_type, minlength=g.num_relations)
mp = [int(v) for v in torch.argsort(counts, descending=True, stable=True)[:3]]
which = sys.argv[1] if len(sys.argv) > 1 else "single"


def run():
    if which == "single":
        return main.mpgnn_parallel_multiple(d, 128, 128, g.num_relations, 128, 2, [mp], epochs=6)
    return main_rgcn.mpgnn_parallel_multiple(d, 128, 128, g.num_relations, 128, 2, 3, epochs=6, verbose=False)


def state(tag):
    torch.cuda.synchronize()
    graphs = sum(1 for o in gc.get_objects() if isinstance(o, torch.cuda.CUDAGraph))
    print(tag, "alloc", torch.cuda.memory_allocated(), "ws", fn.workspace_bytes_cached(), "ws_keys", list(fn._WS),
          "retired", {k: len(v) for k, v in fn._RETIRED.items()}, "graphs", graphs, flush=True)


for i in range(4):
    run()
    state(f"call {i} no-gc")
    gc.collect()
    state(f"call {i} gc")
os.environ["MPGNN_LOOP_GRAPH"] = "0"
for i in range(2):
    run()
    state(f"eager call {i} gc")
    gc.collect()
