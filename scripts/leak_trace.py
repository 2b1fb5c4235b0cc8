"""Active allocations left behind by a graph-replaying drop-in loop call, with their Python stacks."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpgnn_amd  # noqa: E402,F401
from mpgnn_amd import data, main  # noqa: E402

DEV = torch.device("cuda", 0)
g = data.synthetic_graph(3000, 6, 14, feat_dim=128, seed=4)
gen = torch.Generator().manual_seed(1)
y = torch.randint(0, 2, (g.num_nodes,), generator=gen)
perm = torch.randperm(g.num_nodes, generator=gen)
n = g.num_nodes
tr, va, te = perm[: n // 2], perm[n // 2: 3 * n // 4], perm[3 * n // 4:]
d = main.Data(x=g.x, edge_index=g.edge_index, edge_type=g.edge_type, train_idx=tr, train_y=y[tr], val_idx=va,
              val_y=y[va], test_idx=te, test_y=y[te]).to(DEV)


def run():
    return main.mpgnn_parallel_multiple(d, 128, 128, g.num_relations, 128, 2, [[0, 1]], epochs=5)


run()
torch.cuda.synchronize()
base = torch.cuda.memory_allocated()
torch.cuda.memory._record_memory_history(max_entries=200000)
run()
torch.cuda.synchronize()
print("leak bytes", torch.cuda.memory_allocated() - base, flush=True)
snap = torch.cuda.memory._snapshot()
seen = 0
for seg in snap["segments"]:
    for blk in seg["blocks"]:
        if blk["state"] != "active_allocated":
            continue
        frames = blk.get("frames") or []
        if not frames:
            continue
        seen += 1
        py = [f"{f['filename'].split('/')[-1]}:{f['line']}:{f['name']}" for f in frames
              if f["filename"].endswith(".py")][:8]
        print(blk["size"], "pool", seg.get("segment_pool_id"), " <- ".join(py), flush=True)
print("blocks with history", seen)
