#!/usr/bin/env python3
"""Bench: edges aggregated/sec of the metapath-RGCN relational stack on MI355X.

Workload (BASELINE.json configs[2]): FB15K-237-shaped graph, N = 14,541,
R = 237, E = 310,116, 128-d features; the RGCN stack of model.py:Net (main_rgcn.py:547,
L = 3: conv1 then the shared conv2 twice, ReLU after each) with 128-d hidden/output.

One timed STEP = one forward pass of the 3 relational layers over the whole graph, inputs
resident in HBM.  value = edges aggregated per second = 3 · E · steps / time (an edge
aggregated = one (node_1, rel, node_2) edge folded into its (node_1, rel) segment in one
layer).  With --gpus N (torchrun, one process per GPU) the graph is sharded by
aggregating-node (node_1) range, edge-balanced: each rank computes complete output rows for its
range and one RCCL all-gather over xGMI per layer assembles the next layer's input
(distributed.sharded_stack_forward, shard_side="rows"; measured per-rank compute at 8 shards
1.91x below one GPU vs 1.51x for node_2 shards, scripts/shard_compute.py); the training epoch
runs RGCNConv(shard=, group=, shard_side="rows") with the per-layer all-reduce of the disjoint
rows and the gradient all-reduces. Total work is fixed: "scaling" is "strong".

Also reported (separate loops, outside the timed step): the training epoch of
main_rgcn.py:458-461 — train step (forward + NLL + backward + Adam) + validation forward.

roofline: the dominant kernel (rel_gemm_kernel, forward) timed live with HIP events on its
launch stream over a second pass of the same K steps (events between kernels drain the queue,
so they are kept out of the headline's timed region); algorithmic FLOPs = 2·(S + N)·F_in·F_out per launch
(segment rows H @ W_r plus node rows x @ root, both computed by that launch) against the
dense fp32 MFMA peak (157.3 TFLOP/s); algorithmic bytes (A rows in, Y rows out, weights)
reported beside it.  traffic: HBM bytes per launch from rocprofv3 PMC counters
(profiles/pmc_seg_fwd.json when present, else null).
cpu_baseline: the CPU oracle (PyG-2.3.1 loop semantics, same ATen ops) timed on this host.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import mpgnn_amd  # noqa: E402
from mpgnn_amd import _lib, data  # noqa: E402
from mpgnn_amd.distributed import shard_ranges, sharded_stack_forward  # noqa: E402

METRIC = "edges aggregated/sec + epoch time, FB15K-237 128-d at 1/2/4/8 MI355X"
PEAK_FP32_MFMA = 157.3  # TFLOP/s dense (MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32)
PEAK_HBM = 8000.0       # GB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="fb15k237", choices=["fb15k237", "C2", "C5"],
                    help="fb15k237 = C3/C4 (the headline); C2 / C5 = the other BASELINE.json configs")
    ap.add_argument("--recipe", default="survey", choices=["survey", "relcond"],
                    help="FB15K-237 edge recipe: survey = SURVEY §8d C3 (S ~ 208k, the headline); "
                         "relcond = round-1 relation-conditional graph (S ~ 48k, lighter)")
    ap.add_argument("--layers", type=int, default=None, help="default 3 (C3, C5) / 2 (C2)")
    ap.add_argument("--feat", type=int, default=None, help="default 128 (C2, C3) / 256 (C5)")
    ap.add_argument("--epoch-steps", type=int, default=None, help="0 skips the epoch leg (default 10; 2 at C5)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-reps", type=int, default=2)
    a = ap.parse_args()
    dflt = {"fb15k237": (3, 128, 30), "C2": (2, 128, 10), "C5": (3, 256, 2)}[a.workload]
    a.layers = dflt[0] if a.layers is None else a.layers
    a.feat = dflt[1] if a.feat is None else a.feat
    a.epoch_steps = dflt[2] if a.epoch_steps is None else a.epoch_steps
    return a


WORKLOADS = {
    "fb15k237": ("C3 FB15K-237 (N=14541, R=237, E=310116)",
                 "synthetic: FB15K-237-shaped graph (38,000 real dev+test triples + relation-conditional "
                 "samples to E=310,116), U[0,1) features, seed-10 random-init weights"),
    "C2": ("C2 synthetic (N=100000, R=16, out-degree U{1..32})",
           "synthetic: seeded generator of create_graph (SURVEY §8d C2), U[0,1) features, seed-10 weights"),
    "C5": ("C5 synthetic (N=2000000, R=64, out-degree U{1..31})",
           "synthetic: seeded generator of create_graph (SURVEY §8d C5), U[0,1) features, seed-10 weights"),
}


def setup_dist(n):
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n:
        raise SystemExit(f"--gpus {n} but WORLD_SIZE={world}: launch N>1 with torch.distributed.run")
    # rehearsal of the N > 1 flow on a one-GPU box: every rank on device 0 over gloo
    # (MPGNN_BENCH_REHEARSE=1); the numbers of such a run are not a measurement
    rehearse = os.environ.get("MPGNN_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    torch.cuda.set_device(local)
    group = None
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        group = dist.group.WORLD
    return rank, world, local, group


def cpu_baseline_sampled(g, net_cpu, layers, reps):
    """C2 / C5: the full CPU stack would take minutes to hours (R dense N×F×F GEMMs per layer),
    so the oracle's loop body is timed for ONE relation of the first layer (index_select,
    scatter_add_, div, mm — rgcn_oracle.rgcn_forward's iteration) and scaled by R·layers, plus
    the root GEMM per layer; labelled as extrapolated."""
    from oracle import rgcn_oracle as orc
    w = net_cpu.conv1.weight.detach()
    root = net_cpu.conv1.root.detach()
    x, ei, et = g.x, g.edge_index, g.edge_type
    size = (x.size(0), x.size(0))
    with torch.no_grad():
        times = []
        for _ in range(reps + 1):
            t0 = time.perf_counter()
            tmp = orc.masked_edge_index(ei, et == 0)
            h = orc.propagate_mean(tmp, x, size)
            _ = h @ w[0]
            t_rel = time.perf_counter() - t0
            t0 = time.perf_counter()
            _ = x @ root
            t_root = time.perf_counter() - t0
            times.append((t_rel, t_root))
    times = sorted(times[1:])
    t_rel, t_root = times[len(times) // 2]
    est = layers * (g.num_relations * t_rel + t_root)
    return {"value": layers * g.num_edges / est, "unit": "edges/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"oracle loop body for relation 0 of layer 1 ({reps} timed + 1 warm-up, median "
                      f"{t_rel * 1e3:.1f} ms) + root GEMM ({t_root * 1e3:.1f} ms), extrapolated x{g.num_relations} "
                      f"relations x{layers} layers = {est:.1f} s per forward (extrapolated, not run in full)"}


def cpu_baseline(g, net_cpu, layers, reps):
    """Oracle (CPU, all host threads torch uses) on the same graph: `reps` timed forwards of
    the relational stack after one warm-up; edges/s = layers·E / median time."""
    from oracle import rgcn_oracle as orc
    params = {k: v.detach() for k, v in net_cpu.state_dict().items()}
    x, ei, et = g.x, g.edge_index, g.edge_type

    def fwd():
        h = x
        for layer in range(layers):
            p = "conv1." if layer == 0 else "conv2."
            h = torch.relu(orc.rgcn_forward(h, ei, et, params[p + "weight"], params[p + "root"],
                                            params[p + "bias"]))
        return h

    with torch.no_grad():
        fwd()
        times = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fwd()
            times.append(time.perf_counter() - t0)
    times.sort()
    med = times[len(times) // 2]
    return {"value": layers * g.num_edges / med, "unit": "edges/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"{reps} timed + 1 warm-up forward passes of the {layers}-layer RGCN stack on the full "
                      f"FB15K-shaped graph (oracle/rgcn_oracle.py, PyG-2.3.1 loop: index_select/scatter_add_/"
                      f"div/mm per relation); median {med * 1e3:.1f} ms"}


def main():
    args = parse()
    rank, world, local, group = setup_dist(args.gpus)
    dev = torch.device("cuda", local)
    if args.workload == "fb15k237":
        g = data.fb15k237_graph(feat_dim=args.feat, seed=0, recipe=args.recipe)
    else:
        g = data.config_graph(args.workload)
        if g.x.shape[1] != args.feat:
            g.x = torch.rand((g.num_nodes, args.feat), generator=torch.Generator().manual_seed(1))
    F = args.feat
    torch.manual_seed(10)  # main_rgcn.py:31
    net_cpu = mpgnn_amd.Net(F, F, g.num_relations, F, 2, args.layers)
    net = mpgnn_amd.Net(F, F, g.num_relations, F, 2, args.layers)
    net.load_state_dict(net_cpu.state_dict())
    net = net.to(dev)
    x, ei, et = g.x.to(dev), g.edge_index.to(dev), g.edge_type.to(dev)
    shard = None
    ranges = None
    if world > 1:  # shard by the aggregating node: complete rows per rank (scripts/shard_compute.py)
        ranges = shard_ranges(g.edge_index, g.num_nodes, world, side="rows")
        shard = ranges[rank]
    convs = [net.conv1] + [net.conv2] * (args.layers - 1)

    def step():
        if world > 1:  # each rank's complete rows all-gathered per layer
            return sharded_stack_forward(convs, x, ei, et, ranges, group, shard_side="rows")
        h = x
        for conv in convs:
            h = conv(h, ei, et, activation="relu")  # F.relu(conv(...)), model.py:144,146
        return h

    # plan (built once per graph, cached) + warm-up
    with torch.no_grad():
        for _ in range(max(args.warmup, 1)):
            step()
    torch.cuda.synchronize()
    plan = mpgnn_amd.get_plan(ei, et, g.num_nodes, shard=shard, device=dev, shard_side="rows")

    # ---- timed region: K forward steps --------------------------------------------------
    if group is not None:
        dist.barrier(group=group)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.no_grad():
        for _ in range(args.steps):
            step()
    torch.cuda.synchronize()
    if group is not None:
        dist.barrier(group=group)
    elapsed = time.perf_counter() - t0

    # ---- roofline pass: the same K steps again with the dominant kernel bracketed by HIP
    # events on its launch stream (C-ABI timing hook).  Kept out of the timed region: an event
    # between two kernels drains the queue (~4 us per event pair on this stack), which would
    # charge the headline number for the measurement itself.
    _lib.lib.mpgnn_timing_reset()
    _lib.lib.mpgnn_set_option(3, 1 << _lib.KERNEL_KINDS["seg_fwd"])  # time only the roofline kernel
    _lib.lib.mpgnn_timing_enable(1)
    with torch.no_grad():
        for _ in range(args.steps):
            step()
    torch.cuda.synchronize()
    _lib.lib.mpgnn_timing_enable(0)
    _lib.lib.mpgnn_set_option(3, -1)
    seg_ms, seg_n = _lib.kernel_timing("seg_fwd")
    row_ms, row_n = _lib.kernel_timing("row_fwd")

    # ---- per-kernel breakdown: a third pass with every kernel kind timed (events between all
    # kernels make each launch slightly longer than in the headline pass; attribution only)
    _lib.lib.mpgnn_timing_reset()
    _lib.lib.mpgnn_timing_enable(1)
    with torch.no_grad():
        for _ in range(args.steps):
            step()
    torch.cuda.synchronize()
    _lib.lib.mpgnn_timing_enable(0)
    per_layer = {}
    for kind, label in (("mean", "segment means: flat_rows_kernel + split-row finalize"), ("final", "split-row finalize alone"),
                        ("seg_fwd", "transform GEMM"), ("row_fwd", "combine (flat_rows_kernel)")):
        k_ms, k_n = _lib.kernel_timing(kind)
        if k_n:
            per_layer[kind] = {"what": label, "us_per_layer": round(k_ms * 1e3 / (args.steps * args.layers), 2)}
    if group is not None:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        elapsed = float(t.item())
    ms_per_step = elapsed * 1e3 / args.steps
    edges_per_step = args.layers * g.num_edges
    value = edges_per_step * args.steps / elapsed
    # SURVEY §8d layer roofline: algorithmic bytes per forward layer
    # B = E·(4·F_in + 4) + S·8 + N·4·F_out (gathered rows + their column ids, segment ptr/rel,
    # output write); at 8 TB/s that bounds edges/s at E / (B / 8e12)
    b_layer = g.num_edges * (4 * F + 4) + plan.num_segments * 8 + g.num_nodes * 4 * F
    ideal = g.num_edges / (b_layer / (PEAK_HBM * 1e9))
    hbm_roofline = {"bound": "hbm", "alg_bytes_per_layer": b_layer,
                    "achieved_GBps": round(value / g.num_edges * b_layer / 1e9, 1), "peak_GBps": PEAK_HBM,
                    "ideal_edges_per_s": round(ideal, 1), "frac": round(value / ideal, 4),
                    "note": "whole-step edges/s against the aggregation's HBM roofline of SURVEY §8d (516 B per "
                            "edge at F=128); at C3 x (7.4 MB) stays in L2/MALL, so the layer is bound on-die"}

    # ---- the same step replayed as one HIP graph (launch overhead removed) ---------------
    graph = None
    if world == 1:
        try:
            s_cap = torch.cuda.Stream()
            s_cap.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s_cap), torch.no_grad():
                for _ in range(2):  # workspace / allocator warm-up on the capture stream
                    step()
            torch.cuda.current_stream().wait_stream(s_cap)
            torch.cuda.synchronize()
            cg = torch.cuda.CUDAGraph()
            with torch.cuda.graph(cg), torch.no_grad():
                step()
            for _ in range(3):
                cg.replay()
            torch.cuda.synchronize()
            tg = time.perf_counter()
            for _ in range(args.steps):
                cg.replay()
            torch.cuda.synchronize()
            g_el = time.perf_counter() - tg
            graph = {"value": round(edges_per_step * args.steps / g_el, 1),
                     "ms_per_step": round(g_el * 1e3 / args.steps, 4),
                     "note": "same 3-layer forward captured once with torch.cuda.graph (hipGraph) and "
                             "replayed: every kernel runs every step, host launch overhead removed"}
        except Exception as e:  # capture unsupported here: report, keep the eager number
            graph = {"error": f"{type(e).__name__}: {e}"[:200]}
        cg = None  # free the graph's private pool and the capture stream's workspace
        mpgnn_amd.functional.release_workspaces()
        torch.cuda.empty_cache()

    # ---- epoch (main_rgcn.py:458-461): train fwd+bwd+Adam + validation forward ------------
    opt = mpgnn_amd.main._adam(net)  # Adam(lr 0.01, wd 5e-4), fused multi-tensor kernel on the GPU
    y = torch.randint(0, 2, (g.num_nodes,), generator=torch.Generator().manual_seed(0)).to(dev)
    train_idx = torch.arange(0, g.num_nodes, 3, device=dev)
    train_y = y[train_idx]  # data.train_y of the reference loop: fixed labels, indexed once

    def epoch():
        net.train()
        opt.zero_grad()
        out = net(x, ei, et, shard=shard, group=group, shard_side="rows")
        loss = torch.nn.functional.nll_loss(out.index_select(0, train_idx), train_y)
        loss.backward()
        opt.step()
        net.eval()
        with torch.no_grad():
            net(x, ei, et, shard=shard, group=group, shard_side="rows")

    epoch_ms = None
    if args.epoch_steps > 0:
        for _ in range(5):
            epoch()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.epoch_steps):
            epoch()
        torch.cuda.synchronize()
        epoch_ms = (time.perf_counter() - t1) * 1e3 / args.epoch_steps

    # ---- the same epoch captured once as a HIP graph (host issue removed) -------------------
    # torch's whole-network capture recipe: warm-up on a side stream, grads allocated inside
    # the capture, Adam(fused, capturable); replay = train fwd + NLL + bwd + Adam + val fwd.
    epoch_graph = None
    if args.epoch_steps > 0 and world == 1:
        try:
            netg = mpgnn_amd.Net(F, F, g.num_relations, F, 2, args.layers).to(dev)
            netg.load_state_dict(net.state_dict())
            optg = torch.optim.Adam(netg.parameters(), lr=0.01, weight_decay=0.0005, fused=True, capturable=True)

            def epoch_g():
                netg.train()
                out = netg(x, ei, et)
                loss = torch.nn.functional.nll_loss(out.index_select(0, train_idx), train_y)
                loss.backward()
                optg.step()
                netg.eval()
                with torch.no_grad():
                    netg(x, ei, et)
                return loss

            s_cap = torch.cuda.Stream()
            s_cap.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s_cap):
                for _ in range(3):
                    optg.zero_grad(set_to_none=True)
                    epoch_g()
            torch.cuda.current_stream().wait_stream(s_cap)
            torch.cuda.synchronize()
            cg_e = torch.cuda.CUDAGraph()
            optg.zero_grad(set_to_none=True)
            with torch.cuda.graph(cg_e):
                static_loss = epoch_g()
            for _ in range(3):
                cg_e.replay()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for _ in range(args.epoch_steps):
                cg_e.replay()
            torch.cuda.synchronize()
            epoch_graph = {"ms": round((time.perf_counter() - t1) * 1e3 / args.epoch_steps, 4),
                           "loss_finite": bool(torch.isfinite(static_loss).item()),
                           "note": "the epoch above captured once as a HIP graph (Adam fused + capturable) and "
                                   "replayed: every kernel of train fwd/bwd/step + val fwd runs every replay"}
            cg_e = None
            mpgnn_amd.functional.release_workspaces()
            torch.cuda.empty_cache()
        except Exception as e:  # capture unsupported: report, keep the eager number
            epoch_graph = {"error": f"{type(e).__name__}: {e}"[:200]}

    # ---- roofline of the dominant kernel (per launch, this rank) --------------------------
    S = plan.num_segments
    E_loc = plan.num_edges
    # the layer's transform may be split over several launches (root rows + relation groups,
    # MPGNN_OPT_OVERLAP): the roofline is per LAYER = the summed durations of its launches
    layer_calls = args.steps * args.layers
    seg_avg_ms = seg_ms / max(layer_calls, 1)
    n_root = plan.num_nodes if world == 1 else (shard[1] - shard[0])
    flops = 2.0 * (S + n_root) * F * F   # Y = H @ W_r over S segment rows + Y_root = x @ root
    alg_bytes = 4 * F * (2 * S + 2 * n_root) + 4 * F * F * (plan.num_relations_present + 1)  # A rows in, Y out, W
    achieved_tf = flops / (seg_avg_ms * 1e-3) / 1e12 if seg_n else None
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_seg_fwd.json")
    if os.path.exists(pmc_path):
        try:
            pmc = json.load(open(pmc_path))
            if pmc.get("workload") == args.workload and pmc.get("feat") == F and world == 1 and \
                    pmc.get("kernel", "").startswith("mpgnn::rel_gemm_kernel"):
                traffic = pmc.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    roofline = {
        "bound": "mfma", "achieved": round(achieved_tf, 3) if achieved_tf else None, "peak": PEAK_FP32_MFMA,
        "unit": "TFLOP/s", "frac": round(achieved_tf / PEAK_FP32_MFMA, 4) if achieved_tf else None,
        "traffic": traffic,
        "kernel": ("rel_gemm_kernel (Y = H @ W_r, Y_root = x @ root; W_r slice held in registers; "
                   "v_mfma_f32_32x32x2_f32)") if F in (64, 128) else
                  "tile_gemm_kernel (Y = H @ W_r, Y_root = x @ root; persistent LDS-tiled; v_mfma_f32_32x32x2_f32)",
        "avg_launch_us": round(seg_avg_ms * 1e3, 2), "launches": seg_n,
        "launches_per_layer": round(seg_n / max(layer_calls, 1), 2),
        "note": "avg_launch_us = summed duration of one layer's transform launches (root rows + relation "
                "groups; they run on a second stream beside the segment means, so contention is included)",
        "alg_flops_per_launch": flops, "alg_bytes_per_launch": alg_bytes,
        "alg_GBps": round(alg_bytes / (seg_avg_ms * 1e-3) / 1e9, 1) if seg_n else None,
        "hbm_frac_if_streamed": round(alg_bytes / (seg_avg_ms * 1e-3) / 1e9 / PEAK_HBM, 4) if seg_n else None,
        "row_kernel_avg_us": round(row_ms / max(row_n, 1) * 1e3, 2),
    }

    result = None
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            if args.workload == "fb15k237":
                cpu = cpu_baseline(g, net_cpu, args.layers, args.cpu_reps)
            else:
                cpu = cpu_baseline_sampled(g, net_cpu, args.layers, args.cpu_reps)
        result = {
            "metric": METRIC, "value": round(value, 1), "unit": "edges/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": WORKLOADS[args.workload][1],
            "config": {"workload": WORKLOADS[args.workload][0] + ": RGCN Net stack forward, "
                                   f"L={args.layers}, F_in=F_hidden=F_out={F}",
                       "graph": {"nodes": g.num_nodes, "relations": g.num_relations, "edges": g.num_edges,
                                 "segments": S if world == 1 else None},
                       "parallelism": "single GPU" if world == 1 else
                       f"row-range shards x{world} (aggregating node, edge-balanced): each rank computes its "
                       "complete output rows, one RCCL all-gather per layer (epoch: per-layer all-reduce of the "
                       "disjoint rows, gradient all-reduces)"},
            "graph_replay": graph,
            "epoch_ms": round(epoch_ms, 3) if epoch_ms is not None else None,
            "epoch_graph": epoch_graph,
            "epoch_def": "main_rgcn.py:458-461 train (fwd+NLL+bwd+Adam) + validation forward",
            "roofline": roofline,
            "hbm_roofline": hbm_roofline,
            "kernels_per_layer": per_layer,
            "cpu_baseline": cpu,
        }
        print(json.dumps(result), flush=True)
    if group is not None:
        dist.barrier(group=group)
        dist.destroy_process_group()
    return result


if __name__ == "__main__":
    main()
