#!/usr/bin/env python3
"""Bench: edges aggregated/sec of the metapath-RGCN relational layers on MI355X.

Workload (BASELINE.json configs[2]): the FB15K-237-shaped graph of the §8d
recipe (N = 14,541, R = 237, E = 310,116, S ≈ 208 k segments), 128-d features; mode ALL = the
RGCN stack of model.py:Net (main_rgcn.py:547, L = 3: conv1 then the shared conv2 twice, ReLU
after each). ``--mode single`` times the MPGNN metapath layer instead: MPNetm's CustomRGCNConv
chain over one metapath (model.py:203-228, mp_rgcn_layer.py:225-246; C2: 2 hops, C5: 3 hops).

One timed STEP = one forward pass of the relational layers over the whole graph, inputs
resident in HBM.  value = edges aggregated per second = Σ_layers E_layer · steps / time (an edge
aggregated = one (node_1, rel, node_2) edge folded into its (node_1, rel) segment in one layer,
SURVEY §8d; mode ALL: E per layer, mode SINGLE: the edges of that layer's relation).

--gpus N (torch.distributed.run, one process per GPU): the C4 line — the graph sharded by
GATHERED-node (node_2) range, edge-balanced (the north-star partition): every rank
computes partial sums for all rows from its own edges (global per-segment counts), one RCCL
reduce-scatter over xGMI per layer hands each rank the summed rows of its own range (the only
rows its next layer gathers), one all-gather after the last layer; the training epoch all-reduces
each layer's partial output and the gradients. ``--shard-side rows`` times the aggregating-node
(node_1) partition instead (labelled). Total work is fixed: "scaling" is "strong".

Also reported (separate loops, outside the timed step): ``epoch_ms``, the kernel epoch — train
step (forward + NLL + backward + Adam) + one validation forward, no scoring; ``loop_epoch``, the
reference's whole epoch through the drop-in loops (main_rgcn.py:458-461: weighted-NLL train,
validation and test forwards with macro F1; main.py:1121-1126: train + validation).
cpu_baseline threads: the affinity mask capped by the cgroup CPU quota (both recorded).

roofline: the kernel with the largest share of the forward layer (per-kernel HIP-event pass on
the launch stream; rocprofv3 summary in profiles/), against its own bound — the transform GEMM
(rel_gemm_bf3_kernel / single_bf3_kernel on the bf16 matrix cores: 6 bf16 products per fp32
product of 2·(S+N)·F_in·F_out, priced against the dense bf16 peak, the fp32-equivalent rate
beside it; --gemm fp32: rel_gemm_kernel against the fp32 MFMA peak) or the gathers (segment
means / combine, HBM 8 TB/s, SURVEY §8d bytes). Every forward kernel kind is listed in
roofline_kernels.
traffic: HBM bytes per launch from the rocprofv3 PMC passes committed under profiles/ (FETCH_SIZE
×2 + WRITE_SIZE, MI355X_MICROARCH.md §HBM), or null when no pass matches the workload.
cpu_baseline: the CPU oracle (PyG-2.3.1 loop semantics, same ATen ops) on this host.
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
from mpgnn_amd.distributed import shard_ranges, sharded_stack_forward, sharded_stack_forwards  # noqa: E402

METRIC = "edges aggregated/sec + epoch time, FB15K-237 128-d at 1/2/4/8 MI355X"
PEAK_FP32_MFMA = 157.3  # TFLOP/s dense (MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32)
PEAK_BF16_MFMA = 2516.6  # TFLOP/s dense = 16 x the f32 rate (v_mfma_f32_32x32x16_bf16, 32 cycles, MI355X_MICROARCH.md)
PEAK_HBM = 8000.0       # GB/s spec

WORKLOADS = {
    "fb15k237": ("C3 FB15K-237 (N=14541, R=237, E=310116, SURVEY 8d recipe)",
                 "synthetic: FB15K-237-shaped graph, SURVEY 8d C3 recipe (relation ~ dev+test histogram, node_1/"
                 "node_2 ~ dev+test entity frequency add-one smoothed over 14,541 entities), U[0,1) features, "
                 "seed-10 random-init weights"),
    "fb15k237_relcond": ("C3' FB15K-237 relation-conditional graph (round-1 headline, S ~ 48k)",
                         "synthetic: 38,000 real dev+test triples + relation-conditional samples to E=310,116, "
                         "U[0,1) features, seed-10 random-init weights"),
    "C2": ("C2 synthetic (N=100000, R=16, out-degree U{1..32})",
           "synthetic: seeded generator of create_graph (SURVEY 8d C2), U[0,1) features, seed-10 weights"),
    "C5": ("C5 synthetic (N=2000000, R=64, out-degree U{1..31})",
           "synthetic: seeded generator of create_graph (SURVEY 8d C5), U[0,1) features, seed-10 weights"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="fb15k237", choices=list(WORKLOADS))
    ap.add_argument("--mode", default="all", choices=["all", "single", "score", "score_all", "score_bags"],
                    help="all = RGCN Net (mode B, main_rgcn.py); single = MPNetm metapath chain (mode A, main.py); "
                         "score = the metapath score function (model.py:26-125, main.py:727-760); score_all = every "
                         "relation of the first search round at once (main.py:1309-1330, score_relations_batched)")
    ap.add_argument("--relation", type=int, default=None, help="mode score: relation scored (default: the largest)")
    ap.add_argument("--metapath", default=None,
                    help="mode single: comma-separated relations, one per layer (default C2 '1,0', C5 '2,1,0', "
                         "FB15K the three most frequent relations)")
    ap.add_argument("--shard-side", default="gathered", choices=["gathered", "rows"],
                    help="--gpus N > 1: gathered = node_2 ranges + reduce-scatter (north star, C4); rows = node_1")
    ap.add_argument("--layers", type=int, default=None, help="mode all: default 3 (C3, C5) / 2 (C2)")
    ap.add_argument("--feat", type=int, default=None, help="default 128 (C2, C3) / 256 (C5)")
    ap.add_argument("--epoch-steps", type=int, default=None, help="0 skips the epoch leg (default 30; 10 C2; 2 C5)")
    ap.add_argument("--loop-epochs", type=int, default=None,
                    help="epochs of the drop-in training loop timed (0 skips; default 20 C3, 5 C2, 8 C5)")
    ap.add_argument("--gemm", default="bf3", choices=["bf3", "fp32"],
                    help="transform / dgrad GEMM: bf3 = bf16 matrix cores, 3-way exact split (default); fp32 = fp32 MFMA")
    ap.add_argument("--chunk-rows", type=int, default=None,
                    help="backward weight-gradient reduction chunk length (MPGNN_OPT_CHUNK_ROWS; default: the library's)")
    ap.add_argument("--bwd-fused", type=int, default=1, choices=[0, 1],
                    help="backward at F = 128: dgrad + dW in one launch (MPGNN_OPT_BWD_FUSED); 0 for A/B")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-reps", type=int, default=5, help="timed CPU repetitions (median), after 2 warm-ups")
    a = ap.parse_args()
    base = "C3" if a.workload.startswith("fb15k237") else a.workload
    # loop epochs K: (t(6 + K) - t(6)) / K — the two calls' fixed costs (model build, capture,
    # allocator) vary by a few ms, so K sets the noise: C3 K = 40 read 1.25 and 1.90 ms on one box
    # (profiles/r06_bench_c3*.json), K = 120 holds ~150 ms of epochs against that
    dflt = {"C3": (3, 128, 30, 120), "C2": (2, 128, 10, 40), "C5": (3, 256, 2, 8)}[base]
    a.layers = dflt[0] if a.layers is None else a.layers
    a.feat = dflt[1] if a.feat is None else a.feat
    a.epoch_steps = dflt[2] if a.epoch_steps is None else a.epoch_steps
    a.loop_epochs = dflt[3] if a.loop_epochs is None else a.loop_epochs
    return a


def setup_dist(n):
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n:
        raise SystemExit(f"--gpus {n} but WORLD_SIZE={world}: launch N>1 with torch.distributed.run")
    # rehearsal of the N > 1 flow on a one-GPU box: every rank on device 0 over gloo
    # (MPGNN_BENCH_REHEARSE=1); the numbers of such a run are not a measurement
    rehearse = os.environ.get("MPGNN_BENCH_REHEARSE") == "1"
    # MPGNN_BENCH_FORCE_DIST=1: the sharded path through a real process group even at N = 1
    # (RCCL with one rank: every collective runs, each an identity) — the world-1 RCCL test
    force = os.environ.get("MPGNN_BENCH_FORCE_DIST") == "1"
    if rehearse:
        local = 0
    torch.cuda.set_device(local)
    group = None
    if world > 1 or force:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        group = dist.group.WORLD
    return rank, world, local, group


def _cgroup_cpus():
    """CPUs the cgroup quota grants (cgroup v2 cpu.max / v1 cfs quota), or None if unlimited."""
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            return max(1, -(-int(quota) // int(period)))
    except (OSError, ValueError):
        pass
    try:
        quota = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        period = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if quota > 0:
            return max(1, -(-quota // period))
    except (OSError, ValueError):
        pass
    return None


def usable_cpus():
    """Host threads the CPU baseline may use: the affinity mask, capped by the cgroup quota."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    quota = _cgroup_cpus()
    return (min(aff, quota) if quota else aff), aff, quota


def host_info():
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    use, aff, quota = usable_cpus()
    return {"nproc": os.cpu_count(), "affinity_cpus": aff, "cgroup_quota_cpus": quota, "cpu_model": model,
            "torch_threads": torch.get_num_threads()}


class _cpu_threads:
    """torch's intra-op pool at the usable host CPUs for the CPU baseline (all the
    cores the process may run on), restored afterwards."""

    def __enter__(self):
        self.prev = torch.get_num_threads()
        torch.set_num_threads(usable_cpus()[0])
        return self

    def __exit__(self, *exc):
        torch.set_num_threads(self.prev)


def _median(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2]


def cpu_baseline_full(g, params, layers, reps):
    """Oracle (CPU, the host threads torch uses) on the same graph: 2 warm-ups, `reps` timed
    forwards of the mode-ALL stack; edges/s = layers·E / median time."""
    from oracle import rgcn_oracle as orc
    x, ei, et = g.x, g.edge_index, g.edge_type

    def fwd():
        h = x
        for layer in range(layers):
            p = "conv1." if layer == 0 else "conv2."
            h = torch.relu(orc.rgcn_forward(h, ei, et, params[p + "weight"], params[p + "root"], params[p + "bias"]))
        return h

    with torch.no_grad():
        for _ in range(2):
            fwd()
        times = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fwd()
            times.append(time.perf_counter() - t0)
    med = _median(times)
    return {"value": layers * g.num_edges / med, "unit": "edges/s", "cores": torch.get_num_threads(), "kind": "port",
            **host_info(),
            "sample": f"{reps} timed (after 2 warm-up) forward passes of the {layers}-layer RGCN stack on the full "
                      f"graph (oracle/rgcn_oracle.py, PyG-2.3.1 loop: index_select/scatter_add_/div/mm per relation); "
                      f"median {med * 1e3:.1f} ms"}


def cpu_baseline_rel0(g, params, layers, reps):
    """C2 / C5 mode ALL: the full CPU stack would take minutes to hours (R dense N×F×F GEMMs per
    layer), so the oracle's loop body is timed for ONE relation of the first layer (index_select,
    scatter_add_, div, mm — rgcn_oracle.rgcn_forward's iteration) and scaled by R·layers, plus
    the root GEMM per layer; labelled as extrapolated."""
    from oracle import rgcn_oracle as orc
    w, root = params["conv1.weight"], params["conv1.root"]
    x, ei, et = g.x, g.edge_index, g.edge_type
    size = (x.size(0), x.size(0))
    with torch.no_grad():
        times = []
        for k in range(reps + 2):
            t0 = time.perf_counter()
            tmp = orc.masked_edge_index(ei, et == 0)
            h = orc.propagate_mean(tmp, x, size)
            _ = h @ w[0]
            t_rel = time.perf_counter() - t0
            t0 = time.perf_counter()
            _ = x @ root
            t_root = time.perf_counter() - t0
            if k >= 2:
                times.append((t_rel, t_root))
    t_rel, t_root = _median(times)
    est = layers * (g.num_relations * t_rel + t_root)
    return {"value": layers * g.num_edges / est, "unit": "edges/s", "cores": torch.get_num_threads(), "kind": "port",
            **host_info(),
            "sample": f"oracle loop body for relation 0 of layer 1 ({reps} timed after 2 warm-up, median "
                      f"{t_rel * 1e3:.1f} ms) + root GEMM ({t_root * 1e3:.1f} ms), extrapolated x{g.num_relations} "
                      f"relations x{layers} layers = {est:.1f} s per forward (extrapolated, not run in full)"}


def cpu_baseline_single(g, convs_cpu, metapath, edges, reps):
    """Mode SINGLE: the oracle CustomRGCNConv chain (mp_rgcn_layer.py:225-271: masked_edge_index,
    propagate mean, h @ W, x @ root, bias, ReLU) over the metapath, full graph."""
    from oracle import rgcn_oracle as orc
    x, ei, et = g.x, g.edge_index, g.edge_type

    def fwd():
        h = x
        for conv, rel in zip(convs_cpu, metapath):
            h = torch.relu(orc.custom_rgcn_forward(h, ei, et, rel, conv.weight.detach(), conv.root.detach(),
                                                   conv.bias.detach()))
        return h

    with torch.no_grad():
        for _ in range(2):
            fwd()
        times = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fwd()
            times.append(time.perf_counter() - t0)
    med = _median(times)
    return {"value": edges / med, "unit": "edges/s", "cores": torch.get_num_threads(), "kind": "port", **host_info(),
            "sample": f"{reps} timed (after 2 warm-up) forward passes of the {len(metapath)}-hop CustomRGCNConv chain "
                      f"(oracle/rgcn_oracle.py custom_rgcn_forward) on the full graph; median {med * 1e3:.1f} ms"}


def time_drop_in_loop(single, g, x, ei, et, F, layers, metapath, epochs, shard_kw, dev, group):
    """Per-epoch time of the drop-in training loops as a user of the reference runs them:
    mode ALL = ``mpgnn_amd.main_rgcn.mpgnn_parallel_multiple`` (main_rgcn.py:452-472: per epoch
    train with the class-weighted NLL :376-380, validation forward + macro F1, test forward +
    macro F1, :458-461), mode SINGLE = ``mpgnn_amd.main.mpgnn_parallel_multiple`` (main.py:1117-
    1136: train + validation with F1). Both include their per-epoch host syncs (loss.item-style
    float, the F1 counts). Per epoch = (t(6 + K epochs) - t(6 epochs)) / K: model construction,
    the optimizer and the final test cancel (each of the two times the min of 3 alternated calls).
    Labels: 2 classes, seeded; 60/20/20 node split."""
    from mpgnn_amd import main as mmain
    from mpgnn_amd import main_rgcn as mrg
    n = g.num_nodes
    gen = torch.Generator().manual_seed(0)
    y = torch.randint(0, 2, (n,), generator=gen)
    perm = torch.randperm(n, generator=gen)
    a, b = int(0.6 * n), int(0.8 * n)
    tr, va, te = (perm[:a].sort().values, perm[a:b].sort().values, perm[b:].sort().values)
    d = mmain.Data(x=x, edge_index=ei, edge_type=et, train_idx=tr.to(dev), train_y=y[tr].to(dev),
                   val_idx=va.to(dev), val_y=y[va].to(dev), test_idx=te.to(dev), test_y=y[te].to(dev))
    if shard_kw:
        d.shard_kw = shard_kw
    R = g.num_relations
    if single:
        def run(k):
            return mmain.mpgnn_parallel_multiple(d, F, F, R, F, 2, [metapath], epochs=k)
    else:
        def run(k):
            return mrg.mpgnn_parallel_multiple(d, F, F, R, F, 2, layers, epochs=k, verbose=False)

    def timed(k):
        if group is not None:
            dist.barrier(group=group)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        score = run(k)
        torch.cuda.synchronize()
        return time.perf_counter() - t0, score

    run(6)  # warm-up: plan cached, allocator and kernels warm, one graph capture done (graph pool)
    # the loops run their first 3 epochs eagerly and replay one captured epoch after that
    # (main._epochs): t(6 + K) - t(6) holds K steady-state epochs, the capture cancels
    # min of 3 alternated timings each: one call's fixed costs (model build, capture, allocator)
    # vary by more than K epochs' worth between calls, a single pair misstates the difference
    t1s, tks = [], []
    for _ in range(3):
        t1s.append(timed(6)[0])
        tk, score = timed(6 + epochs)
        tks.append(tk)
    t1, tk = min(t1s), min(tks)
    per = (tk - t1) / epochs
    if group is not None:
        t = torch.tensor([per], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        per = float(t.item())
    if per <= 0:  # the two runs' fixed costs (model build, allocator, capture) did not cancel
        return {"ms": None, "epochs_timed": epochs, "note": "t(6 + K) - t(6) <= 0: not measured (raise --loop-epochs)"}
    fn = "mpgnn_amd.main.mpgnn_parallel_multiple" if single else "mpgnn_amd.main_rgcn.mpgnn_parallel_multiple"
    ref = ("main.py:1117-1136 (train + validation F1 per epoch)" if single else
           "main_rgcn.py:452-472 (weighted-NLL train + validation F1 + test F1 per epoch, :458-461)")
    return {"ms": round(per * 1e3, 4), "epochs_timed": epochs, "loop": fn, "reference": ref,
            "final_score": round(float(score), 4),
            "note": "(t(6+K) - t(6)) / K of the drop-in loop call, each t the min of 3 alternated calls "
                    "(steady-state epochs: after 3 eager epochs the loop "
                    "replays one captured HIP graph per epoch; its prints' host syncs included); synthetic 2-class labels"}


def bench_score(args):
    """Mode score: the metapath score function of the reference's search loop —
    ``score_relation_parallel`` (main.py:727-760): edge dictionary of one relation, then 100
    epochs of train() (model.py:74-89 forward = per-source argmax of the destination weights,
    MSE, backward, Adam, clamp). One STEP = one train() epoch of the drop-in (GPU kernels
    mpgnn_score_argmax / _bwd + torch's MSE / fused Adam / clamp). value = edges scored per
    second = E_r · steps / time (every edge of the relation whose source is in the mask is read
    once per epoch by the argmax). Single GPU (candidate relations are independent: replicas).
    roofline: mpgnn_score_argmax (memset + kernel) per launch, HIP events on the launch stream,
    against HBM with its algorithmic bytes. cpu_baseline: the oracle's reference-style loop
    (oracle/score_oracle.py, the Python dict loop of model.py:82-87) on a bounded number of epochs."""
    import random as _random
    from mpgnn_amd import score as sc
    rank, world, local, group = setup_dist(args.gpus)
    if world > 1:
        raise SystemExit("--mode score shards nothing (candidate relations are replicas)")
    dev = torch.device("cuda", local)
    if args.workload.startswith("fb15k237"):
        g = data.fb15k237_graph(feat_dim=4, seed=0, recipe="relcond" if args.workload == "fb15k237_relcond" else "survey")
    else:
        g = data.config_graph(args.workload)
    N = g.num_nodes
    counts = torch.bincount(g.edge_type, minlength=g.num_relations)
    rel = int(torch.argmax(counts)) if args.relation is None else int(args.relation)
    y = torch.randint(0, 2, (N,), generator=torch.Generator().manual_seed(0))

    class D:
        pass
    d = D()
    d.x = torch.zeros(N, 2)
    d.edge_index, d.edge_type, d.num_nodes = g.edge_index.to(dev), g.edge_type.to(dev), N
    d.labels = y.unsqueeze(-1)
    mask = torch.unique(g.edge_index[0][g.edge_type == rel]).tolist()  # first-iteration mask (main.py:734-735)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ed, dd = sc.create_edge_dictionary(d, rel, mask, BAGS=False, dataset="synthetic")
    _random.seed(0)
    w0 = sc.initialize_weights(d, dd, BAGS=False)
    torch.manual_seed(77)
    model = sc.get_model(w0, 2).to(dev)
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t0
    opt = sc.get_optimizer(model)
    crit, crit_node = sc.get_loss(), sc.get_loss_per_node()
    E_r = ed.num_entries

    def step():
        return sc.train(d, ed, model, opt, crit, mask, crit_node, [], w0, None, BAGS=False, dataset="synthetic")

    for _ in range(max(args.warmup, 1)):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()[0]
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ms = elapsed * 1e3 / args.steps
    # the argmax launch alone (max_weights memset + kernel): 50 calls captured as one HIP graph
    # and replayed between HIP events, so the GPU time is measured, not the host's issue rate
    # of the per-call Python work (eager: ~47 us per call, the kernel a few)
    w = model.input.weights.detach()
    reps, per_graph = 200, 50
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    k_how = "graph"
    with torch.no_grad():
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(5):
                sc.score_argmax(w, ed)
        torch.cuda.current_stream().wait_stream(side)
        try:
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                for _ in range(per_graph):
                    sc.score_argmax(w, ed)
            graph.replay()
            ev0.record()
            for _ in range(reps // per_graph):
                graph.replay()
            ev1.record()
        except RuntimeError:  # capture refused: eager calls (host-bound upper bound)
            k_how = "eager"
            torch.cuda.synchronize()
            ev0.record()
            for _ in range(reps):
                sc.score_argmax(w, ed)
            ev1.record()
    torch.cuda.synchronize()
    k_us = ev0.elapsed_time(ev1) * 1e3 / reps
    K = len(ed)
    alg = E_r * 8.0 + K * (4 + 8 + 12) + N * 4.0
    roofline = {"bound": "hbm", "achieved": round(alg / (k_us * 1e-6) / 1e9, 2), "peak": PEAK_HBM, "unit": "GB/s",
                "frac": round(alg / (k_us * 1e-6) / 1e9 / PEAK_HBM, 5), "traffic": None,
                "kernel": "score_argmax_kernel (+ max_weights memset)", "avg_launch_us": round(k_us, 3),
                "algorithmic": "E_r·(4 dst id + 4 weight) + K·(4 key + 8 ptr + 12 outputs) + N·4 max_weights",
                "timing": f"HIP events around {reps} launches ({'replays of a HIP graph of ' + str(per_graph) + ' calls' if k_how == 'graph' else 'eager calls'})",
                "note": "tiny launch (K sources, E_r edges): bound by launch latency, not HBM"}
    # the whole score_relation_parallel (dictionary build + weights + 100 epochs + final loss.item)
    _random.seed(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sc.score_relation_parallel(d, rel, [], 2, "synthetic")
    srp_s = time.perf_counter() - t0
    cpu = None
    if not args.no_cpu_baseline:
        from oracle import score_oracle as so
        with _cpu_threads():
            ei_c, et_c = g.edge_index, g.edge_type
            ed_o, dd_o = so.create_edge_dictionary(ei_c, et_c, rel, mask, d.labels, "synthetic")
            w_o = so.initialize_weights(N, dd_o, _random.Random(0))
            torch.manual_seed(77)
            m_o = so.Score(w_o, "synthetic", 2)
            o_o = torch.optim.Adam(m_o.parameters(), lr=0.1)
            so.train(m_o, o_o, ed_o, N, d.labels, mask, "synthetic")  # warm-up
            times = []
            for _ in range(max(2, min(args.cpu_reps, 5))):
                t1 = time.perf_counter()
                so.train(m_o, o_o, ed_o, N, d.labels, mask, "synthetic")
                times.append(time.perf_counter() - t1)
        med = _median(times)
        cpu = {"value": E_r / med, "unit": "edges/s", "cores": usable_cpus()[0], "kind": "port", **host_info(),
               "sample": f"{len(times)} epochs (after 1 warm-up) of the oracle's reference-style train() "
                         f"(oracle/score_oracle.py: the per-source Python loop of model.py:82-87, MSE, Adam, clamp), "
                         f"relation {rel} ({E_r} edges, {K} sources); median {med * 1e3:.1f} ms per epoch"}
    result = {
        "metric": "score-function edges scored/sec (main.py:727-760 epochs)", "value": round(E_r * args.steps / elapsed, 1),
        "unit": "edges/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": WORKLOADS[args.workload][1].split(",")[0] + "; 2-class synthetic labels, seed-0 random weights",
        "config": {"workload": f"{WORKLOADS[args.workload][0]}: score function, relation {rel} (the largest), "
                               f"first-iteration mask (all {K} sources)", "mode": "score",
                   "graph": {"nodes": N, "edges_relation": E_r, "sources": K}},
        "epoch_def": "one train() of main.py:641-673 (non-bag): argmax forward, MSE, backward, Adam(lr 0.1), clamp",
        "score_relation_parallel_s": round(srp_s, 4),
        "setup_s": round(setup_s, 4),
        "final_loss": round(float(loss.item()), 6),
        "roofline": roofline,
        "cpu_baseline": cpu,
    }
    print(json.dumps(result), flush=True)
    return result


def bench_score_all(args):
    """Mode score_all: the first round of the metapath search —
    every relation scored by score_relation_parallel (main.py:1309-1330: 100 epochs each, split
    over MPI ranks) — as ONE batched problem (score.score_relations_batched: per epoch one argmax
    launch over every relation's dictionary, one gradient scatter, one fused Adam over the stacked
    [R, N] weights, one clamp; replayed as a HIP graph). One STEP = one epoch of all relations.
    value = edges scored per second = E (every edge of every relation read by the argmax) ·
    epochs / time. Beside it: the per-relation drop-in path (score_relation_parallel per
    relation, its own graph) on a sample of relations, extrapolated; the CPU oracle's per-source
    Python loop on a bounded sample (2 relations × 3 epochs), extrapolated. roofline: the
    all-relation argmax launch (mpgnn_score_argmax_multi) per launch, HIP events around 50 graph-
    captured calls, against HBM with its algorithmic bytes."""
    import random as _random
    from mpgnn_amd import score as sc
    rank, world, local, group = setup_dist(args.gpus)
    if world > 1:
        raise SystemExit("--mode score_all shards nothing (one scoring round is one batched problem per GPU)")
    dev = torch.device("cuda", local)
    g = data.fb15k237_graph(feat_dim=2, seed=0, recipe="survey") if args.workload.startswith("fb15k237") \
        else data.config_graph(args.workload)
    N = g.num_nodes
    rels = torch.unique(g.edge_type).tolist()

    class D:
        pass
    d = D()
    d.x = torch.zeros(N, 2)
    d.edge_index, d.edge_type, d.num_nodes = g.edge_index.to(dev), g.edge_type.to(dev), N
    d.labels = torch.randint(0, 2, (N, 1), generator=torch.Generator().manual_seed(0))
    epochs = 100  # main.py:755
    _random.seed(0)
    torch.manual_seed(77)
    sc.score_relations_batched(d, rels, 2, "synthetic", epochs=5)  # warm-up: dictionaries, capture path
    torch.cuda.synchronize()
    times = []
    for _ in range(max(1, min(args.steps, 3))):
        _random.seed(0)
        torch.manual_seed(77)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = sc.score_relations_batched(d, rels, 2, "synthetic", epochs=epochs)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    total_s = _median(times)
    E = g.num_edges
    # per-relation drop-in path on a sample of relations (evenly spaced), extrapolated by edges
    counts = torch.bincount(g.edge_type).tolist()
    sample = rels[:: max(1, len(rels) // 12)]
    _random.seed(0)
    t0 = time.perf_counter()
    for r in sample:
        sc.score_relation_parallel(d, r, [], 2, "synthetic")
    torch.cuda.synchronize()
    per_rel_sample_s = time.perf_counter() - t0
    per_rel_s = per_rel_sample_s * len(rels) / len(sample)
    # the all-relation argmax launch alone: 50 calls captured once, replayed between HIP events
    rd = sc.RelationDictionaries(d.edge_index, d.edge_type, rels, N, dev)
    K = rd.num_keys
    w = torch.rand(len(rels) * N, device=dev)
    lab = d.labels.reshape(-1).to(dev).float()
    alpha = torch.ones(len(rels), device=dev)
    bufs = [torch.empty(K, dtype=t, device=dev) for t in (torch.int32, torch.int32, torch.float32, torch.float32,
                                                           torch.float32)]

    def one():
        _lib.check(_lib.lib.mpgnn_score_argmax_multi(w.data_ptr(), N, rd.keys_t.data_ptr(), rd.key_ptr_t.data_ptr(),
                                                     rd.dst_t.data_ptr(), rd.key_rel_t.data_ptr(), K, lab.data_ptr(),
                                                     alpha.data_ptr(), *(b.data_ptr() for b in bufs),
                                                     torch.cuda.current_stream(dev).cuda_stream))
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            one()
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(50):
            one()
    graph.replay()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(4):
        graph.replay()
    ev1.record()
    torch.cuda.synchronize()
    k_us = ev0.elapsed_time(ev1) * 1e3 / 200
    alg = E * 8.0 + K * (4 + 8 + 4 + 4 + 20)
    roofline = {"bound": "hbm", "achieved": round(alg / (k_us * 1e-6) / 1e9, 2), "peak": PEAK_HBM, "unit": "GB/s",
                "frac": round(alg / (k_us * 1e-6) / 1e9 / PEAK_HBM, 5), "traffic": None,
                "kernel": "score_multi_argmax_kernel", "avg_launch_us": round(k_us, 3),
                "algorithmic": "E·(4 dst id + 4 weight) + K·(4 key + 8 ptr + 4 relation + 4 label + 20 outputs)",
                "timing": "HIP events around 200 launches (4 replays of a HIP graph of 50 calls)"}
    cpu = None
    if not args.no_cpu_baseline:
        from oracle import score_oracle as so
        with _cpu_threads():
            ei_c, et_c = g.edge_index, g.edge_type
            t_cpu, e_cpu = 0.0, 0
            for r in (rels[0], rels[len(rels) // 2]):
                mask = torch.unique(ei_c[0][et_c == r]).tolist()
                ed_o, dd_o = so.create_edge_dictionary(ei_c, et_c, r, mask, d.labels, "synthetic")
                w_o = so.initialize_weights(N, dd_o, _random.Random(0))
                m_o = so.Score(w_o, "synthetic", 2)
                o_o = torch.optim.Adam(m_o.parameters(), lr=0.1)
                t1 = time.perf_counter()
                for _ in range(3):
                    so.train(m_o, o_o, ed_o, N, d.labels, mask, "synthetic")
                t_cpu += time.perf_counter() - t1
                e_cpu += 3 * int(counts[r])
        cpu = {"value": e_cpu / t_cpu, "unit": "edges/s", "cores": usable_cpus()[0], "kind": "port", **host_info(),
               "sample": f"3 epochs of 2 relations ({e_cpu // 3} edges) through the oracle's reference-style train() "
                         f"(oracle/score_oracle.py, the per-source Python loop of model.py:82-87); "
                         f"{t_cpu:.2f} s, extrapolated: the full round (237 relations x 100 epochs) "
                         f"~{E * epochs / (e_cpu / t_cpu):.0f} s"}
    losses = [r_[1] for r_ in res]
    result = {
        "metric": "score-function edges scored/sec, every relation of one search round (main.py:1309-1330)",
        "value": round(E * epochs / total_s, 1), "unit": "edges/s", "n_gpus": 1, "steps": epochs, "warmup": 5,
        "ms_per_step": round(total_s * 1e3 / epochs, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32",
        "data": WORKLOADS[args.workload][1].split(",")[0] + "; 2-class synthetic labels, seeded random weights",
        "config": {"workload": f"{WORKLOADS[args.workload][0]}: all {len(rels)} relations x {epochs} epochs, "
                               "first-iteration masks (every source of each relation)", "mode": "score_all",
                   "graph": {"nodes": N, "edges": E, "relations": len(rels), "keys": K}},
        "epoch_def": "one train() epoch of main.py:641-673 (non-bag) for EVERY relation: argmax forward, MSE, "
                     "backward, Adam(lr 0.1), clamp",
        "round_s": round(total_s, 4),
        "per_relation_path_s": round(per_rel_s, 3),
        "per_relation_path_def": f"score_relation_parallel per relation (its own HIP-graph loop), {len(sample)} "
                                 f"relations timed ({per_rel_sample_s:.3f} s), x {len(rels)}/{len(sample)}",
        "speedup_vs_per_relation": round(per_rel_s / total_s, 2),
        "losses_finite": int(sum(1 for v in losses if v == v)),
        "roofline": roofline,
        "cpu_baseline": cpu,
    }
    print(json.dumps(result), flush=True)
    return result


def bench_score_bags(args):
    """Mode score_bags (the bag branch): score_relation_bags_parallel (main.py:853-917)
    — restarts of 50 train(BAGS=True) epochs (model.py:45-72: per bag, per member source, the
    first argmax of weights · LinearLayerAttri(feat), the strict-max pick) until two restarts fail
    to lower the loss — for the candidate relation, on bags made by create_bags (main.py:545-575)
    from a first non-bag scoring of the largest relation. One STEP = one train() epoch. value =
    edges scored per second = Σ over the bags' member sources of their destination counts ·
    epochs / time. roofline: mpgnn_score_bag_argmax per launch (HIP events around 50 graph-
    captured calls) against HBM with its algorithmic bytes. cpu_baseline: the oracle's per-bag
    Python loop (oracle/score_oracle.py train_bags) on 3 epochs."""
    import random as _random
    from mpgnn_amd import score as sc
    rank, world, local, group = setup_dist(args.gpus)
    if world > 1:
        raise SystemExit("--mode score_bags shards nothing (candidate relations are replicas)")
    dev = torch.device("cuda", local)
    g = data.fb15k237_graph(feat_dim=2, seed=0, recipe="survey") if args.workload.startswith("fb15k237") \
        else data.config_graph(args.workload)
    N = g.num_nodes
    counts = torch.bincount(g.edge_type, minlength=g.num_relations)
    order = torch.argsort(counts, descending=True, stable=True).tolist()
    rel0 = order[0]

    class D:
        pass
    d = D()
    gen = torch.Generator().manual_seed(0)
    d.x = torch.nn.functional.one_hot(torch.randint(0, 2, (N,), generator=gen), 2).float()  # colour features
    d.edge_index, d.edge_type, d.num_nodes = g.edge_index.to(dev), g.edge_type.to(dev), N
    d.labels = torch.randint(0, 2, (N, 1), generator=gen)
    mask = torch.unique(g.edge_index[0][g.edge_type == rel0]).tolist()
    ed0, dd0 = sc.create_edge_dictionary(d, rel0, mask, BAGS=False, dataset="synthetic")
    sc.create_bags(ed0, dd0, d)
    # the candidate: the relation whose edges start from the most bag members
    members = torch.tensor(sorted({n for b in d.bags for n in b}))
    src_in = torch.isin(g.edge_index[0], members)
    rel = int(torch.argmax(torch.bincount(g.edge_type[src_in], minlength=g.num_relations)))
    trace = []
    _random.seed(0)
    torch.manual_seed(5)
    sc.score_relation_bags_parallel(d, rel, 2, "synthetic", trace=trace)  # warm-up + epoch count
    n_epochs = len(trace)
    times = []
    for _ in range(max(1, min(args.steps, 3))):
        _random.seed(0)
        torch.manual_seed(5)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r_, cur, model, preds, v = sc.score_relation_bags_parallel(d, rel, 2, "synthetic")
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    run_s = _median(times)
    # the bags / dictionary the epochs ran on, and the edges one epoch reads
    mask_b = list(dict.fromkeys(n for b in d.bags for n in b))
    edb, _ = sc.create_edge_dictionary(d, rel, mask_b, BAGS=True, dataset="synthetic")
    cb, cl = sc.clean_bags_for_relation_type(d, edb)
    bs = sc.BagSet(cb, edb)
    kp = edb.key_ptr_t.long()
    mk = bs.mem_key.long()
    deg = torch.where(mk >= 0, kp[mk.clamp(min=0) + 1] - kp[mk.clamp(min=0)], torch.zeros_like(mk))
    edges_epoch = int(deg.sum())
    w = torch.rand(N, 1, device=dev)
    lin = torch.rand(1, 2, device=dev)
    feat = d.x.to(dev)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side), torch.no_grad():
        for _ in range(3):
            sc.score_bag_argmax(w, lin, feat, bs)
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph), torch.no_grad():
        for _ in range(50):
            sc.score_bag_argmax(w, lin, feat, bs)
    graph.replay()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(4):
        graph.replay()
    ev1.record()
    torch.cuda.synchronize()
    k_us = ev0.elapsed_time(ev1) * 1e3 / 200
    B, M = bs.num_bags, bs.num_members
    alg = edges_epoch * 8.0 + M * (4 + 4 + 8 + 8 + 16) + B * (8 + 12)
    roofline = {"bound": "hbm", "achieved": round(alg / (k_us * 1e-6) / 1e9, 2), "peak": PEAK_HBM, "unit": "GB/s",
                "frac": round(alg / (k_us * 1e-6) / 1e9 / PEAK_HBM, 5), "traffic": None,
                "kernel": "score_bag_argmax_kernel (+ its output allocations)", "avg_launch_us": round(k_us, 3),
                "algorithmic": "edges·(4 dst + 4 weight) + M·(node, key, key_ptr, feature row, 4 outputs) + B·(ptr, "
                               "3 outputs)",
                "timing": "HIP events around 200 calls (4 replays of a HIP graph of 50)",
                "note": "small launch (B bags, M members): bound by launch latency and the bag-serial member walk"}
    cpu = None
    if not args.no_cpu_baseline:
        from oracle import score_oracle as so
        with _cpu_threads():
            ed_o, dd_o = so.create_edge_dictionary_bags(g.edge_index, g.edge_type, rel, mask_b, d.bags, d.bag_labels)
            cb_o, cl_o = so.clean_bags_for_relation_type(d.bags, d.bag_labels, ed_o)
            torch.manual_seed(5)
            m_o = so.Score(so.initialize_weights(N, dd_o, _random.Random(0)), "synthetic", 2)
            o_o = torch.optim.Adam(m_o.parameters(), lr=0.1)
            gm = torch.ones(N, 1)
            t1 = time.perf_counter()
            for _ in range(3):
                so.train_bags(m_o, o_o, ed_o, cb_o, cl_o, d.x, [], None, gm)
            t_cpu = (time.perf_counter() - t1) / 3
        cpu = {"value": edges_epoch / t_cpu, "unit": "edges/s", "cores": usable_cpus()[0], "kind": "port",
               **host_info(),
               "sample": f"3 epochs of train(BAGS=True) through the oracle (oracle/score_oracle.py train_bags: the "
                         f"per-bag, per-source Python loop of model.py:56-70 + autograd), relation {rel}: "
                         f"{t_cpu * 1e3:.1f} ms per epoch"}
    result = {
        "metric": "bag score edges scored/sec (score_relation_bags_parallel, main.py:853-917)",
        "value": round(edges_epoch * n_epochs / run_s, 1), "unit": "edges/s", "n_gpus": 1, "steps": n_epochs,
        "warmup": n_epochs, "ms_per_step": round(run_s * 1e3 / n_epochs, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": WORKLOADS[args.workload][1].split(",")[0] + "; one-hot 2-colour features, 2-class synthetic labels",
        "config": {"workload": f"{WORKLOADS[args.workload][0]}: bags from create_bags over relation {rel0}'s "
                               f"dictionaries, candidate relation {rel}", "mode": "score_bags",
                   "bags": B, "members": M, "edges_per_epoch": edges_epoch, "epochs_run": n_epochs,
                   "restarts": n_epochs // 50},
        "epoch_def": "one train(BAGS=True) of main.py:641-673: bag-pick forward, MSE, backward, grad mask, "
                     "Adam(lr 0.1), clamps",
        "run_s": round(run_s, 4), "current_loss": cur, "v": bool(v),
        "roofline": roofline,
        "cpu_baseline": cpu,
    }
    print(json.dumps(result), flush=True)
    return result


def pmc_traffic(workload, mode, feat, kernel_prefix):
    """HBM bytes per launch of `kernel_prefix` from the committed PMC summary, or None."""
    rows = []
    for rnd in ("r06", "r05", "r04", "r03", "r02"):  # the newest round's PMC summary first
        try:
            rows += json.load(open(os.path.join(ROOT, "profiles", f"{rnd}_pmc_traffic.json")))
        except (OSError, ValueError):
            pass
    for r in rows:
        if r.get("workload") == workload and r.get("mode") == mode and r.get("feat") == feat and \
                r.get("kernel", "").startswith(kernel_prefix):
            return r.get("hbm_bytes_per_launch")
    return None


def main():
    args = parse()
    # A/B hook: library option defaults "K=V,K=V" (include/mpgnn_rgcn.h enum mpgnn_option), set
    # before any plan exists; recorded in the line's config
    ab_opts = os.environ.get("MPGNN_BENCH_SET_OPT", "")
    for kv in filter(None, ab_opts.split(",")):
        k, v = kv.split("=")
        _lib.set_option(int(k), int(v))
    _lib.set_option(24, 1 if args.gemm == "bf3" else 0)  # MPGNN_OPT_GEMM_BF3
    _lib.set_option(25, args.bwd_fused)  # MPGNN_OPT_BWD_FUSED
    if args.chunk_rows is not None:
        _lib.set_option(20, args.chunk_rows)  # MPGNN_OPT_CHUNK_ROWS (before the plan is built)
    if args.mode == "score":
        return bench_score(args)
    if args.mode == "score_all":
        return bench_score_all(args)
    if args.mode == "score_bags":
        return bench_score_bags(args)
    rank, world, local, group = setup_dist(args.gpus)
    sharded = group is not None
    dev = torch.device("cuda", local)
    if args.workload.startswith("fb15k237"):
        g = data.fb15k237_graph(feat_dim=args.feat, seed=0,
                                recipe="relcond" if args.workload == "fb15k237_relcond" else "survey")
    else:
        g = data.config_graph(args.workload)
        if g.x.shape[1] != args.feat:
            g.x = torch.rand((g.num_nodes, args.feat), generator=torch.Generator().manual_seed(1))
    F = args.feat
    x, ei, et = g.x.to(dev), g.edge_index.to(dev), g.edge_type.to(dev)
    single = args.mode == "single"
    shard = ranges = None
    side = args.shard_side
    if sharded:
        ranges = shard_ranges(g.edge_index, g.num_nodes, world, side=side)
        shard = ranges[rank]
    torch.manual_seed(10)  # main_rgcn.py:31 / main.py:31-style seeding of the init
    rel_counts = torch.bincount(g.edge_type, minlength=g.num_relations)
    if single:
        if args.metapath:
            metapath = [int(v) for v in args.metapath.split(",")]
        elif args.workload == "C2":
            metapath = [1, 0]
        elif args.workload == "C5":
            metapath = [2, 1, 0]
        else:
            metapath = [int(v) for v in torch.argsort(rel_counts, descending=True, stable=True)[:3]]
        model_cpu = mpgnn_amd.MPNetm(F, F, g.num_relations, F, 2, 1, [metapath])
        model = mpgnn_amd.MPNetm(F, F, g.num_relations, F, 2, 1, [metapath])
        model.load_state_dict(model_cpu.state_dict())
        model = model.to(dev).eval()
        convs = list(model.layers_list[0])
        edges_per_step = int(sum(int(rel_counts[r]) for r in metapath))
        if sharded:
            raise SystemExit("--mode single shards nothing (MPGNN candidates are replicas: distributed.metapath_fanout)")

        def step():
            h = x
            for li, (conv, rel) in enumerate(zip(convs, metapath)):
                h = conv(li, rel, h, ei, et, activation="relu")  # F.relu(conv(...)), model.py:211,214
            return h
        layers = len(metapath)
    else:
        model_cpu = mpgnn_amd.Net(F, F, g.num_relations, F, 2, args.layers)
        model = mpgnn_amd.Net(F, F, g.num_relations, F, 2, args.layers)
        model.load_state_dict(model_cpu.state_dict())
        model = model.to(dev)
        convs = [model.conv1] + [model.conv2] * (args.layers - 1)
        edges_per_step = args.layers * g.num_edges
        layers = args.layers

        def step():
            if sharded:  # partial sums per rank, reduce-scatter per layer (or all-gather of rows)
                return sharded_stack_forward(convs, x, ei, et, ranges, group, shard_side=side)
            h = x
            for conv in convs:
                h = conv(h, ei, et, activation="relu")  # F.relu(conv(...)), model.py:144,146
            return h

    # N > 1 (sharded, mode ALL): the steps run with two passes in flight — each layer's
    # reduce-scatter (RCCL, its own stream) overlaps the other pass's layer on the compute stream;
    # every pass is the single-pass computation (bit-identical, tests/test_distributed_gloo.py)
    inflight = int(os.environ.get("MPGNN_BENCH_INFLIGHT", "2")) if sharded and not single else 1

    def run_steps(k):
        if inflight > 1:
            sharded_stack_forwards(convs, x, ei, et, ranges, group, steps=k, inflight=inflight, shard_side=side)
            return
        for _ in range(k):
            step()

    # plan (built once per graph, cached) + warm-up
    t_plan = time.perf_counter()
    with torch.no_grad():
        step()
    torch.cuda.synchronize()
    first_step_s = time.perf_counter() - t_plan
    # Clock pre-warm (untimed, like the plan build): back-to-back steps for >= PREWARM_S seconds.
    # The chip leaves its idle clocks only over the first ~0.1-0.2 s of sustained load: the same
    # 20 timed steps ran 307 us/step right after a 5-step warm-up and 269-275 us/step once the GPU
    # had been busy for ~0.2 s (scripts/step_probe.py, profiles/r06_step_probe_c3.json), so a
    # 6-ms timed region straight after a short warm-up measures the ramp, not the kernels.
    prewarm_s = float(os.environ.get("MPGNN_BENCH_PREWARM_S", "0.3"))
    n_prewarm = 0
    t_pw = time.perf_counter()
    with torch.no_grad():
        while prewarm_s > 0:
            run_steps(10)
            n_prewarm += 10
            torch.cuda.synchronize()
            more = torch.tensor([1 if time.perf_counter() - t_pw < prewarm_s else 0], dtype=torch.int32)
            if group is not None:  # every rank runs the same number of steps (collectives inside step)
                if dist.get_backend(group) == "nccl":
                    more = more.to(dev)
                dist.all_reduce(more, op=dist.ReduceOp.MAX, group=group)
            if int(more.item()) == 0:
                break
    prewarm = {"s": round(time.perf_counter() - t_pw, 3), "steps": n_prewarm,
               "why": "untimed back-to-back steps before the warm-up so the timed region runs at the "
                      "clocks the chip holds under sustained load (MPGNN_BENCH_PREWARM_S, default 0.3)"}
    with torch.no_grad():
        run_steps(max(args.warmup, 1))
    torch.cuda.synchronize()
    plan = mpgnn_amd.get_plan(ei, et, g.num_nodes, shard=shard, device=dev,
                              shard_side=side if shard is not None else "gathered")

    # ---- timed region: K forward steps --------------------------------------------------
    if group is not None:
        dist.barrier(group=group)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.no_grad():
        run_steps(args.steps)
    torch.cuda.synchronize()
    if group is not None:
        dist.barrier(group=group)
    elapsed = time.perf_counter() - t0

    # ---- per-kernel pass: every kernel kind bracketed by HIP events on its launch stream (kept
    # out of the timed region: an event pair between kernels drains the queue)
    _lib.lib.mpgnn_timing_reset()
    _lib.lib.mpgnn_timing_enable(1)
    with torch.no_grad():
        for _ in range(args.steps):
            step()
    torch.cuda.synchronize()
    _lib.lib.mpgnn_timing_enable(0)
    # mode SINGLE at F = 256 (rgcn_kernels.hip root_epi): root items finish the segment-less rows
    root_epi = bool(single and F == 256 and not sharded)
    kinds = {"mean": "segment means (flat_rows_kernel over the multi-edge segments)",
             "seg_fwd": ("split-K transform GEMM of the whole layer (single_bf3_kernel)"
                         if single and args.gemm == "bf3" and F in (64, 128) and not sharded else
                         "transform GEMM (rel_gemm_bf3_kernel / rel_gemm_bf3w_kernel at F = 256 / rel_gemm_kernel)"),
             "row_fwd": (("rows with a segment: single_fix_kernel (the root items' epilogue finished the others)"
                          if root_epi else "combine / output (single_combine_kernel: node -> segment map, one "
                          "streaming pass)") if single else
                         "combine / output (flat_rows_kernel over the augmented row-major list)"),
             "final": "split-row finalize", "piece": "ordered pieces"}
    per_layer = {}
    for kind, label in kinds.items():
        k_ms, k_n = _lib.kernel_timing(kind)
        if k_n:
            per_layer[kind] = {"what": label, "us_per_layer": round(k_ms * 1e3 / (args.steps * layers), 2),
                               "launches_per_layer": round(k_n / (args.steps * layers), 2)}
    if group is not None:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        elapsed = float(t.item())
    ms_per_step = elapsed * 1e3 / args.steps
    value = edges_per_step * args.steps / elapsed

    # ---- rooflines per forward kernel kind (per layer, this rank; first layer's selection) ----
    mode_id = _lib.MODE_SINGLE if single else _lib.MODE_ALL
    sel_rel = metapath[0] if single else -1
    seg_b, seg_e = plan.select(mode_id, sel_rel, g.num_relations)
    S = seg_e - seg_b
    Sm = plan.hsave_rows(mode_id, sel_rel, g.num_relations)
    m_ptr = plan.table("m_ptr")
    rel_m = plan.table("rel_m_ptr")
    d_lo = int(torch.searchsorted(torch.from_numpy(plan.table("rel_seg_ptr")).to(torch.int64), seg_b).item())
    m_lo = int(rel_m[d_lo]) if len(rel_m) else 0
    Em = int(m_ptr[m_lo + Sm] - m_ptr[m_lo]) if Sm else 0
    n_rows = plan.num_nodes if not sharded else (shard[1] - shard[0])
    E_layer = (edges_per_step // layers) if not single else int(rel_counts[metapath[0]])
    model_costs = {
        "seg_fwd": ("mfma", 2.0 * (S + n_rows) * F * F, "2·(S + N)·F_in·F_out: segment rows (mean @ W_r) + node rows "
                    "(x @ root)"),
        "mean": ("hbm", Em * (4.0 * F + 4) + Sm * (4.0 * F + 8), "Em·(4F + 4) gathered x rows + col ids of the "
                 "multi-edge segments, Sm·(4F + 8) mean rows written + counts / pointers"),
        "row_fwd": (("hbm", S * (12.0 * F + 4), "S·(12F + 4): Y rows + s_row read, the segment rows of out read "
                     "and written") if root_epi else
                    ("hbm", (S + n_rows) * (4.0 * F + 4) + n_rows * 4.0 * F, "(S + N)·(4F + 4) Y / Y_root rows + ids "
                     "gathered, N·4F output rows written")),
    }
    # the transform on the bf16-split matrix cores: rel_gemm_bf3_kernel (mode ALL), mode SINGLE
    # unsharded: single_bf3_kernel (split-K: x @ root and mean @ W halves, one launch per layer)
    # (F = 256, mode ALL: rel_gemm_bf3w_kernel, the split-K form of the same six-product scheme)
    # (F = 256, mode SINGLE unsharded, round 5: rel_gemm_bf3w_kernel with the root epilogue)
    bf3 = args.gemm == "bf3" and ((F in (64, 128) and (not single or not sharded)) or
                                  (F == 256 and (not single or root_epi)))
    rooflines = []
    for kind, (bound, work, model_txt) in model_costs.items():
        if kind not in per_layer:
            continue
        us = per_layer[kind]["us_per_layer"]
        extra = {}
        if bound == "mfma" and bf3:
            # the transform on the bf16 matrix cores: 6 bf16 MFMA products per fp32 product (exact
            # 3-way operand split) — priced against the dense bf16 peak with the flops it issues
            ach = 6.0 * work / (us * 1e-6) / 1e12
            peak, unit = PEAK_BF16_MFMA, "TFLOP/s"
            fp32_eq = work / (us * 1e-6) / 1e12
            extra = {"hw_flops_per_launch": 6.0 * work, "fp32_equivalent_TFLOPs": round(fp32_eq, 2),
                     "frac_of_fp32_mfma_peak": round(fp32_eq / PEAK_FP32_MFMA, 4),
                     "path": "v_mfma_f32_32x32x16_bf16, fp32 operands split a = a0 + a1 + a2 (bf16, exact), "
                             "6 products (a0b0 | a2b0 + a1b1 + a0b2 + a1b0 + a0b1), fp32 accumulation"}
        elif bound == "mfma":
            ach = work / (us * 1e-6) / 1e12
            peak, unit = PEAK_FP32_MFMA, "TFLOP/s"
            extra = {"path": "v_mfma_f32_32x32x2_f32"}
        else:
            ach = work / (us * 1e-6) / 1e9
            peak, unit = PEAK_HBM, "GB/s"
        seg_name = ("single_bf3_kernel" if bf3 and single and F != 256 else
                    ("rel_gemm_bf3w_kernel" if F == 256 else "rel_gemm_bf3_kernel") if bf3 else "rel_gemm_kernel")
        kname = {"seg_fwd": seg_name, "mean": "flat_rows_kernel",
                 "row_fwd": ("single_fix_kernel" if root_epi else "single_combine_kernel") if single
                 else "flat_rows_kernel"}[kind]
        rooflines.append({"kind": kind, "kernel": kname, "bound": bound, "achieved": round(ach, 2), "peak": peak,
                          "unit": unit, "frac": round(ach / peak, 4), "us_per_layer": us,
                          "share_of_layer": None, "algorithmic": model_txt,
                          ("alg_flops_per_launch" if bound == "mfma" else "alg_bytes_per_launch"): work, **extra})
    total_us = sum(v["us_per_layer"] for v in per_layer.values())
    for r in rooflines:
        r["share_of_layer"] = round(r["us_per_layer"] / total_us, 3) if total_us else None
    dom = max(rooflines, key=lambda r: r["us_per_layer"]) if rooflines else None
    roofline = None
    if dom is not None:
        mode_tag = "single" if single else "all"
        traffic = pmc_traffic(args.workload, mode_tag, F, "mpgnn::" + dom["kernel"]) if not sharded else None
        roofline = {"bound": dom["bound"], "achieved": dom["achieved"], "peak": dom["peak"], "unit": dom["unit"],
                    "frac": dom["frac"], "traffic": traffic, "kernel": dom["kernel"], "kind": dom["kind"],
                    **{k: dom[k] for k in ("fp32_equivalent_TFLOPs", "frac_of_fp32_mfma_peak", "path") if k in dom},
                    "avg_launch_us": dom["us_per_layer"], "share_of_layer": dom["share_of_layer"],
                    "algorithmic": dom["algorithmic"],
                    "note": "dominant kernel of the forward layer by the per-kernel HIP-event pass (events on the "
                            "launch stream, one pair per launch; the headline timed region has none); traffic = "
                            "PMC FETCH_SIZE x2 + WRITE_SIZE per launch (profiles/r06_pmc_traffic.json; older rounds for kernels not re-profiled)"}
        # SURVEY 8d whole-step HBM roofline of the aggregation (kept beside the kernel roofline)
    b_edge = 4 * F + 4
    hbm_roofline = {"bound": "hbm", "bytes_per_edge": b_edge,
                    "alg_bytes_per_step": edges_per_step * b_edge + layers * (S * 8 + g.num_nodes * 4 * F),
                    "note": f"SURVEY 8d: B = E_l·(4·F + 4) + S_l·8 + N·4·F per layer ({b_edge} B per edge at F={F}); "
                            "at C3 x stays in L2/MALL, so the gathers are bound on-die, not by HBM"}
    hbm_roofline["achieved_GBps"] = round(hbm_roofline["alg_bytes_per_step"] / (ms_per_step * 1e-3) / 1e9, 1)
    hbm_roofline["frac"] = round(hbm_roofline["achieved_GBps"] / PEAK_HBM, 4)

    # ---- the same step replayed as one HIP graph (launch overhead removed) ---------------
    graph = None
    if not sharded:
        try:
            s_cap = torch.cuda.Stream()
            s_cap.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s_cap), torch.no_grad():
                for _ in range(2):  # workspace / allocator warm-up on the capture stream
                    step()
            torch.cuda.current_stream().wait_stream(s_cap)
            torch.cuda.synchronize()
            cg = torch.cuda.CUDAGraph()
            with torch.cuda.graph(cg, stream=s_cap), torch.no_grad():  # the warmed-up stream's workspace
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
                     "note": "same forward captured once with torch.cuda.graph (hipGraph) and replayed: every "
                             "kernel runs every step, host launch overhead removed"}
        except Exception as e:  # capture unsupported here: report, keep the eager number
            graph = {"error": f"{type(e).__name__}: {e}"[:200]}
        cg = None
        mpgnn_amd.functional.release_workspaces()
        torch.cuda.empty_cache()

    # ---- epoch: train fwd + NLL + bwd + Adam, then a validation forward --------------------
    opt = mpgnn_amd.main._adam(model)  # Adam(lr 0.01, wd 5e-4), fused multi-tensor kernel on the GPU
    y = torch.randint(0, 2, (g.num_nodes,), generator=torch.Generator().manual_seed(0)).to(dev)
    train_idx = torch.arange(0, g.num_nodes, 3, device=dev)
    train_y = y[train_idx]  # data.train_y of the reference loops: labels indexed once

    def fwd_model():
        if single:
            return model(x, ei, et)
        return model(x, ei, et, shard=shard, group=group, shard_side=side)

    def epoch():
        model.train()
        opt.zero_grad()
        out = fwd_model()
        loss = mpgnn_amd.metrics.nll_loss_rows(out, train_idx, train_y)
        loss.backward()
        opt.step()
        model.eval()
        with torch.no_grad():
            fwd_model()

    epoch_ms = None
    if args.epoch_steps > 0:
        for _ in range(3):
            epoch()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.epoch_steps):
            epoch()
        torch.cuda.synchronize()
        epoch_ms = (time.perf_counter() - t1) * 1e3 / args.epoch_steps
        if group is not None:
            t = torch.tensor([epoch_ms], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
            epoch_ms = float(t.item())
    model.eval()

    # ---- the same epoch captured once as a HIP graph (host issue removed) -------------------
    epoch_graph = None
    if args.epoch_steps > 0 and not sharded:
        try:
            if single:
                netg = mpgnn_amd.MPNetm(F, F, g.num_relations, F, 2, 1, [metapath]).to(dev)
            else:
                netg = mpgnn_amd.Net(F, F, g.num_relations, F, 2, args.layers).to(dev)
            netg.load_state_dict(model.state_dict())
            optg = mpgnn_amd.main._adam_graphable(netg)  # LeanAdam: the HIP step, capturable

            def epoch_g():
                netg.train()
                out = netg(x, ei, et)
                loss = mpgnn_amd.metrics.nll_loss_rows(out, train_idx, train_y)
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
            with torch.cuda.graph(cg_e, stream=s_cap):
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

    # ---- the reference's whole epoch, through the drop-in loops ------------------------------
    loop = None
    if args.loop_epochs > 0:
        shard_kw = dict(shard=shard, group=group, shard_side=side) if sharded else None
        loop = time_drop_in_loop(single, g, x, ei, et, F, args.layers, metapath if single else None,
                                 args.loop_epochs, shard_kw, dev, group)

    result = None
    if rank == 0:
        cpu = None
        if not sharded and not args.no_cpu_baseline:
            with _cpu_threads():
                if single:
                    convs_cpu = list(model_cpu.layers_list[0])
                    cpu = cpu_baseline_single(g, convs_cpu, metapath, edges_per_step, args.cpu_reps)
                else:
                    params = {k: v.detach() for k, v in model_cpu.state_dict().items()}
                    if args.workload.startswith("fb15k237"):
                        cpu = cpu_baseline_full(g, params, args.layers, args.cpu_reps)
                    else:
                        cpu = cpu_baseline_rel0(g, params, args.layers, args.cpu_reps)
        if single:
            what = (f"MPNetm metapath chain (mode A, CustomRGCNConv x{layers}), metapath={metapath}, "
                    f"F_in=F_hidden={F}")
        else:
            what = f"RGCN Net stack forward (mode B), L={layers}, F_in=F_hidden=F_out={F}"
        if not sharded:
            par = "single GPU"
        elif side == "gathered":
            par = (f"node_2-range shards x{world} (gathered node, edge-balanced; SURVEY 8e): partial sums per rank, "
                   "one RCCL reduce-scatter per layer + one all-gather, issued asynchronously with two passes in "
                   "flight (a pass's collective overlaps the other pass's layer; epoch: per-layer all-reduce of the "
                   "partial output, gradient all-reduces)")
        else:
            par = (f"node_1-range shards x{world} (aggregating node, edge-balanced): complete rows per rank, one "
                   "RCCL all-gather per layer")
        result = {
            "metric": METRIC, "value": round(value, 1), "unit": "edges/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": WORKLOADS[args.workload][1],
            "config": {"workload": WORKLOADS[args.workload][0] + ": " + what, "mode": args.mode,
                       "graph": {"nodes": g.num_nodes, "relations": g.num_relations, "edges": g.num_edges,
                                 "edges_per_step": edges_per_step, "segments_layer1": S,
                                 "multi_edge_segments_layer1": Sm},
                       "parallelism": par, "shard_side": side if sharded else None,
                       "library_options": ab_opts or None},
            "graph_replay": graph,
            "epoch_ms": round(epoch_ms, 3) if epoch_ms is not None else None,
            "epoch_graph": epoch_graph,
            "epoch_def": ("kernel epoch: train (fwd + unweighted NLL + bwd + Adam) + one no-grad validation "
                          "forward, no F1 scoring, no host sync (the reference's full epoch is loop_epoch)"),
            "loop_epoch": loop,
            "first_step_s": round(first_step_s, 3),
            "prewarm": prewarm,
            "passes_in_flight": inflight,
            "first_step_def": ("graph plan built on the GPU from the resident edge tensors "
                               "(mpgnn_plan_create_device) + first forward"
                               if os.environ.get("MPGNN_PLAN_BUILD", "") != "host" else
                               "host plan build + upload + first forward"),
            "roofline": roofline,
            "roofline_kernels": rooflines,
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
