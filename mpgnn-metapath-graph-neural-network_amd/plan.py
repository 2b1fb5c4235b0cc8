"""GraphPlan — the sorted segment tables of one (edge_index, edge_type) graph.

Replaces the per-call, per-relation compaction ``edge_index[:, edge_type == r]``
(mp_rgcn_layer.py:29-35, :231, and the RGCNConv loop ≙ :250-251) with a one-time build
(csrc/plan.cpp) that is uploaded to the GPU and cached across the 999 training epochs of
``mpgnn_parallel_multiple`` (main.py:1121) keyed by tensor identity and ``_version``.
"""
from __future__ import annotations

import ctypes
import os
import threading
import weakref
from collections import OrderedDict

import numpy as np
import torch

from . import _lib
from ._lib import check, lib

FLOWS = ("target_to_source", "source_to_target")


class GraphPlan:
    """Host + device segment tables for one graph (optionally one dst-range shard)."""

    def __init__(self, edge_index: torch.Tensor, edge_type: torch.Tensor, num_nodes: int,
                 shard: tuple[int, int] | None = None, flow: str = "target_to_source",
                 shard_side: str = "gathered", build: str = "auto", device=None):
        """build: "host" (csrc/plan.cpp, multi-threaded counting sorts), "device" (csrc/
        plan_device.hip, radix sorts on the GPU; the plan is then resident on that device) or
        "auto" = "device" when edge_index is a CUDA tensor (MPGNN_PLAN_BUILD=host forces the host
        build). Both give bit-identical tables. ``device``: the GPU the plan must live on (the
        features' device; default: edge_index's) — the edge tensors are copied there for the
        build. If the device build runs out of memory outside PyTorch's caching allocator
        ("auto" only), the plan is built on the host and uploaded instead."""
        if flow not in FLOWS:
            raise ValueError(f"Expected 'flow' to be either {FLOWS} (got '{flow}')")
        if edge_index.dim() != 2 or edge_index.size(0) != 2:
            raise ValueError(f"edge_index must be [2, E], got {tuple(edge_index.shape)}")
        if edge_type.dim() != 1 or edge_type.numel() != edge_index.size(1):
            raise ValueError("edge_type must be [E] matching edge_index")
        if build not in ("auto", "host", "device"):
            raise ValueError(f"build must be 'auto', 'host' or 'device', got {build!r}")
        on_device = build == "device" or (build == "auto" and edge_index.is_cuda
                                          and os.environ.get("MPGNN_PLAN_BUILD", "") != "host")
        dev = None
        if on_device:
            if device is not None and torch.device(device).type == "cuda":
                dev = torch.device(device)
                if dev.index is None:
                    dev = torch.device("cuda", torch.cuda.current_device())
            else:
                dev = edge_index.device if edge_index.is_cuda else torch.device("cuda", torch.cuda.current_device())
        ei = edge_index.detach().to(dev if on_device else "cpu", torch.int64)
        if flow == "source_to_target":  # aggregate into edge_index[1]: swap the roles
            ei = ei.flip(0)
        ei = ei.contiguous()
        et = edge_type.detach().to(dev if on_device else "cpu", torch.int64).contiguous()
        self.num_nodes = int(num_nodes)
        self.flow = flow
        lo, hi = shard if shard is not None else (0, self.num_nodes)
        self.shard = (int(lo), int(hi))
        if shard_side not in _lib.SHARD_SIDES:
            raise ValueError(f"shard_side must be one of {tuple(_lib.SHARD_SIDES)}")
        self.shard_side = shard_side
        handle = ctypes.c_void_p()
        self._device = None
        if on_device:
            # returns after the build has finished on the stream: ei / et may be freed after it
            st = lib.mpgnn_plan_create_device(ei.data_ptr() if ei.numel() else None,
                                              et.data_ptr() if et.numel() else None,
                                              et.numel(), self.num_nodes, self.shard[0], self.shard[1],
                                              _lib.SHARD_SIDES[shard_side], dev.index,
                                              ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream),
                                              ctypes.byref(handle))
            if st == _lib.MPGNN_ERR_ALLOC and build == "auto":
                # the builder's scratch is raw hipMalloc: with PyTorch's cache holding the device,
                # fall back to the host build (uploaded below by to_device)
                on_device = False
                ei, et = ei.cpu(), et.cpu()
            else:
                check(st, "mpgnn_plan_create_device")
                self._device = dev.index
        if not on_device:
            check(lib.mpgnn_plan_create_sharded(ei.data_ptr() if ei.numel() else None,
                                                et.data_ptr() if et.numel() else None,
                                                et.numel(), self.num_nodes, self.shard[0], self.shard[1],
                                                _lib.SHARD_SIDES[shard_side], ctypes.byref(handle)),
                  "mpgnn_plan_create")
        self._h = handle
        self._lock = threading.Lock()
        self._sel_cache: dict = {}
        self._ws_cache: dict = {}
        info = _lib.PlanInfo()
        check(lib.mpgnn_plan_get_info(self._h, ctypes.byref(info)))
        self.num_edges = int(info.num_edges)
        self.num_segments = int(info.num_segments)
        self.num_relations_present = int(info.num_relations)
        self.num_tiles = int(info.num_tiles)
        self.num_chunks = int(info.num_chunks)

    # -- lifetime -------------------------------------------------------------------------
    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib.mpgnn_plan_destroy(h)
            except Exception:
                pass
            self._h = None

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._h

    def to_device(self, device: torch.device) -> "GraphPlan":
        if isinstance(device, torch.device) and device.type == "cuda" and device.index is not None \
                and device.index == self._device:
            return self  # already resident (hot path of every layer call)
        if torch.device(device).type != "cuda":
            raise RuntimeError(
                f"mpgnn_amd: tensors are on {device}; the relational aggregation runs only as HIP "
                "kernels on a ROCm GPU (there is no CPU fallback). Move the model and data to 'cuda'.")
        idx = torch.device(device).index
        if idx is None:
            idx = torch.cuda.current_device()
        with self._lock:
            if self._device is None:
                check(lib.mpgnn_plan_upload(self._h, idx), "mpgnn_plan_upload")
                self._device = idx
            elif self._device != idx:
                raise RuntimeError(f"plan lives on cuda:{self._device}, tensor on cuda:{idx}")
        return self

    # -- queries ---------------------------------------------------------------------------
    def select(self, mode: int, relation: int, num_relations: int) -> tuple[int, int]:
        key = (mode, int(relation), int(num_relations))
        hit = self._sel_cache.get(key)  # the plan is immutable: answers are cached
        if hit is not None:
            return hit
        b, e = ctypes.c_int64(), ctypes.c_int64()
        check(lib.mpgnn_plan_select(self._h, mode, int(relation), int(num_relations),
                                    ctypes.byref(b), ctypes.byref(e)), "mpgnn_plan_select")
        self._sel_cache[key] = (int(b.value), int(e.value))
        return self._sel_cache[key]

    def table(self, name: str) -> np.ndarray:
        tid, dtype = _lib.TABLES[name]
        n, eb = ctypes.c_int64(), ctypes.c_int32()
        check(lib.mpgnn_plan_table_size(self._h, tid, ctypes.byref(n), ctypes.byref(eb)))
        out = np.empty(int(n.value), dtype=dtype)
        check(lib.mpgnn_plan_export(self._h, tid, out.ctypes.data if out.size else None,
                                    out.nbytes), "mpgnn_plan_export")
        return out

    def digest(self) -> int:
        """Fingerprint of every plan table (equal for both builders on the same graph)."""
        out = ctypes.c_uint64()
        check(lib.mpgnn_plan_digest(self._h, ctypes.byref(out)), "mpgnn_plan_digest")
        return int(out.value)

    def set_option(self, option: int, value: int) -> None:
        """This plan's kernel switch (``enum mpgnn_option``; the plan was created with the
        process defaults of ``_lib.set_option``)."""
        check(lib.mpgnn_plan_set_option(self._h, int(option), int(value)), "mpgnn_plan_set_option")

    def get_option(self, option: int) -> int:
        v = ctypes.c_int64()
        check(lib.mpgnn_plan_get_option(self._h, int(option), ctypes.byref(v)), "mpgnn_plan_get_option")
        return int(v.value)

    def set_exact_order(self, on: bool) -> None:
        """MPGNN_OPT_EXACT_ORDER on this plan (see include/mpgnn_rgcn.h)."""
        self.set_option(_lib.OPT_EXACT_ORDER, 1 if on else 0)

    def hsave_rows(self, mode: int, relation: int, num_relations: int) -> int:
        """Rows of the saved means of a layer call: its multi-edge segments (the single-edge
        segments' means are x rows, read through the plan's s_src table)."""
        key = ("hsave", mode, int(relation), int(num_relations))
        hit = self._sel_cache.get(key)
        if hit is not None:
            return hit
        n = ctypes.c_int64()
        check(lib.mpgnn_rgcn_hsave_rows(self._h, mode, int(relation), int(num_relations), ctypes.byref(n)),
              "mpgnn_rgcn_hsave_rows")
        self._sel_cache[key] = int(n.value)
        return self._sel_cache[key]

    def workspace_bytes(self, mode, relation, num_relations, f_in, f_out, row_lo, row_hi,
                        forward_only: bool = False) -> int:
        key = (mode, int(relation), int(num_relations), f_in, f_out, row_lo, row_hi, forward_only)
        hit = self._ws_cache.get(key)
        if hit is not None:
            return hit
        b = ctypes.c_int64()
        fn = lib.mpgnn_rgcn_fwd_workspace_bytes if forward_only else lib.mpgnn_rgcn_workspace_bytes
        check(fn(self._h, mode, int(relation), int(num_relations), f_in, f_out, row_lo, row_hi, ctypes.byref(b)),
              "mpgnn_rgcn_workspace_bytes")
        self._ws_cache[key] = int(b.value)
        return self._ws_cache[key]


class _PlanCache:
    """LRU of plans keyed by the identity/version of the graph tensors."""

    def __init__(self, capacity: int = 16):
        self.capacity = capacity
        self._d: OrderedDict = OrderedDict()
        self._lock = threading.Lock()

    def get(self, edge_index, edge_type, num_nodes, flow="target_to_source", shard=None,
            device=None, shard_side="gathered") -> GraphPlan:
        key = (id(edge_index), edge_index._version, tuple(edge_index.shape), edge_index.data_ptr(),
               id(edge_type), edge_type._version, edge_type.data_ptr(), int(num_nodes), flow,
               tuple(shard) if shard is not None else None, shard_side if shard is not None else None)
        with self._lock:
            hit = self._d.get(key)
            if hit is not None:
                ref_ei, ref_et, plan = hit
                if ref_ei() is edge_index and ref_et() is edge_type:
                    self._d.move_to_end(key)
                    return plan.to_device(device) if device is not None else plan
                del self._d[key]
        plan = GraphPlan(edge_index, edge_type, num_nodes, shard=shard, flow=flow, shard_side=shard_side,
                         device=device)
        if device is not None:
            plan.to_device(device)
        with self._lock:
            self._d[key] = (weakref.ref(edge_index), weakref.ref(edge_type), plan)
            while len(self._d) > self.capacity:
                self._d.popitem(last=False)
        return plan

    def clear(self):
        with self._lock:
            self._d.clear()


plan_cache = _PlanCache()


def get_plan(edge_index, edge_type, num_nodes, flow="target_to_source", shard=None, device=None,
             shard_side="gathered"):
    return plan_cache.get(edge_index, edge_type, num_nodes, flow=flow, shard=shard, device=device,
                          shard_side=shard_side)
