"""mpgnn_amd — MI355X (gfx950) drop-in for the relational hot path of
francescoferrini/MPGNN-Metapath-Graph-Neural-Network.

  mp_rgcn_layer.CustomRGCNConv   ← reference mp_rgcn_layer.py (MPGNN layer, one relation/layer)
  nn.RGCNConv                    ← torch_geometric.nn.RGCNConv as used by model.py:137-138
  model.MPNetm / model.Net       ← reference model.py wrappers (unchanged PyTorch around the layers)
  functional.rgcn_conv           autograd op over the C ABI (include/mpgnn_rgcn.h)
  plan.GraphPlan                 one-time sorted segment tables of a graph (cached)
  data, distributed              graph inputs (C1-C5, native link.dat reader) and dst-range sharding
  main, main_rgcn, metrics       training / evaluation loops of main.py and main_rgcn.py
  score.Score / score_relation_parallel   the metapath score function (model.py:26-125,
                                 main.py:387-760) on the GPU: segment argmax kernels

The directory name is not a Python identifier; import it as ``mpgnn_amd`` (repo-root shim).
"""
from . import _lib  # noqa: F401  (loads libmpgnn_rgcn.so — ImportError if missing: no CPU fallback)
from .functional import MODE_ALL, MODE_SINGLE, rgcn_conv, segment_means
from .model import MPNetm, Net
from .mp_rgcn_layer import CustomRGCNConv, masked_edge_index
from .nn import CustomFastRGCNConv, FastRGCNConv, RGCNConv
from . import data, distributed, metrics  # noqa: E402
from . import score  # noqa: E402  (score function, model.py:26-125 / main.py:387-760)
from . import main, main_rgcn  # noqa: E402  (training-loop drop-ins, main.py / main_rgcn.py)
from .plan import GraphPlan, get_plan, plan_cache

__all__ = ["CustomRGCNConv", "RGCNConv", "FastRGCNConv", "CustomFastRGCNConv", "MPNetm", "Net", "GraphPlan", "get_plan", "plan_cache",
           "rgcn_conv", "segment_means", "masked_edge_index", "MODE_SINGLE", "MODE_ALL"]
__version__ = "0.1.0"
