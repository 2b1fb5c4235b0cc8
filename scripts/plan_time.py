#!/usr/bin/env python3
"""Plan build time for a named workload (MPGNN_PLAN_TIMING=1 prints the phases)."""
import os
sys_path_root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
import sys
sys.path.insert(0, sys_path_root)
import time, torch, mpgnn_amd  # noqa: E402
from mpgnn_amd import data
g=data.config_graph(sys.argv[1] if len(sys.argv)>1 else "C5")
t=time.time(); p=mpgnn_amd.GraphPlan(g.edge_index, g.edge_type, g.num_nodes); print("plan", round(time.time()-t,3), flush=True)
