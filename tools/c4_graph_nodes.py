"""What the captured C4 SASRec step (sasrec._CapturedStep) holds, node by
node: the HIP graph is kept (keep_graph) and its nodes counted by type (hipGraphGetNodes /
hipGraphNodeGetType) and dumped as DOT (hipGraphDebugDotPrint) —
kernels by name, and every memcpy / memset node (a device copy inside the
replayed step shows up as one of these; outside the graph the step's own
host-side copies are listed by _CapturedStep.run).  One JSON line.

    python tools/c4_graph_nodes.py [--batch 2048] [--out gpurun_out/c4_graph.dot]
"""
import argparse
import collections
import ctypes
import json
import os
import re
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


TYPES = {0: "kernel", 1: "memcpy", 2: "memset", 3: "host", 4: "graph", 5: "empty",
         6: "wait_event", 7: "event_record", 8: "ext_semas_signal", 9: "ext_semas_wait",
         10: "mem_alloc", 11: "mem_free", 12: "memcpy_from_symbol", 13: "memcpy_to_symbol"}


class _DS:
    def __init__(self, n_users, m_items):
        self.n_users, self.m_items = n_users, m_items


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--users", type=int, default=1_000_000)
    ap.add_argument("--items", type=int, default=100_000)
    ap.add_argument("--out", default="gpurun_out/c4_graph.dot")
    a = ap.parse_args()
    from furusato_recommend_amd import SASRec, sasrec as S
    from furusato_recommend_amd.sasrec import SequenceData

    class KeptGraph(torch.cuda.CUDAGraph):  # keep the hipGraph_t after instantiation
        def __new__(cls, keep_graph=False):
            return super().__new__(cls, True)

        def __init__(self, keep_graph=False):
            super().__init__(True)
    S.torch.cuda.CUDAGraph = KeptGraph  # the module's torch is this torch
    hip = ctypes.CDLL("libamdhip64.so")
    dev = torch.device("cuda", 0)
    torch.manual_seed(2020)
    seq = SequenceData.synthetic(a.users, a.items, dev, max_len=50, min_len=5, seed=0)
    m = SASRec({"recdim": 128, "layer": 2, "heads": 2, "lr": 1e-3, "decay": 1e-4,
                "device": "cuda:0", "bpr_batch_size": a.batch, "dropout_p": 0.2, "graph": True},
               _DS(a.users, a.items), sequences=seq)
    rng = np.random.default_rng(7)
    for step in range(3):
        u_h = rng.integers(0, a.users, a.batch)
        u = m._upload(u_h)
        pn = m.sample_pairs(u, 7, step * a.batch)
        m.stageOne(u_h, pn[0], pn[1])
    torch.cuda.synchronize()
    graphs = list(m.__dict__.get("_graphs", {}).values())
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    res = []
    for i, cs in enumerate(graphs):
        for tag, g in (("A", cs.graph), ("B", cs.graph_b)):
            if g is None:
                continue
            path = a.out.replace(".dot", f"_{i}{tag}.dot")
            hg = ctypes.c_void_p(g.raw_cuda_graph())
            # node types (hipGraphNodeType: 0 kernel, 1 memcpy, 2 memset, ...)
            n = ctypes.c_size_t(0)
            hip.hipGraphGetNodes(hg, None, ctypes.byref(n))
            nodes = (ctypes.c_void_p * n.value)()
            hip.hipGraphGetNodes(hg, nodes, ctypes.byref(n))
            types = collections.Counter()
            for nd in nodes:
                t = ctypes.c_int(-1)
                hip.hipGraphNodeGetType(ctypes.c_void_p(nd), ctypes.byref(t))
                types[TYPES.get(t.value, str(t.value))] += 1
            rc = hip.hipGraphDebugDotPrint(hg, path.encode(), ctypes.c_uint(1))
            txt = open(path).read() if rc == 0 and os.path.exists(path) else ""
            kinds = collections.Counter()
            names = collections.Counter()
            for lab in re.findall(r'label="([^"]*)"', txt):
                low = lab.lower()
                if "memcpy" in low:
                    kinds["memcpy"] += 1
                    names["memcpy: " + lab[:160]] += 1
                elif "memset" in low:
                    kinds["memset"] += 1
                    names["memset: " + lab[:160]] += 1
                elif "kernel" in low or "func" in low:
                    kinds["kernel"] += 1
                    m_ = re.search(r"(mirec::\w+|at::native::\w+|rocprim::\w+|\w+_kernel\w*)", lab)
                    names[m_.group(1) if m_ else lab[:80]] += 1
                else:
                    kinds["other"] += 1
            res.append({"graph": f"{i}{tag}", "capacity": cs.C, "node_types": dict(types),
                        "dot_rc": rc, "nodes": dict(kinds),
                        "copy_nodes": {k: v for k, v in names.items()
                                       if k.startswith(("memcpy", "memset"))},
                        "top_kernels": names.most_common(12), "dot": path})
    print(json.dumps({"c4_graph_nodes": res}), flush=True)


if __name__ == "__main__":
    main()
