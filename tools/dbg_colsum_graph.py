"""Debug: is torch's column reduction (x.sum(0), the bias-gradient form the
captured SASRec data-parallel step used before mirec_col_sums) exact when
replayed in a HIP graph whose input changes between replays?

For each shape: R replays of a graph holding `y = x.sum(0)` (torch) and the
same graph with mirec_col_sums, x refilled (eager, new random data) before
every replay; each result is checked against a float64 sum on the device.
Also the same R reductions eagerly.  Variants: with / without a host
synchronize between replays, and with the refill done inside the graph (a
kernel writes x, then the reduction reads it: the captured step's shape).
Prints one JSON line per (shape, variant): bad replays / R and the worst
relative error."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from furusato_recommend_amd.linear import col_sums  # noqa: E402

R = int(os.environ.get("REPS", "200"))


def check(y, x):
    ref = x.double().sum(0)
    err = (y.double() - ref).abs().max() / ref.abs().max().clamp_min(1e-30)
    return float(err)


def run(n, m, how, impl):
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(n + m)
    x = torch.empty(n, m, device=dev)
    src = torch.empty(n, m, device=dev)
    red = (lambda t: t.sum(0)) if impl == "torch" else col_sums
    bad, worst = 0, 0.0
    if how == "eager":
        for r in range(R):
            x.normal_(generator=g)
            y = red(x)
            e = check(y, x)
            bad += e > 1e-5
            worst = max(worst, e)
        return bad, worst
    pool = torch.cuda.graph_pool_handle()
    graph = torch.cuda.CUDAGraph()
    x.normal_(generator=g)
    src.normal_(generator=g)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm-up outside the capture
        if how == "inside":
            x.copy_(src)
        red(x)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(graph, pool=pool):
        if how == "inside":
            x.copy_(src)  # the reduction's input written inside the graph
        y = red(x)
    outs = []
    for r in range(R):
        if how == "inside":
            src.normal_(generator=g)
        else:
            x.normal_(generator=g)
        graph.replay()
        if how.endswith("sync"):
            torch.cuda.synchronize()
        outs.append((y.clone(), x.clone()))
        if len(outs) == 20:
            for yy, xx in outs:
                e = check(yy, xx)
                bad += e > 1e-5
                worst = max(worst, e)
            outs = []
    for yy, xx in outs:
        e = check(yy, xx)
        bad += e > 1e-5
        worst = max(worst, e)
    return bad, worst


if __name__ == "__main__":
    for n, m in ((14336, 192), (56320, 192), (56320, 384), (7168, 64)):
        for impl in ("torch", "mirec"):
            for how in ("eager", "graph", "graph_sync", "inside"):
                b, w = run(n, m, how, impl)
                print(json.dumps({"n": n, "m": m, "impl": impl, "how": how, "reps": R,
                                  "bad": int(b), "worst_rel": w}), flush=True)
