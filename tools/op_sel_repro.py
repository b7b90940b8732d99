"""Run tools/op_sel_repro.hip's probe (built beforehand:
hipcc -O3 --offload-arch=gfx950 -shared -fPIC tools/op_sel_repro.hip -o tools/op_sel_repro.so):
per (MFMA iterations, op_sel or not), REPS launches of 2048 workgroups, the
number of launches with a lane that did not get its pair's high dword, and
those lanes' positions within the wave.  One JSON line per configuration."""
import ctypes
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "op_sel_repro.so"))
REPS = int(os.environ.get("REPS", "50"))
blocks = 2048
n = blocks * 256
inp = torch.randn(2 * n, device="cuda")
out = torch.empty(3 * n, device="cuda")
for iters in (0, 8, 64):
    for use in (1, 0):
        bad_launches, lanes = 0, torch.zeros(64, dtype=torch.int64)
        for _ in range(REPS):
            bad = torch.zeros(64, dtype=torch.int32, device="cuda")
            rc = lib.op_sel_probe_launch(ctypes.c_void_p(inp.data_ptr()),
                                         ctypes.c_void_p(out.data_ptr()),
                                         ctypes.c_void_p(bad.data_ptr()), blocks, iters, use)
            if rc != 0:
                sys.exit(f"launch failed: {rc}")
            torch.cuda.synchronize()
            b = bad.cpu().long()
            if int(b.sum()):
                bad_launches += 1
                lanes += b
        print(json.dumps({"mfma_iters": iters, "op_sel": bool(use), "reps": REPS,
                          "launches_with_wrong_lanes": bad_launches,
                          "wrong_lane_counts_by_lane": lanes.tolist()}), flush=True)
