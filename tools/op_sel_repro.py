"""Run tools/op_sel_repro.hip's probe (built beforehand:
hipcc -O3 --offload-arch=gfx950 -shared -fPIC tools/op_sel_repro.hip -o tools/op_sel_repro.so):
per configuration, REPS launches of 2048 workgroups; the number of launches
with a lane that did not get its pair's high dword, the wrong lanes by
position in the wave (for waves in even / odd hardware slots), and what the wrong lanes
read instead (the pair's LOW dword, zero, or something else).  One JSON line
per configuration."""
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
torch.manual_seed(0)
inp = torch.randn(2 * n, device="cuda")
out = torch.empty(3 * n, device="cuda")
lo_h, hi_h = inp.view(n, 2)[:, 0], inp.view(n, 2)[:, 1]
# (MFMA iterations, op_sel, MFMA only in odd wave slots, s_nop 7 rounds, pair by v_mov_b64)
CONFIGS = [(0, 1, 0, 0, 1), (8, 1, 0, 0, 1), (8, 0, 0, 0, 1), (64, 1, 0, 0, 1),
           (8, 1, 0, 0, 0), (8, 1, 1, 0, 1), (64, 1, 1, 0, 1), (8, 1, 0, 4, 1), (8, 1, 0, 32, 1),
           (8, 1, 0, 256, 1)]
for iters, use, odd, nops, p64 in CONFIGS:
    bad_launches, lanes = 0, torch.zeros(128, dtype=torch.int64)
    kinds = {"low_dword": 0, "zero": 0, "other": 0}
    for _ in range(REPS):
        bad = torch.zeros(128, dtype=torch.int32, device="cuda")
        rc = lib.op_sel_probe_launch(ctypes.c_void_p(inp.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                     ctypes.c_void_p(bad.data_ptr()), blocks, iters, use, odd, nops, p64)
        if rc != 0:
            sys.exit(f"launch failed: {rc}")
        torch.cuda.synchronize()
        b = bad.cpu().long()
        if int(b.sum()):
            bad_launches += 1
            lanes += b
            r = out.view(n, 3)[:, :2]
            wrong = (r[:, 0] != hi_h) | (r[:, 1] != hi_h)
            got = torch.where(r[:, 0] != hi_h, r[:, 0], r[:, 1])[wrong]
            kinds["low_dword"] += int((got == lo_h[wrong]).sum())
            kinds["zero"] += int((got == 0).sum())
            kinds["other"] += int(((got != lo_h[wrong]) & (got != 0)).sum())
    print(json.dumps({"mfma_iters": iters, "op_sel": bool(use), "mfma_odd_wave_slots_only": bool(odd),
                      "s_nop7_rounds": nops, "pair_v_mov_b64": bool(p64), "reps": REPS,
                      "launches_with_wrong_lanes": bad_launches,
                      "wrong_lanes_even_slot": {i: c for i, c in enumerate(lanes[:64].tolist()) if c},
                      "wrong_lanes_odd_slot": {i: c for i, c in enumerate(lanes[64:].tolist()) if c},
                      "wrong_values": kinds}), flush=True)
