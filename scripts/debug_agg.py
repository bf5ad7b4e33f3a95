"""Diagnostics: dump a sorted-gamma plan's path table and fine index and recompute the
aggregation's coverage in numpy (tests/test_gpu_pipeline.py::test_sorted_gamma_aggregation data)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "incentive-design-mpc_amd"), os.path.join(ROOT, "oracle")]
import lompc_oracle as O  # noqa: E402
from lompc_amd import BatchPlan, LoMPC, LoMPCConstants, _lib  # noqa: E402

N = 24
rng = np.random.default_rng(0)
c = O.large_consts()
lompc = LoMPC(N, LoMPCConstants(c.delta, c.theta, c.y_max, c.w_max, c.ev_type), device=0)
sizes = [300000, 5000]
parts = [np.sort(c.y_max * rng.random(m)) for m in sizes]
off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
gn = np.concatenate(parts)
g = torch.as_tensor(gn, device="cuda:0")
S = len(sizes)
lm = torch.as_tensor(c.theta * rng.random((S, 3 * N)), device="cuda:0")
lr = torch.zeros(S, dtype=torch.float64, device="cuda:0")
agg = BatchPlan(lompc, g, off, want_w=False, want_cost=False, sorted_gamma=True)
out = agg.run(lm, lr)
print("check", agg.check())
G = agg.cells
F = G * 256
lib = _lib.load()
lib.lompc_debug_plan_tables.restype = ctypes.c_int
cnt = np.zeros(S * G, np.int32)
lo = np.zeros(S * G)
ge = np.zeros(S * G * 8)
pos = np.zeros(S * (F + 1), np.int32)
sinfo = np.zeros(S * 4, np.int32)
rc = lib.lompc_debug_plan_tables(agg._plan, ctypes.c_void_p(cnt.ctypes.data), ctypes.c_void_p(lo.ctypes.data),
                                 ctypes.c_void_p(ge.ctypes.data), ctypes.c_void_p(pos.ctypes.data),
                                 ctypes.c_void_p(sinfo.ctypes.data), None)
print("rc", rc, "G", G, "sinfo", sinfo.reshape(S, 4))
pos = pos.reshape(S, F + 1)
for s in range(S):
    gs = parts[s]
    print("set", s, "pos head", pos[s, :8], "pos at cells", pos[s, ::256][:G + 1])
    unc = 0
    for cc in range(G):
        cell = s * G + cc
        cs, ce = pos[s, cc * 256], pos[s, (cc + 1) * 256]
        n = cnt[cell]
        gg = ge[cell * 8: cell * 8 + n]
        q0 = cs + np.searchsorted(gs[cs:ce], lo[cell], side="left")
        qn = cs + np.searchsorted(gs[cs:ce], gg[-1], side="right") if n else ce
        u = (q0 - cs) + (ce - qn) if n else ce - cs
        unc += u
        if cc < 3 or u:
            print(f"  cell {cc}: range [{cs},{ce}) g[{gs[cs] if ce > cs else None}, {gs[ce - 1] if ce > cs else None}] "
                  f"lo {lo[cell]} cnt {n} ge {gg} uncovered {u}")
    print("set", s, "uncovered (numpy)", unc, "stats", out["set_stats"][s].cpu().numpy())

# emulate k_agg's boundary search exactly (fine bucket of the piece end, clamped to the cell, then
# the search inside [pos[fb], pos[fb + 1]])
win = []
for s in range(S):
    gs = parts[s]
    mg = 1e-7 * c.y_max
    wlo = min(max(gs[0] - mg, 0.0), c.y_max)
    whi = min(max(gs[-1] + mg, wlo + mg), c.y_max)
    W = whi - wlo
    fs = F / W
    def fine(v):
        x = (v - wlo) * fs
        return 0 if x <= 0 else (F - 1 if x >= F - 1 else int(x))
    unc = 0
    for cc in range(G):
        cell = s * G + cc
        cs, ce = pos[s, cc * 256], pos[s, (cc + 1) * 256]
        n = cnt[cell]
        vb = [lo[cell]] + list(ge[cell * 8: cell * 8 + n])
        q = []
        for j, v in enumerate(vb):
            fb = min(max(fine(v), cc * 256), (cc + 1) * 256 - 1)
            a, b = min(max(pos[s, fb], cs), ce), min(max(pos[s, fb + 1], cs), ce)
            seg = gs[a:b]
            q.append(a + int(np.sum(seg < v) if j == 0 else np.sum(seg <= v)))
        u = (q[0] - cs) + (ce - q[-1]) if n else ce - cs
        if u:
            print(f"  emu set {s} cell {cc}: q {q} cs {cs} ce {ce} u {u}")
        unc += u
    print("emulated uncovered", s, unc)
