import os, sys, numpy as np, torch
ROOT = "/root/repo" if os.path.exists("/root/repo") else os.environ["GRAFT_REPO_ROOT"]
sys.path.insert(0, os.path.join(ROOT, "incentive-design-mpc_amd"))
from lompc_amd import _lib
if os.environ.get("DBG_LIB"):
    _lib._lib = _lib.load(os.path.join(ROOT, "incentive-design-mpc_amd", "lompc_amd", os.environ["DBG_LIB"]))
from lompc_amd import BatchPlan, LoMPC, LoMPCConstants
N, P, B, K = 24, 12, 262144, 3
rng = np.random.default_rng(0)
cs = [LoMPCConstants(0.05, 10.0, 0.9, 0.25, "small"), LoMPCConstants(0.025, 50.0, 0.9, 0.15, "large")]
lompcs = [LoMPC(N, c, device=0) for c in cs]
M = B // 2
off1 = np.array([(M * p) // P for p in range(P + 1)], dtype=np.int64)
off = np.concatenate([off1, M + off1[1:]])
gn = np.concatenate([c.y_max - (0.3 + 0.2 * rng.random(M)) for c in cs])
g = torch.as_tensor(gn, device="cuda")
lm = torch.as_tensor(np.stack([np.concatenate([c.theta * rng.random((P, 3 * N)) for c in cs]) for _ in range(K)]), device="cuda")
lr = torch.zeros((K, 2 * P), dtype=torch.float64, device="cuda")
plan = BatchPlan(lompcs, g, off, sets_per_ctx=[P, P], want_w=True, want_cost=True, want_status=True)
o = plan.run_steps(lm, lr, K, lm[0].numel(), lr[0].numel(), per_run_sets=True, per_run=True)
print("check", plan.check(), plan.info())
st = o["status"].cpu().numpy()
for k in range(K):
    rep = st[k] == _lib.LOMPC_QP_REPAIRED if hasattr(_lib, "LOMPC_QP_REPAIRED") else st[k] != 0
    print("run", k, "status counts", np.unique(st[k], return_counts=True))
# block map: recompute ~ blocks per set
nb = plan.info()["workgroups"]
print("blocks", nb)
k = 0
bad = np.nonzero(st[k] != st[k].min())[0] if False else None
vals, cnts = np.unique(st[0], return_counts=True)
mode = vals[np.argmax(cnts)]
print("mode status", mode)
LIB = os.environ.get("DBG_LIB")
for s in range(24):
    a, b = off[s], off[s + 1]
    ss = st[1, a:b]
    # per position within the set: which rows are not OK
    nbs = int(round((b - a) / 520))
    bounds = [a + (b - a) * j // nbs for j in range(nbs + 1)]
    print("set", s, "bad", int((ss != 0).sum()), "of", b - a)
    for j in range(0):
        blk = st[1, bounds[j]:bounds[j + 1]]
        n = len(blk); per = -(-n // 7)
        print("set", s, "block", j, "n", n, "per-wave non-OK:", [int((blk[w*per:(w+1)*per] != 0).sum()) for w in range(7)])
    gs = gn[a:b]
    okm = ss == 0
    print("  gamma range ok", gs[okm].min() if okm.any() else None, gs[okm].max() if okm.any() else None,
          "bad", gs[~okm].min() if (~okm).any() else None, gs[~okm].max() if (~okm).any() else None)
