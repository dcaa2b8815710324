import sys, numpy as np, torch
sys.path.insert(0, "tests"); sys.path.insert(0, "monotonic-rnnt_amd/pytorch_binding"); sys.path.insert(0, "oracle")
from _parity import knobs, random_problem
import monotonic_rnnt_op as op
dev = torch.device("cuda:0")
rng = np.random.default_rng(1)
acts, labels, T, S = random_problem(rng, 16, (200, 200), 40, 256, force={b: (200, 40) for b in range(16)})
a = torch.from_numpy(acts).to(dev); lab = torch.from_numpy(labels).to(dev)
Tt, St = torch.from_numpy(T), torch.from_numpy(S)
scale = torch.linspace(0.5, 2.0, 16, device=dev)
def run():
    x = a.clone().requires_grad_(True)
    c = op.monotonic_rnnt_loss(x, lab, Tt, St); (c * scale).sum().backward(); torch.cuda.synchronize()
    return c.detach().clone(), x.grad.clone()
def cmp(n, p, q):
    dc = (p[0] - q[0]).abs().max().item(); dg = (p[1] - q[1]).abs().max().item()
    ng = (p[1].view(torch.int32) != q[1].view(torch.int32)).sum().item()
    print(f"{n}: costs maxdiff {dc:.3e} grads maxdiff {dg:.3e} differing grads {ng}", flush=True)
P = [run() for _ in range(3)]
cmp("product run0 vs run1", P[0], P[1]); cmp("product run0 vs run2", P[0], P[2])
for kn in [dict(chase_pair=2), dict(chase_pair=2, chase_early_free=0), dict(chase_pair=2, chase_ring=16), dict(chase_pair=2, chase_wait_us=100000)]:
    with knobs(chase=1, **kn):
        D = [run() for _ in range(3)]
    cmp(f"dev {kn} run0 vs run1", D[0], D[1]); cmp(f"dev {kn} run0 vs run2", D[0], D[2]); cmp(f"dev {kn} vs product", D[0], P[0])
with knobs(chase=1, chase_pair=1):
    D1 = [run() for _ in range(2)]
cmp("dev pair1 run0 vs run1", D1[0], D1[1])
with knobs(chase=0):
    R = run()
cmp("dev pair1 vs two-kernel", D1[0], R); cmp("product vs two-kernel", P[0], R)
