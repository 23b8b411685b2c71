"""Developer diagnostic: which user rows of the C4 one-step embedding gradient differ (fused D = 128
gate vs the fp32 oracle), mapped back to their batch positions (16-row slabs of the gate kernels)."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "two-tower-augmented-with-adaptive-mimic-mechanism_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
import test_fullsize_parity_gpu as F  # noqa: E402

os.environ.pop("TTAMM_GENERIC_GATE", None)
om, oopts, tm, topts, ores, tl, _ = F._one_step("c4", seed=404, in_batch=True)
og, tg = F._grads(om, oopts), F._grads(tm, topts)
c = bench.CONFIGS["c4"]
gen = torch.Generator().manual_seed(404)
perm = torch.randperm(c["I"], generator=gen)
users = torch.randint(0, c["U"], (c["B"],), generator=gen)
name = "user_encoder.embedding.weight"
a, b = tg[name].to("cuda").to_dense() if tg[name].is_sparse else tg[name].to("cuda"), og[name].to("cuda")
b = b.to_dense() if b.is_sparse else b
den = float(b.abs().max())
rowerr = ((a - b).abs().max(dim=1).values / den).cpu()
bad = torch.nonzero(rowerr > 1e-5).flatten()
print(f"{name}: {bad.numel()} rows above 1e-5 of max (max row err {float(rowerr.max()):.2e})")
pos = []
for u in bad.tolist():
    pos += torch.nonzero(users == u).flatten().tolist()
pos.sort()
print("batch positions:", pos[:80])
print("slabs:", sorted(set(p // 16 for p in pos))[:80])
print("rows within slab:", sorted(set(p % 16 for p in pos)))
# per-column pattern of the worst row
if bad.numel():
    u = int(bad[torch.argmax(rowerr[bad])])
    d = ((a[u] - b[u]).abs() / den).cpu()
    print("worst row", u, "cols above 1e-6:", torch.nonzero(d > 1e-6).flatten().tolist()[:64])
    print("ttamm", a[u][:8].tolist())
    print("oracle", b[u][:8].tolist())
    # one ReLU unit of the gate's hidden layer flipped at its kink? then the row's dE difference is
    # parallel to one column h of G1[:, :D] and dG1's difference sits in row h
    G1 = dict(om.named_parameters())["user_encoder.adaptive_mimic.gate_network.0.weight"].detach().double()
    diff = (a[u] - b[u]).double().cpu()
    cos = (G1[:, :diff.numel()] @ diff) / (G1[:, :diff.numel()].norm(dim=1) * diff.norm())
    h = int(cos.abs().argmax())
    print(f"dE diff vs G1 columns: best unit h={h} |cos|={float(cos.abs()[h]):.6f}")
    n1 = "user_encoder.adaptive_mimic.gate_network.0.weight"
    dW = (tg[n1].to("cuda") - og[n1].to("cuda")).double()
    rn = dW.norm(dim=1)
    print(f"dG1 diff: row {int(rn.argmax())} holds {float(rn.max()**2 / (rn**2).sum()):.6f} of the diff energy")
    nb = "user_encoder.adaptive_mimic.gate_network.0.bias"
    db = (tg[nb].to("cuda") - og[nb].to("cuda")).double().abs()
    print(f"dc1 diff: argmax {int(db.argmax())}, share {float(db.max() / db.sum()):.6f}")
