"""Developer diagnostic: one D = 128 gated tower (module autograd path) forward + backward with the
fused gate and with the generic gate (TTAMM_GENERIC_GATE=1) on the same inputs; per-parameter
max-abs relative difference, for several row counts and gradient scales."""
import copy
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "two-tower-augmented-with-adaptive-mimic-mechanism_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
import ttamm  # noqa: E402

dev = torch.device("cuda")
c = dict(bench.CONFIGS["c4"])
c["dropout"] = 0.0
c["F"] = 64
tcfg = bench.tower_cfg(c)
U, F = 25000, c["F"]


def run(enc, idx, feats, dT, generic):
    if generic:
        os.environ["TTAMM_GENERIC_GATE"] = "1"
    else:
        os.environ.pop("TTAMM_GENERIC_GATE", None)
    enc.zero_grad(set_to_none=True)
    out = enc({"indices": idx, "features": feats})
    out.backward(dT)
    torch.cuda.synchronize()
    return out.detach().clone(), {n: (p.grad.to_dense() if p.grad.is_sparse else p.grad).clone()
                                  for n, p in enc.named_parameters() if p.grad is not None}


torch.manual_seed(0)
enc0 = ttamm.build_tower_encoder(tcfg, num_embeddings=U, feature_dim=F, device=dev)
for R in (2000, 8192, 16384, 20000):
    for scale in (1.0, 1e-6):
        g = torch.Generator(device=dev).manual_seed(R)
        idx = torch.randint(0, U, (R,), device=dev, generator=g)
        feats = torch.randn((R, F), device=dev, generator=g)
        dT = torch.randn((R, c["D"]), device=dev, generator=g) * scale
        enc_a = copy.deepcopy(enc0)
        enc_b = copy.deepcopy(enc0)
        oa, ga = run(enc_a, idx, feats, dT, False)
        ob, gb = run(enc_b, idx, feats, dT, True)
        worst = []
        fo = float((oa - ob).abs().max() / ob.abs().max())
        for n in gb:
            d = float((ga[n] - gb[n]).abs().max() / gb[n].abs().max().clamp_min(1e-30))
            worst.append((d, n))
        worst.sort(reverse=True)
        print(f"R={R:6d} scale={scale:g} out {fo:.2e} | " + ", ".join(f"{n}={d:.2e}" for d, n in worst[:4]), flush=True)
