"""Developer timing: one bf16 gated tower (C5 widths: D = Hg = 256, MLP 605 -> 512 -> 256) through the
module path, forward + backward on R rows, repeated; run under rocprofv3 --kernel-trace --stats to
time the gate kernels alone on the chip (TTAMM_GENERIC_GATE=1: the generic path)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "two-tower-augmented-with-adaptive-mimic-mechanism_amd"))
sys.path.insert(0, str(ROOT / "tests"))

import torch  # noqa: E402

import ttamm  # noqa: E402
from helpers import Shape  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 57344
shape = Shape(U=200000, I=200000, F=605, H=512, D=256, hidden_dims=(512,), matmul_dtype="bf16", dropout=0.0)
enc = ttamm.build_tower_encoder(shape.tower_cfg(), num_embeddings=200000, feature_dim=605, device="cuda")
g = torch.Generator(device="cuda").manual_seed(1)
idx = torch.randint(0, 200000, (R,), device="cuda", generator=g)
feats = torch.randn((R, 605), device="cuda", generator=g)
dT = torch.randn((R, 256), device="cuda", generator=g)
for _ in range(12):
    enc.zero_grad(set_to_none=True)
    out = enc({"indices": idx, "features": feats})
    out.backward(dT)
torch.cuda.synchronize()
print("done", R)
