"""Per-kernel parity on MI355X: row gather (bit-exact), eval tower forward, mimic augment,
MSE, optimizer kernels in isolation, and the negative sampler's contract."""

import ctypes

import pytest
import torch

from helpers import Shape, make_problem, rel_err
from oracle import cpu_reference as ref

pytestmark = pytest.mark.gpu


def _ulps(a, b):
    """max |a - b| in units of fp32 ulp(b) (ulp floored at ulp(1e-3))."""
    ulp = torch.finfo(torch.float32).eps * b.abs().clamp_min(1e-3)
    return ((a - b).abs() / ulp).max().item()


def _lib():
    from ttamm import _lib

    return _lib, _lib.load()


@pytest.mark.parametrize("rows,dim,n", [(1000, 96, 5000), (7, 8, 33), (513, 12, 1), (300, 5, 77), (64, 128, 0),
                                        # every width of the wide kernel, with ragged row tails
                                        (999, 32, 4097), (999, 64, 1234), (999, 128, 70001), (999, 192, 4099),
                                        (999, 256, 3333), (999, 96, 70001), (50, 128, 7)])
def test_gather_rows_bit_exact(rows, dim, n):
    L, lib = _lib()
    table = torch.randn(rows, dim, device="cuda")
    idx = torch.randint(0, rows, (n,), device="cuda")
    out = torch.full((n, dim), float("nan"), device="cuda")
    L.check(lib.ttamm_gather_rows(table.data_ptr(), rows, dim, idx.data_ptr(), n, out.data_ptr(), dim,
                                  L.stream_handle()))
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), table.cpu().index_select(0, idx.cpu()))


def test_gather_rows_strided_output_bit_exact():
    L, lib = _lib()
    table = torch.randn(4096, 96, device="cuda")
    idx = torch.randint(0, 4096, (1000,), device="cuda")
    out = torch.zeros(1000, 192, device="cuda")
    L.check(lib.ttamm_gather_rows(table.data_ptr(), 4096, 96, idx.data_ptr(), 1000, out.data_ptr(), 192,
                                  L.stream_handle()))
    torch.cuda.synchronize()
    assert torch.equal(out[:, :96].cpu(), table.cpu()[idx.cpu()])
    assert torch.count_nonzero(out[:, 96:]) == 0


@pytest.mark.parametrize("shape", [Shape(dropout=0.0), Shape(F=605, H=192, D=96, hidden_dims=(192,), dropout=0.0),
                                   Shape(F=37, D=12, gate_hidden=20, hidden_dims=(24, 16), dropout=0.0),
                                   Shape(dropout=0.0, fusion="sum"), Shape(dropout=0.0, fusion="concat")],
                         ids=["tiny", "c2dims", "odd", "sum", "concat"])
def test_tower_forward_eval_matches_oracle(shape):
    from gpu_helpers import ttamm_model_from

    prob = make_problem(shape, steps=1)
    tm = ttamm_model_from(prob).eval()
    om = prob.model.eval()
    idx = torch.randint(0, shape.I, (257,))
    with torch.no_grad():
        want = ref.tower_forward(om.item_encoder, idx, prob.item_features[idx], training=False)
        got = tm.item_encoder({"indices": idx.cuda(), "features": prob.item_features[idx].cuda()})
        assert got.shape == (257, shape.D)
        assert rel_err(got, want) <= 1e-5
        want_aug = want + om.adaptive_mimic.item_augmented.weight[idx]
        got_aug = tm.adaptive_mimic.augment_items(idx.cuda(), got)
        assert rel_err(got_aug, want_aug) <= 1e-6


def test_mimic_forward_and_losses():
    """tests/test_adaptive_mimic.py:6-33, on the device, plus values vs F.mse_loss."""
    import ttamm

    torch.manual_seed(0)
    mech = ttamm.AdaptiveMimicMechanism(num_users=4, num_items=6, embedding_dim=8, init_std=0.01).cuda()
    users = torch.tensor([0, 1], dtype=torch.long, device="cuda")
    items = torch.tensor([2, 3], dtype=torch.long, device="cuda")
    ue = torch.zeros((2, 8), device="cuda")
    ie = torch.ones((2, 8), device="cuda")
    with torch.no_grad():
        au, ai, lu, li = mech(user_indices=users, item_indices=items, user_embedding=ue, item_embedding=ie)
        assert au.shape == ue.shape and ai.shape == ie.shape
        assert lu.item() >= 0 and li.item() >= 0
        wu = mech.user_augmented.weight[users]
        wi = mech.item_augmented.weight[items]
        assert torch.equal(au, ue + wu) and torch.equal(ai, ie + wi)
        assert abs(lu.item() - torch.nn.functional.mse_loss(wu, ie).item()) <= 1e-6
        assert abs(li.item() - torch.nn.functional.mse_loss(wi, ue).item()) <= 1e-6
        neg = mech.augment_items(torch.tensor([0, 1, 2, 3], device="cuda"), torch.randn((4, 8), device="cuda"))
        assert neg.shape == (4, 8)
    with pytest.raises(ValueError):
        mech.augment_items(torch.tensor([0, 1], dtype=torch.int32, device="cuda"), torch.zeros((2, 8), device="cuda"))


def test_encoder_with_features_shape():
    """tests/test_encoders.py:6-26 on the device."""
    import ttamm

    cfg = {"type": "tower", "id_embedding": {"params": {"embedding_dim": 8}},
           "feature_encoder": {"type": "linear", "output_dim": 8}, "fusion": "gated",
           "adaptive_mimic": {"hidden_dim": 16}}
    enc = ttamm.build_tower_encoder(cfg, num_embeddings=5, feature_dim=4, device=torch.device("cuda")).eval()
    with torch.no_grad():
        out = enc({"indices": torch.tensor([0, 1, 2], device="cuda"), "features": torch.randn(3, 4, device="cuda")})
    assert out.shape == (3, 8)


@pytest.mark.parametrize("decoupled", [1, 0])
def test_adamw_dense_kernel_matches_torch(decoupled):
    L, lib = _lib()
    torch.manual_seed(3)
    n = 100003
    p0 = torch.randn(n)
    g = [torch.randn(n) * 1e-2 for _ in range(3)]
    pt = p0.clone().requires_grad_(True)
    cls = torch.optim.AdamW if decoupled else torch.optim.Adam
    opt = cls([pt], lr=1e-3, weight_decay=0.01)
    p = p0.cuda()
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    for step, gg in enumerate(g, start=1):
        pt.grad = gg.clone()
        opt.step()
        gc = gg.cuda()
        L.check(lib.ttamm_adamw_dense(p.data_ptr(), m.data_ptr(), v.data_ptr(), gc.data_ptr(), n, 1e-3, 0.9, 0.999,
                                      1e-8, 0.01, decoupled, step, L.stream_handle()))
    torch.cuda.synchronize()
    st = opt.state[pt]
    assert rel_err(m, st["exp_avg"]) <= 1e-6
    assert rel_err(v, st["exp_avg_sq"]) <= 1e-6
    # a few ulp: rounding of sqrt / division vs ATen's vectorised CPU kernels
    assert _ulps(p.cpu(), pt.detach()) <= 4


def test_sparse_adam_kernel_matches_torch():
    L, lib = _lib()
    torch.manual_seed(4)
    rows, dim = 500, 24
    w0 = torch.randn(rows, dim)
    wt = torch.nn.Parameter(w0.clone())
    opt = torch.optim.SparseAdam([wt], lr=1e-3)
    w = w0.cuda()
    m = torch.zeros_like(w)
    v = torch.zeros_like(w)
    for step in range(1, 4):
        uniq = torch.randperm(rows)[:97].sort().values
        grad = torch.randn(97, dim) * 1e-2
        wt.grad = torch.sparse_coo_tensor(uniq[None, :], grad, (rows, dim))
        opt.step()
        uc, gc = uniq.cuda(), grad.cuda()
        L.check(lib.ttamm_sparse_adam_rows(w.data_ptr(), m.data_ptr(), v.data_ptr(), dim, uc.data_ptr(), gc.data_ptr(),
                                           97, 1e-3, 0.9, 0.999, 1e-8, step, L.stream_handle()))
    torch.cuda.synchronize()
    st = opt.state[wt]
    assert rel_err(m, st["exp_avg"]) <= 1e-6
    assert rel_err(v, st["exp_avg_sq"]) <= 1e-6
    assert _ulps(w.cpu(), wt.detach()) <= 4


def test_sampler_excludes_positives():
    """tests/test_samplers.py:6-19 on the device."""
    import ttamm

    users = torch.tensor([0, 1], dtype=torch.long)
    positives = {0: {1, 2}, 1: {0}}
    for _ in range(20):
        neg = ttamm.sample_negative_items(users, num_items=5, positives=positives, num_negatives=2,
                                          device=torch.device("cuda"))
        assert neg.shape == (2, 2)
        assert all(i not in positives[0] for i in neg[0].tolist())
        assert all(i not in positives[1] for i in neg[1].tolist())


def test_sampler_uniform_over_allowed_items():
    import ttamm

    num_items = 50
    positives = {0: set(range(0, 50, 5))}  # 10 blocked, 40 allowed
    users = torch.zeros(4000, dtype=torch.long)
    neg = ttamm.sample_negative_items(users, num_items=num_items, positives=positives, num_negatives=10,
                                      device=torch.device("cuda")).cpu().reshape(-1)
    assert not torch.isin(neg, torch.tensor(sorted(positives[0]))).any()
    counts = torch.bincount(neg, minlength=num_items).double()
    allowed = [i for i in range(num_items) if i not in positives[0]]
    obs = counts[allowed]
    exp = neg.numel() / len(allowed)
    chi2 = ((obs - exp) ** 2 / exp).sum().item()
    assert chi2 < 80.0  # 39 dof: p ~ 1e-4


def test_sampler_errors():
    import ttamm

    users = torch.tensor([0], dtype=torch.long)
    with pytest.raises(ValueError):
        ttamm.sample_negative_items(users, num_items=5, positives={}, num_negatives=0, device=torch.device("cuda"))
    with pytest.raises(ValueError):
        ttamm.sample_negative_items(users, num_items=1, positives={}, num_negatives=2, device=torch.device("cuda"))
    with pytest.raises(RuntimeError):
        ttamm.sample_negative_items(users, num_items=3, positives={0: {0, 1, 2}}, num_negatives=2,
                                    device=torch.device("cuda"))
    # 999 of 1000 items are positives: 11 draws almost never find the free one
    with pytest.raises(RuntimeError):
        ttamm.sample_negative_items(torch.zeros(64, dtype=torch.long), num_items=1000,
                                    positives={0: set(range(999))}, num_negatives=8, device=torch.device("cuda"))
