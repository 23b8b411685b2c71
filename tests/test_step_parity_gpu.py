"""Fused training step on MI355X vs the CPU oracle (same parameters, injected negatives and
dropout keep-masks).  Tolerances: loss and gradients 1e-5 norm-wise relative
(max|ours - oracle| / max|oracle| per tensor, tests/helpers.rel_err)."""

import pytest
import torch

from helpers import Shape, make_problem, named_optimizer_state, rel_err, run_oracle

pytestmark = pytest.mark.gpu

GRAD_TOL = 1e-5


def _grads_by_name(model, opts):
    """With lr = 0 and beta1 = 0 a single Adam/SparseAdam step leaves exp_avg == grad
    exactly (lerp weight 1; (g - 0) * 1), and parameters unchanged."""
    return {n: st["exp_avg"] for n, st in named_optimizer_state(model, opts).items()}


@pytest.mark.parametrize(
    "shape",
    [
        Shape(),
        Shape(dropout=0.0, hidden_dims=(16,)),
        Shape(U=50, I=300, F=37, H=24, D=12, B=40, N=3, gate_hidden=20, hidden_dims=(24,)),
        Shape(U=64, I=512, F=20, D=16, B=64, N=5, hidden_dims=(32, 24)),
        Shape(mimic=False),
        Shape(sparse=False),
        Shape(padding_idx=5),
        Shape(sparse=False, padding_idx=5),
        Shape(fusion="sum"),
        Shape(fusion="concat"),
        Shape(U=50, I=300, F=37, H=24, D=12, B=40, N=3, hidden_dims=(24, 16), fusion="concat"),
        # concat with the reference's default output_dim (embedding + feature width, encoders.py:212),
        # and with a feature width and output_dim of their own (the mimic tables output-wide)
        Shape(fusion="concat", concat_out=None),
        Shape(U=50, I=300, F=37, H=24, D=12, B=40, N=3, hidden_dims=(24,), fusion="concat", feature_out=20, concat_out=28),
        Shape(fusion="concat", feature_out=12, concat_out=20, sparse=False, mimic=False),
        # the reference's other activations (encoders.py:68-78), with dropout (injected keep masks)
        Shape(activation="gelu"),
        Shape(activation="tanh"),
        Shape(activation="selu"),
        Shape(U=50, I=300, F=37, H=24, D=12, B=40, N=3, hidden_dims=(24, 16), activation="gelu", fusion="sum"),
        # five hidden layers (six Linear)
        Shape(hidden_dims=(16, 12, 20, 8, 16)),
        Shape(hidden_dims=(16, 12, 20, 8, 16), activation="tanh", dropout=0.0),
        # identity feature encoder (encoders.py:114-119, F == D) and a single Linear encoder
        Shape(F=8, feature_type="identity"),
        Shape(F=8, feature_type="identity", fusion="sum"),
        Shape(feature_type="linear"),
    ],
    ids=["tiny", "nodrop", "odd", "2hidden", "nomimic", "dense-id", "padding", "dense-id-padding", "sum", "concat",
         "concat-odd", "concat-default-out", "concat-out28", "concat-out20-dense-nomimic", "gelu", "tanh", "selu", "gelu-2hidden-sum", "5hidden", "5hidden-tanh", "identity-enc",
         "identity-enc-sum", "linear-enc"],
)
def test_step_gradients_match_oracle(shape):
    from gpu_helpers import run_ttamm

    prob = make_problem(shape, steps=1)
    om, oo, ores = run_oracle(prob, lr=0.0, betas=(0.0, 0.999))
    tm, to, tres = run_ttamm(prob, lr=0.0, betas=(0.0, 0.999))
    assert abs(tres[0]["total"] - ores[0].total) <= GRAD_TOL * abs(ores[0].total)
    assert abs(tres[0]["bce"] - ores[0].bce) <= GRAD_TOL * abs(ores[0].bce)
    if shape.mimic:
        assert abs(tres[0]["mimic_user"] - ores[0].mimic_user) <= GRAD_TOL * abs(ores[0].mimic_user)
        assert abs(tres[0]["mimic_item"] - ores[0].mimic_item) <= GRAD_TOL * abs(ores[0].mimic_item)
    og = _grads_by_name(om, oo)
    tg = _grads_by_name(tm, to)
    assert set(og) == set(tg)
    for name in og:
        err = rel_err(tg[name], og[name])
        assert err <= GRAD_TOL, f"{name}: rel err {err:.3e}"
    # lr = 0: parameters untouched
    for (n, p), (_, q) in zip(om.state_dict().items(), tm.state_dict().items()):
        assert torch.equal(q.cpu(), p), n


@pytest.mark.parametrize("shape", [Shape(), Shape(sparse=False), Shape(padding_idx=5), Shape(sparse=False, padding_idx=5),
                                   Shape(fusion="concat"), Shape(sparse=False, max_norm=0.05)],
                         ids=["tiny", "dense-id", "padding", "dense-id-padding", "concat", "max-norm"])
def test_three_steps_match_oracle(shape):
    from gpu_helpers import run_ttamm

    prob = make_problem(shape, steps=3)
    om, oo, ores = run_oracle(prob)
    tm, to, tres = run_ttamm(prob)
    for o, t in zip(ores, tres):
        assert abs(t["total"] - o.total) <= 1e-5 * abs(o.total)
    osd, tsd = om.state_dict(), tm.state_dict()
    for n in osd:
        # Adam normalises each update to ~lr: compare the parameter *change* relative to lr.
        d = (tsd[n].cpu() - osd[n]).abs().max().item()
        assert d <= 1e-3 * 1e-3 * 50, f"{n}: max abs diff {d:.3e}"
    ost, tst = named_optimizer_state(om, oo), named_optimizer_state(tm, to)
    for n in ost:
        assert rel_err(tst[n]["exp_avg"], ost[n]["exp_avg"]) <= 1e-4, n
        assert rel_err(tst[n]["exp_avg_sq"], ost[n]["exp_avg_sq"]) <= 1e-4, n
        assert float(tst[n]["step"]) == float(ost[n]["step"]), n
    if shape.padding_idx is not None and shape.sparse:
        # SparseAdam never sees the padding row (torch drops it from the sparse gradient)
        init = prob.model.state_dict()
        for n in ("user_encoder.embedding.weight", "item_encoder.embedding.weight"):
            assert torch.equal(tsd[n][shape.padding_idx].cpu(), init[n][shape.padding_idx]), n
            assert not tst[n]["exp_avg"][shape.padding_idx].any(), n


# bf16 towers (ttamm.h ttamm_tower.matmul_bf16; BASELINE config C5): checked against the
# oracle's bf16 restatement (oracle/cpu_reference.py _BF16Linear: operands rounded to bf16,
# fp32 accumulation).  Both sides round the SAME definition, but an fp32 activation that differs
# by one ulp (summation order) can round to the neighbouring bf16 value, so the tolerance is the
# bf16 one: max-norm relative 2e-3 per tensor, and the mean error stays at fp32 level.
# D == Hg in {128, 256} runs the fused bf16 gate (gate16.hip) unless TTAMM_GENERIC_GATE=1 ("generic").
BF16_TOL = 2e-3


@pytest.mark.parametrize("generic", [False, True], ids=["fused", "generic"])
@pytest.mark.parametrize(
    "shape",
    [
        Shape(matmul_dtype="bf16"),
        Shape(U=50, I=300, F=37, H=24, D=12, B=40, N=3, gate_hidden=20, hidden_dims=(24,), matmul_dtype="bf16"),
        Shape(U=96, I=768, F=605, H=512, D=256, B=48, N=5, hidden_dims=(512,), matmul_dtype="bf16"),
        Shape(U=3000, I=20000, F=64, H=128, D=128, B=1500, N=3, hidden_dims=(128,), matmul_dtype="bf16"),
        Shape(U=2000, I=8000, F=605, H=512, D=256, B=300, N=3, hidden_dims=(512,), matmul_dtype="bf16", mimic=False),
    ],
    ids=["tiny", "odd", "c5-dims", "d128-rows", "d256-nomimic"],
)
def test_bf16_step_gradients_match_bf16_oracle(shape, generic, monkeypatch):
    from gpu_helpers import run_ttamm

    if generic:
        monkeypatch.setenv("TTAMM_GENERIC_GATE", "1")
    else:
        monkeypatch.delenv("TTAMM_GENERIC_GATE", raising=False)

    prob = make_problem(shape, steps=1)
    om, oo, ores = run_oracle(prob, lr=0.0, betas=(0.0, 0.999))
    tm, to, tres = run_ttamm(prob, lr=0.0, betas=(0.0, 0.999))
    for key in ("total", "bce", "mimic_user", "mimic_item"):
        assert abs(tres[0][key] - getattr(ores[0], key)) <= 1e-4 * abs(getattr(ores[0], key)), key
    og, tg = _grads_by_name(om, oo), _grads_by_name(tm, to)
    assert set(og) == set(tg)
    for name in og:
        err = rel_err(tg[name], og[name])
        mean = ((tg[name].double() - og[name].double()).abs().mean() / og[name].double().abs().max().clamp_min(1e-30)).item()
        assert err <= BF16_TOL, f"{name}: rel err {err:.3e}"
        assert mean <= 2e-5, f"{name}: mean rel err {mean:.3e}"
    # the bf16 path really rounds: fp32 GEMMs on the same inputs give gradients measurably
    # farther from the bf16 oracle than ttamm's bf16 step is
    prob32 = make_problem(Shape(**{**shape.__dict__, "matmul_dtype": "fp32"}), steps=1)
    m32, o32, _ = run_oracle(prob32, lr=0.0, betas=(0.0, 0.999))
    g32 = _grads_by_name(m32, o32)
    far = max(rel_err(g32[n], og[n]) for n in og)
    near = max(rel_err(tg[n], og[n]) for n in og)
    assert far > 5e-4 and far > 4 * near, (far, near)


# Fused gate kernel (csrc/gate.hip: fp32 towers with D == Hg in {32, 64, 96, 128}) and the generic
# two-GEMM gate path (TTAMM_GENERIC_GATE=1), both against the oracle at the fp32 tolerance.
# Row counts are not multiples of the kernel's 16-row slabs (user rows = B, item rows = B(1+N)).
# D = 128 (C4's width) runs the 4-wave variant with G2 read from global memory and the backward's
# two matrices staged one after the other; "d128-rounds" has more 16-row slabs than the grid has
# waves (the backward's per-round staging runs twice in both towers).
GATE_SHAPES = [
    Shape(U=64, I=256, F=40, H=48, D=32, B=45, N=5, hidden_dims=(48,)),
    Shape(U=64, I=512, F=70, H=64, D=64, B=40, N=4, hidden_dims=(64,)),
    Shape(U=96, I=768, F=605, H=192, D=96, B=37, N=5, hidden_dims=(192,)),
    Shape(U=64, I=256, F=40, H=48, D=32, B=32, N=5, hidden_dims=(48,), mimic=False),
    Shape(U=64, I=256, F=40, H=48, D=32, B=32, N=5, hidden_dims=(48,), sparse=False),
    Shape(U=64, I=512, F=40, H=64, D=128, B=45, N=5, hidden_dims=(64,)),
    Shape(U=2500, I=24000, F=40, H=64, D=128, B=2000, N=8, hidden_dims=(64,)),
]


@pytest.mark.parametrize("generic", [False, True], ids=["fused", "generic"])
@pytest.mark.parametrize("shape", GATE_SHAPES,
                         ids=["d32", "d64", "d96-c2dims", "d32-nomimic", "d32-dense-id", "d128", "d128-rounds"])
def test_gate_paths_match_oracle(shape, generic, monkeypatch):
    if generic:
        monkeypatch.setenv("TTAMM_GENERIC_GATE", "1")
    else:
        monkeypatch.delenv("TTAMM_GENERIC_GATE", raising=False)
    _gate_case(shape)


def test_gate16_split_form_matches_oracle_at_d96(monkeypatch):
    """fp32 towers at D = 96 on gate16.hip's split-bf16 form (TTAMM_GATE16_SPLIT=1, opt-in: measured
    slower than gate.hip at C2), at the fp32 tolerance.  A developer switch: needs the make DEV=1
    library (TTAMM_LIBRARY=.../build_dev/libttamm.so)."""
    _require_developer_build()
    monkeypatch.setenv("TTAMM_GATE16_SPLIT", "1")
    monkeypatch.delenv("TTAMM_GENERIC_GATE", raising=False)
    _gate_case(GATE_SHAPES[2])


def _require_developer_build():
    from ttamm import _lib

    if not _lib.load().ttamm_developer_build():
        pytest.skip("developer switch: needs the make DEV=1 library (TTAMM_LIBRARY)")


def _gate_case(shape):
    from gpu_helpers import run_ttamm

    prob = make_problem(shape, steps=1)
    om, oo, ores = run_oracle(prob, lr=0.0, betas=(0.0, 0.999))
    tm, to, tres = run_ttamm(prob, lr=0.0, betas=(0.0, 0.999))
    assert abs(tres[0]["total"] - ores[0].total) <= GRAD_TOL * abs(ores[0].total)
    og, tg = _grads_by_name(om, oo), _grads_by_name(tm, to)
    assert set(og) == set(tg)
    for name in og:
        err = rel_err(tg[name], og[name])
        assert err <= GRAD_TOL, f"{name}: rel err {err:.3e}"


@pytest.mark.parametrize("rows", [1024, 768], ids=["rps1024", "rps768"])
def test_long_wgrad_splits_match_oracle(rows, monkeypatch):
    """Weight-gradient split-K chunks longer than 512 rows (the C2 step picks 576): every row
    of a chunk must reach the gradient, including the gathered feature rows past row 512.  A
    developer switch (make DEV=1 library); the default library's C2 choice (576 rows) is covered
    by the full-size parity tests."""
    from gpu_helpers import run_ttamm

    _require_developer_build()

    monkeypatch.setenv("TTAMM_WGRAD_ROWS_PER_SPLIT", str(rows))
    shape = Shape(U=400, I=3000, F=40, H=64, D=32, B=400, N=5, hidden_dims=(64,))
    prob = make_problem(shape, steps=1)
    om, oo, _ = run_oracle(prob, lr=0.0, betas=(0.0, 0.999))
    tm, to, _ = run_ttamm(prob, lr=0.0, betas=(0.0, 0.999))
    og, tg = _grads_by_name(om, oo), _grads_by_name(tm, to)
    for name in og:
        err = rel_err(tg[name], og[name])
        assert err <= GRAD_TOL, f"{name}: rel err {err:.3e}"


# gradient_clip_norm (training.py:824-825): clip_grad_norm_ over every parameter between backward
# and the optimizers.  Dense ID tables (torch cannot clip the sparse ones: see
# test_host_cpu.test_reference_clipping_rejects_sparse_id_gradients).  max_norm 0.05 clips every
# step of this problem; 100 never does (coefficient 1).
@pytest.mark.parametrize("max_norm", [0.05, 100.0], ids=["clipped", "unclipped"])
def test_gradient_clipping_matches_oracle(max_norm):
    from gpu_helpers import run_ttamm

    shape = Shape(sparse=False)
    prob = make_problem(shape, steps=3)
    om, oo, ores = run_oracle(prob, gradient_clip_norm=max_norm)
    tm, to, tres = run_ttamm(prob, gradient_clip_norm=max_norm)
    for o, t in zip(ores, tres):
        assert abs(t["total"] - o.total) <= 1e-5 * abs(o.total)
    osd, tsd = om.state_dict(), tm.state_dict()
    for n in osd:
        d = (tsd[n].cpu() - osd[n]).abs().max().item()
        assert d <= 1e-3 * 1e-3 * 50, f"{n}: max abs diff {d:.3e}"
    ost, tst = named_optimizer_state(om, oo), named_optimizer_state(tm, to)
    for n in ost:
        assert rel_err(tst[n]["exp_avg"], ost[n]["exp_avg"]) <= 1e-4, n
        assert rel_err(tst[n]["exp_avg_sq"], ost[n]["exp_avg_sq"]) <= 1e-4, n
    if max_norm < 1:  # the clip was active: the moments differ from an unclipped run
        om2, oo2, _ = run_oracle(prob)
        ost2 = named_optimizer_state(om2, oo2)
        assert any(rel_err(ost2[n]["exp_avg"], ost[n]["exp_avg"]) > 1e-2 for n in ost)


def test_gradient_clipping_rejects_sparse_id_tables():
    from gpu_helpers import run_ttamm

    prob = make_problem(Shape(), steps=1)
    with pytest.raises(NotImplementedError, match="sparse"):
        run_ttamm(prob, gradient_clip_norm=1.0)


def test_max_norm_renormalises_looked_up_rows():
    """nn.Embedding(max_norm) (encoders.py:48,58): the step renorms the rows it looks up in place,
    as torch's embedding_renorm_ does in the reference's forward: after one step with lr = 0 the
    looked-up rows of both ID tables equal the oracle's (the renorm is the only change), and
    rows no batch touched keep their norm."""
    from gpu_helpers import run_ttamm

    shape = Shape(sparse=False, max_norm=0.05)
    prob = make_problem(shape, steps=1)
    init = {k: v.clone() for k, v in prob.model.state_dict().items()}
    om, oo, ores = run_oracle(prob, lr=0.0, betas=(0.0, 0.999), weight_decay=0.0)
    tm, to, tres = run_ttamm(prob, lr=0.0, betas=(0.0, 0.999), weight_decay=0.0)
    assert abs(tres[0]["total"] - ores[0].total) <= GRAD_TOL * abs(ores[0].total)
    osd, tsd = om.state_dict(), tm.state_dict()
    for n in ("user_encoder.embedding.weight", "item_encoder.embedding.weight"):
        changed = (osd[n] != init[n]).any(dim=1)
        assert changed.any(), n  # the renorm did act
        assert (tsd[n].cpu().norm(dim=1)[changed] <= 0.05 * (1 + 1e-6)).all(), n
        assert rel_err(tsd[n].cpu(), osd[n]) <= 1e-6, n


def test_ragged_batches_full_short_full():
    """A short batch between full ones (the epoch's last batch is short, training.py:1382
    drop_last=False; here in the middle, so a full batch follows it on the same workspace).
    Every step must be counted (steps_applied; the prologue's completion counter sits at a
    batch-size-independent offset) and the tables / optimizer state must match the oracle."""
    import ttamm
    from gpu_helpers import ttamm_model_from, ttamm_optimizers
    from helpers import LOSS_WEIGHTS

    shape = Shape(dropout=0.0)
    prob = make_problem(shape, steps=3)
    b = 13
    users, pos, neg, um, im = prob.batches[1]
    prob.batches[1] = (users[:b], pos[:b], neg[:b], [m[:b] for m in um], [m[: b * (1 + shape.N)] for m in im])
    om, oo, ores = run_oracle(prob)
    tm = ttamm_model_from(prob)
    to = ttamm_optimizers(tm)
    eng = ttamm.FusedTrainStep(tm, to, negatives_per_positive=shape.N, positives=prob.positives,
                               user_features=prob.user_features.cuda(), item_features=prob.item_features.cuda(),
                               loss_weights=LOSS_WEIGHTS, max_batch=shape.B)
    for k, (u, p, n, a, c) in enumerate(prob.batches):
        eng.step(u.cuda(), p.cuda(), n.cuda().reshape(-1),
                 keep_masks={"user": [m.cuda() for m in a], "item": [m.cuda() for m in c]})
        torch.cuda.synchronize()
        assert int(eng.steps_applied.item()) == k + 1, f"step {k} not counted"
        got = eng.last_losses()["total"]
        assert abs(got - ores[k].total) <= 1e-5 * abs(ores[k].total), (k, got, ores[k].total)
    eng.finish()
    osd, tsd = om.state_dict(), tm.state_dict()
    for n in osd:
        d = (tsd[n].cpu() - osd[n]).abs().max().item()
        assert d <= 1e-3 * 1e-3 * 50, f"{n}: max abs diff {d:.3e}"
    ost, tst = named_optimizer_state(om, oo), named_optimizer_state(tm, to)
    for n in ost:
        assert rel_err(tst[n]["exp_avg"], ost[n]["exp_avg"]) <= 1e-4, n
        assert float(tst[n]["step"]) == float(ost[n]["step"]) == 3.0, n
