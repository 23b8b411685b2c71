"""The CPU oracle against (1) the reference's own known-answer / property tests, restated,
and (2) the committed golden fixtures (regression guard for the oracle itself)."""

import numpy as np
import pytest
import torch

from golden_io import NAMES, load
from helpers import named_optimizer_state, rel_err, run_oracle
from oracle import cpu_reference as ref


# ---- reference tests restated on the oracle (tests/test_metrics.py, test_training_utils.py,
#      test_samplers.py, test_adaptive_mimic.py, test_encoders.py) ---------------------------
def test_ranking_metrics_known_answer():
    """tests/test_metrics.py:4-19."""
    m = ref.ranking_metrics({0: [3, 2, 1], 1: [4, 5, 6]}, {0: {1, 2}, 1: {4}}, [1, 2, 3])
    assert m.recall[1] == 0.5
    assert m.precision[1] == 0.5
    assert m.hit_rate[1] == 0.5
    assert m.recall[3] > m.recall[1]
    assert abs(m.mrr - 0.75) < 1e-6


def test_metric_lookup_known_answer():
    """tests/test_training_utils.py:44-52: recall@2 == 1.0 for {0: [1, 2, 3]} vs {0: {2}}."""
    m = ref.ranking_metrics({0: [1, 2, 3]}, {0: {2}}, [1, 2, 3])
    assert m.recall[2] == pytest.approx(1.0)
    assert 5 not in m.precision


def test_sampler_excludes_positives():
    """tests/test_samplers.py:6-19."""
    torch.manual_seed(0)
    positives = {0: {1, 2}, 1: {0}}
    neg = ref.sample_negative_items(torch.tensor([0, 1]), num_items=5, positives=positives, num_negatives=2)
    assert neg.shape == (2, 2)
    assert all(i not in positives[0] for i in neg[0].tolist())
    assert all(i not in positives[1] for i in neg[1].tolist())


def test_sampler_errors():
    with pytest.raises(ValueError):
        ref.sample_negative_items(torch.tensor([0]), num_items=5, positives={}, num_negatives=0)
    with pytest.raises(ValueError):
        ref.sample_negative_items(torch.tensor([0]), num_items=1, positives={}, num_negatives=1)
    with pytest.raises(RuntimeError):
        ref.sample_negative_items(torch.tensor([0]), num_items=3, positives={0: {0, 1, 2}}, num_negatives=1)


def test_mimic_shapes_and_losses():
    """tests/test_adaptive_mimic.py:6-33."""
    mech = ref.OracleMimic(4, 6, 8, init_std=0.01)
    u = torch.tensor([0, 1])
    i = torch.tensor([2, 3])
    ue, ie = torch.zeros((2, 8)), torch.ones((2, 8))
    au, a_u = ref.gather_aug(mech.user_augmented, u, ue)
    ai, a_i = ref.gather_aug(mech.item_augmented, i, ie)
    assert au.shape == ue.shape and ai.shape == ie.shape
    assert torch.nn.functional.mse_loss(a_u, ie).item() >= 0
    with pytest.raises(ValueError):
        ref.gather_aug(mech.item_augmented, i.int(), ie)
    with pytest.raises(ValueError):
        ref.OracleMimic(0, 6, 8)


def test_gated_tower_shape():
    """tests/test_encoders.py:6-26."""
    cfg = {"type": "tower", "id_embedding": {"params": {"embedding_dim": 8}},
           "feature_encoder": {"type": "linear", "output_dim": 8}, "fusion": "gated",
           "adaptive_mimic": {"hidden_dim": 16}}
    tower = ref.build_tower(cfg, num_embeddings=5, feature_dim=4)
    out = ref.tower_forward(tower, torch.tensor([0, 1, 2]), torch.randn(3, 4), training=False)
    assert out.shape == (3, 8)


# ---- golden fixtures -------------------------------------------------------------------------
@pytest.mark.parametrize("name", NAMES)
def test_oracle_reproduces_golden(name):
    prob, arr = load(name)
    gm, go, gres = run_oracle(prob, lr=0.0, betas=(0.0, 0.999), steps=1)
    want = torch.from_numpy(arr["grads/loss"])
    got = torch.tensor([gres[0].total, gres[0].bce, gres[0].mimic_user, gres[0].mimic_item], dtype=torch.float64)
    assert torch.allclose(got, want, rtol=1e-6, atol=1e-7)
    for pname, st in named_optimizer_state(gm, go).items():
        assert rel_err(st["exp_avg"], torch.from_numpy(arr[f"grads/{pname}"])) <= 1e-6, pname
    sm, so, sres = run_oracle(prob, steps=3)
    for k, v in sm.state_dict().items():
        assert torch.allclose(v, torch.from_numpy(arr[f"steps3/param/{k}"]), rtol=1e-6, atol=1e-8), k


# ---- exact-IP retrieval restatement (training.py:613-679, :944-970) ----------------------
def test_flat_ip_search_known_answer():
    items = np.array([[1, 0], [0, 1], [1, 1], [2, 0], [-1, 0]], dtype=np.float32)
    q = np.array([[1, 0], [0, 0]], dtype=np.float32)
    s, i = ref.flat_ip_search(items, q, 7)
    # query 0: scores [1, 0, 1, 2, -1] -> 3 (2), 0 (1), 2 (1), 1 (0), 4 (-1); ties by lower id
    assert i[0].tolist() == [3, 0, 2, 1, 4, -1, -1]
    assert s[0, :5].tolist() == [2, 1, 1, 0, -1]
    # query 1: all scores 0 -> id order
    assert i[1, :5].tolist() == [0, 1, 2, 3, 4]


def test_retrieve_with_faiss_filters_blocked_and_appends_truth():
    items = np.eye(6, dtype=np.float32)[:, :4] * np.arange(6, 0, -1, dtype=np.float32)[:, None]
    user = np.ones(4, dtype=np.float32)
    # scores: 6, 5, 4, 3, 0, 0 for items 0..5
    got = ref.retrieve_with_faiss(items, user, blocked={0, 2}, ground_truth={5}, max_k=3, faiss_search_k=80)
    assert got == [1, 3, 4]
    # only 2 unblocked candidates exist beyond the block: the ground truth is appended
    got = ref.retrieve_with_faiss(items[:4], user, blocked={0, 1}, ground_truth={9}, max_k=3, faiss_search_k=2)
    assert got == [2, 3, 9]


def test_normalize_l2_known_answer():
    """faiss.normalize_L2 restatement (training.py:670-672): unit rows, zero rows untouched."""
    x = np.array([[3, 4], [0, 0], [0, -2], [1, 1]], dtype=np.float32)
    y = ref.normalize_l2(x)
    assert y[0].tolist() == [np.float32(0.6), np.float32(0.8)]
    assert y[1].tolist() == [0.0, 0.0]
    assert y[2].tolist() == [0.0, -1.0]
    assert abs(float(y[3, 0]) - 2 ** -0.5) < 1e-7 and y[3, 0] == y[3, 1]
    assert x[0].tolist() == [3, 4]  # input not modified


def test_chunked_inbatch_definition_equals_train_step_block():
    """oracle.inbatch_bce_chunked (the definition the in-batch op tests use at full size) is the
    in-batch block of train_step(in_batch=True): autograd of BCEWithLogits over u @ p^T."""
    import torch
    from oracle import cpu_reference as ref

    g = torch.Generator().manual_seed(3)
    u = (torch.randn((37, 12), generator=g) * 0.4).double().requires_grad_()
    p = (torch.randn((37, 12), generator=g) * 0.4).double().requires_grad_()
    s = u @ p.t()
    loss = torch.nn.BCEWithLogitsLoss()(s.reshape(-1), torch.eye(37, dtype=s.dtype).reshape(-1))
    loss.backward()
    got_sum, du, dp = ref.inbatch_bce_chunked(u.detach(), p.detach(), chunk=10)
    assert abs(got_sum / 37 ** 2 - float(loss)) <= 1e-12
    assert torch.allclose(du, u.grad, rtol=0, atol=1e-14)
    assert torch.allclose(dp, p.grad, rtol=0, atol=1e-14)
    # a rank's block of a sharded batch: users 10..19 of the global batch score all 37 positives
    _, du2, _ = ref.inbatch_bce_chunked(u.detach()[10:20], p.detach(), row_base=10, inv_count=1 / 37 ** 2)
    assert torch.allclose(du2, u.grad[10:20], rtol=0, atol=1e-14)
