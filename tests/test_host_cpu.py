"""Host-side logic of the ttamm drop-in modules on CPU: construction, parameter layout,
state_dict / optimizer-group compatibility with the reference, error conventions, and the
no-fallback rule (compute on a CPU tensor raises; it never silently runs PyTorch ops)."""

import pytest
import torch

import ttamm
from helpers import Shape
from oracle import cpu_reference as ref


def _model(shape: Shape):
    cfg = shape.tower_cfg()
    ue = ttamm.build_tower_encoder(cfg, num_embeddings=shape.U, feature_dim=shape.F)
    ie = ttamm.build_tower_encoder(cfg, num_embeddings=shape.I, feature_dim=shape.F)
    mm = ttamm.AdaptiveMimicMechanism(num_users=shape.U, num_items=shape.I, embedding_dim=shape.D)
    return ttamm.TwoTowerModel(ue, ie, similarity=ttamm.DotProductSimilarity(), adaptive_mimic=mm)


@pytest.mark.parametrize("shape", [Shape(), Shape(dropout=0.0), Shape(hidden_dims=(16, 12)), Shape(gate_hidden=20)])
def test_state_dict_keys_match_reference_layout(shape):
    ours = _model(shape).state_dict()
    oracle = ref.build_model(shape.tower_cfg(), num_users=shape.U, num_items=shape.I, user_feature_dim=shape.F,
                             item_feature_dim=shape.F).state_dict()
    assert list(ours.keys()) == list(oracle.keys())
    for k in ours:
        assert ours[k].shape == oracle[k].shape, k
    # dropout > 0 puts the second Linear at network.3, dropout == 0 at network.2 (encoders.py:132-142)
    keys = " ".join(ours)
    if shape.dropout and len(shape.hidden_dims) == 1:
        assert "feature_encoder.network.3.weight" in keys
    if not shape.dropout:
        assert "feature_encoder.network.2.weight" in keys


def test_same_seed_same_init_as_oracle():
    """Construction order matches the reference, so the same seed gives the same weights."""
    shape = Shape()
    torch.manual_seed(7)
    ours = _model(shape).state_dict()
    torch.manual_seed(7)
    oracle = ref.build_model(shape.tower_cfg(), num_users=shape.U, num_items=shape.I, user_feature_dim=shape.F,
                             item_feature_dim=shape.F).state_dict()
    for k in ours:
        assert torch.equal(ours[k], oracle[k]), k


def test_parameter_groups_follow_reference_order():
    model = _model(Shape())
    dense, sparse = ttamm._collect_parameter_groups(model)
    names = {id(p): n for n, p in model.named_parameters()}
    assert [names[id(p)] for p in sparse] == ["user_encoder.embedding.weight", "item_encoder.embedding.weight"]
    dn = [names[id(p)] for p in dense]
    assert dn[0].startswith("user_encoder.feature_encoder")
    assert dn[-2:] == ["adaptive_mimic.user_augmented.weight", "adaptive_mimic.item_augmented.weight"]
    assert len(dn) + len(sparse) == len(list(model.parameters()))
    o_dense, o_sparse = ref.parameter_groups(
        ref.build_model(Shape().tower_cfg(), num_users=64, num_items=256, user_feature_dim=12, item_feature_dim=12))
    assert [p.shape for p in dense] == [p.shape for p in o_dense]


def test_encoder_config_errors():
    with pytest.raises(ValueError, match="max_norm"):
        ttamm.build_id_embedding({"params": {"embedding_dim": 4, "sparse": True, "max_norm": 1.0}}, num_embeddings=3)
    with pytest.raises(ValueError, match="Unsupported fusion"):
        ttamm.TowerEncoder(embedding=torch.nn.Embedding(3, 4), feature_encoder=None, fusion="bogus", output_dim=None,
                           adaptive_mimic=None)
    with pytest.raises(ValueError, match="Identity feature encoder"):
        ttamm.build_feature_encoder({"type": "identity"}, input_dim=5, fallback_output_dim=4)
    with pytest.raises(ValueError, match="Unsupported activation"):
        ttamm.build_feature_encoder({"type": "mlp", "hidden_dims": [4], "activation": "swish"}, input_dim=5,
                                    fallback_output_dim=4)
    with pytest.raises(ValueError, match="must equal embedding dimension"):
        ttamm.build_tower_encoder({"id_embedding": {"params": {"embedding_dim": 8}},
                                   "feature_encoder": {"type": "linear", "output_dim": 4}, "fusion": "gated"},
                                  num_embeddings=3, feature_dim=5)
    with pytest.raises(ValueError, match="Unsupported encoder type"):
        ttamm.build_tower_encoder({"type": "graph"}, num_embeddings=3, feature_dim=0)
    with pytest.raises(ValueError, match="positive"):
        ttamm.AdaptiveMimicMechanism(num_users=0, num_items=3, embedding_dim=4)


def test_sparse_flag_reaches_embedding():
    """tests/test_encoders.py:29-42."""
    enc = ttamm.build_tower_encoder({"type": "tower", "id_embedding": {"params": {"embedding_dim": 4, "sparse": True}},
                                     "fusion": "identity"}, num_embeddings=10, feature_dim=0)
    assert enc.embedding.sparse
    assert enc.fusion == "identity"


def test_deprecated_fusion_alias_warns():
    fe = ttamm.build_feature_encoder({"type": "linear", "output_dim": 4}, input_dim=3, fallback_output_dim=4)
    with pytest.warns(DeprecationWarning):
        t = ttamm.TowerEncoder(embedding=torch.nn.Embedding(3, 4), feature_encoder=fe, fusion="adaptive_mimic",
                               output_dim=None, adaptive_mimic=ttamm.FeatureFusionGate(4))
    assert t.fusion == "gated"


def test_no_cpu_fallback():
    """Compute on CPU tensors raises instead of running PyTorch ops (the product path is HIP)."""
    model = _model(Shape()).eval()
    with torch.no_grad(), pytest.raises(RuntimeError, match="ROCm"):
        model.item_encoder({"indices": torch.tensor([0, 1]), "features": torch.randn(2, 12)})
    with torch.no_grad(), pytest.raises(RuntimeError, match="ROCm"):
        model.adaptive_mimic.augment_items(torch.tensor([0, 1]), torch.zeros(2, 8))
    with pytest.raises(RuntimeError, match="ROCm"):
        ttamm.sample_negative_items(torch.tensor([0]), num_items=5, positives={}, num_negatives=2,
                                    device=torch.device("cpu"))
    dense, sparse = ttamm._collect_parameter_groups(model)
    opts = [torch.optim.AdamW(dense), torch.optim.SparseAdam(sparse)]
    with pytest.raises(RuntimeError, match="ROCm"):
        ttamm.FusedTrainStep(model, opts, negatives_per_positive=2, positives={}, user_features=None,
                             item_features=None, max_batch=4)


def test_mimic_index_dtype_error_precedes_device_check():
    mech = ttamm.AdaptiveMimicMechanism(num_users=4, num_items=6, embedding_dim=8)
    with pytest.raises(ValueError, match="torch.long"):
        mech.augment_items(torch.tensor([0, 1], dtype=torch.int32), torch.zeros(2, 8))


def test_sampler_argument_errors():
    with pytest.raises(ValueError, match="greater than zero"):
        ttamm.sample_negative_items(torch.tensor([0]), num_items=5, positives={}, num_negatives=0,
                                    device=torch.device("cpu"))
    with pytest.raises(ValueError, match="greater than one"):
        ttamm.sample_negative_items(torch.tensor([0]), num_items=1, positives={}, num_negatives=2,
                                    device=torch.device("cpu"))


def test_positives_csr_from_mapping():
    csr = ttamm.PositivesCSR.from_mapping({0: {3, 1}, 2: {5}}, device=torch.device("cpu"), num_users=4)
    assert csr.offsets.tolist() == [0, 2, 2, 3, 3]
    assert csr.values.tolist() == [1, 3, 5]
    assert csr.num_users == 4 and csr.max_degree == 2


def test_train_one_epoch_rejects_unsupported_options():
    model = _model(Shape())
    dense, sparse = ttamm._collect_parameter_groups(model)
    opts = [torch.optim.AdamW(dense), torch.optim.SparseAdam(sparse)]
    kw = dict(optimizers=opts, negatives_per_positive=2, num_items=256, user_positive_items={}, user_features=None,
              item_features=None, device=torch.device("cpu"))
    with pytest.raises(NotImplementedError, match="BCEWithLogitsLoss"):
        ttamm.train_one_epoch(model, [], criterion=torch.nn.BCEWithLogitsLoss(reduction="sum"), **kw)
    assert ttamm.train_one_epoch(model, [], criterion=torch.nn.BCEWithLogitsLoss(), **kw) == 0.0


def test_reference_clipping_rejects_sparse_id_gradients():
    """training.py:824-825 calls clip_grad_norm_(model.parameters(), ...): with the default sparse
    ID tables (configs/default.yaml:30,47) torch raises NotImplementedError on their sparse
    gradients — the fused step raises the same type there and clips dense-ID models."""
    from helpers import make_problem
    from oracle import cpu_reference as ref

    prob = make_problem(Shape(), steps=1)
    opts = ref.build_optimizers(prob.model, lr=1e-3)
    users, pos, neg, um, im = prob.batches[0]
    with pytest.raises(NotImplementedError):
        ref.train_step(prob.model, opts, users, pos, neg, user_features=prob.user_features,
                       item_features=prob.item_features, user_keep_masks=um, item_keep_masks=im,
                       gradient_clip_norm=1.0)
