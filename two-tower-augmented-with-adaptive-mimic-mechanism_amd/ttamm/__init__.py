"""ttamm — MI355X-native training step for the two-tower model with an adaptive mimic
mechanism (drop-in for alperkartkaya2-afk/two-tower-augmented-with-adaptive-mimic-mechanism's
models + training hot loop).  Compute runs in libttamm.so (gfx950 HIP kernels); see
include/ttamm.h for the C ABI and DESIGN.md for the design."""

from .adaptive_mimic import AdaptiveMimicMechanism
from .data import DeviceInteractionLoader, load_features, load_interactions, save_features, save_interactions
from .encoders import (
    FeatureEncoderConfig,
    FeatureEncoderWrapper,
    FeatureFusionGate,
    TowerEncoder,
    build_feature_encoder,
    build_id_embedding,
    build_tower_encoder,
)
from .inbatch import inbatch_bce
from .retrieval import encode_item_embeddings, evaluate_model, prepare_faiss_resources
from .samplers import PositivesCSR, sample_negative_items
from .training import DotProductSimilarity, FusedTrainStep, _collect_parameter_groups, train_one_epoch
from .two_tower import TwoTowerModel

__all__ = [
    "AdaptiveMimicMechanism",
    "DeviceInteractionLoader",
    "DotProductSimilarity",
    "FeatureEncoderConfig",
    "FeatureEncoderWrapper",
    "FeatureFusionGate",
    "FusedTrainStep",
    "PositivesCSR",
    "TowerEncoder",
    "TwoTowerModel",
    "build_feature_encoder",
    "build_id_embedding",
    "build_tower_encoder",
    "encode_item_embeddings",
    "evaluate_model",
    "inbatch_bce",
    "load_features",
    "load_interactions",
    "prepare_faiss_resources",
    "sample_negative_items",
    "save_features",
    "save_interactions",
    "train_one_epoch",
]
