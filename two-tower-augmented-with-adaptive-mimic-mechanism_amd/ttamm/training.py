"""Training step — drop-in for the hot loop of ``src/pipelines/training.py``.

``train_one_epoch`` has the signature and return value of the reference's
``_train_one_epoch`` (training.py:700-833).  Each batch is one call of the native executor
``ttamm_train_step`` (libttamm), which runs the whole step on the MI355X:

    negatives (samplers.py:11-85) -> both towers (encoders.py:221-255) -> mimic augment and
    stop-grad MSE (adaptive_mimic.py:40-68) -> dot-product scores, BCE (training.py:770-803)
    -> backward -> AdamW over the dense group incl. the FULL mimic tables and SparseAdam over
    the ID tables (training.py:1311-1350).

The caller's torch optimizers stay the owners of the optimizer state: their ``state`` holds
the same ``exp_avg`` / ``exp_avg_sq`` / ``step`` entries torch would create, updated in place
by the kernels, so ``optimizer.state_dict()`` and checkpoints (training.py:150-182) keep
their format.
"""

from __future__ import annotations

import ctypes
from typing import Any, Callable, Iterable, Mapping, Sequence

import torch
from torch import nn

from . import _lib
from .encoders import TowerEncoder, describe_tower, feature_layers
from .samplers import PositivesCSR, draw_seed, positives_csr
from .two_tower import TwoTowerModel


class DotProductSimilarity(nn.Module):
    """<u, v> over the last dim (training.py:53-59)."""

    def forward(self, user_embedding: torch.Tensor, item_embedding: torch.Tensor) -> torch.Tensor:
        return (user_embedding * item_embedding).sum(dim=-1)


def _collect_parameter_groups(model: TwoTowerModel) -> tuple[list[nn.Parameter], list[nn.Parameter]]:
    """(dense, sparse) parameter lists in the reference's order (training.py:276-309):
    each tower's ID table first (sparse group if ``sparse=True``), then the tower's other
    parameters, then every remaining model parameter (the mimic tables) — dense."""
    dense: list[nn.Parameter] = []
    sparse: list[nn.Parameter] = []
    seen: set[int] = set()

    def put(p: nn.Parameter, bucket: list[nn.Parameter]) -> None:
        if id(p) not in seen:
            seen.add(id(p))
            bucket.append(p)

    for tower in (model.user_encoder, model.item_encoder):
        emb = getattr(tower, "embedding", None)
        if isinstance(emb, nn.Embedding):
            put(emb.weight, sparse if getattr(emb, "sparse", False) else dense)
        for name, p in tower.named_parameters():
            if name != "embedding.weight":
                put(p, dense)
    for p in model.parameters():
        put(p, dense)
    return dense, sparse


# ---------------------------------------------------------------------------------------
# optimizer state, torch-compatible
# ---------------------------------------------------------------------------------------
def _adam_state(opt: torch.optim.Optimizer, p: torch.Tensor) -> dict:
    st = opt.state[p]
    if len(st) == 0:  # torch/optim/adam.py _init_group
        st["step"] = torch.tensor(0.0, dtype=torch.float32)
        st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
    return st


def _sparse_adam_state(opt: torch.optim.Optimizer, p: torch.Tensor) -> dict:
    st = opt.state[p]
    if len(st) == 0:  # torch/optim/sparse_adam.py step()
        st["step"] = 0
        st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
    return st


def _single_group(opt: torch.optim.Optimizer) -> dict:
    if len(opt.param_groups) != 1:
        raise NotImplementedError("ttamm: one parameter group per optimizer (as training.py:1311-1350 builds)")
    return opt.param_groups[0]


def _pad_features(features: torch.Tensor | None) -> torch.Tensor | None:
    """Feature rows with a 16-byte aligned row stride (zero-padded columns).  A view of an
    already padded matrix (stride(0) % 4 == 0) is used as is."""
    if features is None or features.numel() == 0:
        return None
    if features.dtype != torch.float32:
        raise ValueError("ttamm: feature matrices must be float32")
    _lib.require_rocm(features, "feature matrix")
    if features.stride(-1) == 1 and features.stride(0) % 4 == 0 and features.data_ptr() % 16 == 0:
        return features
    rows, width = features.shape
    padded = torch.zeros((rows, (width + 3) // 4 * 4), dtype=torch.float32, device=features.device)
    padded[:, :width].copy_(features)
    return padded[:, :width]


def _dense_params(opt: torch.optim.Optimizer) -> list[torch.Tensor]:
    return [p for g in opt.param_groups for p in g["params"]]


class FusedTrainStep:
    """Owns the native step descriptor and workspace for one (model, optimizers) pair."""

    def __init__(
        self,
        model: TwoTowerModel,
        optimizers: Sequence[torch.optim.Optimizer],
        *,
        negatives_per_positive: int,
        positives: Mapping[int, set[int]] | PositivesCSR | None,
        user_features: torch.Tensor | None,
        item_features: torch.Tensor | None,
        loss_weights: Mapping[str, Any] | None = None,
        max_batch: int,
        seed: int | None = None,
        num_items: int | None = None,
        deferred_adamw: bool = True,
        replay_slices: int = 64,
        table_adamw_math: str = "exact",
        overlap: bool = True,
        aux_cus: int | None = None,
        item_category_tensor: torch.Tensor | None = None,
        major_category_id: int | None = None,
        in_batch_negatives: bool = False,
        gradient_clip_norm: float | None = None,
        feature_planes: bool = False,
    ) -> None:
        # feature_planes (developer option, off by default): fp32 towers keep their feature rows
        # pre-split into bf16 hi / mid / lo planes (1.5x the fp32 rows' bytes in HBM) for the first
        # layer's forward and weight gradient instead of splitting them inside the GEMMs (same
        # results, bit for bit).  Measured slower at C2: the forward GEMM reads 1.5x the gathered
        # bytes, 126 -> 135 us, the step 0.656 -> 0.664 ms (profiles/r05_s7_feature_planes.txt).
        # in_batch_negatives: ttamm's in-batch mode (ttamm.h ttamm_step_args.in_batch; not the
        # reference's behaviour): every user is also scored against every positive of the batch
        self.in_batch = bool(in_batch_negatives)
        if negatives_per_positive < 0 or (negatives_per_positive == 0 and not self.in_batch):
            raise ValueError("num_negatives must be greater than zero.")
        self.model = model
        self.num_neg = int(negatives_per_positive)
        ue, ie = model.user_encoder, model.item_encoder
        if not isinstance(ue, TowerEncoder) or not isinstance(ie, TowerEncoder):
            raise NotImplementedError("ttamm: towers must be ttamm.encoders.TowerEncoder")
        self.device = ue.embedding.weight.device
        _lib.require_rocm(ue.embedding.weight, "FusedTrainStep")
        # the sampler's range: the item table, or the global item count of a sharded step
        self.num_items = int(num_items) if num_items is not None else ie.num_embeddings
        if self.num_items <= 1:
            raise ValueError("num_items must be greater than one.")
        mimic = getattr(model, "adaptive_mimic", None)
        self.mimic = mimic
        if mimic is not None and (ue.output_dim != ie.output_dim):
            raise ValueError("Adaptive mimic requires user and item embedding dimensions to match.")

        # ---- optimizers ---------------------------------------------------------------
        dense_opt = sparse_opt = None
        for opt in optimizers:
            if isinstance(opt, torch.optim.SparseAdam):
                sparse_opt = opt
            elif isinstance(opt, (torch.optim.AdamW, torch.optim.Adam, torch.optim.SGD)):
                dense_opt = opt
            else:
                raise NotImplementedError(
                    f"ttamm: optimizer {type(opt).__name__} is not implemented (Adam / AdamW / SGD + SparseAdam)")
        self.dense_opt, self.sparse_opt = dense_opt, sparse_opt
        # the dense group's optimizer (training.py:1311-1333): Adam / AdamW, or SGD with momentum
        self.sgd = isinstance(dense_opt, torch.optim.SGD)
        # SGD with / without momentum decides, once, what the kernels' moment slots alias (the
        # momentum buffer, or the parameter itself) and whether the tables' g = 0 rows are deferred
        self._sgd_momentum_on = self.sgd and float(dense_opt.param_groups[0]["momentum"]) != 0.0
        self._sgd_buffers: list[tuple[torch.Tensor, torch.Tensor]] = []  # (param, buffer) not yet in state
        dense_ids = {id(p) for g in (dense_opt.param_groups if dense_opt else []) for p in g["params"]}
        sparse_ids = {id(p) for g in (sparse_opt.param_groups if sparse_opt else []) for p in g["params"]}
        self.decoupled = False
        if dense_opt is not None:
            g = _single_group(dense_opt)
            if g.get("amsgrad") or g.get("maximize"):
                raise NotImplementedError("ttamm: amsgrad / maximize are not implemented")
            if self.sgd and g.get("differentiable"):
                raise NotImplementedError("ttamm: differentiable SGD is not implemented")
            self.decoupled = isinstance(dense_opt, torch.optim.AdamW) or bool(g.get("decoupled_weight_decay", False))
        if sparse_opt is not None and _single_group(sparse_opt).get("maximize"):
            raise NotImplementedError("ttamm: maximize is not implemented")

        self.features = {"user": _pad_features(user_features), "item": _pad_features(item_features)}
        state: dict[int, dict] = {}
        handled: set[int] = set()
        self._adam_steps: list[dict] = []
        self._sparse_steps: list[dict] = []

        def dense_param(p: torch.Tensor) -> None:
            if id(p) not in dense_ids:
                raise ValueError("ttamm: a trained parameter is missing from the dense optimizer")
            if self.sgd:
                state[id(p)] = self._sgd_state(dense_opt, p)
            else:
                st = _adam_state(dense_opt, p)
                state[id(p)] = st
                self._adam_steps.append(st)
            handled.add(id(p))

        self.towers = {}
        for name, tower in (("user", ue), ("item", ie)):
            emb = tower.embedding.weight
            if id(emb) in sparse_ids:
                st = _sparse_adam_state(sparse_opt, emb)
                state[id(emb)] = st
                self._sparse_steps.append(st)
                handled.add(id(emb))
                id_opt = _lib.OPT_SPARSE_ADAM
            else:
                dense_param(emb)
                id_opt = _lib.OPT_DENSE
            feats = self.features[name]
            uses_features = tower.fusion != "identity" and feats is not None
            if uses_features:
                linears, _ = feature_layers(tower)
                for layer in linears:
                    dense_param(layer.weight)
                    dense_param(layer.bias)
                if tower.fusion == "gated":
                    for i in (0, 2):
                        dense_param(tower.adaptive_mimic.gate_network[i].weight)
                        dense_param(tower.adaptive_mimic.gate_network[i].bias)
                elif tower.fusion == "concat":
                    dense_param(tower.projection.weight)
                    dense_param(tower.projection.bias)
            elif tower.fusion != "identity":
                # no feature rows: the reference's tower falls back to the ID embedding
                # (encoders.py:228-231), so these parameters get no gradient and torch's
                # optimizers skip them (no state, no step) — as here
                for p in tower.parameters():
                    if p is not emb:
                        handled.add(id(p))
            self.towers[name] = (tower, feats if uses_features else None, id_opt)
        self.mimic_tables = {}
        if mimic is not None:
            for name, table in (("user", mimic.user_augmented.weight), ("item", mimic.item_augmented.weight)):
                dense_param(table)
                self.mimic_tables[name] = table
        unhandled = [i for i in dense_ids | sparse_ids if i not in handled]
        if unhandled:
            raise NotImplementedError(
                "ttamm: the optimizers hold parameters outside the fused step"
            )
        self.state = state

        # ---- descriptor ---------------------------------------------------------------
        args = _lib.StepArgs()
        for name in ("user", "item"):
            tower, feats, id_opt = self.towers[name]
            desc = describe_tower(
                tower if feats is not None else _IdentityView(tower),
                features=feats,
                mimic_table=self.mimic_tables.get(name),
                state=state,
                id_optimizer=id_opt,
            )
            if feats is not None and getattr(tower, "matmul_dtype", "fp32") == "bf16":
                # bf16 towers: the feature rows rounded to bf16 once (RNE, the values every bf16
                # GEMM of the step rounds them to), so the first layer streams half the bytes
                f16 = self._bf16_copy(feats)
                desc.features_bf16 = f16.data_ptr()
                desc.feat_bf16_ld = f16.stride(0)
            elif feats is not None and feature_planes:
                # fp32 towers: the feature rows split once into their bf16 hi / mid / lo planes (the
                # split every split-bf16 GEMM of the step forms), so the first layer's forward and
                # weight gradient stage them instead of splitting in every k-tile (same bits)
                fp = self._planes_copy(feats)
                desc.features_planes = fp.data_ptr()
                desc.feat_planes_ld = fp.stride(0)
            setattr(args, name, desc)
        args.mimic_enabled = 1 if mimic is not None else 0
        args.in_batch = 1 if self.in_batch else 0
        lw = dict(loss_weights or {})
        args.hp.lambda_mimic_user = float(lw.get("mimic_user", 0.0))
        args.hp.lambda_mimic_item = float(lw.get("mimic_item", 0.0))
        # category-alignment loss (training.py:530-579, :805-820): the reference returns 0
        # without a category tensor / major id, so the fused step runs it only with both
        args.hp.lambda_category_alignment = float(lw.get("category_alignment", 0.0))
        # clip_grad_norm_(model.parameters(), gradient_clip_norm) between backward and the
        # optimizers (training.py:824-825).  torch's clip_grad_norm_ cannot take the sparse
        # gradients of sparse ID tables (linalg_vector_norm has no sparse kernel: the reference
        # raises NotImplementedError there), so the fused step clips dense-ID models only
        if gradient_clip_norm is not None and gradient_clip_norm > 0:
            if any(self.towers[n][2] == _lib.OPT_SPARSE_ADAM for n in ("user", "item")):
                raise NotImplementedError(
                    "gradient clipping with sparse ID embeddings: clip_grad_norm_ cannot take sparse gradients "
                    "(torch: 'aten::linalg_vector_norm' has no SparseCPU/SparseCUDA kernel)")
            args.hp.grad_clip_norm = float(gradient_clip_norm)
        self.item_categories = None
        if item_category_tensor is not None and major_category_id is not None and \
                args.hp.lambda_category_alignment > 0:
            cats = item_category_tensor.to(self.device, torch.long).contiguous()
            if cats.numel() != self.num_items:  # sharded: the global tensor on every rank
                raise ValueError("ttamm: item_category_tensor must hold one category per item")
            ncat = int(cats.max().item()) + 1 if cats.numel() else 0
            if int(cats.min().item()) < 0 or not 0 <= int(major_category_id) < ncat:
                raise ValueError("ttamm: category ids must be >= 0 and major_category_id must occur")
            if ncat > 65535:
                raise NotImplementedError("ttamm: at most 65535 item categories")
            self.item_categories = cats
            args.item_categories = cats.data_ptr()
            args.num_categories = ncat
            args.major_category = int(major_category_id)
        args.b.num_neg = self.num_neg
        self.csr = None
        if positives is not None:
            self.csr = positives_csr(positives, device=self.device, num_users=ue.num_embeddings)
            if self.csr.max_degree >= self.num_items:
                raise RuntimeError("a user interacted with all items; cannot sample negatives.")
            args.b.pos_offsets = self.csr.offsets.data_ptr()
            args.b.pos_values = self.csr.values.data_ptr()
        args.b.seed = draw_seed() if seed is None else int(seed)
        self.loss_out = torch.zeros(5, dtype=torch.float32, device=self.device)
        self.loss_accum = torch.zeros(2, dtype=torch.float64, device=self.device)
        self.status = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.steps_applied = torch.zeros(1, dtype=torch.int64, device=self.device)
        args.loss_out = self.loss_out.data_ptr()
        args.loss_accum = self.loss_accum.data_ptr()
        args.status = self.status.data_ptr()
        args.steps_applied = self.steps_applied.data_ptr()
        self.max_batch = int(max_batch)
        args.b.batch = self.max_batch
        self.lib = _lib.load()
        self.dense_step0 = int(self._adam_steps[0]["step"].item()) if self._adam_steps else 0
        self.sparse_step0 = int(self._sparse_steps[0]["step"]) if self._sparse_steps else 0
        # arithmetic of the g = 0 AdamW updates of untouched table rows (ttamm.h table_g0_math):
        # "exact" (default) = IEEE sqrt / division, bit-identical to torch's AdamW; "fast" =
        # v_sqrt / v_rcp (<= 1 ulp each): exp_avg / exp_avg_sq stay bit-identical, a warm row's
        # parameter moves by the same update term within a few ulp per step (the
        # contract: tests/test_deferred_gpu.py::test_fast_g0_drift_bounded_over_many_steps).  Not the
        # default: over C1's 3 epochs those ulps move Recall@20 by 0.003 (5 of 1,600 users), outside
        # the north-star's +-0.002 gate that "exact" meets (round 6)
        if table_adamw_math not in ("exact", "fast"):
            raise ValueError("ttamm: table_adamw_math must be 'exact' or 'fast'")
        args.table_g0_math = _lib.G0_FAST if table_adamw_math == "fast" else _lib.G0_EXACT
        # deferred exact AdamW(g = 0) on the dense-group tables (ttamm.h ttamm_table.last_step):
        # the rows are current to dense_step0 now
        self._deferred: list[torch.Tensor] = []
        if deferred_adamw and self.dense_opt is not None and not (
                self.sgd and float(self.dense_opt.param_groups[0]["momentum"]) == 0.0
                and float(self.dense_opt.param_groups[0]["weight_decay"]) == 0.0):
            # (plain SGD without momentum or weight decay leaves g = 0 rows unchanged: nothing to defer)
            if not 1 <= replay_slices <= 255:
                raise ValueError("ttamm: replay_slices must be in [1, 255]")
            tables = []
            for name in ("user", "item"):
                desc = getattr(args, name)
                if self.mimic is not None:
                    tables.append((desc.mimic, self.mimic_tables[name]))
                if desc.id.optimizer == _lib.OPT_DENSE:
                    tables.append((desc.id, self.towers[name][0].embedding.weight))
            for tb, param in tables:
                last = torch.full((tb.rows,), self.dense_step0, dtype=torch.int32, device=self.device)
                tb.last_step = last.data_ptr()
                self._deferred.append(last)
                if not self.sgd and self.decoupled:
                    # rows never given a gradient (exp_avg = exp_avg_sq = +0.0 throughout: AdamW(g = 0)
                    # moves only p) replay from the parameter row alone (ttamm.h ttamm_table.touched)
                    st = state[id(param)]
                    touched = ((st["exp_avg"].view(tb.rows, -1).view(torch.int32) != 0).any(dim=1)
                               | (st["exp_avg_sq"].view(tb.rows, -1).view(torch.int32) != 0).any(dim=1))
                    touched = touched.to(torch.uint8).contiguous()
                    tb.touched = touched.data_ptr()
                    self._deferred.append(touched)
            if tables:
                cap = replay_slices + 2
                self.adam_history = torch.zeros(cap * int(self.lib.ttamm_adam_history_entry_bytes()),
                                                dtype=torch.uint8, device=self.device)
                args.adam_history = self.adam_history.data_ptr()
                args.history_capacity = cap
                args.replay_slices = replay_slices
        # second HIP stream for the index-only prologue (row sort + deferred catch-up),
        # overlapping the feature MLP (ttamm.h ttamm_step_args.aux_stream)
        # (aux_cus: restrict it to that many CUs spread over the device, ttamm_stream_create_cu_limited,
        # so it shares only part of the chip with the GEMMs it overlaps; None = every CU)
        self._aux_handle = None
        if overlap and aux_cus:
            h = ctypes.c_void_p()
            _lib.check(self.lib.ttamm_stream_create_cu_limited(int(aux_cus), ctypes.byref(h)))
            self._aux_handle = h.value
            self.aux_stream = None
            args.aux_stream = self._aux_handle
        else:
            self.aux_stream = torch.cuda.Stream(device=self.device) if overlap else None
            args.aux_stream = self.aux_stream.cuda_stream if self.aux_stream is not None else None
        self._configure(args)
        self.ws_bytes = int(self.lib.ttamm_train_step_workspace_size(ctypes.byref(args)))
        # zeroed once: the row-grouping scratch at its head must start (and stays) zero
        self.workspace = torch.zeros(self.ws_bytes, dtype=torch.uint8, device=self.device)
        args.workspace = self.workspace.data_ptr()
        args.workspace_bytes = self.ws_bytes
        self.neg_buffer = torch.empty(self.max_batch * self.num_neg, dtype=torch.long, device=self.device)
        self.args = args
        self.steps_done = 0

    # ------------------------------------------------------------------------------------
    def _bf16_copy(self, feats: torch.Tensor) -> torch.Tensor:
        rows, width = feats.shape
        ld = (width + 7) // 8 * 8
        out = torch.empty((rows, ld), dtype=torch.bfloat16, device=feats.device)
        lib = _lib.load()
        _lib.check(lib.ttamm_to_bf16(feats.data_ptr(), rows, width, feats.stride(0), out.data_ptr(), ld,
                                     _lib.stream_handle(feats.device)))
        self._keep = getattr(self, "_keep", []) + [out]
        return out

    def _planes_copy(self, feats: torch.Tensor) -> torch.Tensor:
        rows, width = feats.shape
        ld = 48 * ((width + 15) // 16)
        out = torch.empty((rows, ld), dtype=torch.int16, device=feats.device)
        lib = _lib.load()
        _lib.check(lib.ttamm_to_planes(feats.data_ptr(), rows, width, feats.stride(0), out.data_ptr(), ld,
                                       _lib.stream_handle(feats.device)))
        self._keep = getattr(self, "_keep", []) + [out]
        return out

    def _sgd_state(self, opt: torch.optim.Optimizer, p: torch.Tensor) -> dict:
        """The kernels' view of torch.optim.SGD's state (sgd.py): the momentum buffer as exp_avg
        (exp_avg_sq aliases it), created by the first step as torch does (buf = grad.clone());
        without momentum torch keeps no state and both alias the parameter (ttamm.h
        TTAMM_DENSE_SGD)."""
        if float(opt.param_groups[0]["momentum"]) == 0.0:
            return {"exp_avg": p, "exp_avg_sq": p}
        buf = opt.state[p].get("momentum_buffer")
        if buf is None:
            buf = torch.zeros_like(p, memory_format=torch.preserve_format)
            self._sgd_buffers.append((p, buf))
        elif buf.shape != p.shape or not buf.is_contiguous():
            raise ValueError("ttamm: SGD momentum_buffer must be a contiguous tensor of the parameter's shape")
        return {"exp_avg": buf, "exp_avg_sq": buf}

    def _configure(self, args: _lib.StepArgs) -> None:
        """Hook: descriptor fields that shape the workspace (set before it is sized)."""

    def _hparams(self) -> None:
        hp = self.args.hp
        if self.sgd:
            g = self.dense_opt.param_groups[0]
            hp.dense_optimizer = _lib.DENSE_SGD
            hp.lr = float(g["lr"])
            hp.weight_decay = float(g["weight_decay"])
            hp.momentum = float(g["momentum"])
            if (hp.momentum != 0.0) != self._sgd_momentum_on:
                # the moment slots alias the parameter without momentum and a momentum buffer with it
                # (and the deferred replay would overwrite lagging rows' buffers): not switchable
                raise ValueError("ttamm: SGD momentum changed between zero and non-zero after the step was "
                                 "built; build a new FusedTrainStep for the new setting")
            hp.dampening = float(g["dampening"])
            hp.nesterov = 1 if g["nesterov"] else 0
            # torch creates a momentum buffer at its parameter's first step (buf = grad.clone()),
            # later buf = momentum buf + (1 - dampening) grad.  With dampening == 0 (the reference
            # never sets it) a zero buffer's normal update IS grad, so buffers created here start at
            # zero and no first-step flag is needed; with dampening the flag is one per step, so a
            # state where some buffers exist and others do not cannot be stepped exactly
            if self._sgd_buffers and hp.dampening != 0.0:
                created = {id(p) for p, _ in self._sgd_buffers}
                if any(id(p) not in created for p in _dense_params(self.dense_opt)):
                    raise NotImplementedError(
                        "ttamm: SGD with dampening and momentum buffers for only some parameters (a partly "
                        "initialised optimizer state) is not implemented")
                hp.sgd_first_step = 1
            else:
                hp.sgd_first_step = 0
        elif self.dense_opt is not None:
            g = self.dense_opt.param_groups[0]
            hp.lr = float(g["lr"])
            hp.beta1, hp.beta2 = (float(b) for b in g["betas"])
            hp.eps = float(g["eps"])
            hp.weight_decay = float(g["weight_decay"])
            hp.decoupled_weight_decay = 1 if self.decoupled else 0
        if self.sparse_opt is not None:
            g = self.sparse_opt.param_groups[0]
            hp.sparse_lr = float(g["lr"])
            hp.sparse_beta1, hp.sparse_beta2 = (float(b) for b in g["betas"])
            hp.sparse_eps = float(g["eps"])
        hp.dense_step = self.dense_step0 + self.steps_done + 1
        hp.sparse_step = self.sparse_step0 + self.steps_done + 1

    def step(
        self,
        users: torch.Tensor,
        pos_items: torch.Tensor,
        neg_items: torch.Tensor | None = None,
        *,
        keep_masks: Mapping[str, Sequence[torch.Tensor]] | None = None,
        timing_events: Sequence[Any] | None = None,
    ) -> None:
        """Enqueue one training step on the current stream (no host synchronisation).
        ``timing_events``: hipEvent_t handles, pairs as in ttamm.h ttamm_step_args."""
        if not self._bind_batch(users, pos_items, neg_items, keep_masks):
            return
        a = self.args
        ev = list(timing_events or [])
        for i in range(len(a.timing_events)):
            a.timing_events[i] = ev[i] if i < len(ev) else None
        self._hparams()
        _lib.check(self.lib.ttamm_train_step(ctypes.byref(a), _lib.stream_handle(self.device)))
        self.steps_done += 1
        self._register_sgd_buffers()

    def _register_sgd_buffers(self) -> None:
        """After the first enqueued step: it wrote buf = grad into the SGD momentum buffers
        (stream-ordered), so torch's optimizer state holds them from now on."""
        for p, buf in self._sgd_buffers:
            self.dense_opt.state[p]["momentum_buffer"] = buf
        self._sgd_buffers = []

    def _bind_batch(self, users, pos_items, neg_items, keep_masks) -> bool:
        B = users.numel()
        if B == 0:
            return False
        if B > self.max_batch:
            raise ValueError("ttamm: batch larger than the step was sized for")
        if users.dtype != torch.long or pos_items.dtype != torch.long:
            raise ValueError("Adaptive mimic indices must be torch.long tensors.")
        if pos_items.numel() != B:
            raise ValueError("ttamm: one positive item per interaction")
        _lib.require_rocm(users, "train step")
        a = self.args
        a.b.users = users.data_ptr()
        a.b.pos_items = pos_items.data_ptr()
        a.b.batch = B
        if self.num_neg == 0:  # in-batch negatives only
            a.b.neg_items = None
            a.b.sample_negatives = 0
        elif neg_items is not None:
            if neg_items.numel() != B * self.num_neg or neg_items.dtype != torch.long:
                raise ValueError("ttamm: negatives must be int64 [batch, negatives_per_positive]")
            a.b.neg_items = neg_items.data_ptr()
            a.b.sample_negatives = 0
        else:
            if self.csr is None:
                raise ValueError("ttamm: positives are required to sample negatives")
            a.b.neg_items = self.neg_buffer.data_ptr()
            a.b.sample_negatives = 1
        a.b.counter = self.steps_done
        for side, field in (("user", a.b.user_keep_mask), ("item", a.b.item_keep_mask)):
            masks = (keep_masks or {}).get(side) or []
            for i in range(_lib.MAX_LINEAR):
                field[i] = masks[i].data_ptr() if i < len(masks) and masks[i] is not None else None
        return True

    def __del__(self) -> None:
        h = getattr(self, "_aux_handle", None)
        if h:
            try:
                torch.cuda.synchronize(self.device)
                self.lib.ttamm_stream_destroy(ctypes.c_void_p(h))
            except Exception:  # interpreter shutdown
                pass
            self._aux_handle = None

    def flush(self) -> None:
        """Bring every row of the deferred dense-group tables current (enqueued, no sync).
        Needed before the tables or their AdamW state are read outside the step."""
        if not self._deferred or self.steps_done == 0:
            return
        self.args.hp.dense_step = self.dense_step0 + self.steps_done
        # the flush runs on the aux stream (beside the last step's weight-gradient tail) unless that
        # stream is restricted to a CU subset (aux_cus): then on the caller's stream, on every CU
        aux = self.args.aux_stream
        if self._aux_handle:
            self.args.aux_stream = None
        try:
            _lib.check(self.lib.ttamm_flush_tables(ctypes.byref(self.args), _lib.stream_handle(self.device)))
        finally:
            self.args.aux_stream = aux

    def _status_error(self) -> int:
        """Synchronise and return the device status bits.  After an error the device skipped
        every later step (ttamm.h TTAMM_STATUS_*): count only the steps that ran."""
        torch.cuda.current_stream(self.device).synchronize()
        status = int(self.status.item())
        if status:
            self.steps_done = int(self.steps_applied.item())
        return status

    def finish(self) -> float:
        """Flush deferred table updates, synchronise, surface device-side errors, write the
        optimizer step counters back, and return the epoch's mean loss weighted by positives
        (training.py:829-833).  A batch id outside its table raises IndexError (nn.Embedding,
        encoders.py:222-223), sampler exhaustion RuntimeError (samplers.py:78-81); either way the
        parameters and optimizer state are those after the last good step."""
        status = self._status_error()
        self.flush()
        torch.cuda.current_stream(self.device).synchronize()
        for st in self._adam_steps:
            st["step"].fill_(float(self.dense_step0 + self.steps_done))
        for st in self._sparse_steps:
            st["step"] = self.sparse_step0 + self.steps_done
        if status & _lib.STATUS_LOOKAHEAD_MISMATCH:
            raise ValueError("ttamm: a row-sharded step was called with a batch other than the one its look-ahead "
                             "(next_batch=) prepared; that step was skipped on the rank that got it")
        if status & _lib.STATUS_INDEX_OUT_OF_RANGE:
            raise IndexError("index out of range in self")
        if status & _lib.STATUS_SAMPLER_EXHAUSTED:
            raise RuntimeError("Exceeded resampling attempts while drawing negatives.")
        total, count = self.loss_accum.tolist()
        return total / max(count, 1.0)

    def last_losses(self) -> dict[str, float]:
        v = self.loss_out.tolist()
        return {"total": v[0], "bce": v[1], "mimic_user": v[2], "mimic_item": v[3], "category_alignment": v[4]}


class _IdentityView(nn.Module):
    """A tower seen without its feature path (features absent: encoders.py:228-231)."""

    def __init__(self, tower: TowerEncoder) -> None:
        super().__init__()
        object.__setattr__(self, "_t", tower)
        self.fusion = "identity"
        self.feature_encoder = None
        self.embedding = tower.embedding
        self.matmul_dtype = tower.matmul_dtype
        self.id_dim = tower.id_dim
        self.output_dim = tower.id_dim
        self.num_embeddings = tower.num_embeddings


def train_one_epoch(
    model: TwoTowerModel,
    dataloader: Iterable,
    *,
    optimizers: list[torch.optim.Optimizer],
    criterion: nn.BCEWithLogitsLoss,
    negatives_per_positive: int,
    num_items: int,
    user_positive_items: Mapping[int, set[int]],
    user_features: torch.Tensor | None,
    item_features: torch.Tensor | None,
    device: torch.device,
    gradient_clip_norm: float | None = None,
    loss_weights: Mapping[str, Any] | None = None,
    item_category_tensor: torch.Tensor | None = None,
    major_category_id: int | None = None,
    batch_hook: Callable[[int, torch.Tensor, torch.Tensor], tuple[Any, Any]] | None = None,
    step_losses: list | None = None,
    in_batch_negatives: bool = False,
    table_adamw_math: str = "exact",
) -> float:
    """Drop-in for ``_train_one_epoch`` (training.py:700-833) executed on the MI355X.

    Two keyword-only extras (absent from the reference, default off) make a run reproducible
    against a CPU run of the reference loop:
      batch_hook(step, users, pos) -> (negatives [B, N] | None, {"user": [...], "item": [...]} |
          None): injects the batch's negatives (instead of the on-device sampler) and dropout
          keep-masks (instead of the Philox stream) — the RNG streams a CPU run draws differently;
      step_losses: receives each step's device loss vector [total, bce, mimic_user, mimic_item,
          category_alignment] (no host synchronisation inside the loop).
    ``in_batch_negatives`` selects ttamm's in-batch mode (FusedTrainStep; BASELINE C2/C4), with
    ``negatives_per_positive`` sampled negatives on top (0 allowed).  ``table_adamw_math``: the
    g = 0 AdamW arithmetic of untouched mimic-table rows — "exact" (default, bit-identical to
    torch) or "fast" (v_sqrt / v_rcp, within a few ulp of torch per step; FusedTrainStep)."""
    model.train()
    if not isinstance(criterion, nn.BCEWithLogitsLoss) or criterion.reduction != "mean" or \
            criterion.weight is not None or criterion.pos_weight is not None:
        raise NotImplementedError("ttamm: the step implements BCEWithLogitsLoss(reduction='mean')")
    lw = dict(loss_weights or {})
    if num_items != model.item_encoder.num_embeddings:
        raise ValueError("num_items does not match the item embedding table")
    device = torch.device(device)
    batches = iter(dataloader)
    engine = None
    step = 0
    for users_in, pos_in in batches:
        users = users_in.to(device, non_blocking=True).reshape(-1)
        pos = pos_in.to(device, non_blocking=True).reshape(-1)
        if engine is None:
            size = getattr(dataloader, "batch_size", None) or users.numel()
            engine = FusedTrainStep(
                model, optimizers, negatives_per_positive=negatives_per_positive, positives=user_positive_items,
                user_features=user_features, item_features=item_features, loss_weights=lw,
                max_batch=max(int(size), users.numel()),
                item_category_tensor=item_category_tensor, major_category_id=major_category_id,
                in_batch_negatives=in_batch_negatives, gradient_clip_norm=gradient_clip_norm,
                table_adamw_math=table_adamw_math,
            )
        neg = masks = None
        if batch_hook is not None:
            neg, masks = batch_hook(step, users_in, pos_in)
            if neg is not None:
                neg = neg.to(device, torch.long).reshape(-1)
            if masks:
                masks = {k: [m.to(device) for m in v] for k, v in masks.items()}
        engine.step(users, pos, neg, keep_masks=masks)  # stream-ordered: inputs are recycled safely
        if step_losses is not None:
            step_losses.append(engine.loss_out.clone())
        step += 1
    if engine is None:
        return 0.0
    return engine.finish()
