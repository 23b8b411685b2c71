// Native executor of one training step (the body of `_train_one_epoch`,
// training.py:726-831), issued as a fixed sequence of gfx950 kernels on one HIP stream.
//
//   sample negatives                      samplers.py:11-85                (a11)
//   tower forward (user & item grouped)   encoders.py:221-255              (a1, a3, a4)
//     hidden Linear+ReLU+Dropout GEMMs    gathered feature rows, MFMA fp32
//     final Linear -> f ; ID gather -> e  into one [rows, 2D] "ef" buffer
//     gate GEMM 1 (ReLU), gate GEMM 2 (sigmoid, mix, mimic augment)      adaptive_mimic.py:88-95 (a2)
//   score + BCE + mimic MSE fwd/bwd       training.py:770-803              (a5-a7)
//   tower backward (dgrad chain grouped, then all weight grads in one launch)
//   coalesce row grads, SparseAdam (ID tables), AdamW touched rows        (a9, a5)
//   AdamW(g=0) stream over the full mimic tables, side-row scatter         (a5, a10)
//   AdamW on the MLP / gate weights                                        (a10)
//
// A row-sharded multi-GPU step runs the same pieces as phases (ttamm.h TTAMM_PHASE_*): the
// item tower of a rank runs over the item rows it owns, for whoever requested them; the
// host moves (t | a) and (dT | dA) rows between phases and all-reduces the gradient arena.
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "kernels.h"

namespace ttamm {

namespace {

enum Role { ROLE_USER = 0, ROLE_ITEM = 1 };

struct TowerWs {
    int role = ROLE_USER;
    int64_t R = 0;
    const int64_t* idx = nullptr;   // ID / mimic table rows
    const int64_t* fidx = nullptr;  // feature rows (null: row r)
    int64_t* idx_own = nullptr;     // staged (range-checked) rows: users / 1-process items [pos; neg] /
                                    // sharded owner's requested local item rows
    // dropout stream key of row r (see GemmProblem::row_key)
    const int64_t* row_key = nullptr;
    int64_t key_base0 = 0, key_base1 = 0, key_split = 0;
    // ID-table max_norm: per-row claim marks (persistent, zero once) and this call's tag base
    int32_t* renorm_mark = nullptr;
    int32_t renorm_tag = 0;
    int64_t renorm_split = 0;  // item tower: positives [0, split) are one lookup, negatives the next
    int64_t renorm_key_split = 0;  // sharded owner: requests with row_key < this (positives) are one lookup
    float* hid[TTAMM_MAX_LINEAR] = {};
    float* dhid[TTAMM_MAX_LINEAR] = {};
    // non-ReLU activations: each hidden layer's pre-activation, its drawn keep bytes (dropout
    // without an injected mask), and the keep bytes the backward reads (injected or drawn)
    float* pre[TTAMM_MAX_LINEAR] = {};
    uint8_t* mask[TTAMM_MAX_LINEAR] = {};
    const uint8_t* keep[TTAMM_MAX_LINEAR] = {};
    float* ef = nullptr;    // gated: [R, 2D] = [e | f]
    float* e = nullptr;     // non-gated: [R, D]
    float* f = nullptr;     // sum fusion: [R, D]
    float* z = nullptr;     // gate hidden [R, Hg]
    float* dz = nullptr;
    float* g = nullptr;
    float* t = nullptr;     // [R, t_ld] (a alongside at the same stride)
    float* a = nullptr;
    int64_t t_ld = 0;
    float* aug = nullptr;   // [R, D] or null (sharded item owner)
    const float* dT = nullptr;  // [R, dT_ld]
    float* dT_own = nullptr;
    int64_t dT_ld = 0;
    const float* dA = nullptr;  // mimic-table grad rows (user: all rows; item: positives or all)
    float* dA_own = nullptr;
    int64_t dA_ld = 0;
    int64_t dA_split = 0;       // rows < dA_split read dA, the rest read dT
    const int64_t* xu = nullptr;  // sharded owner, compact exchange rows: row units (GateTower::xu)
    float* dq = nullptr;
    float* dEF = nullptr;  // [R, 2D]
    float* gw[TTAMM_MAX_LINEAR] = {};
    float* gb[TTAMM_MAX_LINEAR] = {};
    float* ggw[2] = {};
    float* ggb[2] = {};
    float* slab[TTAMM_MAX_LINEAR + 2] = {};
    CoalesceWs co{};
    CatchupList cl{};  // deferred AdamW: the batch's rows to bring current, grouped by lag
    float* side_id = nullptr;
    float* side_mimic = nullptr;
    float* piece_e = nullptr;
    float* piece_a = nullptr;
    float* wpad = nullptr;  // first feature layer weight, in_features padded to a multiple of 4
    uint16_t* w16 = nullptr;  // bf16 towers with bf16 feature rows: the weight rounded, padded to % 8
    uint16_t* gw16 = nullptr;  // bf16 gated towers (D == Hg in {128, 256}): the fused gate's weight images
    bool gw16_ready = false;   // formed by this call's forward (the weights do not change before its backward)
    // wpad / w16 formed by this step's prologue launch (ttamm_train_step; the standalone tower
    // entry points form them themselves)
    bool weight_prepped = false;
    int wgrad_rps[kWgradClasses] = {512, 512, 512, 512};  // split-K rows of the weight gradients, per tile class
};

struct StepWs {
    TowerWs user, item;
    float* partials = nullptr;
    uint32_t* prologue_done = nullptr;  // completion counter of step_prologue_kernel (zero between calls)
    int64_t* keys_own = nullptr;        // sharded owner: staged request keys [item_rows_capacity]
    // compact exchange rows (ttamm_step_args.exchange_counts): the first unit of each owned row
    // (~unit for a negative), formed with the ITEM_FWD staging
    int64_t* own_units = nullptr;
    int score_blocks = 0;
    // in-batch negatives (ttamm_step_args.in_batch)
    bool ib_on = false;
    InBatchArgs ib{};
    float* ib_du = nullptr;   // [B, D]
    float* ib_dp = nullptr;   // [B, D] (one process; sharded: the caller's inbatch_dp)
    int ib_parts = 0;
    bool cal_on = false;  // category-alignment loss this step
    CalArgs cal{};
    // gradient clipping (ttamm_hparams.grad_clip_norm)
    bool clip_on = false;
    float* clip_partials = nullptr;
    int clip_parts = 0;
    float* clip_coef = nullptr;
};

// The category-alignment loss runs when categories are given and its weight is positive
// (training.py:805: `if lambda_cal > 0`; _category_alignment_loss returns 0 without them).
bool cal_enabled(const ttamm_step_args& A) {
    return A.item_categories != nullptr && A.hp.lambda_category_alignment > 0.0;
}

int tower_in_dim(const ttamm_tower& T, int l) { return l == 0 ? T.feat_dim : T.linear[l - 1].out_features; }
inline int round4(int x) { return (x + 3) / 4 * 4; }
inline int round8(int x) { return (x + 7) / 8 * 8; }
// the first feature layer's forward on bf16 operands in memory (ttamm_tower.features_bf16)
bool uses_w16(const ttamm_tower& T) {
    return T.matmul_bf16 && T.features_bf16 != nullptr && T.fusion != TTAMM_FUSION_IDENTITY && T.n_linear > 0;
}
// gated and concat towers keep [e | f] rows (the gate's / projection's input) and their gradient
bool uses_ef(const ttamm_tower& T) { return T.fusion == TTAMM_FUSION_GATED || T.fusion == TTAMM_FUSION_CONCAT; }
// Linear layers after the feature encoder: the gate's two, or the concat projection
int fusion_linears(const ttamm_tower& T) {
    return T.fusion == TTAMM_FUSION_GATED ? 2 : T.fusion == TTAMM_FUSION_CONCAT ? 1 : 0;
}
// widths of a tower: the ID rows (Did), the feature encoder's output (Fo), the [e | f] rows of
// gated / concat fusion (Did + Fo) and the tower output (concat: the projection's output_dim,
// encoders.py:211-217; otherwise Did).  Everything downstream of the tower (scores, mimic
// tables, the exchange rows) is output-wide; only concat lets the output differ from Did.
int fo_dim(const ttamm_tower& T) { return T.n_linear ? T.linear[T.n_linear - 1].out_features : T.feat_dim; }
int efw(const ttamm_tower& T) { return T.id.dim + fo_dim(T); }
int out_dim(const ttamm_tower& T) { return T.fusion == TTAMM_FUSION_CONCAT ? T.gate[0].out_features : T.id.dim; }
bool needs_wpad(const ttamm_tower& T) {
    return T.fusion != TTAMM_FUSION_IDENTITY && T.n_linear > 0 && T.linear[0].in_features % 4 != 0;
}

// Validate one tower against the reference's own constraints.
int validate_tower(const ttamm_tower& T, const char* name, int D, bool training) {
    std::string n(name);
    TTAMM_REQUIRE(T.id.weight, n + ": embedding table missing");
    if (training) TTAMM_REQUIRE(T.id.exp_avg && T.id.exp_avg_sq, n + ": embedding optimizer state missing");
    TTAMM_REQUIRE(T.fusion == TTAMM_FUSION_CONCAT || T.id.dim == D, n + ": embedding dim mismatch");
    TTAMM_REQUIRE(D % 4 == 0 && T.id.dim % 4 == 0, n + ": ttamm requires embedding_dim % 4 == 0");
    TTAMM_REQUIRE(T.id.rows > 0, n + ": empty embedding table");
    TTAMM_REQUIRE(T.id.rows < (int64_t(1) << 31), n + ": tables of 2^31 rows or more are not supported (int32 row keys)");
    TTAMM_REQUIRE(T.n_linear >= 0 && T.n_linear <= TTAMM_MAX_LINEAR, n + ": too many feature-encoder layers");
    TTAMM_REQUIRE(T.activation >= TTAMM_ACT_RELU && T.activation <= TTAMM_ACT_SELU, n + ": unsupported activation");
    TTAMM_REQUIRE(T.fusion >= TTAMM_FUSION_IDENTITY && T.fusion <= TTAMM_FUSION_CONCAT, n + ": unsupported fusion");
    if (T.fusion != TTAMM_FUSION_IDENTITY) {
        TTAMM_REQUIRE(T.features != nullptr && T.feat_dim > 0, n + ": fusion needs feature rows");
        TTAMM_REQUIRE(T.feat_ld >= T.feat_dim, n + ": feature row stride too small");
        TTAMM_REQUIRE(T.feat_ld % 4 == 0 && (uintptr_t)T.features % 16 == 0,
                      n + ": feature rows must be 16-byte aligned (row stride % 4 == 0)");
        if (T.features_bf16)
            TTAMM_REQUIRE(T.matmul_bf16 && T.feat_bf16_ld % 8 == 0 && T.feat_bf16_ld >= round8(T.feat_dim) &&
                              (uintptr_t)T.features_bf16 % 16 == 0,
                          n + ": bf16 feature rows need matmul_bf16, 16-byte aligned rows of >= round8(F) elements");
        if (T.features_planes)
            TTAMM_REQUIRE(!T.matmul_bf16 && T.feat_planes_ld % 8 == 0 &&
                              T.feat_planes_ld >= 48 * ceil_div(T.feat_dim, 16) && (uintptr_t)T.features_planes % 16 == 0,
                          n + ": feature planes need fp32 GEMMs and 16-byte aligned rows of >= 48 ceil(F / 16) "
                              "elements (a multiple of 8)");
        for (int l = 0; l < T.n_linear; ++l) {
            const ttamm_linear& L = T.linear[l];
            TTAMM_REQUIRE(L.weight && L.bias, n + ": linear parameters missing");
            if (training)
                TTAMM_REQUIRE(L.weight_exp_avg && L.weight_exp_avg_sq && L.bias_exp_avg && L.bias_exp_avg_sq,
                              n + ": linear optimizer state missing");
            TTAMM_REQUIRE(L.in_features == tower_in_dim(T, l), n + ": feature-encoder layer shapes do not chain");
            TTAMM_REQUIRE(L.out_features % 4 == 0, n + ": ttamm requires feature-encoder widths % 4 == 0");
        }
        const int fo = fo_dim(T);
        if (T.fusion == TTAMM_FUSION_CONCAT)
            TTAMM_REQUIRE(fo % 4 == 0, n + ": ttamm requires the feature encoder's output width % 4 == 0");
        else
            TTAMM_REQUIRE(fo == D, n + ": Feature encoder output dimension must match id embedding dimension for "
                                       "'sum' or 'gated' fusion.");
        TTAMM_REQUIRE(T.dropout >= 0.f && T.dropout < 1.f, n + ": dropout must be in [0, 1)");
    }
    if (T.fusion == TTAMM_FUSION_GATED) {
        const ttamm_linear &G1 = T.gate[0], &G2 = T.gate[1];
        TTAMM_REQUIRE(G1.weight && G1.bias && G2.weight && G2.bias, n + ": gate parameters missing");
        if (training)
            TTAMM_REQUIRE(G1.weight_exp_avg && G1.weight_exp_avg_sq && G1.bias_exp_avg && G1.bias_exp_avg_sq &&
                              G2.weight_exp_avg && G2.weight_exp_avg_sq && G2.bias_exp_avg && G2.bias_exp_avg_sq,
                          n + ": gate optimizer state missing");
        TTAMM_REQUIRE(G1.in_features == 2 * D && G2.out_features == D && G2.in_features == G1.out_features,
                      n + ": gate shapes do not match the embedding dimension");
        TTAMM_REQUIRE(G1.out_features % 4 == 0, n + ": ttamm requires the gate hidden width % 4 == 0");
    }
    if (T.fusion == TTAMM_FUSION_CONCAT) {
        const ttamm_linear& P = T.gate[0];
        TTAMM_REQUIRE(P.weight && P.bias, n + ": concat projection parameters missing");
        if (training)
            TTAMM_REQUIRE(P.weight_exp_avg && P.weight_exp_avg_sq && P.bias_exp_avg && P.bias_exp_avg_sq,
                          n + ": concat projection optimizer state missing");
        TTAMM_REQUIRE(P.in_features == efw(T) && P.out_features == D,
                      n + ": concat projection must map [e | f] (embedding dim + feature output) to the output dim");
    }
    return TTAMM_OK;
}

bool sharded(const ttamm_step_args& A) { return A.phase != TTAMM_PHASE_ALL; }
// compact exchange rows (ttamm.h ttamm_step_args.exchange_counts)
bool compact_exchange(const ttamm_step_args& A) { return sharded(A) && A.exchange_counts != nullptr; }
int64_t global_batch(const ttamm_step_args& A) { return A.global_batch > 0 ? A.global_batch : A.b.batch; }

// The replicated-weight gradient arena: per tower (user, item) the feature-encoder layers'
// weight, bias, then the gate's, each piece padded to 64 floats (256 B).
inline size_t pad64(size_t n) { return (n + 63) / 64 * 64; }
size_t tower_grad_floats(const ttamm_tower& T) {
    size_t n = 0;
    if (T.fusion == TTAMM_FUSION_IDENTITY) return 0;
    for (int l = 0; l < T.n_linear; ++l)
        n += pad64((size_t)T.linear[l].out_features * T.linear[l].in_features) + pad64(T.linear[l].out_features);
    for (int q = 0; q < fusion_linears(T); ++q)
        n += pad64((size_t)T.gate[q].out_features * T.gate[q].in_features) + pad64(T.gate[q].out_features);
    return n;
}
void carve_grads(const ttamm_tower& T, TowerWs& w, float*& cur) {
    if (T.fusion == TTAMM_FUSION_IDENTITY) return;
    for (int l = 0; l < T.n_linear; ++l) {
        w.gw[l] = cur;
        cur += pad64((size_t)T.linear[l].out_features * T.linear[l].in_features);
        w.gb[l] = cur;
        cur += pad64(T.linear[l].out_features);
    }
    for (int q = 0; q < fusion_linears(T); ++q) {
            w.ggw[q] = cur;
            cur += pad64((size_t)T.gate[q].out_features * T.gate[q].in_features);
            w.ggb[q] = cur;
            cur += pad64(T.gate[q].out_features);
        }
}

// Workspace layout.  Deterministic in the arguments, so every phase call of a sharded step
// finds the previous phases' activations where it left them.
// The weight-gradient problems of one tower (tower_backward's list), for the split choice.
int wgrad_shapes(const ttamm_tower& T, int64_t R, WgradShape* out) {
    int n = 0;
    if (T.fusion == TTAMM_FUSION_IDENTITY) return 0;
    for (int l = 0; l < T.n_linear; ++l) out[n++] = WgradShape{R, T.linear[l].out_features, T.linear[l].in_features};
    for (int q = 0; q < fusion_linears(T); ++q) out[n++] = WgradShape{R, T.gate[q].out_features, T.gate[q].in_features};
    return n;
}

// Per-row scratch of the row grouping (CoalesceWs cnt / first / fill) comes first in the
// workspace: its offsets depend only on the table sizes, so it stays in place (and zero between
// calls, as launch_coalesce leaves it) whatever the batch size.  The caller zeroes the
// workspace once.
void plan_scratch(Arena& ar, const ttamm_step_args& A, StepWs& ws) {
    coalesce_bind_scratch(ws.user.co, ar.take<int32_t>(coalesce_scratch_ints(A.user.id.rows)), A.user.id.rows);
    coalesce_bind_scratch(ws.item.co, ar.take<int32_t>(coalesce_scratch_ints(A.item.id.rows)), A.item.id.rows);
    if (cal_enabled(A)) {
        const int64_t ncat = std::min<int64_t>(A.num_categories, 65535);
        coalesce_bind_scratch(ws.cal.co, ar.take<int32_t>(coalesce_scratch_ints(ncat)), ncat);
    }
    if (A.user.id.max_norm > 0.0) ws.user.renorm_mark = ar.take<int32_t>(A.user.id.rows);
    if (A.item.id.max_norm > 0.0) ws.item.renorm_mark = ar.take<int32_t>(A.item.id.rows);
    // step_prologue_kernel's completion counter: its last block resets it, so it must sit at a
    // batch-size-independent offset (a short last batch must find it zero, not old activations)
    ws.prologue_done = ar.take<uint32_t>(1);
}

void plan_coalesce(Arena& ar, CoalesceWs& co, int64_t R) {
    co.keys_out = ar.take<int32_t>(R);
    co.vals_out = ar.take<int32_t>(R);
    co.vals_tmp = ar.take<int32_t>(R);
    co.lead = ar.take<int32_t>(R);
    // lead_cnt / seglong double as the segment scan's tile totals: ceil(entries / 256) of them
    co.lead_cnt = ar.take<int32_t>(std::max<int64_t>(R, 257));
    co.seglong = ar.take<int32_t>(std::max<int64_t>(R, 257));
    co.seg_start = ar.take<int32_t>(R + 1);
    co.n_unique = ar.take<int32_t>(1);
}

int plan(Arena& ar, const ttamm_step_args& A, StepWs& ws) {
    const int64_t B = A.b.batch;
    const int N = A.b.num_neg;
    const int D = out_dim(A.user);
    const bool mimic = A.mimic_enabled != 0;
    const bool shard = sharded(A);
    plan_scratch(ar, A, ws);
    {
        WgradShape shapes[2 * (TTAMM_MAX_LINEAR + 2)];
        int n = wgrad_shapes(A.user, B, shapes);
        n += wgrad_shapes(A.item, shard ? A.item_rows_capacity : B * (1 + N), shapes + n);
        int rps[kWgradClasses];
        wgrad_rows_per_split(shapes, n, rps);
        for (int c = 0; c < kWgradClasses; ++c) ws.user.wgrad_rps[c] = ws.item.wgrad_rps[c] = rps[c];
    }
    // ext_io: the item tower's t / a / dT / dA live in the caller's exchange buffers
    auto tower = [&](const ttamm_tower& T, TowerWs& w, int64_t R, bool ext_io, int64_t dA_rows) {
        w.R = R;
        w.idx_own = ar.take<int64_t>(R);
        for (int l = 0; l + 1 < T.n_linear; ++l) {
            w.hid[l] = ar.take<float>((size_t)R * T.linear[l].out_features);
            w.dhid[l] = ar.take<float>((size_t)R * T.linear[l].out_features);
            if (T.activation != TTAMM_ACT_RELU) {
                w.pre[l] = ar.take<float>((size_t)R * T.linear[l].out_features);
                if (T.dropout > 0.f) w.mask[l] = ar.take<uint8_t>((size_t)R * T.linear[l].out_features);
            }
        }
        const int Hg = T.fusion == TTAMM_FUSION_GATED ? T.gate[0].out_features : 0;
        if (uses_ef(T)) {
            w.ef = ar.take<float>((size_t)R * efw(T));
            w.dEF = ar.take<float>((size_t)R * efw(T));
        }
        if (T.fusion == TTAMM_FUSION_GATED) {
            w.z = ar.take<float>((size_t)R * Hg);
            w.dz = ar.take<float>((size_t)R * Hg);
            w.g = ar.take<float>((size_t)R * D);
            w.dq = ar.take<float>((size_t)R * D);
            const int np = T.matmul_bf16 ? 1 : 3;
            if (gate16_supported(D, Hg, np)) w.gw16 = ar.take<uint16_t>((size_t)gate16_image_elems(D, Hg, np));
        } else if (!uses_ef(T)) {
            w.e = ar.take<float>((size_t)R * D);
            if (T.fusion == TTAMM_FUSION_SUM) w.f = ar.take<float>((size_t)R * D);
        }
        if (!ext_io) {
            w.t = ar.take<float>((size_t)R * D);
            w.a = mimic ? ar.take<float>((size_t)R * D) : nullptr;
            w.t_ld = D;
            w.aug = ar.take<float>((size_t)R * D);
            w.dT_own = ar.take<float>((size_t)R * D);
            w.dT = w.dT_own;
            w.dT_ld = D;
            w.dA_own = mimic ? ar.take<float>((size_t)dA_rows * D) : nullptr;
            w.dA = w.dA_own;
            w.dA_ld = D;
            w.dA_split = dA_rows;
        }
        if (T.fusion != TTAMM_FUSION_IDENTITY) {
            for (int l = 0; l < T.n_linear; ++l) {
                const ttamm_linear& L = T.linear[l];
                w.slab[l] = ar.take<float>(
                    wgrad_slab_floats((int)R, L.out_features, L.in_features, w.wgrad_rps[wgrad_class(L.out_features)]));
            }
        }
        {
            for (int q = 0; q < fusion_linears(T); ++q) {
                const ttamm_linear& L = T.gate[q];
                w.slab[TTAMM_MAX_LINEAR + q] =
                    ar.take<float>(wgrad_slab_floats((int)R, L.out_features, L.in_features,
                                                     w.wgrad_rps[wgrad_class(L.out_features)]));
            }
        }
        plan_coalesce(ar, w.co, R);
        if (A.adam_history && A.history_capacity > 1) {
            const int cap = A.history_capacity;
            catchup_bind(w.cl, ar.take<int32_t>(catchup_list_ints(R, cap)), R, cap);
        }
        if (needs_wpad(T)) w.wpad = ar.take<float>((size_t)T.linear[0].out_features * round4(T.linear[0].in_features));
        if (uses_w16(T)) w.w16 = ar.take<uint16_t>((size_t)T.linear[0].out_features * round8(T.linear[0].in_features));
        w.piece_e = ar.take<float>((size_t)R * T.id.dim);
        if (mimic) w.piece_a = ar.take<float>((size_t)R * D);
        if (T.id.optimizer == TTAMM_OPT_DENSE) w.side_id = ar.take<float>((size_t)R * 3 * T.id.dim);
        if (mimic) w.side_mimic = ar.take<float>((size_t)R * 3 * D);
    };
    ws.user.role = ROLE_USER;
    ws.item.role = ROLE_ITEM;
    tower(A.user, ws.user, B, false, B);
    if (shard) {
        tower(A.item, ws.item, A.item_rows_capacity, true, 0);
        ws.keys_own = ar.take<int64_t>(A.item_rows_capacity);
        ws.own_units = ar.take<int64_t>(A.item_rows_capacity);
    }
    else
        tower(A.item, ws.item, B * (1 + N), false, B);
    ws.score_blocks = score_blocks(B, D);
    ws.partials = ar.take<float>((size_t)ws.score_blocks * 3);
    if (A.hp.grad_clip_norm > 0.0) {
        ws.clip_on = true;
        // [tables' total (sharded: all-reduced)] + both towers' row partials + the dense partials
        ws.clip_parts = 1 + rows_sumsq_blocks(B, A.user.id.dim) +
                        rows_sumsq_blocks(shard ? A.item_rows_capacity : B * (1 + N), A.item.id.dim) +
                        kDenseSumsqBlocks;
        ws.clip_partials = ar.take<float>((size_t)ws.clip_parts);
        ws.clip_coef = ar.take<float>(1);
    }
    if (A.in_batch) {
        ws.ib_on = true;
        const int64_t Bc = shard ? global_batch(A) : B;
        size_t su, sp, parts;
        inbatch_workspace_floats(B, Bc, D, &su, &sp, &parts);
        ws.ib.slab_u = ar.take<float>(su);
        ws.ib.slab_p = ar.take<float>(sp);
        ws.ib.loss_part = ar.take<float>(parts);
        ws.ib_parts = (int)parts;
        ws.ib_du = ar.take<float>((size_t)B * D);
        if (!shard) ws.ib_dp = ar.take<float>((size_t)B * D);
    }
    if (cal_enabled(A)) {
        // one process: the batch's item rows; sharded: this requester's rows, with the per-category
        // sums and scatters in the caller's all-reduce buffers (slot space = category ids)
        CalArgs& c = ws.cal;
        ws.cal_on = true;
        const int64_t R = B * (1 + N);
        c.R = R;
        c.D = D;
        c.nseg_max = (int)std::min<int64_t>(R, std::max<int64_t>(1, std::min<int64_t>(A.num_categories, 65535)));
        const int64_t slots = shard ? A.num_categories : c.nseg_max;
        const int pieces = cal_max_pieces(R, c.nseg_max);
        c.catrow = ar.take<int64_t>(R);
        plan_coalesce(ar, c.co, R);
        c.co.sorted = 1;  // categories ascending, as the reference's loop (training.py:567)
        c.pcount = ar.take<int32_t>(c.nseg_max);
        c.pstart = ar.take<int32_t>(c.nseg_max);
        c.psum = ar.take<float>((size_t)pieces * D);
        c.mean = ar.take<float>((size_t)c.nseg_max * D);
        c.pslab = ar.take<float>((size_t)pieces * D * D);
        if (shard) {
            c.gstats = A.cal_stats;
            c.cov = A.cal_scatter;
        } else {
            c.cov = ar.take<float>((size_t)c.nseg_max * D * D);
        }
        c.part = ar.take<float>(slots);
        c.flag = ar.take<int32_t>(slots);
        c.gmajor = ar.take<float>((size_t)D * D);
        c.out = ar.take<float>(2);
    }
    // gradient arena: the caller's all-reduce buffer when sharded, else workspace
    float* arena = shard ? A.dense_grads : ar.take<float>(tower_grad_floats(A.user) + tower_grad_floats(A.item));
    carve_grads(A.user, ws.user, arena);
    carve_grads(A.item, ws.item, arena);
    return TTAMM_OK;
}

GemmProblem gp_base() {
    GemmProblem p;
    std::memset(&p, 0, sizeof(p));
    p.keep_prob = 1.f;
    p.inv_keep = 1.f;
    p.a_ones_col = -1;
    return p;
}

struct Batcher {
    GemmBatch b;
    Batcher() { std::memset(&b, 0, sizeof(b)); }
    void add(const GemmProblem& p) { b.p[b.count++] = p; }
    int run(hipStream_t s) {
        if (b.count == 0) return TTAMM_OK;
        int rc = launch_gemm(b, s);
        std::memset(&b, 0, sizeof(b));
        return rc;
    }
};

// Dropout RNG words: key = seed; counter words 2,3 = step counter / (domain | tower | layer)
void set_dropout(GemmProblem& p, const ttamm_tower& T, const ttamm_batch& bt, int tower_id, int layer,
                 const uint8_t* mask) {
    const float pdrop = T.dropout;
    p.keep_prob = 1.0f - pdrop;
    // torch computes noise/(1-p) in fp32: 1.f / (1.f - p)
    p.inv_keep = pdrop > 0.f ? 1.0f / (1.0f - pdrop) : 1.0f;
    p.keep_mask = mask;
    p.rng_k0 = (uint32_t)bt.seed;
    p.rng_k1 = (uint32_t)(bt.seed >> 32);
    p.rng_c2 = (uint32_t)bt.counter;
    p.rng_c3 = RNG_DROPOUT | ((uint32_t)tower_id << 24) | ((uint32_t)layer << 20) |
               ((uint32_t)(bt.counter >> 32) & 0xFFFFFu);
}

void set_keys(GemmProblem& p, const TowerWs& w) {
    p.row_key = w.row_key;
    p.key_base0 = w.key_base0;
    p.key_base1 = w.key_base1;
    p.key_split = w.key_split;
}

// ---- fused gate (gate.hip) ------------------------------------------------------------------
// Used when every gated tower of a grouped launch has a supported D == Hg: fp32 towers gate.hip
// (D in {32, 64, 96, 128}), bf16 towers gate16.hip (D in {128, 256}); any other configuration runs
// the generic GEMM path.  TTAMM_GENERIC_GATE=1 forces the generic path (the tests run both).
bool generic_gate_forced() {
    const char* v = product_env("TTAMM_GENERIC_GATE");
    return v && v[0] == '1';
}

bool gate_group(const ttamm_tower* const* T, TowerWs* const* W, int ntowers, int D, bool mimic, GateArgs& ga) {
    std::memset(&ga, 0, sizeof(ga));
    if (generic_gate_forced()) return false;
    // TTAMM_GATE16_SPLIT=1: fp32 towers at D = 96 on gate16.hip's split-bf16 form instead of gate.hip
    // (fp32 MFMA).  Measured slower at C2 (forward 71 vs 61 us, backward 72 vs 70, step 0.695 vs
    // 0.655 ms, profiles/r05_s20_gate16_split.txt): the kernels are latency-bound, not MFMA-bound
    const char* e16 = dev_env("TTAMM_GATE16_SPLIT");
    const bool split16 = e16 && e16[0] == '1';
    int hg = -1, planes = -1;
    for (int k = 0; k < ntowers; ++k) {
        const ttamm_tower& t = *T[k];
        if (t.fusion != TTAMM_FUSION_GATED) continue;
        const int h = t.gate[0].out_features;
        int np;
        if (t.matmul_bf16) {
            if (!(gate16_supported(D, h, 1) && W[k]->gw16)) return false;
            np = 1;
        } else if (split16 && gate16_supported(D, h, 3) && W[k]->gw16) {
            np = 3;
        } else if (gate_fused_supported(D, h)) {
            np = 0;
        } else {
            return false;
        }
        if ((hg >= 0 && h != hg) || (planes >= 0 && np != planes)) return false;
        hg = h;
        planes = np;
    }
    if (hg < 0) return false;
    ga.planes = planes;
    ga.images_ready = 1;
    for (int k = 0; k < ntowers; ++k) {
        const ttamm_tower& t = *T[k];
        const TowerWs& w = *W[k];
        if (t.fusion != TTAMM_FUSION_GATED || w.R <= 0) continue;
        GateTower& g = ga.tw[ga.count++];
        g.R = w.R;
        g.ef = w.ef;
        g.G1 = t.gate[0].weight;
        g.c1 = t.gate[0].bias;
        g.G2 = t.gate[1].weight;
        g.c2 = t.gate[1].bias;
        g.z = w.z;
        g.g = w.g;
        g.t = w.t;
        g.a = w.a;
        g.ld_t = w.t_ld;
        g.table = mimic ? t.mimic.weight : nullptr;
        g.idx = w.idx;
        g.aug = w.aug;
        g.dT = w.dT;
        g.ld_dT = w.dT_ld;
        g.dq = w.dq;
        g.dz = w.dz;
        g.dEF = w.dEF;
        g.xu = w.xu;
        g.w16 = w.gw16;
        if (!w.gw16_ready) ga.images_ready = 0;
    }
    ga.D = D;
    ga.HG = hg;
    return true;
}

// compact exchange rows (TowerWs::xu) are addressed by the fused gate kernels only
int require_fused_for_units(const ttamm_tower* const* T, TowerWs* const* W, int ntowers, bool fused_gate) {
    for (int k = 0; k < ntowers; ++k)
        TTAMM_REQUIRE(!W[k]->xu || (T[k]->fusion == TTAMM_FUSION_GATED && fused_gate),
                      "compact exchange rows (exchange_counts) need the item tower on the fused gate kernels "
                      "(ttamm_exchange_compact_supported)");
    return TTAMM_OK;
}

// ---- forward -------------------------------------------------------------------------------
// part FWD_GATHER: ID-row renorm + gather; FWD_FEAT: feature encoder; FWD_FUSION: gate / combine
// (reads the mimic rows)
// TTAMM_GATE_OUT_EPILOGUE=1: the generic gate's sigmoid mix / mimic augment in the second gate
// GEMM's epilogue (EPI_GATE_OUT) instead of gate_mix_kernel after an EPI_STORE launch
bool gate_out_epilogue() {
    static const bool on = dev_env("TTAMM_GATE_OUT_EPILOGUE") != nullptr;
    return on;
}
enum { FWD_GATHER = 1, FWD_FUSION = 2, FWD_FEAT = 4, FWD_MLP = FWD_GATHER | FWD_FEAT, FWD_ALL = 7 };
int tower_forward(const ttamm_tower* T[2], TowerWs* W[2], const ttamm_batch& bt, int D, bool mimic, hipStream_t s,
                  int ntowers, void* const* l0_events = nullptr, int part = FWD_ALL, hipEvent_t after_l0 = nullptr) {
    int rc;
    if (part & FWD_GATHER) {
        // ID rows -> e (ef[:, :D] when gated): both towers' gathers in one launch
        GatherSegs gs;
        gs.count = 0;
        for (int k = 0; k < ntowers; ++k) {
            const ttamm_tower& t = *T[k];
            TowerWs& w = *W[k];
            if (t.id.max_norm > 0.0 && w.R > 0 && w.row_key && w.renorm_key_split > 0) {
                // sharded owner: every requester's positives (keys < global batch) are the reference's
                // first item lookup (training.py:750), the negatives its second (:776)
                for (int ph = 0; ph < 2; ++ph)
                    if ((rc = launch_renorm_rows(t.id.weight, t.id.rows, t.id.dim, w.idx, w.R, t.id.max_norm, w.renorm_mark,
                                                 w.renorm_tag + ph, s, w.row_key, w.renorm_key_split, ph)))
                        return rc;
            } else if (t.id.max_norm > 0.0 && w.R > 0) {  // nn.Embedding max_norm: renorm, then look up
                const int64_t split = w.renorm_split > 0 && w.renorm_split < w.R ? w.renorm_split : w.R;
                if ((rc = launch_renorm_rows(t.id.weight, t.id.rows, t.id.dim, w.idx, split, t.id.max_norm, w.renorm_mark,
                                             w.renorm_tag, s)))
                    return rc;
                if (split < w.R &&
                    (rc = launch_renorm_rows(t.id.weight, t.id.rows, t.id.dim, w.idx + split, w.R - split, t.id.max_norm,
                                             w.renorm_mark, w.renorm_tag + 1, s)))
                    return rc;
            }
            float* dst = uses_ef(t) ? w.ef : w.e;
            const int64_t ld = uses_ef(t) ? efw(t) : t.id.dim;
            gs.seg[gs.count++] = GatherSeg{t.id.weight, t.id.rows, t.id.dim, w.idx, w.R, dst, ld};
        }
        if ((rc = launch_gather_rows_segs(gs, s))) return rc;
    }
    if (part & FWD_FEAT) {
        for (int k = 0; k < ntowers; ++k) {
            const ttamm_tower& t = *T[k];
            TowerWs& w = *W[k];
            if (t.fusion != TTAMM_FUSION_IDENTITY && t.n_linear == 0 && w.R > 0) {
                // identity feature encoder (encoders.py:114-119): f = the feature row
                const int64_t ld = uses_ef(t) ? efw(t) : t.id.dim;
                float* fdst = uses_ef(t) ? w.ef + t.id.dim : w.f;
                if ((rc = launch_add_rows(t.features, t.feat_ld, nullptr, 0, w.R, fo_dim(t), fdst, ld, s, w.fidx)))
                    return rc;
            }
        }
        // feature encoder layers
        int maxL = 0;
        for (int k = 0; k < ntowers; ++k)
            if (T[k]->fusion != TTAMM_FUSION_IDENTITY) maxL = T[k]->n_linear > maxL ? T[k]->n_linear : maxL;
        for (int l = 0; l < maxL; ++l) {
            Batcher bb;
            PadSegs pads;  // first-layer weights padded to 16-B rows, both towers in one launch
            pads.count = 0;
            for (int k = 0; k < ntowers; ++k) {
                const ttamm_tower& t = *T[k];
                TowerWs& w = *W[k];
                if (t.fusion == TTAMM_FUSION_IDENTITY || l >= t.n_linear) continue;
                const ttamm_linear& L = t.linear[l];
                GemmProblem p = gp_base();
                p.bf16 = t.matmul_bf16;
                if (l == 0) {
                    p.A = t.features;
                    p.a_idx = w.fidx;
                    p.lda = t.feat_ld;
                } else {
                    p.A = w.hid[l - 1];
                    p.lda = t.linear[l - 1].out_features;
                }
                p.B = L.weight;
                p.ldb = L.in_features;
                if (l == 0 && w.w16) {  // bf16 operands in memory (C5 layer 1)
                    const int kp = round8(L.in_features);
                    if (!w.weight_prepped &&
                        (rc = launch_to_bf16(L.weight, L.out_features, L.in_features, L.in_features, w.w16, kp, s)))
                        return rc;
                    p.A16 = t.features_bf16;
                    p.lda = t.feat_bf16_ld;
                    p.B16 = w.w16;
                    p.ldb = kp;
                } else if (l == 0 && w.wpad) {
                    if (!w.weight_prepped)
                        pads.seg[pads.count++] = PadSeg{L.weight, L.out_features, L.in_features, L.in_features, w.wpad,
                                                        round4(L.in_features)};
                    p.B = w.wpad;
                    p.ldb = round4(L.in_features);
                }
                p.b_kn = 0;
                p.M = (int)w.R;
                p.N = L.out_features;
                p.K = L.in_features;
                // the feature rows and the padded weight are zero beyond F: run K to the padded
                // width so every k-tile is whole (fast GEMM path)
                if (l == 0 && w.wpad && t.feat_ld >= round4(L.in_features)) p.K = round4(L.in_features);
                if (l == 0 && w.w16) p.K = round8(L.in_features);  // both operands zero beyond F
                // pre-split feature rows (ttamm_tower.features_planes): zero beyond F up to whole
                // 16-k chunks, so K may run to the padded width
                if (l == 0 && t.features_planes && !t.matmul_bf16 && p.K <= 16 * (t.feat_planes_ld / 48)) {
                    p.A3p = t.features_planes;
                    p.lda3 = t.feat_planes_ld;
                }
                p.bias = L.bias;
                if (l + 1 < t.n_linear) {
                    p.epi = EPI_HIDDEN;
                    p.C = w.hid[l];
                    p.ldc = L.out_features;
                    const uint8_t* injected = w.role == ROLE_USER ? bt.user_keep_mask[l] : bt.item_keep_mask[l];
                    set_dropout(p, t, bt, w.role, l, injected);
                    set_keys(p, w);
                    p.act = t.activation;
                    if (t.activation != TTAMM_ACT_RELU) {  // the backward's inputs
                        p.pre = w.pre[l];
                        if (t.dropout > 0.f && injected == nullptr) p.mask_out = w.mask[l];
                        w.keep[l] = injected ? injected : w.mask[l];
                    }
                } else {
                    p.epi = EPI_STORE;
                    if (uses_ef(t)) {
                        p.C = w.ef + t.id.dim;
                        p.ldc = efw(t);
                    } else {
                        p.C = w.f;
                        p.ldc = D;
                    }
                }
                bb.add(p);
            }
            if ((rc = launch_pad_rows_segs(pads, s))) return rc;
            const bool timed = l == 0 && l0_events && l0_events[0] && l0_events[1];
            if (timed) TTAMM_HIP(hipEventRecord((hipEvent_t)l0_events[0], s));
            if ((rc = bb.run(s))) return rc;
            if (timed) TTAMM_HIP(hipEventRecord((hipEvent_t)l0_events[1], s));
            if (l == 0 && after_l0) TTAMM_HIP(hipEventRecord(after_l0, s));
        }
    }
    if (!(part & FWD_FUSION)) return TTAMM_OK;
    // fusion
    GateArgs ga;
    const bool fused_gate = gate_group(T, W, ntowers, D, mimic, ga);
    if ((rc = require_fused_for_units(T, W, ntowers, fused_gate))) return rc;
    if (fused_gate && ga.count > 0) {
        if ((rc = launch_gate(ga, false, s))) return rc;
        for (int k = 0; k < ntowers; ++k) W[k]->gw16_ready = W[k]->gw16 != nullptr;
    }
    Batcher g1, g2, gc;
    for (int k = 0; k < ntowers; ++k) {
        const ttamm_tower& t = *T[k];
        TowerWs& w = *W[k];
        const float* table = mimic ? t.mimic.weight : nullptr;
        if (t.fusion == TTAMM_FUSION_CONCAT) {  // t = [e | f] P^T + b (encoders.py:242-244)
            GemmProblem p = gp_base();
            p.bf16 = t.matmul_bf16;
            p.A = w.ef;
            p.lda = efw(t);
            p.B = t.gate[0].weight;
            p.ldb = efw(t);
            p.M = (int)w.R;
            p.N = D;
            p.K = efw(t);
            p.bias = t.gate[0].bias;
            p.epi = EPI_STORE;
            p.C = w.t;
            p.ldc = w.t_ld;
            gc.add(p);
            continue;
        }
        if (t.fusion == TTAMM_FUSION_GATED) {
            if (fused_gate) continue;
            const int Hg = t.gate[0].out_features;
            GemmProblem p = gp_base();
            p.bf16 = t.matmul_bf16;
            p.A = w.ef;
            p.lda = 2 * D;
            p.B = t.gate[0].weight;
            p.ldb = 2 * D;
            p.M = (int)w.R;
            p.N = Hg;
            p.K = 2 * D;
            p.bias = t.gate[0].bias;
            p.epi = EPI_GATE_HIDDEN;
            p.C = w.z;
            p.ldc = Hg;
            g1.add(p);
            GemmProblem q = gp_base();
            q.bf16 = t.matmul_bf16;
            q.A = w.z;
            q.lda = Hg;
            q.B = t.gate[1].weight;
            q.ldb = Hg;
            q.M = (int)w.R;
            q.N = D;
            q.K = Hg;
            q.bias = t.gate[1].bias;
            if (gate_out_epilogue()) {  // TTAMM_GATE_OUT_EPILOGUE=1: the mix in the GEMM's epilogue
                q.epi = EPI_GATE_OUT;
                q.C = w.aug;
                q.ldc = D;
                q.aux0 = w.ef;
                q.ld_aux0 = 2 * D;
                q.out1 = w.g;
                q.out2 = w.t;
                q.out3 = w.a;
                q.table = table;
                q.idx = w.idx;
                q.ld_out = D;
                q.ld_out2 = w.t_ld;
            } else {  // the pre-activation into g; gate_mix_kernel below (rows.hip)
                q.epi = EPI_STORE;
                q.C = w.g;
                q.ldc = D;
            }
            g2.add(q);
        } else {
            if ((rc = launch_combine(w.e, D, t.fusion == TTAMM_FUSION_SUM ? w.f : nullptr, D, table, t.mimic.rows, w.idx,
                                     w.R, D, w.t, w.a, w.t_ld, w.aug, s)))
                return rc;
        }
    }
    if ((rc = g1.run(s))) return rc;
    if ((rc = g2.run(s))) return rc;
    if (!gate_out_epilogue() && !fused_gate) {
        for (int k = 0; k < ntowers; ++k) {
            const ttamm_tower& t = *T[k];
            TowerWs& w = *W[k];
            if (t.fusion != TTAMM_FUSION_GATED) continue;
            if ((rc = launch_gate_mix(w.g, w.ef, mimic ? t.mimic.weight : nullptr, w.idx, w.R, D, w.t, w.a, w.t_ld, w.aug, s)))
                return rc;
        }
    }
    if ((rc = gc.run(s))) return rc;
    for (int k = 0; k < ntowers; ++k) {  // concat: a = A[idx], aug = t + a (in place on t)
        const ttamm_tower& t = *T[k];
        TowerWs& w = *W[k];
        if (t.fusion != TTAMM_FUSION_CONCAT) continue;
        if ((rc = launch_combine(w.t, w.t_ld, nullptr, D, mimic ? t.mimic.weight : nullptr, t.mimic.rows, w.idx, w.R,
                                 D, w.t, w.a, w.t_ld, w.aug, s)))
            return rc;
    }
    return TTAMM_OK;
}

// TTAMM_WGRAD_X16=1: the bf16 towers' first-layer weight gradient reads X from the bf16 feature copy
bool wgrad_x16() {
    const char* e = dev_env("TTAMM_WGRAD_X16");
    return e && e[0] == '1';
}

// ---- backward ------------------------------------------------------------------------------
// wg_events (optional, 2 events): around the wide weight-gradient GEMM launch (bench)
// part BWD_GATE: the fusion's backward (dEF, the ID rows' gradient with it); BWD_MLP: the feature
// MLP's dgrad chain and every weight gradient
enum { BWD_GATE = 1, BWD_MLP = 2, BWD_ALL = 3 };
int tower_backward(const ttamm_tower* T[2], TowerWs* W[2], int D, hipStream_t s, int ntowers,
                   void* const* wg_events = nullptr, int part = BWD_ALL) {
    int rc;
    if (part & BWD_GATE) {
    // gate: dq, dz, dEF
    GateArgs ga;
    const bool fused_gate = gate_group(T, W, ntowers, D, false, ga);
    if ((rc = require_fused_for_units(T, W, ntowers, fused_gate))) return rc;
    if (fused_gate && ga.count > 0)
        if ((rc = launch_gate(ga, true, s))) return rc;
    Batcher b1, b2;
    for (int k = 0; k < ntowers; ++k) {
        const ttamm_tower& t = *T[k];
        TowerWs& w = *W[k];
        if (t.fusion != TTAMM_FUSION_GATED || fused_gate) continue;
        const int Hg = t.gate[0].out_features;
        if ((rc = launch_gate_dq(w.dT, w.dT_ld, w.ef, w.g, w.R, D, w.dq, s))) return rc;
        GemmProblem p = gp_base();  // dz = (dq . G2) * (z > 0)
        p.bf16 = t.matmul_bf16;
        p.A = w.dq;
        p.lda = D;
        p.B = t.gate[1].weight;  // [D, Hg] = [K, N]
        p.ldb = Hg;
        p.b_kn = 1;
        p.M = (int)w.R;
        p.N = Hg;
        p.K = D;
        p.epi = EPI_DGRAD_RELU;
        p.C = w.dz;
        p.ldc = Hg;
        p.aux0 = w.z;
        p.ld_aux0 = Hg;
        b1.add(p);
        GemmProblem q = gp_base();  // [de | df] = dz . G1 + gate-mix terms
        q.bf16 = t.matmul_bf16;
        q.A = w.dz;
        q.lda = Hg;
        q.B = t.gate[0].weight;  // [Hg, 2D] = [K, N]
        q.ldb = 2 * D;
        q.b_kn = 1;
        q.M = (int)w.R;
        q.N = 2 * D;
        q.K = Hg;
        q.epi = EPI_DGRAD_GATE_EF;
        q.C = w.dEF;
        q.ldc = 2 * D;
        q.aux1 = w.dT;
        q.ld_aux1 = w.dT_ld;
        q.aux2 = w.g;
        q.ld_aux2 = D;
        b2.add(q);
    }
    for (int k = 0; k < ntowers; ++k) {  // concat: d[e | f] = dT P
        const ttamm_tower& t = *T[k];
        TowerWs& w = *W[k];
        if (t.fusion != TTAMM_FUSION_CONCAT) continue;
        GemmProblem q = gp_base();
        q.bf16 = t.matmul_bf16;
        q.A = w.dT;
        q.lda = w.dT_ld;
        q.B = t.gate[0].weight;  // [D, Did + Fo] = [K, N]
        q.ldb = efw(t);
        q.b_kn = 1;
        q.M = (int)w.R;
        q.N = efw(t);
        q.K = D;
        q.epi = EPI_STORE;
        q.C = w.dEF;
        q.ldc = efw(t);
        b2.add(q);
    }
    if ((rc = b1.run(s))) return rc;
    if ((rc = b2.run(s))) return rc;
    }
    if (!(part & BWD_MLP)) return TTAMM_OK;
    // MLP dgrad chain (layers L-1 .. 1)
    int maxL = 0;
    for (int k = 0; k < ntowers; ++k)
        if (T[k]->fusion != TTAMM_FUSION_IDENTITY) maxL = T[k]->n_linear > maxL ? T[k]->n_linear : maxL;
    for (int step = 0; step + 1 < maxL; ++step) {
        Batcher bb;
        for (int k = 0; k < ntowers; ++k) {
            const ttamm_tower& t = *T[k];
            TowerWs& w = *W[k];
            if (t.fusion == TTAMM_FUSION_IDENTITY) continue;
            const int l = t.n_linear - 1 - step;  // layer whose input grad we compute
            if (l < 1) continue;
            const ttamm_linear& L = t.linear[l];
            GemmProblem p = gp_base();
            p.bf16 = t.matmul_bf16;
            if (l == t.n_linear - 1) {
                p.A = uses_ef(t) ? w.dEF + t.id.dim : w.dT;
                p.lda = uses_ef(t) ? efw(t) : w.dT_ld;
            } else {
                p.A = w.dhid[l];
                p.lda = L.out_features;
            }
            p.B = L.weight;  // [out, in] = [K, N]
            p.ldb = L.in_features;
            p.b_kn = 1;
            p.M = (int)w.R;
            p.N = L.in_features;
            p.K = L.out_features;
            p.epi = EPI_DGRAD_HIDDEN;
            p.C = w.dhid[l - 1];
            p.ldc = L.in_features;
            p.aux0 = w.hid[l - 1];
            p.ld_aux0 = L.in_features;
            const float pdrop = t.dropout;
            p.inv_keep = pdrop > 0.f ? 1.0f / (1.0f - pdrop) : 1.0f;
            p.act = t.activation;
            if (t.activation != TTAMM_ACT_RELU) {  // act'(pre-activation), the forward's keep bytes
                p.aux0 = w.pre[l - 1];
                p.keep_prob = 1.0f - pdrop;
                p.keep_mask = pdrop > 0.f ? w.keep[l - 1] : nullptr;
            }
            bb.add(p);
        }
        if ((rc = bb.run(s))) return rc;
    }
    // all weight gradients in one grouped launch
    WgradBatch wb;
    std::memset(&wb, 0, sizeof(wb));
    for (int k = 0; k < ntowers; ++k) {
        const ttamm_tower& t = *T[k];
        TowerWs& w = *W[k];
        if (t.fusion == TTAMM_FUSION_IDENTITY) continue;
        if (t.fusion == TTAMM_FUSION_GATED) {
            const int Hg = t.gate[0].out_features;
            WgradProblem g2{};
            g2.bf16 = t.matmul_bf16;
            g2.dY = w.dq;
            g2.ld_dy = D;
            g2.X = w.z;
            g2.ld_x = Hg;
            g2.R = (int)w.R;
            g2.M = D;
            g2.N = Hg;
            g2.grad_w = w.ggw[1];
            g2.grad_b = w.ggb[1];
            g2.slab = w.slab[TTAMM_MAX_LINEAR + 1];
            g2.rows_per_split = w.wgrad_rps[wgrad_class(g2.M)];
            wb.p[wb.count++] = g2;
            WgradProblem g1{};
            g1.bf16 = t.matmul_bf16;
            g1.dY = w.dz;
            g1.ld_dy = Hg;
            g1.X = w.ef;
            g1.ld_x = 2 * D;
            g1.R = (int)w.R;
            g1.M = Hg;
            g1.N = 2 * D;
            g1.grad_w = w.ggw[0];
            g1.grad_b = w.ggb[0];
            g1.slab = w.slab[TTAMM_MAX_LINEAR];
            g1.rows_per_split = w.wgrad_rps[wgrad_class(g1.M)];
            wb.p[wb.count++] = g1;
        }
        if (t.fusion == TTAMM_FUSION_CONCAT) {  // dP = dT^T [e | f], db = sum dT
            WgradProblem pp{};
            pp.bf16 = t.matmul_bf16;
            pp.dY = w.dT;
            pp.ld_dy = w.dT_ld;
            pp.X = w.ef;
            pp.ld_x = efw(t);
            pp.R = (int)w.R;
            pp.M = D;
            pp.N = efw(t);
            pp.grad_w = w.ggw[0];
            pp.grad_b = w.ggb[0];
            pp.slab = w.slab[TTAMM_MAX_LINEAR];
            pp.rows_per_split = w.wgrad_rps[wgrad_class(pp.M)];
            wb.p[wb.count++] = pp;
        }
        for (int l = t.n_linear - 1; l >= 0; --l) {
            const ttamm_linear& L = t.linear[l];
            WgradProblem p{};
            p.bf16 = t.matmul_bf16;
            if (l == t.n_linear - 1) {
                p.dY = uses_ef(t) ? w.dEF + t.id.dim : w.dT;
                p.ld_dy = uses_ef(t) ? efw(t) : w.dT_ld;
            } else {
                p.dY = w.dhid[l];
                p.ld_dy = L.out_features;
            }
            if (l == 0) {
                p.X = t.features;
                p.x_idx = w.fidx;
                p.ld_x = t.feat_ld;
                if (uses_w16(t) && wgrad_x16()) {  // the same bf16 values, from the tower's bf16 copy
                    p.X16 = t.features_bf16;
                    p.ld_x16 = t.feat_bf16_ld;
                }
                if (t.features_planes && !t.matmul_bf16) {
                    p.X3p = t.features_planes;
                    p.ld_x3 = t.feat_planes_ld;
                }
            } else {
                p.X = w.hid[l - 1];
                p.ld_x = t.linear[l - 1].out_features;
            }
            p.R = (int)w.R;
            p.M = L.out_features;
            p.N = L.in_features;
            p.grad_w = w.gw[l];
            p.grad_b = w.gb[l];
            p.slab = w.slab[l];
            p.rows_per_split = w.wgrad_rps[wgrad_class(p.M)];
            wb.p[wb.count++] = p;
        }
    }
    if ((rc = launch_wgrad(wb, s, wg_events))) return rc;
    return TTAMM_OK;
}

// Deferred exact AdamW(g = 0) (ttamm.h ttamm_table.last_step).
struct Deferred {
    bool on = false;
    AdamConsts* hist = nullptr;
    int cap = 0;
    int slices = 1;
    int32_t step = 0;  // the dense step this call executes
    int decoupled = 1;
    int fast = 0;  // TTAMM_G0_FAST arithmetic for the g = 0 updates
    int sgd = 0;   // torch.optim.SGD dense group: the g = 0 replay is sgd_elem's (replay_sgd_kernel)
    const uint32_t* status = nullptr;  // poisoned: the step writes nothing
    // one-process step with the aux stream: the rolling slice runs there (replay_slice_aux)
    // instead of at the end of the main stream's step
    bool slice_on_aux = false;
    // TTAMM_SLICE_LATE=1: launched when the main stream reaches the table updates (overlapping
    // the memory-bound row updates and the next step's prologue) rather than behind the grouping
    // (overlapping the backward GEMMs).  Measured at C2: the weight-gradient GEMM runs uncontended
    // (132 -> 76 us) but the row updates slow by as much, step 0.7326 vs 0.7280 ms
    // (profiles/r03_c2_slice_late_vs_early_s16.txt) — so behind the grouping stays the default.
    // (Started once the gate backward is enqueued, overlapping dgrad + the weight gradients
    // instead of the gate backward: 0.745 vs 0.712-0.720 ms, profiles/r03_c2_slice_point_s20.txt.)
    bool slice_late = false;
};

// The tables of a tower that belong to the dense (AdamW) group.
int dense_tables(const ttamm_tower& t, bool mimic, const ttamm_table* out[2]) {
    int n = 0;
    if (mimic) out[n++] = &t.mimic;
    if (t.id.optimizer == TTAMM_OPT_DENSE) out[n++] = &t.id;
    return n;
}

ReplaySeg replay_seg(const ttamm_table& tb) {
    ReplaySeg g;
    std::memset(&g, 0, sizeof(g));
    g.p = tb.weight;
    g.m = tb.exp_avg;
    g.v = tb.exp_avg_sq;
    g.last = tb.last_step;
    g.touched = tb.touched;
    g.dim = tb.dim;
    return g;
}

// The rolling slice of the deferred AdamW(g = 0): this step's 1/slices of every dense-group
// table's rows brought to `target` (every row's lag stays below the history ring).
int replay_slice(const ttamm_tower* const* T, int n, bool mimic, const Deferred& df, int32_t target, int stamp,
                 void* const* events, hipStream_t s) {
    ReplayArgs ra;
    std::memset(&ra, 0, sizeof(ra));
    ra.hist = df.hist;
    ra.cap = df.cap;
    ra.decoupled = df.decoupled;
    ra.sgd = df.sgd;
    ra.fast_g0 = df.fast;
    ra.status = df.status;
    ra.target = target;
    ra.stamp = stamp;
    const int slice = (int)(((int64_t)target % df.slices + df.slices) % df.slices);
    for (int k = 0; k < n; ++k) {
        const ttamm_table* tabs[2];
        const int nt = dense_tables(*T[k], mimic, tabs);
        for (int i = 0; i < nt; ++i) {
            ReplaySeg g = replay_seg(*tabs[i]);
            const int64_t per = (tabs[i]->rows + df.slices - 1) / df.slices;
            g.row_lo = std::min<int64_t>(tabs[i]->rows, slice * per);
            g.row_hi = std::min<int64_t>(tabs[i]->rows, g.row_lo + per);
            ra.seg[ra.count++] = g;
        }
    }
    return launch_replay(ra, s, events);
}

// Before a tower reads its rows (part A): count the batch's rows — which marks each row's first
// position — and, deferred, bring the dense-group rows it touches current to step - 1 (each row
// once): the rows behind, listed by lag (the list build stamps them current — a replay that runs
// before this step's row updates, the aux stream's slice or a flush after a poisoned step, must
// see them current to step - 1), then one replay over the list.  Part B groups the rows for the
// row updates at the step's end.  ev: 2 events around the replay kernel (bench).
int tower_prepare_a(const ttamm_tower& t, TowerWs& w, bool mimic, const Deferred& df, hipStream_t s,
                    void* const* ev = nullptr) {
    int rc;
    if ((rc = launch_coalesce_count(w.idx, w.R, t.id.rows, w.co, s))) return rc;
    if (!df.on || w.R == 0) return TTAMM_OK;
    const ttamm_table* tabs[2];
    const int n = dense_tables(t, mimic, tabs);
    if (n == 0) return TTAMM_OK;
    TTAMM_REQUIRE(w.cl.cnt != nullptr, "deferred AdamW: catch-up list workspace missing");
    int32_t* lasts[2] = {tabs[0]->last_step, n > 1 ? tabs[1]->last_step : nullptr};
    if ((rc = launch_catchup_list(w.idx, w.R, w.co.first, lasts, n, df.step - 1, df.cap, w.cl, df.status, s)))
        return rc;
    ReplayArgs ra;
    std::memset(&ra, 0, sizeof(ra));
    ra.hist = df.hist;
    ra.cap = df.cap;
    ra.decoupled = df.decoupled;
    ra.sgd = df.sgd;
    ra.fast_g0 = df.fast;
    ra.status = df.status;
    ra.target = df.step - 1;
    ra.stamp = 0;  // stamped by the list build
    for (int i = 0; i < n; ++i) {
        ReplaySeg g = replay_seg(*tabs[i]);
        g.row_lo = 0;
        g.row_hi = w.R;
        g.list_rows = w.cl.rows;
        g.list_lag = w.cl.lag;
        g.list_cnt = w.cl.cnt;
        ra.seg[ra.count++] = g;
    }
    return launch_replay(ra, s, ev);
}

// tower_prepare_a of `n` towers in four launches (launch_prepare_segs: the counts, the catch-up
// lists' counts and scatters; then one replay over every tower's list) instead of 5-6 per tower:
// the aux stream's prologue is a chain of small launches that the gate waits for.
// ev: 2 events around the replay kernel (bench).
int towers_prepare_a(const ttamm_tower* const* T, TowerWs* const* W, int n, bool mimic, const Deferred& df,
                     hipStream_t s, void* const* ev = nullptr) {
    PrepSegs ps;
    std::memset(&ps, 0, sizeof(ps));
    ps.target = df.step - 1;
    ps.cap = df.cap;
    ps.status = df.status;
    ReplayArgs ra;
    std::memset(&ra, 0, sizeof(ra));
    ra.hist = df.hist;
    ra.cap = df.cap;
    ra.decoupled = df.decoupled;
    ra.sgd = df.sgd;
    ra.fast_g0 = df.fast;
    ra.status = df.status;
    ra.target = df.step - 1;
    ra.stamp = 0;  // stamped by the list build
    for (int k = 0; k < n; ++k) {
        const ttamm_tower& t = *T[k];
        TowerWs& w = *W[k];
        const int64_t rows = t.id.rows;
        TTAMM_REQUIRE(rows < (int64_t(1) << 31) && w.co.key_range >= rows && w.co.cnt && w.co.first,
                      "coalesce: per-row scratch missing");
        TTAMM_REQUIRE(!w.co.sorted || rows <= 65536, "coalesce: sorted grouping needs <= 65536 keys");
        PrepSeg& g = ps.seg[ps.count++];
        g.idx = w.idx;
        g.n = w.R;
        g.cnt = w.co.cnt;
        g.first = w.co.first;
        if (!df.on || w.R == 0) continue;
        const ttamm_table* tabs[2];
        const int nt = dense_tables(t, mimic, tabs);
        if (nt == 0) continue;
        TTAMM_REQUIRE(w.cl.cnt != nullptr, "deferred AdamW: catch-up list workspace missing");
        g.list_cnt = w.cl.cnt;
        g.list_rows = w.cl.rows;
        g.list_lag = w.cl.lag;
        g.nlast = nt;
        for (int i = 0; i < nt; ++i) {
            g.last[i] = tabs[i]->last_step;
            ReplaySeg r = replay_seg(*tabs[i]);
            r.row_lo = 0;
            r.row_hi = w.R;
            r.list_rows = w.cl.rows;
            r.list_lag = w.cl.lag;
            r.list_cnt = w.cl.cnt;
            ra.seg[ra.count++] = r;
        }
    }
    int rc;
    if ((rc = launch_prepare_segs(ps, s))) return rc;
    return launch_replay(ra, s, ev);
}

int tower_prepare_b(const ttamm_tower& t, TowerWs& w, hipStream_t s) {
    return launch_coalesce_group(w.idx, w.R, t.id.rows, w.co, s);
}

int tower_prepare(const ttamm_tower& t, TowerWs& w, bool mimic, const Deferred& df, hipStream_t s,
                  void* const* ev = nullptr) {
    int rc;
    if ((rc = tower_prepare_a(t, w, mimic, df, s, ev))) return rc;
    return tower_prepare_b(t, w, s);
}

// Fork / join events of the aux stream, one set per host thread, device and aux stream (reused
// across steps: a wait binds to the record that precedes it; per aux stream, so the engines of
// in-process ranks — each with its own aux stream — never wait on one another's records).  [0] fork, [1] rows current (before the
// fusion), [2] rows grouped (before the table updates), [3] main stream at the table updates
// (the late slice's start), [4] main stream after the fusion backward (the row updates' start
// on the aux stream), [5] aux stream after the row updates (joined at the step's end).
constexpr int kAuxEvents = 6;
// Device-scope fork / join: both streams are on this device, so an agent-scope release / acquire
// (what every kernel boundary already does) orders their memory.  The default system-scope fence
// of an event record / wait added ≈2 µs of main-stream idle at each of the step's event
// operations (an L2 writeback + invalidate per event, profiles/r06_s23_*).
constexpr unsigned kSyncEventFlags = hipEventDisableTiming | hipEventDisableSystemFence;
hipError_t create_sync_event(hipEvent_t* e) {
    const hipError_t rc = hipEventCreateWithFlags(e, kSyncEventFlags);
    if (rc != hipErrorInvalidValue) return rc;
    (void)hipGetLastError();  // a runtime without the flag: the system-scope event
    return hipEventCreateWithFlags(e, hipEventDisableTiming);
}
int aux_events(hipEvent_t ev[kAuxEvents], hipStream_t aux) {
    struct Set {
        int dev;
        hipStream_t aux;
        hipEvent_t e[kAuxEvents];
    };
    thread_local std::vector<Set> cache;
    int dev = 0;
    TTAMM_HIP(hipGetDevice(&dev));
    for (const Set& p : cache)
        if (p.dev == dev && p.aux == aux) {
            for (int i = 0; i < kAuxEvents; ++i) ev[i] = p.e[i];
            return TTAMM_OK;
        }
    Set p;
    p.dev = dev;
    p.aux = aux;
    for (int i = 0; i < kAuxEvents; ++i) TTAMM_HIP(create_sync_event(&p.e[i]));
    cache.push_back(p);
    for (int i = 0; i < kAuxEvents; ++i) ev[i] = p.e[i];
    return TTAMM_OK;
}

bool overlapped(const ttamm_tower* const* T, int n, const Deferred& df, hipStream_t s, hipStream_t aux) {
    bool overlap = aux != nullptr && aux != s;
    for (int k = 0; k < n; ++k)
        if (df.on && T[k]->id.optimizer == TTAMM_OPT_DENSE) overlap = false;
    return overlap;
}

// tower_prepare of `n` towers, then their forward.  With an aux stream the index-only prologue
// runs there while `s` gathers ID rows and runs the feature MLP: part A (count + deferred
// catch-up) first, joined before the fusion, whose epilogue reads the mimic rows; then part B
// (grouping), joined by table_updates.  A deferred dense ID table is read by the first gather,
// so that case stays serial.
// cu_events (optional): ttamm_step_args.timing_events + 8 — [0, 1] around the user tower's
// catch-up replay, [2, 3] around the item tower's (overlapped: [0, 1] around the one replay of
// both towers' lists)
int prepare_forward(const ttamm_tower* T[2], TowerWs* W[2], int n, const ttamm_batch& bt, int D, bool mimic,
                    const Deferred& df, hipStream_t s, hipStream_t aux, void* const* l0_events,
                    void* const* maint_events = nullptr, void* const* cu_events = nullptr,
                    void* const* gather_events = nullptr) {
    int rc;
    auto cu_ev = [&](int k) -> void* const* {
        return cu_events ? cu_events + (W[k]->role == ROLE_USER ? 0 : 2) : nullptr;
    };
    if (!overlapped(T, n, df, s, aux)) {
        for (int k = 0; k < n; ++k)
            if ((rc = tower_prepare(*T[k], *W[k], mimic, df, s, cu_ev(k)))) return rc;
        return tower_forward(T, W, bt, D, mimic, s, n, l0_events, FWD_ALL);
    }
    // The MLP launches are enqueued first: the prologue is a dozen small launches whose
    // host-side enqueue would otherwise hold the GEMMs back behind the host.
    hipEvent_t ev[kAuxEvents];
    if ((rc = aux_events(ev, aux))) return rc;
    // bf16 towers: the prologue starts after the first layer's GEMM (its one-block-per-CU tiles
    // otherwise wait for CUs behind the catch-up replay); fp32 towers: at once
    const bool late_fork = T[0]->matmul_bf16 && dev_env("TTAMM_EARLY_FORK") == nullptr;
    // fp32 towers: the ID-row gather also runs on the aux stream (ahead of the catch-up), beside the
    // first-layer GEMM, which reads only the feature rows; the fusion joins it with the catch-up
    static const bool gather_main = dev_env("TTAMM_GATHER_MAIN") != nullptr;
    const bool gather_aux = !late_fork && !gather_main;
    if (!late_fork) TTAMM_HIP(hipEventRecord(ev[0], s));
    if ((rc = tower_forward(T, W, bt, D, mimic, s, n, l0_events, gather_aux ? FWD_FEAT : FWD_MLP,
                            late_fork ? ev[0] : nullptr)))
        return rc;
    TTAMM_HIP(hipStreamWaitEvent(aux, ev[0], 0));
    if (gather_aux) {
        const bool timed = gather_events && gather_events[0] && gather_events[1];
        if (timed) TTAMM_HIP(hipEventRecord((hipEvent_t)gather_events[0], aux));
        if ((rc = tower_forward(T, W, bt, D, mimic, aux, n, nullptr, FWD_GATHER))) return rc;
        if (timed) TTAMM_HIP(hipEventRecord((hipEvent_t)gather_events[1], aux));
    }
    if ((rc = towers_prepare_a(T, W, n, mimic, df, aux, cu_ev(0)))) return rc;
    TTAMM_HIP(hipEventRecord(ev[1], aux));
    // the fusion is enqueued before the grouping's dozen launches: enqueued after them, the host
    // still issued them when the GPU finished the MLP (~55 us idle per C2 step)
    TTAMM_HIP(hipStreamWaitEvent(s, ev[1], 0));
    if ((rc = tower_forward(T, W, bt, D, mimic, s, n, l0_events, FWD_FUSION))) return rc;
    for (int k = 0; k < n; ++k)
        if ((rc = tower_prepare_b(*T[k], *W[k], aux))) return rc;
    TTAMM_HIP(hipEventRecord(ev[2], aux));
    if (df.slice_on_aux && !df.slice_late) {
        // The previous step's slice (target step - 1), behind this step's catch-up on the aux
        // stream, overlapping the main stream's GEMMs instead of closing the step.  The rows this
        // batch touches are current to step - 1 after the catch-up, so the slice skips them and
        // never races the row updates; its stamp is an atomicMax (a row update may have moved a
        // row to `step` meanwhile).  The next step's catch-up and the flush are ordered after it.
        if ((rc = replay_slice(T, n, mimic, df, df.step - 1, 2, maint_events, aux))) return rc;
    }
    return TTAMM_OK;
}

// the row updates need the grouping (prepare part B), possibly still running on the aux stream
int join_grouping(hipStream_t s, hipStream_t aux) {
    if (aux == nullptr || aux == s) return TTAMM_OK;
    hipEvent_t ev[kAuxEvents];
    int rc;
    if ((rc = aux_events(ev, aux))) return rc;
    TTAMM_HIP(hipStreamWaitEvent(s, ev[2], 0));
    return TTAMM_OK;
}

RowUpdateArgs row_update_args(const ttamm_tower& t, TowerWs& w, int D, bool mimic, const SparseConsts& sp,
                              const AdamConsts& ad, const Deferred& df, const float* grad_scale) {
    RowUpdateArgs ru;
    std::memset(&ru, 0, sizeof(ru));
    ru.n = w.R;
    ru.dim = t.id.dim;  // == D unless concat fusion has another output_dim (tower_optimizer_rows)
    ru.n_unique = w.co.n_unique;
    ru.seg_start = w.co.seg_start;
    ru.keys = w.co.keys_out;
    ru.rows = w.co.vals_out;
    ru.seglong = w.co.seglong;
    if (uses_ef(t)) {
        ru.dE = w.dEF;
        ru.ld_dE = efw(t);
    } else {
        ru.dE = w.dT;
        ru.ld_dE = w.dT_ld;
    }
    ru.id = t.id;
    if (mimic) {
        ru.mimic = t.mimic;
        ru.dA_lo = w.dA;
        ru.dA_hi = w.dT;
        ru.ld_dA = w.dA_ld;
        ru.split_row = w.dA_split;
        ru.xu = w.xu;
    }
    ru.side_id = w.side_id;
    ru.side_mimic = w.side_mimic;
    ru.piece_e = w.piece_e;
    ru.piece_a = w.piece_a;
    ru.sp = sp;
    ru.ad = ad;
    ru.dense_step = df.step;
    ru.status = df.status;
    ru.grad_scale = grad_scale;
    return ru;
}
int tower_optimizer_rows(const ttamm_tower& t, TowerWs& w, int D, bool mimic, const SparseConsts& sp,
                         const AdamConsts& ad, const Deferred& df, hipStream_t s, const float* grad_scale) {
    const RowUpdateArgs ru = row_update_args(t, w, D, mimic, sp, ad, df, grad_scale);
    if (!mimic || t.id.dim == D) return launch_row_update(ru, s);
    // concat with output_dim != embedding_dim: the ID rows and the (output-wide) mimic rows differ
    // in width, so the two tables are updated by two passes over the same row grouping
    RowUpdateArgs a = ru, b = ru;
    std::memset(&a.mimic, 0, sizeof(a.mimic));
    a.piece_a = a.side_mimic = nullptr;
    std::memset(&b.id, 0, sizeof(b.id));
    b.dE = nullptr;
    b.piece_e = b.side_id = nullptr;
    b.dim = D;
    int rc;
    if ((rc = launch_row_update(a, s))) return rc;
    return launch_row_update(b, s);
}
void add_seg(SweepArgs& sw, const ttamm_table& tb) {
    sw.seg[sw.count].p = tb.weight;
    sw.seg[sw.count].m = tb.exp_avg;
    sw.seg[sw.count].v = tb.exp_avg_sq;
    sw.seg[sw.count].n = tb.rows * tb.dim;
    sw.count++;
}

// Touched-row updates of the tables of `n` towers, then the AdamW(g=0) step of the rows the
// batch did not touch: eagerly, one sweep over the dense-group tables and a scatter of the
// staged touched rows; deferred, the replay of this step's 1/slices of the rows to `step`.
int table_updates(const ttamm_tower* T[2], TowerWs* W[2], int n, int D, bool mimic, const SparseConsts& sp,
                  const AdamConsts& ad, const Deferred& df, void* const events[2], hipStream_t s, hipStream_t aux,
                  const float* grad_scale = nullptr) {
    int rc;
    if ((rc = join_grouping(s, aux))) return rc;
    if (df.on && df.slice_on_aux && df.slice_late) {
        // the previous step's slice (target step - 1, as in prepare_forward), started on the aux
        // stream now: the catch-up and the grouping before it on that stream, the row updates
        // beside it (the rows they touch are current to step - 1, so the slice skips them)
        hipEvent_t ev[kAuxEvents];
        if ((rc = aux_events(ev, aux))) return rc;
        TTAMM_HIP(hipEventRecord(ev[3], s));
        TTAMM_HIP(hipStreamWaitEvent(aux, ev[3], 0));
        if ((rc = replay_slice(T, n, mimic, df, df.step - 1, 2, events, aux))) return rc;
    }
    for (int k = 0; k < n; ++k)
        if ((rc = tower_optimizer_rows(*T[k], *W[k], D, mimic, sp, ad, df, s, grad_scale))) return rc;
    if (df.on) {
        if (df.slice_on_aux) return TTAMM_OK;  // replayed on the aux stream (replay_slice_aux)
        return replay_slice(T, n, mimic, df, df.step, 1, events, s);
    }
    SweepArgs sw;
    std::memset(&sw, 0, sizeof(sw));
    sw.ad = ad;
    sw.status = df.status;
    if (mimic)
        for (int k = 0; k < n; ++k) add_seg(sw, T[k]->mimic);
    for (int k = 0; k < n; ++k)
        if (T[k]->id.optimizer == TTAMM_OPT_DENSE) add_seg(sw, T[k]->id);
    // SGD without momentum or weight decay leaves g = 0 rows where they are: no sweep
    const bool sweep = !(ad.sgd && ad.sgd_mom == 0.f && ad.wd == 0.f);
    if (events && events[0]) TTAMM_HIP(hipEventRecord((hipEvent_t)events[0], s));
    if (sweep && (rc = launch_dense_sweep(sw, s))) return rc;
    if (events && events[1]) TTAMM_HIP(hipEventRecord((hipEvent_t)events[1], s));
    for (int k = 0; k < n; ++k) {
        const ttamm_tower& t = *T[k];
        TowerWs& w = *W[k];
        if (mimic)
            if ((rc = launch_side_scatter(w.co.n_unique, w.co.keys_out, w.co.seg_start, w.side_mimic, w.R, D, t.mimic,
                                          df.status, s)))
                return rc;
        if (t.id.optimizer == TTAMM_OPT_DENSE)
            if ((rc = launch_side_scatter(w.co.n_unique, w.co.keys_out, w.co.seg_start, w.side_id, w.R, t.id.dim, t.id,
                                          df.status, s)))
                return rc;
    }
    return TTAMM_OK;
}

DenseAdamArgs dense_args(const ttamm_tower* T[2], TowerWs* W[2], const AdamConsts& ad, const uint32_t* status,
                         const float* grad_scale) {
    DenseAdamArgs da;
    std::memset(&da, 0, sizeof(da));
    da.ad = ad;
    da.status = status;
    da.grad_scale = grad_scale;
    auto add_dense = [&](float* p, float* m, float* v, const float* g, int64_t n) {
        da.t[da.count++] = DenseTensor{p, m, v, g, n};
    };
    for (int k = 0; k < 2; ++k) {
        const ttamm_tower& t = *T[k];
        TowerWs& w = *W[k];
        if (t.fusion == TTAMM_FUSION_IDENTITY) continue;
        for (int l = 0; l < t.n_linear; ++l) {
            const ttamm_linear& L = t.linear[l];
            add_dense(L.weight, L.weight_exp_avg, L.weight_exp_avg_sq, w.gw[l], (int64_t)L.out_features * L.in_features);
            add_dense(L.bias, L.bias_exp_avg, L.bias_exp_avg_sq, w.gb[l], L.out_features);
        }
        {
            for (int q = 0; q < fusion_linears(t); ++q) {
                const ttamm_linear& L = t.gate[q];
                add_dense(L.weight, L.weight_exp_avg, L.weight_exp_avg_sq, w.ggw[q],
                          (int64_t)L.out_features * L.in_features);
                add_dense(L.bias, L.bias_exp_avg, L.bias_exp_avg_sq, w.ggb[q], L.out_features);
            }
        }
    }
    return da;
}
int dense_update(const ttamm_tower* T[2], TowerWs* W[2], const AdamConsts& ad, const uint32_t* status, hipStream_t s,
                 const float* grad_scale = nullptr) {
    return launch_dense_adam(dense_args(T, W, ad, status, grad_scale), s);
}

// the tables' row partials of the squared gradient norm into ws.clip_partials[1, *off)
int clip_table_partials(const ttamm_tower* T[2], TowerWs* W[2], int D, bool mimic, const SparseConsts& sp,
                        const AdamConsts& ad, const Deferred& df, StepWs& ws, hipStream_t s, hipStream_t aux,
                        int* off_out) {
    int rc;
    if ((rc = join_grouping(s, aux))) return rc;  // the row grouping
    int off = 1;
    for (int k = 0; k < 2; ++k) {
        if (!T[k] || W[k]->R <= 0) continue;
        const RowUpdateArgs ru = row_update_args(*T[k], *W[k], D, mimic, sp, ad, df, nullptr);
        if ((rc = launch_rows_sumsq(ru, ws.clip_partials + off, s))) return rc;
        off += rows_sumsq_blocks(W[k]->R, T[k]->id.dim);
    }
    TTAMM_REQUIRE(off <= ws.clip_parts, "clip: partials overflow");
    *off_out = off;
    return TTAMM_OK;
}

// clip_grad_norm_(model.parameters(), max_norm) (training.py:824-825): the global gradient norm
// over both towers' table rows and dense tensors -> ws.clip_coef, read by the optimizer kernels
int clip_coefficient(const ttamm_tower* T[2], TowerWs* W[2], int D, bool mimic, const SparseConsts& sp,
                     const AdamConsts& ad, const Deferred& df, const ttamm_step_args& A, StepWs& ws, hipStream_t s,
                     hipStream_t aux) {
    int rc;
    int off;
    if ((rc = clip_table_partials(T, W, D, mimic, sp, ad, df, ws, s, aux, &off))) return rc;
    if ((rc = launch_dense_sumsq(dense_args(T, W, ad, A.status, nullptr), ws.clip_partials + off, s))) return rc;
    off += kDenseSumsqBlocks;
    TTAMM_REQUIRE(off <= ws.clip_parts, "clip: partials overflow");
    return launch_clip_coef(ws.clip_partials + 1, off - 1, (float)A.hp.grad_clip_norm, ws.clip_coef, s);
}

// sharded clipping, TOWERS_BWD: this rank's share of the squared gradient norm over the table
// rows it owns (its users', its items' — every requester's contributions to a row summed first),
// into *A.table_sumsq for the caller's all-reduce
int clip_table_share(const ttamm_tower* T[2], TowerWs* W[2], int D, bool mimic, const SparseConsts& sp,
                     const AdamConsts& ad, const Deferred& df, const ttamm_step_args& A, StepWs& ws, hipStream_t s,
                     hipStream_t aux) {
    int rc;
    int off;
    if ((rc = clip_table_partials(T, W, D, mimic, sp, ad, df, ws, s, aux, &off))) return rc;
    return launch_sum_partials(ws.clip_partials + 1, off - 1, A.table_sumsq, s);
}

// sharded clipping, TABLES: clip_grad_norm_'s coefficient from the all-reduced table share and the
// (all-reduced) replicated-weight gradients
int clip_coefficient_sharded(const ttamm_tower* T[2], TowerWs* W[2], const AdamConsts& ad, const ttamm_step_args& A,
                             StepWs& ws, hipStream_t s) {
    int rc;
    TTAMM_HIP(hipMemcpyAsync(ws.clip_partials, A.table_sumsq, sizeof(float), hipMemcpyDeviceToDevice, s));
    if ((rc = launch_dense_sumsq(dense_args(T, W, ad, A.status, nullptr), ws.clip_partials + 1, s))) return rc;
    return launch_clip_coef(ws.clip_partials, 1 + kDenseSumsqBlocks, (float)A.hp.grad_clip_norm, ws.clip_coef, s);
}

// Deferred mode is all-or-nothing over the dense-group tables of both towers.
int deferred_of(const ttamm_step_args& A, Deferred& df) {
    const bool mimic = A.mimic_enabled != 0;
    int with = 0, total = 0;
    for (const ttamm_tower* t : {&A.user, &A.item}) {
        const ttamm_table* tabs[2];
        const int n = dense_tables(*t, mimic, tabs);
        for (int i = 0; i < n; ++i) {
            ++total;
            with += tabs[i]->last_step != nullptr ? 1 : 0;
        }
    }
    if (with == 0) return TTAMM_OK;
    TTAMM_REQUIRE(with == total, "deferred AdamW: every dense-group table needs last_step");
    TTAMM_REQUIRE(A.adam_history != nullptr && A.replay_slices >= 1 && A.history_capacity > A.replay_slices &&
                      A.history_capacity <= kMaxAdamHistory,
                  "deferred AdamW: needs adam_history and replay_slices < history_capacity <= 512");
    TTAMM_REQUIRE(A.hp.dense_step < (double)INT32_MAX, "deferred AdamW: step count out of range");
    df.on = true;
    df.hist = static_cast<AdamConsts*>(A.adam_history);
    df.cap = A.history_capacity;
    df.slices = A.replay_slices;
    df.step = (int32_t)A.hp.dense_step;
    df.decoupled = A.hp.decoupled_weight_decay ? 1 : 0;
    df.fast = A.table_g0_math == TTAMM_G0_FAST ? 1 : 0;
    df.sgd = A.hp.dense_optimizer == TTAMM_DENSE_SGD ? 1 : 0;
    return TTAMM_OK;
}

// the category-alignment rows of this step: one process, the item tower's augmented rows
// [positives; negatives]; sharded requester, its requests' (t | a) exchange rows and global ids
CalArgs& bind_cal(const ttamm_step_args& A, StepWs& ws, const TowerWs& I, int64_t B, int D, bool mimic) {
    CalArgs& c = ws.cal;
    c.xa_rows = INT64_MAX;
    if (sharded(A)) {
        c.x = A.item_fwd_in;
        c.xa = mimic ? A.item_fwd_in + D : nullptr;
        c.ld_x = 2 * D;
        c.slot = A.item_slot;
        if (compact_exchange(A)) {  // units of D floats; a negative's row is t + a already
            c.ld_x = D;
            c.slot = A.item_slot;  // units (ttamm_route_rows with counts_ld >= 3)
            c.xa_rows = B;
        }
        c.idx = A.b.pos_items;
        c.idx1 = A.b.neg_items;
        c.split = B;
        c.idx_rows = A.num_items_global > 0 ? A.num_items_global : A.item.id.rows;
    } else {
        c.x = I.aug;
        c.ld_x = D;
        c.idx = I.idx;
        c.idx_rows = A.item.id.rows;
    }
    c.categories = A.item_categories;
    c.num_categories = A.num_categories;
    c.major = A.major_category;
    c.lambda = (float)A.hp.lambda_category_alignment;
    return c;
}

int validate_step(const ttamm_step_args& A) {
    const int D = out_dim(A.user);
    int rc;
    TTAMM_REQUIRE(A.table_g0_math == TTAMM_G0_EXACT || A.table_g0_math == TTAMM_G0_FAST,
                  "table_g0_math must be TTAMM_G0_EXACT or TTAMM_G0_FAST");
    if ((rc = validate_tower(A.user, "user_encoder", D, true))) return rc;
    if ((rc = validate_tower(A.item, "item_encoder", D, true))) return rc;
    TTAMM_REQUIRE(out_dim(A.item) == D, "User and item encoders must produce embeddings with the same dimension.");
    TTAMM_REQUIRE(A.user.matmul_bf16 == A.item.matmul_bf16, "user and item towers must share one matmul precision");
    if (A.hp.grad_clip_norm > 0.0 && A.mimic_enabled)
        TTAMM_REQUIRE(A.user.id.dim == D && A.item.id.dim == D,
                      "gradient clipping with a concat output_dim other than the embedding dim is not supported");
    TTAMM_REQUIRE(A.b.batch > 0, "empty batch");
    if (cal_enabled(A)) {
        TTAMM_REQUIRE(!sharded(A) || (A.cal_stats && A.cal_scatter),
                      "the row-sharded category-alignment loss needs cal_stats and cal_scatter");
        TTAMM_REQUIRE(!sharded(A) || !(A.phase & (TTAMM_PHASE_CAL_STATS | TTAMM_PHASE_CAL_SCATTER |
                                                  TTAMM_PHASE_SCORE | TTAMM_PHASE_USER)) ||
                          (A.item_fwd_in && (A.b.num_neg == 0 || A.b.neg_items)),
                      "the row-sharded category-alignment loss needs item_fwd_in and b.neg_items");
        TTAMM_REQUIRE(A.num_categories > 0 && A.num_categories <= 65535,
                      "category alignment: num_categories must be in [1, 65535]");
        TTAMM_REQUIRE(A.major_category >= 0 && A.major_category < A.num_categories,
                      "category alignment: major_category out of range");
        TTAMM_REQUIRE(D <= 256, "category alignment: embedding dim must be <= 256");
    }
    if (A.in_batch) {
        TTAMM_REQUIRE(A.b.num_neg >= 0, "num_negatives must be >= 0 with in-batch negatives");
        TTAMM_REQUIRE(D % 4 == 0 && D <= 128, "in-batch negatives: embedding dim must be <= 128");
    } else {
        TTAMM_REQUIRE(A.b.num_neg > 0, "num_negatives must be greater than zero.");
    }
    const int64_t num_items = A.num_items_global > 0 ? A.num_items_global : A.item.id.rows;
    TTAMM_REQUIRE(num_items > 1, "num_items must be greater than one.");
    if (A.mimic_enabled) {
        TTAMM_REQUIRE(A.user.mimic.weight && A.item.mimic.weight, "mimic tables missing");
        TTAMM_REQUIRE(A.user.mimic.dim == D && A.item.mimic.dim == D &&
                          A.user.mimic.rows == A.user.id.rows && A.item.mimic.rows == A.item.id.rows,
                      "Adaptive mimic requires user and item embedding dimensions to match.");
    }
    TTAMM_REQUIRE(A.hp.dense_step >= 1 && A.hp.sparse_step >= 1, "optimizer step counts must be >= 1");
    TTAMM_REQUIRE(A.hp.dense_optimizer == TTAMM_DENSE_ADAM || A.hp.dense_optimizer == TTAMM_DENSE_SGD,
                  "hp.dense_optimizer must be TTAMM_DENSE_ADAM or TTAMM_DENSE_SGD");
    for (const ttamm_tower* t : {&A.user, &A.item})
        if (t->id.max_norm > 0.0) {
            TTAMM_REQUIRE(t->id.optimizer == TTAMM_OPT_DENSE, "max_norm is not supported when using sparse embeddings.");
        }
    if (A.hp.grad_clip_norm > 0.0) {
        TTAMM_REQUIRE(!sharded(A) || !(A.phase & (TTAMM_PHASE_USER | TTAMM_PHASE_ITEM_BWD)),
                      "gradient clipping in the row-sharded step needs the grouped schedule (SCORE / TOWERS_BWD)");
        TTAMM_REQUIRE(!sharded(A) || A.table_sumsq != nullptr, "sharded gradient clipping needs table_sumsq");
        TTAMM_REQUIRE(A.user.id.optimizer == TTAMM_OPT_DENSE && A.item.id.optimizer == TTAMM_OPT_DENSE,
                      "gradient clipping needs dense ID tables (clip_grad_norm_ cannot take the sparse gradients "
                      "of sparse ID tables)");
    }
    TTAMM_REQUIRE(A.row_base >= 0 && (A.global_batch == 0 || A.global_batch >= A.row_base + A.b.batch),
                  "row_base / global_batch out of range");
    if (!sharded(A)) return TTAMM_OK;
    const int ph = A.phase;
    TTAMM_REQUIRE((ph & ~8191) == 0, "unknown phase bits");
    TTAMM_REQUIRE(!((ph & TTAMM_PHASE_USER) && (ph & (TTAMM_PHASE_SCORE | TTAMM_PHASE_TOWERS_BWD))),
                  "USER and SCORE / TOWERS_BWD are alternatives");
    TTAMM_REQUIRE(A.in_batch || (ph & (TTAMM_PHASE_INBATCH_SRC | TTAMM_PHASE_INBATCH)) == 0,
                  "INBATCH phases need in_batch");
    TTAMM_REQUIRE(A.item_rows_capacity >= 0 && A.n_item_rows >= 0 && A.n_item_rows <= A.item_rows_capacity,
                  "n_item_rows exceeds item_rows_capacity");
    if (ph & TTAMM_PHASE_SAMPLE)
        TTAMM_REQUIRE(!A.b.sample_negatives || A.b.neg_items, "sharded SAMPLE phase needs b.neg_items for the exchange");
    if (A.exchange_counts) {
        TTAMM_REQUIRE(A.mimic_enabled && A.item.fusion == TTAMM_FUSION_GATED,
                      "compact exchange rows (exchange_counts) need mimic on and a gated item tower");
        TTAMM_REQUIRE(A.exchange_world >= 1 && A.exchange_world <= 1024 && A.exchange_counts_ld >= 3,
                      "exchange_counts needs exchange_world in [1, 1024] and exchange_counts_ld >= 3");
        TTAMM_REQUIRE(A.item_slot, "compact exchange rows need item_slot (the requests' units)");
    }
    if ((ph & (TTAMM_PHASE_ITEM_FWD | TTAMM_PHASE_ITEM_BWD)) && A.n_item_rows > 0)
        TTAMM_REQUIRE(A.item_rows && A.item_row_keys, "item_rows / item_row_keys missing");
    if (ph & TTAMM_PHASE_ITEM_FWD) TTAMM_REQUIRE(A.item_fwd_out || A.n_item_rows == 0, "item_fwd_out missing");
    if (ph & (TTAMM_PHASE_USER | TTAMM_PHASE_SCORE))
        TTAMM_REQUIRE(A.item_fwd_in && A.item_bwd_out, "item_fwd_in / item_bwd_out missing");
    if (ph & (TTAMM_PHASE_ITEM_BWD | TTAMM_PHASE_TOWERS_BWD))
        TTAMM_REQUIRE(A.item_bwd_in || A.n_item_rows == 0, "item_bwd_in missing");
    if (ph & (TTAMM_PHASE_USER | TTAMM_PHASE_SCORE | TTAMM_PHASE_ITEM_BWD | TTAMM_PHASE_TOWERS_BWD |
              TTAMM_PHASE_DENSE))
        TTAMM_REQUIRE(A.dense_grads != nullptr, "dense_grads missing");
    return TTAMM_OK;
}

int run_step(const ttamm_step_args& A, hipStream_t s) {
    int rc;
    if ((rc = validate_step(A))) return rc;
    const int D = out_dim(A.user);
    const bool mimic = A.mimic_enabled != 0;
    const bool shard = sharded(A);
    const int ph = shard ? A.phase : 255;

    Arena ar{static_cast<char*>(A.workspace), A.workspace_bytes, 0, false};
    StepWs ws;
    plan(ar, A, ws);
    TTAMM_REQUIRE(ar.ok(), "workspace too small for this step");

    const int64_t B = A.b.batch;
    const int N = A.b.num_neg;
    const int64_t Bg = global_batch(A);
    const int64_t num_items = A.num_items_global > 0 ? A.num_items_global : A.item.id.rows;
    // ---- row bindings -----------------------------------------------------------------------
    TowerWs& U = ws.user;
    TowerWs& I = ws.item;
    U.idx = U.fidx = U.idx_own;  // staged copy of A.b.users
    U.key_split = B;
    U.key_base0 = A.row_base;
    int64_t* neg = nullptr;
    if (shard) {
        I.R = A.n_item_rows;
        I.idx = I.fidx = I.idx_own;  // staged copy of A.item_rows
        I.row_key = ws.keys_own;  // staged copy of A.item_row_keys (ITEM_FWD)
        I.t = A.item_fwd_out;
        I.a = mimic && A.item_fwd_out ? A.item_fwd_out + D : nullptr;
        I.t_ld = 2 * D;
        I.aug = nullptr;
        I.dT = A.item_bwd_in;
        I.dT_ld = 2 * D;
        I.dA = A.item_bwd_in ? A.item_bwd_in + D : nullptr;
        I.dA_ld = 2 * D;
        I.dA_split = I.R;  // every row's mimic gradient is shipped in (dT | dA)
        if (compact_exchange(A)) {  // D-float units: (t | a) of a positive, t + a of a negative
            I.t_ld = I.dT_ld = I.dA_ld = D;
            I.xu = ws.own_units;
        }
        I.renorm_key_split = Bg;  // request keys: positives [0, Bg), negatives from Bg on
        neg = A.b.neg_items;
    } else {
        I.idx = I.fidx = I.idx_own;
        // item row r < B is interaction r's positive, else negative slot r - B
        I.key_split = B;
        I.key_base0 = A.row_base;
        I.key_base1 = Bg + A.row_base * N;
        neg = I.idx_own + B;
    }
    // max_norm claim tags: unique per lookup (users; positives, then negatives)
    U.renorm_tag = I.renorm_tag = (int32_t)(2 * (A.hp.dense_step % (1 << 29)) + 1);
    if (!shard) I.renorm_split = B;
    const ttamm_tower* T[2] = {&A.user, &A.item};
    TowerWs* W[2] = {&U, &I};
    // TTAMM_PROLOGUE_PREP=1: the SAMPLE phase's prologue forms the first-layer weights (every step
    // runs it first) instead of the pad / bf16 launches before the first GEMM.  Measured slower at
    // C2 (0.660 vs 0.648 ms/step, two A/B pairs on one box; C5 unchanged at 1.413 ms,
    // profiles/r05_s9_prologue_prep.txt): the first GEMM waits for the whole prologue grid
    {
        const char* e = dev_env("TTAMM_PROLOGUE_PREP");
        U.weight_prepped = I.weight_prepped = e && e[0] == '1';
    }
    const ttamm_hparams& hp = A.hp;
    AdamConsts ad = hp.dense_optimizer == TTAMM_DENSE_SGD
                        ? make_sgd_consts(hp.lr, hp.weight_decay, hp.momentum, hp.dampening, hp.nesterov,
                                          hp.sgd_first_step)
                        : make_adam_consts(hp.lr, hp.beta1, hp.beta2, hp.eps, hp.weight_decay,
                                           hp.decoupled_weight_decay, hp.dense_step);
    ad.fast_g0 = A.table_g0_math == TTAMM_G0_FAST ? 1 : 0;
    const SparseConsts sp = make_sparse_consts(hp.sparse_lr, hp.sparse_beta1, hp.sparse_beta2, hp.sparse_eps,
                                               hp.sparse_step);
    Deferred df;
    if ((rc = deferred_of(A, df))) return rc;
    df.status = A.status;

    // ---- indices and negatives ---------------------------------------------------------------
    // one process with the aux stream: the step's count / AdamW constants on the aux stream (below;
    // not with the developer's slice on the main stream, which replays to this step's entry)
    const bool begin_aux = !shard && (ph & TTAMM_PHASE_SAMPLE) &&
                           overlapped(T, 2, df, s, static_cast<hipStream_t>(A.aux_stream)) &&
                           !dev_env("TTAMM_SLICE_MAIN");
    if (ph & TTAMM_PHASE_SAMPLE) {
        // range-checked copies of the batch's ids (nn.Embedding raises IndexError,
        // encoders.py:222-223): an out-of-range id sets TTAMM_STATUS_INDEX_OUT_OF_RANGE, is
        // replaced by row 0 so no kernel reads outside a table, and the step writes nothing
        StageArgs st;
        std::memset(&st, 0, sizeof(st));
        st.status = A.status;
        st.seg[st.count++] = StageSeg{A.b.users, U.idx_own, B, A.user.id.rows};
        if (!shard) {
            st.seg[st.count++] = StageSeg{A.b.pos_items, I.idx_own, B, A.item.id.rows};
            if (!A.b.sample_negatives && N > 0) {
                TTAMM_REQUIRE(A.b.neg_items != nullptr, "negatives must be given when sample_negatives == 0");
                st.seg[st.count++] = StageSeg{A.b.neg_items, neg, B * N, A.item.id.rows};
            }
        } else {  // requester: global item ids, checked only (the owners stage their local rows)
            st.seg[st.count++] = StageSeg{A.b.pos_items, nullptr, B, num_items};
            if (!A.b.sample_negatives && A.b.neg_items && N > 0)
                st.seg[st.count++] = StageSeg{A.b.neg_items, nullptr, B * N, num_items};
        }
        TTAMM_REQUIRE(A.status != nullptr, "the training step needs a status word");
        // staging, the sampler and the step's count + AdamW constants (unless a status error
        // stops it) in one launch
        TTAMM_REQUIRE(!(A.b.sample_negatives && N > 0) || num_items > 1, "num_items must be greater than one.");
        PrologueArgs pa;
        std::memset(&pa, 0, sizeof(pa));
        if (A.b.sample_negatives && N > 0) {
            // one process: into the item tower's rows and (when given) the caller's buffer
            pa.users = A.b.users;
            pa.user_rows = A.user.id.rows;
            pa.batch = B;
            pa.num_neg = N;
            pa.num_items = (uint64_t)num_items;
            pa.pos_offsets = A.b.pos_offsets;
            pa.pos_values = A.b.pos_values;
            pa.k0 = (uint32_t)A.b.seed;
            pa.k1 = (uint32_t)(A.b.seed >> 32);
            pa.counter = A.b.counter;
            pa.slot_base = A.row_base * N;
            pa.out = neg;
            pa.out2 = (!shard && A.b.neg_items != neg) ? A.b.neg_items : nullptr;
        }
        pa.done = ws.prologue_done;
        // the first feature layer's weight in its GEMM's layout, in this launch (both towers; every
        // later phase of the step reads it: tower_forward skips its own pad / bf16 launches)
        for (int k = 0; k < 2; ++k) {
            const ttamm_tower& t = *T[k];
            TowerWs& w = *W[k];
            if (t.fusion == TTAMM_FUSION_IDENTITY || t.n_linear == 0 || !w.weight_prepped) continue;
            const ttamm_linear& L = t.linear[0];
            if (w.w16)
                pa.prep[pa.n_prep++] = WeightPrep{L.weight, L.out_features, L.in_features, L.in_features, w.w16,
                                                  round8(L.in_features), 1};
            else if (w.wpad)
                pa.prep[pa.n_prep++] = WeightPrep{L.weight, L.out_features, L.in_features, L.in_features, w.wpad,
                                                  round4(L.in_features), 0};
        }
        pa.applied = A.steps_applied;
        pa.hist = df.on ? df.hist : nullptr;
        pa.cap = df.on ? df.cap : 2;
        pa.step = df.step;
        pa.c = ad;
        // one process with the aux stream: the step's count and AdamW constants are published by
        // step_begin_kernel on the aux stream (after the fork, below) instead of by the prologue's
        // last block — its completion counter (a release fence and an atomic per block) sat on the
        // main stream's path to the first GEMM.  Nothing in this step reads this step's history
        // entry (the catch-up and the rolling slice replay to step - 1); the next step's catch-up
        // and the flush are ordered after it on the aux stream or after the step's join.
        if (begin_aux) {
            pa.applied = nullptr;
            pa.hist = nullptr;
            pa.done = nullptr;
        }
        if ((rc = launch_step_prologue(st, pa, s))) return rc;
    }
    if (shard && (ph & TTAMM_PHASE_ITEM_FWD) && I.R > 0) {
        // owner: stage the requested local rows (range-checked) and their keys, contiguous
        StageArgs st;
        std::memset(&st, 0, sizeof(st));
        st.status = A.status;
        st.seg[st.count++] = StageSeg{A.item_rows, I.idx_own, I.R, A.item.id.rows, A.item_rows_ld};
        st.seg[st.count++] = StageSeg{A.item_row_keys, ws.keys_own, I.R, INT64_MAX, A.item_rows_ld};
        if (compact_exchange(A)) {  // ... and their exchange units (requester groups as they arrived)
            st.unit_counts = A.exchange_counts + (int64_t)A.exchange_world * A.exchange_counts_ld;
            st.unit_ld = A.exchange_counts_ld;
            st.unit_groups = A.exchange_world;
            st.unit_n = I.R;
            st.unit_out = ws.own_units;
        }
        if ((rc = launch_stage_rows(st, s))) return rc;
    }
    // ---- forward ----------------------------------------------------------------------------
    hipStream_t aux = static_cast<hipStream_t>(A.aux_stream);
    if (!shard) {
        df.slice_on_aux = df.on && overlapped(T, 2, df, s, aux) && !dev_env("TTAMM_SLICE_MAIN");
        df.slice_late = df.slice_on_aux && dev_env("TTAMM_SLICE_LATE") != nullptr;
        if ((rc = prepare_forward(T, W, 2, A.b, D, mimic, df, s, aux, A.timing_events + 2, A.timing_events,
                                  A.timing_events + 8, A.timing_events + 12)))
            return rc;
        if (begin_aux && (rc = launch_step_begin(A.status, A.steps_applied, df.on ? df.hist : nullptr,
                                                 df.on ? df.cap : 2, df.step, ad, aux)))
            return rc;
    } else {
        const ttamm_tower* Ti[2] = {&A.item, nullptr};
        TowerWs* Wi[2] = {&I, nullptr};
        const int both = TTAMM_PHASE_ITEM_FWD | TTAMM_PHASE_USER_FWD;
        if ((ph & both) == both && I.R > 0) {  // grouped: both towers' launches at once
            if ((rc = prepare_forward(T, W, 2, A.b, D, mimic, df, s, aux, A.timing_events + 2, nullptr,
                                      A.timing_events + 8)))
                return rc;
        } else if (ph & TTAMM_PHASE_ITEM_FWD) {
            if (I.R > 0) {
                if ((rc = prepare_forward(Ti, Wi, 1, A.b, D, mimic, df, s, aux, A.timing_events + 2, nullptr,
                                          A.timing_events + 8)))
                    return rc;
            } else if ((rc = tower_prepare(A.item, I, mimic, df, s))) {
                return rc;
            }
        }
        if ((ph & TTAMM_PHASE_USER_FWD) && !((ph & both) == both && I.R > 0))
            if ((rc = prepare_forward(T, W, 1, A.b, D, mimic, df, s, aux, nullptr, nullptr, A.timing_events + 8)))
                return rc;
    }
    // ---- in-batch negatives: S = U P^T, its BCE, dU and dP ------------------------------------
    const int64_t ib_cols = ws.ib_on ? (shard ? Bg : B) : 0;  // positives every user is scored against
    if (ws.ib_on && shard && (ph & TTAMM_PHASE_INBATCH_SRC)) {
        TTAMM_REQUIRE(A.item_fwd_in && A.inbatch_local, "INBATCH_SRC needs item_fwd_in and inbatch_local");
        const bool cx = compact_exchange(A);  // positives keep (t | a) in either layout
        if ((rc = launch_add_rows(A.item_fwd_in, cx ? D : 2 * D, mimic ? A.item_fwd_in + D : nullptr, cx ? D : 2 * D,
                                  B, D, A.inbatch_local, D, s, A.item_slot)))
            return rc;
    }
    if (ws.ib_on && (ph & (shard ? TTAMM_PHASE_INBATCH : TTAMM_PHASE_USER))) {
        InBatchArgs& a = ws.ib;
        a.U = U.aug;
        a.ldu = D;
        a.B = B;
        if (shard) {
            TTAMM_REQUIRE(A.inbatch_items && A.inbatch_dp_all, "INBATCH needs inbatch_items and inbatch_dp_all");
            a.P = A.inbatch_items;
            a.dP = A.inbatch_dp_all;
        } else {
            a.P = I.aug;  // rows [0, B): the positives
            a.dP = ws.ib_dp;
        }
        a.ldp = D;
        a.ld_dp = D;
        a.Bc = ib_cols;
        a.D = D;
        a.row_base = shard ? A.row_base : 0;
        a.inv_T = 1.0f / (float)(Bg * (ib_cols + N));
        a.dU = ws.ib_du;
        a.ld_du = D;
        void* const* ev = A.timing_events + 4;
        if (ev[0] && ev[1]) TTAMM_HIP(hipEventRecord((hipEvent_t)ev[0], s));
        if ((rc = launch_inbatch(a, s))) return rc;
        if (ev[0] && ev[1]) TTAMM_HIP(hipEventRecord((hipEvent_t)ev[1], s));
    }
    // ---- sharded category alignment: global per-category sums, then centered scatters ---------
    if (shard && ws.cal_on && (ph & TTAMM_PHASE_CAL_STATS))
        if ((rc = launch_cal_local(bind_cal(A, ws, I, B, D, mimic), s))) return rc;
    if (shard && ws.cal_on && (ph & TTAMM_PHASE_CAL_SCATTER))
        if ((rc = launch_cal_scatter(bind_cal(A, ws, I, B, D, mimic), s))) return rc;
    // ---- score + loss (fwd + bwd seeds), user-side backward ---------------------------------
    if (ph & (TTAMM_PHASE_USER | TTAMM_PHASE_SCORE)) {
        ScoreArgs sa;
        std::memset(&sa, 0, sizeof(sa));
        sa.B = B;
        sa.Bg = Bg;
        sa.N = N;
        sa.D = D;
        sa.user_aug = U.aug;
        sa.t_user = U.t;
        sa.a_user = U.a;
        sa.lambda_u = (float)A.hp.lambda_mimic_user;
        sa.lambda_i = (float)A.hp.lambda_mimic_item;
        sa.mimic = mimic ? 1 : 0;
        sa.dT_user = U.dT_own;
        sa.dA_user = U.dA_own;
        if (shard) {
            sa.item_aug = nullptr;
            sa.t_item = A.item_fwd_in;
            sa.a_item = mimic ? A.item_fwd_in + D : nullptr;
            sa.ld_item = 2 * D;
            sa.dT_item = A.item_bwd_out;
            sa.dA_item = mimic ? A.item_bwd_out + D : nullptr;
            sa.dA_all = 1;
            sa.ld_dti = 2 * D;
            sa.item_slot = A.item_slot;
            if (compact_exchange(A)) {  // D-float units; negatives: t + a in, dT out (their dA is dT)
                sa.ld_item = sa.ld_dti = D;
                sa.dA_all = 0;
                sa.neg_aug = 1;
            }
        } else {
            sa.item_aug = I.aug;
            sa.t_item = I.t;
            sa.a_item = I.a;
            sa.ld_item = D;
            sa.dT_item = I.dT_own;
            sa.dA_item = I.dA_own;
            sa.ld_dti = D;
        }
        sa.partials = ws.partials;
        sa.blocks = ws.score_blocks;
        const int64_t bce_count = Bg * ((ws.ib_on ? ib_cols : 1) + N);
        sa.inv_numel = 1.0f / (float)bce_count;
        if (ws.ib_on) {
            TTAMM_REQUIRE(!shard || A.inbatch_dp, "sharded in-batch USER phase needs inbatch_dp");
            sa.ib_du = ws.ib_du;
            sa.ib_dp = shard ? A.inbatch_dp : ws.ib_dp;
            sa.ib_ld = D;
        }
        if ((rc = launch_score_loss(sa, s))) return rc;
        if (ws.cal_on) {  // + lambda * L_cal over cat[positives; negatives] (training.py:805-820)
            CalArgs& c = bind_cal(A, ws, I, B, D, mimic);
            if (shard) {
                c.dT = A.item_bwd_out;
                c.dA = mimic ? A.item_bwd_out + D : nullptr;
                c.ld_d = 2 * D;
                c.dA_rows = c.R;  // every request ships its own dA
                if (compact_exchange(A)) {  // only the positives ship a dA
                    c.ld_d = D;
                    c.dA_rows = B;
                }
                if ((rc = launch_cal_finish(c, s))) return rc;
            } else {
                c.dT = I.dT_own;
                c.dA = mimic ? I.dA_own : nullptr;
                c.ld_d = D;
                c.dA_rows = B;
                if ((rc = launch_category_alignment(c, s))) return rc;
            }
        }
        auto finalize = [&](hipStream_t st) {
            return A.loss_out ? launch_loss_finalize(ws.partials, ws.score_blocks, ws.ib_on ? ws.ib.loss_part : nullptr,
                                                     ws.ib_on ? ws.ib_parts : 0, bce_count, B, Bg, D, sa.lambda_u,
                                                     sa.lambda_i, sa.mimic,
                                                     ws.cal_on && A.row_base == 0 ? ws.cal.out : nullptr,
                                                     (float)A.hp.lambda_category_alignment, A.loss_out, A.loss_accum,
                                                     A.status, st)
                              : TTAMM_OK;
        };
        // one process with the touched-row updates on the aux stream: the loss reduction (nothing in
        // the backward reads it) goes there too, ahead of them, instead of between the scores and the
        // fusion backward on the main stream.  TTAMM_ROWS_MAIN=1 / TTAMM_FINALIZE_MAIN=1: main stream.
        static const bool rows_main = dev_env("TTAMM_ROWS_MAIN") != nullptr;
        static const bool fin_main = dev_env("TTAMM_FINALIZE_MAIN") != nullptr;
        const bool rows_aux = !shard && !ws.clip_on && !rows_main && aux != nullptr && aux != s &&
                              overlapped(T, 2, df, s, aux);
        const bool fin_aux = rows_aux && !fin_main;
        if (!fin_aux && (rc = finalize(s))) return rc;
        if (!shard) {
            // ---- the whole backward + optimizers in one process --------------------------------
            // With the aux stream (no clipping: the table updates would wait for the global norm)
            // the touched-row updates run there once the fusion backward has formed the ID and
            // mimic rows' gradients, beside the MLP's dgrad chain and weight gradients (memory-
            // bound row traffic under MFMA-bound GEMMs); the step's end joins them, so the next
            // step's ID-row gather reads the updated rows.  TTAMM_ROWS_MAIN=1: on the main stream.
            if (!rows_aux) {
                if ((rc = tower_backward(T, W, D, s, 2, A.timing_events + 6))) return rc;
                if (ws.clip_on && (rc = clip_coefficient(T, W, D, mimic, sp, ad, df, A, ws, s, aux))) return rc;
                if ((rc = table_updates(T, W, 2, D, mimic, sp, ad, df, A.timing_events, s, aux, ws.clip_coef)))
                    return rc;
                return dense_update(T, W, ad, A.status, s, ws.clip_coef);
            }
            hipEvent_t ev[kAuxEvents];
            if ((rc = aux_events(ev, aux))) return rc;
            if ((rc = tower_backward(T, W, D, s, 2, nullptr, BWD_GATE))) return rc;
            TTAMM_HIP(hipEventRecord(ev[4], s));
            TTAMM_HIP(hipStreamWaitEvent(aux, ev[4], 0));
            if (fin_aux && (rc = finalize(aux))) return rc;
            // on the aux stream: the grouping before it there already, so no join
            if ((rc = table_updates(T, W, 2, D, mimic, sp, ad, df, A.timing_events, aux, aux))) return rc;
            TTAMM_HIP(hipEventRecord(ev[5], aux));
            if ((rc = tower_backward(T, W, D, s, 2, A.timing_events + 6, BWD_MLP))) return rc;
            if ((rc = dense_update(T, W, ad, A.status, s))) return rc;
            TTAMM_HIP(hipStreamWaitEvent(s, ev[5], 0));
            return TTAMM_OK;
        }
        if (ph & TTAMM_PHASE_USER) {
            if ((rc = tower_backward(T, W, D, s, 1))) return rc;
            if ((rc = table_updates(T, W, 1, D, mimic, sp, ad, df, nullptr, s, aux))) return rc;
        }
    }
    // ---- grouped: both towers' backward and table updates ------------------------------------
    if (ph & TTAMM_PHASE_TOWERS_BWD) {
        static const bool rows_main = dev_env("TTAMM_ROWS_MAIN") != nullptr;
        if (I.R > 0 && !ws.clip_on && !rows_main && aux != nullptr && aux != s && overlapped(T, 2, df, s, aux)) {
            // as in one process: the touched-row updates on the aux stream beside the MLP backward,
            // joined before this phase ends (the caller's all-reduce and DENSE follow)
            hipEvent_t ev[kAuxEvents];
            if ((rc = aux_events(ev, aux))) return rc;
            if ((rc = tower_backward(T, W, D, s, 2, nullptr, BWD_GATE))) return rc;
            TTAMM_HIP(hipEventRecord(ev[4], s));
            TTAMM_HIP(hipStreamWaitEvent(aux, ev[4], 0));
            if ((rc = table_updates(T, W, 2, D, mimic, sp, ad, df, A.timing_events, aux, aux))) return rc;
            TTAMM_HIP(hipEventRecord(ev[5], aux));
            if ((rc = tower_backward(T, W, D, s, 2, A.timing_events + 6, BWD_MLP))) return rc;
            TTAMM_HIP(hipStreamWaitEvent(s, ev[5], 0));
        } else {
            if (I.R > 0) {
                if ((rc = tower_backward(T, W, D, s, 2, A.timing_events + 6))) return rc;
            } else {
                if ((rc = tower_backward(T, W, D, s, 1))) return rc;
                const size_t n = tower_grad_floats(A.item);
                if (n) TTAMM_HIP(hipMemsetAsync(I.gw[0] ? I.gw[0] : I.ggw[0], 0, n * sizeof(float), s));
            }
            if (ws.clip_on) {  // the table updates wait for the global norm (TABLES, after the all-reduce)
                if ((rc = clip_table_share(T, W, D, mimic, sp, ad, df, A, ws, s, aux))) return rc;
            } else if ((rc = table_updates(T, W, 2, D, mimic, sp, ad, df, A.timing_events, s, aux))) {
                return rc;
            }
        }
    }
    // ---- sharded clipping: the deferred table updates, scaled by clip_grad_norm_'s coefficient --
    if ((ph & TTAMM_PHASE_TABLES) && ws.clip_on) {
        if ((rc = clip_coefficient_sharded(T, W, ad, A, ws, s))) return rc;
        if ((rc = table_updates(T, W, 2, D, mimic, sp, ad, df, A.timing_events, s, aux, ws.clip_coef))) return rc;
    }
    // ---- item-side backward on the owner ------------------------------------------------------
    if (ph & TTAMM_PHASE_ITEM_BWD) {
        const ttamm_tower* Ti[2] = {&A.item, nullptr};
        TowerWs* Wi[2] = {&I, nullptr};
        if (I.R > 0) {
            if ((rc = tower_backward(Ti, Wi, D, s, 1, A.timing_events + 6))) return rc;
        } else {
            // no requests: this rank's item-tower gradient share is zero
            const size_t n = tower_grad_floats(A.item);
            if (n) TTAMM_HIP(hipMemsetAsync(I.gw[0] ? I.gw[0] : I.ggw[0], 0, n * sizeof(float), s));
        }
        if ((rc = table_updates(Ti, Wi, 1, D, mimic, sp, ad, df, A.timing_events, s, aux))) return rc;
    }
    if (ph & TTAMM_PHASE_DENSE)
        if ((rc = dense_update(T, W, ad, A.status, s, ws.clip_on ? ws.clip_coef : nullptr))) return rc;
    return TTAMM_OK;
}

}  // namespace

size_t train_step_workspace_size(const ttamm_step_args& A) {
    Arena ar{nullptr, 0, 0, true};
    StepWs ws;
    plan(ar, A, ws);
    return ar.off + 256;
}

int exchange_compact_supported(const ttamm_step_args& A) {
    if (!A.mimic_enabled || A.item.fusion != TTAMM_FUSION_GATED) return 0;
    const int D = out_dim(A.user);
    // gate_group's choice as the step makes it: a gated tower has gate16 weight images exactly when
    // plan() gives it some (a stand-in pointer here; gate_group only tests it)
    static uint16_t stand_in;
    TowerWs u, it;
    const ttamm_tower* T2[2] = {&A.user, &A.item};
    TowerWs* W2[2] = {&u, &it};
    for (int k = 0; k < 2; ++k) {
        W2[k]->R = 1;
        const ttamm_tower& t = *T2[k];
        if (t.fusion == TTAMM_FUSION_GATED && gate16_supported(D, t.gate[0].out_features, t.matmul_bf16 ? 1 : 3))
            W2[k]->gw16 = &stand_in;
    }
    GateArgs ga;
    const ttamm_tower* Ti[2] = {&A.item, nullptr};
    TowerWs* Wi[2] = {&it, nullptr};
    if (!gate_group(Ti, Wi, 1, D, true, ga)) return 0;
    return gate_group(T2, W2, 2, D, true, ga) ? 1 : 0;
}

int64_t dense_grad_floats(const ttamm_step_args& A) {
    return (int64_t)(tower_grad_floats(A.user) + tower_grad_floats(A.item));
}

int train_step(const ttamm_step_args& A, hipStream_t s) { return run_step(A, s); }

int flush_tables(const ttamm_step_args& A, hipStream_t s) {
    Deferred df;
    int rc;
    if ((rc = deferred_of(A, df))) return rc;
    if (!df.on) return TTAMM_OK;
    // With an aux stream the flush runs there, behind the last step's table updates and slice (which
    // it must follow) and beside the main stream's tail of that step (weight gradients, their reduce,
    // the dense update: no table rows), and the main stream waits for it: its next reader of the
    // tables is the next step's gather (round 6: the flush overlaps ~0.15 ms of that tail)
    hipStream_t aux = static_cast<hipStream_t>(A.aux_stream);
    const hipStream_t run = (aux != nullptr && aux != s) ? aux : s;
    ReplayArgs ra;
    std::memset(&ra, 0, sizeof(ra));
    ra.hist = df.hist;
    ra.cap = df.cap;
    ra.decoupled = df.decoupled;
    ra.sgd = df.sgd;
    ra.fast_g0 = df.fast;
    ra.target = df.step;
    ra.stamp = 1;
    for (const ttamm_tower* t : {&A.user, &A.item}) {
        const ttamm_table* tabs[2];
        const int n = dense_tables(*t, A.mimic_enabled != 0, tabs);
        for (int i = 0; i < n; ++i) {
            ReplaySeg g = replay_seg(*tabs[i]);
            g.row_lo = 0;
            g.row_hi = tabs[i]->rows;
            ra.seg[ra.count++] = g;
        }
    }
    if ((rc = launch_replay(ra, run))) return rc;
    if (run != s) {
        hipEvent_t e;
        TTAMM_HIP(create_sync_event(&e));
        TTAMM_HIP(hipEventRecord(e, run));
        TTAMM_HIP(hipStreamWaitEvent(s, e, 0));
        TTAMM_HIP(hipEventDestroy(e));
    }
    return TTAMM_OK;
}

// ---- eval-mode tower forward (TowerEncoder.forward + augment) -----------------------------
size_t tower_forward_workspace_size(const ttamm_tower& T, int64_t n) {
    Arena ar{nullptr, 0, 0, true};
    const int D = out_dim(T);
    for (int l = 0; l + 1 < T.n_linear; ++l) ar.take<float>((size_t)n * T.linear[l].out_features);
    ar.take<float>((size_t)n * efw(T));  // ef / e
    ar.take<float>((size_t)n * D);       // f
    if (T.fusion == TTAMM_FUSION_GATED) ar.take<float>((size_t)n * T.gate[0].out_features);
    for (int q = 0; q < 3; ++q) ar.take<float>((size_t)n * D);  // g, t, a
    ar.take<int64_t>(n);                                         // range-checked ids
    if (needs_wpad(T)) ar.take<float>((size_t)T.linear[0].out_features * round4(T.linear[0].in_features));
    if (T.id.max_norm > 0.0) ar.take<int32_t>(T.id.rows);  // renorm claim marks
    return ar.off + 256;
}

int tower_forward_eval(const ttamm_tower& T, const int64_t* idx, const int64_t* fidx, int64_t n, int augment,
                       float* out, void* wsp, size_t ws_bytes, hipStream_t s) {
    const int D = out_dim(T);
    int rc;
    if ((rc = validate_tower(T, "tower", D, false))) return rc;
    if (augment && T.mimic.weight)
        TTAMM_REQUIRE(T.mimic.rows == T.id.rows && T.mimic.dim == D, "tower: mimic table shape does not match the tower");
    if (n <= 0) return TTAMM_OK;
    Arena ar{static_cast<char*>(wsp), ws_bytes, 0, false};
    TowerWs w;
    w.R = n;
    w.idx = idx;
    w.fidx = fidx;
    for (int l = 0; l + 1 < T.n_linear; ++l) w.hid[l] = ar.take<float>((size_t)n * T.linear[l].out_features);
    float* efbuf = ar.take<float>((size_t)n * efw(T));
    float* fbuf = ar.take<float>((size_t)n * D);
    float* zbuf = T.fusion == TTAMM_FUSION_GATED ? ar.take<float>((size_t)n * T.gate[0].out_features) : nullptr;
    float* gbuf = ar.take<float>((size_t)n * D);
    float* tbuf = ar.take<float>((size_t)n * D);
    float* abuf = ar.take<float>((size_t)n * D);
    int64_t* idxc = ar.take<int64_t>(n);
    if (needs_wpad(T)) w.wpad = ar.take<float>((size_t)T.linear[0].out_features * round4(T.linear[0].in_features));
    if (T.id.max_norm > 0.0) {  // nn.Embedding max_norm renorms in eval mode too (one lookup)
        w.renorm_mark = ar.take<int32_t>(T.id.rows);
        w.renorm_tag = 1;
    }
    TTAMM_REQUIRE(ar.ok(), "workspace too small for tower forward");
    if (w.renorm_mark) TTAMM_HIP(hipMemsetAsync(w.renorm_mark, 0, (size_t)T.id.rows * sizeof(int32_t), s));
    {  // ids outside the tables read row 0 (the Python mirror raises IndexError before calling)
        StageArgs st;
        std::memset(&st, 0, sizeof(st));
        st.seg[st.count++] = StageSeg{idx, idxc, n, T.id.rows};
        if ((rc = launch_stage_rows(st, s))) return rc;
        if (fidx == idx) fidx = idxc;
        idx = idxc;
        w.idx = idx;
        w.fidx = fidx;
    }
    if (uses_ef(T)) {
        w.ef = efbuf;
        w.z = zbuf;
        w.g = gbuf;
    } else {
        w.e = efbuf;
        w.f = fbuf;
    }
    w.t = tbuf;
    w.t_ld = D;
    w.a = abuf;
    w.aug = out;
    // eval mode: no dropout
    ttamm_tower te = T;
    te.dropout = 0.f;
    ttamm_batch bt;
    std::memset(&bt, 0, sizeof(bt));
    const ttamm_tower* TT[2] = {&te, nullptr};
    TowerWs* WW[2] = {&w, nullptr};
    const bool mimic = augment && T.mimic.weight;
    if ((rc = tower_forward(TT, WW, bt, D, mimic, s, 1))) return rc;
    return TTAMM_OK;
}


// ---- training-mode tower forward / backward (module-level autograd) ------------------------
// TowerEncoder.forward under autograd (encoders.py:221-255) in two calls: the forward keeps its
// activations in the workspace, the backward (same tower, rows and workspace) runs the tower's
// backward kernels — gate, dgrad chain, one grouped weight-gradient launch — into the caller's
// gradient arena (tower_grad_floats: per Linear weight then bias, 256-B aligned pieces) and
// writes the ID rows' gradient per position (and, identity feature encoder, the feature rows').
namespace {
void plan_tower_train(Arena& ar, const ttamm_tower& T, int64_t n, TowerWs& w) {
    const int D = out_dim(T);
    w.role = ROLE_USER;
    w.R = n;
    w.idx_own = ar.take<int64_t>(n);
    for (int l = 0; l + 1 < T.n_linear; ++l) {
        w.hid[l] = ar.take<float>((size_t)n * T.linear[l].out_features);
        w.dhid[l] = ar.take<float>((size_t)n * T.linear[l].out_features);
        if (T.activation != TTAMM_ACT_RELU) {
            w.pre[l] = ar.take<float>((size_t)n * T.linear[l].out_features);
            if (T.dropout > 0.f) w.mask[l] = ar.take<uint8_t>((size_t)n * T.linear[l].out_features);
        }
    }
    if (uses_ef(T)) {
        w.ef = ar.take<float>((size_t)n * efw(T));
        w.dEF = ar.take<float>((size_t)n * efw(T));
    } else {
        w.e = ar.take<float>((size_t)n * D);
        w.f = ar.take<float>((size_t)n * D);
    }
    if (T.fusion == TTAMM_FUSION_GATED) {
        const int Hg = T.gate[0].out_features;
        w.z = ar.take<float>((size_t)n * Hg);
        w.dz = ar.take<float>((size_t)n * Hg);
        w.g = ar.take<float>((size_t)n * D);
        w.dq = ar.take<float>((size_t)n * D);
        const int np = T.matmul_bf16 ? 1 : 3;
        if (gate16_supported(D, Hg, np)) w.gw16 = ar.take<uint16_t>((size_t)gate16_image_elems(D, Hg, np));
    }
    WgradShape shapes[TTAMM_MAX_LINEAR + 2];
    const int ns = wgrad_shapes(T, n, shapes);
    int rps[kWgradClasses] = {512, 512, 512, 512};
    if (ns) wgrad_rows_per_split(shapes, ns, rps);
    for (int c = 0; c < kWgradClasses; ++c) w.wgrad_rps[c] = rps[c];
    if (T.fusion != TTAMM_FUSION_IDENTITY) {
        for (int l = 0; l < T.n_linear; ++l) {
            const ttamm_linear& L = T.linear[l];
            w.slab[l] = ar.take<float>(wgrad_slab_floats((int)n, L.out_features, L.in_features,
                                                         w.wgrad_rps[wgrad_class(L.out_features)]));
        }
        for (int q = 0; q < fusion_linears(T); ++q) {
            const ttamm_linear& L = T.gate[q];
            w.slab[TTAMM_MAX_LINEAR + q] = ar.take<float>(
                wgrad_slab_floats((int)n, L.out_features, L.in_features, w.wgrad_rps[wgrad_class(L.out_features)]));
        }
    }
    if (needs_wpad(T)) w.wpad = ar.take<float>((size_t)T.linear[0].out_features * round4(T.linear[0].in_features));
    if (T.id.max_norm > 0.0) w.renorm_mark = ar.take<int32_t>(T.id.rows);
}

int bind_tower_train(const ttamm_tower& T, const int64_t* idx, const int64_t* fidx, int64_t n, void* wsp,
                     size_t ws_bytes, TowerWs& w) {
    Arena ar{static_cast<char*>(wsp), ws_bytes, 0, false};
    plan_tower_train(ar, T, n, w);
    TTAMM_REQUIRE(ar.ok(), "workspace too small for the training tower forward / backward");
    w.idx = w.idx_own;
    w.fidx = fidx == idx ? w.idx_own : fidx;  // caller-gathered feature rows: fidx = null (row r)
    w.key_split = n;
    return TTAMM_OK;
}
}  // namespace

size_t tower_grad_floats_of(const ttamm_tower& T) { return tower_grad_floats(T); }

size_t tower_train_workspace_size(const ttamm_tower& T, int64_t n) {
    Arena ar{nullptr, 0, 0, true};
    TowerWs w;
    plan_tower_train(ar, T, n, w);
    return ar.off + 256;
}

int tower_train_forward(const ttamm_tower& T, const int64_t* idx, const int64_t* fidx, int64_t n,
                        const uint8_t* const* keep_masks, uint64_t seed, uint64_t counter, float* out, void* wsp,
                        size_t ws_bytes, hipStream_t s) {
    const int D = out_dim(T);
    int rc;
    if ((rc = validate_tower(T, "tower", D, false))) return rc;
    if (n <= 0) return TTAMM_OK;
    TowerWs w;
    if ((rc = bind_tower_train(T, idx, fidx, n, wsp, ws_bytes, w))) return rc;
    {  // ids outside the table read row 0 (the Python mirror raises IndexError before calling)
        StageArgs st;
        std::memset(&st, 0, sizeof(st));
        st.seg[st.count++] = StageSeg{idx, w.idx_own, n, T.id.rows};
        if ((rc = launch_stage_rows(st, s))) return rc;
    }
    if (w.renorm_mark) {
        TTAMM_HIP(hipMemsetAsync(w.renorm_mark, 0, (size_t)T.id.rows * sizeof(int32_t), s));
        w.renorm_tag = 1;
    }
    w.t = out;
    w.t_ld = D;
    ttamm_batch bt;
    std::memset(&bt, 0, sizeof(bt));
    bt.seed = seed;
    bt.counter = counter;
    for (int l = 0; keep_masks && l + 1 < T.n_linear; ++l) bt.user_keep_mask[l] = keep_masks[l];
    const ttamm_tower* TT[2] = {&T, nullptr};
    TowerWs* WW[2] = {&w, nullptr};
    return tower_forward(TT, WW, bt, D, false, s, 1);
}

int tower_train_backward(const ttamm_tower& T, const int64_t* idx, const int64_t* fidx, int64_t n,
                         const uint8_t* const* keep_masks, const float* d_out, float* grad_arena, float* d_id_rows,
                         float* d_feat_rows, void* wsp, size_t ws_bytes, hipStream_t s) {
    const int D = out_dim(T);
    const int Did = T.id.dim;
    int rc;
    if ((rc = validate_tower(T, "tower", D, false))) return rc;
    const size_t ng = tower_grad_floats(T);
    if (n <= 0) {
        if (ng) TTAMM_HIP(hipMemsetAsync(grad_arena, 0, ng * sizeof(float), s));
        return TTAMM_OK;
    }
    TTAMM_REQUIRE(d_out && (ng == 0 || grad_arena), "tower backward: d_out / grad_arena missing");
    TowerWs w;
    if ((rc = bind_tower_train(T, idx, fidx, n, wsp, ws_bytes, w))) return rc;
    w.dT = d_out;
    w.dT_ld = D;
    float* cur = grad_arena;
    carve_grads(T, w, cur);
    // non-ReLU layers read the forward's keep bytes: the injected masks again, or the ones the
    // forward drew into the workspace
    for (int l = 0; l + 1 < T.n_linear; ++l) w.keep[l] = keep_masks && keep_masks[l] ? keep_masks[l] : w.mask[l];
    const ttamm_tower* TT[2] = {&T, nullptr};
    TowerWs* WW[2] = {&w, nullptr};
    if (T.fusion != TTAMM_FUSION_IDENTITY)
        if ((rc = tower_backward(TT, WW, D, s, 1))) return rc;
    // d(ID rows): [e | f] towers take dEF[:, :Did]; sum / identity fusion pass dT to e
    const float* de = uses_ef(T) ? w.dEF : d_out;
    const int64_t ld_de = uses_ef(T) ? efw(T) : D;
    if (d_id_rows && (rc = launch_add_rows(de, ld_de, nullptr, 0, n, Did, d_id_rows, Did, s))) return rc;
    if (d_feat_rows) {  // identity feature encoder: f = the feature row, its gradient is dEF[:, Did:] / dT
        TTAMM_REQUIRE(T.n_linear == 0 && T.fusion != TTAMM_FUSION_IDENTITY,
                      "tower backward: feature-row gradients exist for the identity feature encoder only");
        const float* df = uses_ef(T) ? w.dEF + Did : d_out;
        const int fo = fo_dim(T);
        if ((rc = launch_add_rows(df, ld_de, nullptr, 0, n, fo, d_feat_rows, fo, s))) return rc;
    }
    return TTAMM_OK;
}

}  // namespace ttamm
