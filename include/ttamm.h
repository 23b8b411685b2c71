/*
 * ttamm.h — C ABI of libttamm.so, the MI355X (gfx950) two-tower training step.
 *
 * The reference (alperkartkaya2-afk/two-tower-augmented-with-adaptive-mimic-mechanism)
 * is pure Python/PyTorch, so the "FFI" this boundary replaces is the set of Python calls
 * its training step makes.  Each entry point below names the reference interface it
 * stands in for (file:line relative to the reference root).  The Python host mirror in
 * two-tower-augmented-with-adaptive-mimic-mechanism_amd/ttamm binds these with ctypes
 * (see INTEGRATION.md for the binding a maintainer would add to the reference).
 *
 * Conventions
 *   - Every pointer argument is a DEVICE pointer unless its comment says "host".
 *   - The caller (PyTorch's caching allocator) owns all memory; the library never
 *     allocates or frees caller buffers.  Scratch comes from a caller workspace sized by
 *     the matching *_workspace_size query.
 *   - `stream` is a hipStream_t passed as void* (torch.cuda.current_stream().cuda_stream).
 *     All calls are asynchronous on that stream and reentrant.
 *   - Return value: TTAMM_OK (0) or an error code; ttamm_last_error() gives a
 *     thread-local message.  The Python wrapper maps TTAMM_E_INVALID to ValueError and
 *     TTAMM_E_RUNTIME / TTAMM_E_HIP to RuntimeError, mirroring the reference's conventions
 *     (encoders.py:51-52,203-204,236-252; adaptive_mimic.py:32-33,101-102; samplers.py:25-28,38-42,78-81).
 *   - Indices are int64 (torch.long), as the reference requires (adaptive_mimic.py:101-102).
 *   - Floating point is fp32 throughout (the reference computes in fp32).
 */
#ifndef TTAMM_H
#define TTAMM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TTAMM_ABI_VERSION 25

#define TTAMM_OK 0
#define TTAMM_E_INVALID 1 /* bad shape / config / dtype  -> ValueError   */
#define TTAMM_E_RUNTIME 2 /* runtime condition          -> RuntimeError */
#define TTAMM_E_HIP 3     /* HIP API failure            -> RuntimeError */

#define TTAMM_MAX_LINEAR 6 /* feature-encoder Linear layers per tower (hidden + final) */

/* Feature-MLP activations (encoders.py:68-78 _get_activation; ttamm_tower.activation). */
#define TTAMM_ACT_RELU 0
#define TTAMM_ACT_GELU 1 /* nn.GELU(approximate='none'): x / 2 (1 + erf(x / sqrt 2)) */
#define TTAMM_ACT_TANH 2
#define TTAMM_ACT_SELU 3

/* Fusion strategies of TowerEncoder (encoders.py:194-219). "concat" is not on the hot path. */
#define TTAMM_FUSION_IDENTITY 0
#define TTAMM_FUSION_SUM 1
#define TTAMM_FUSION_GATED 2
/* concat (encoders.py:211-215,242-244): t = projection([e | f]); the projection (Linear 2D -> D,
 * output_dim == embedding_dim) rides in ttamm_tower.gate[0] */
#define TTAMM_FUSION_CONCAT 3

/* Which optimizer owns a row table (training.py:276-309, :1311-1350). */
#define TTAMM_OPT_SPARSE_ADAM 0 /* nn.Embedding(sparse=True) -> torch.optim.SparseAdam      */
#define TTAMM_OPT_DENSE 1       /* every other parameter       -> AdamW / Adam (dense group) */

/* Phases of one training step (ttamm_step_args.phase).  0 = the whole step in one process.
 * A row-sharded multi-GPU step (item rows owned by rank i % W) runs them with
 * exchanges in between; several bits may be set in one call and run in this order:
 *   SAMPLE   requester: draw negatives for its users into b.neg_items
 *            [all-to-all: requested item ids (+ their global request positions) -> owners]
 *   ITEM_FWD owner: item tower over the requested local rows           -> item_fwd_out (t | a)
 *            [all-to-all: (t | a) rows back to the requesters]  (overlaps USER_FWD)
 *   USER_FWD requester: user tower forward
 *   USER     requester: scores + losses, user-tower backward, user-table updates;
 *            (dT | dA) of its item requests                            -> item_bwd_out
 *            [all-to-all: (dT | dA) rows -> owners]
 *   ITEM_BWD owner: item-tower backward, item-table updates
 *            [all-reduce (sum): the replicated-weight gradient arena dense_grads]
 *   DENSE    AdamW/Adam on the replicated feature-encoder and gate weights */
#define TTAMM_PHASE_ALL 0
#define TTAMM_PHASE_SAMPLE 1
#define TTAMM_PHASE_ITEM_FWD 2
#define TTAMM_PHASE_USER_FWD 4
#define TTAMM_PHASE_USER 8
#define TTAMM_PHASE_ITEM_BWD 16
#define TTAMM_PHASE_DENSE 32
/* In-batch negatives in a sharded step (ttamm_step_args.in_batch): after USER_FWD and the (t | a)
 * exchange,
 *   INBATCH_SRC requester: its augmented positives (t + a)                 -> inbatch_local
 *               [all-gather: inbatch_local -> inbatch_items, rank-major]
 *   INBATCH     requester: S = U P^T over the global positives; dU kept in the workspace,
 *               its share of dP for every global positive                -> inbatch_dp_all
 *               [reduce-scatter (sum): inbatch_dp_all -> inbatch_dp, this rank's positives]
 * then USER adds the sampled negatives (if any) and the mimic terms. */
#define TTAMM_PHASE_INBATCH_SRC 64
#define TTAMM_PHASE_INBATCH 128
/* Grouped variant (ShardedTrainStep(group_towers=True)): ITEM_FWD | USER_FWD in one call run the
 * two towers' forward as one set of grouped launches; USER splits into
 *   SCORE      requester: scores + losses; (dT | dA) of its item requests -> item_bwd_out
 *              [all-to-all: (dT | dA) rows -> owners]
 *   TOWERS_BWD both towers' backward (user rows + owned item rows) grouped, both tables' updates
 * so each tower-wide kernel is launched once per step, as in the one-process step. */
#define TTAMM_PHASE_SCORE 256
#define TTAMM_PHASE_TOWERS_BWD 512
/* Gradient clipping in a sharded step (hp.grad_clip_norm > 0; grouped schedule): TOWERS_BWD then
 * leaves the table updates out and writes this rank's squared gradient norm over the table rows it
 * owns to *table_sumsq; after the caller's all-reduce of dense_grads and table_sumsq,
 *   TABLES  clip_grad_norm_'s coefficient from the global norm, then the table updates
 * and DENSE applies the same coefficient. */
#define TTAMM_PHASE_TABLES 1024
/* Category-alignment loss in a sharded step (item_categories set, lambda > 0): L_cal is taken
 * over the GLOBAL batch's item rows (training.py:541-579 on cat[positives; negatives] of all
 * ranks), so after the (t | a) exchange and before SCORE / USER,
 *   CAL_STATS    requester: per-category sums and row counts of its requests -> cal_stats
 *                [all-reduce (sum): cal_stats]
 *   CAL_SCATTER  requester: centered scatter of its rows about the global means -> cal_scatter
 *                [all-reduce (sum): cal_scatter]
 * and SCORE / USER form the covariances, L_cal and G, and add the gradient of this rank's rows
 * into item_bwd_out.  The rank with row_base 0 carries lambda * L_cal in its loss share. */
#define TTAMM_PHASE_CAL_STATS 2048
#define TTAMM_PHASE_CAL_SCATTER 4096

/* Device-side status word bits (written by kernels, read by the host at epoch end).  Once a
 * bit is set, every later step on that status word is skipped on the device (no parameter,
 * optimizer-state or loss-accumulator write), so the state the host finds is the state after
 * the last good step — as the reference, which raises inside the failing batch before its
 * backward, leaves it. */
#define TTAMM_STATUS_SAMPLER_EXHAUSTED 1u    /* samplers.py:78-81 -> RuntimeError            */
#define TTAMM_STATUS_INDEX_OUT_OF_RANGE 2u   /* a batch id < 0 or >= table rows -> IndexError
                                                (nn.Embedding, encoders.py:222-223)         */
#define TTAMM_STATUS_LOOKAHEAD_MISMATCH 4u   /* row-sharded step called with a batch other than the
                                                one its look-ahead prepared -> ValueError   */

/* ---------------------------------------------------------------------------------- */
/* Parameter descriptors                                                               */
/* ---------------------------------------------------------------------------------- */

/* nn.Linear(in, out): weight [out, in] row-major, bias [out]; plus its AdamW state. */
typedef struct ttamm_linear {
    float* weight;
    float* bias;
    float* weight_exp_avg;
    float* weight_exp_avg_sq;
    float* bias_exp_avg;
    float* bias_exp_avg_sq;
    int32_t in_features;
    int32_t out_features;
} ttamm_linear;

/* A row table [rows, dim] (an nn.Embedding weight) and its optimizer state. */
typedef struct ttamm_table {
    float* weight;
    float* exp_avg;
    float* exp_avg_sq;
    int64_t rows;
    int32_t dim;
    int32_t optimizer; /* TTAMM_OPT_* */
    /* Dense-group (AdamW) tables only.  NULL: every step sweeps AdamW(g = 0) over the whole
     * table (training.py:1316-1323 semantics, executed eagerly).  Non-NULL: per-row dense
     * step count the row is current to; the g = 0 updates a row missed are replayed exactly
     * (same fp32 operations, same per-step constants from adam_history) before the row is
     * read, on a rolling 1/replay_slices of the rows each step, and by ttamm_flush_tables. */
    int32_t* last_step;
    /* nn.Embedding(padding_idx=...) (encoders.py:47,55-57): has_padding_idx != 0 makes row
     * padding_idx receive no gradient — SparseAdam leaves it untouched (torch drops the row from
     * the sparse gradient), AdamW updates it with g = 0.  The lookup itself is unchanged. */
    int32_t has_padding_idx;
    int64_t padding_idx;
    /* nn.Embedding(max_norm=...) (encoders.py:48,58; dense tables only, as the reference
     * requires): > 0 renormalises every looked-up row whose L2 norm exceeds it, in place and
     * before the lookup (torch embedding_renorm_: row *= max_norm / (norm + 1e-7)), once per
     * forward call — the user rows, then the positives', then the negatives' (training.py:
     * 748-775 calls the item encoder twice).  0 = off. */
    double max_norm;
    /* Deferred dense-group tables (last_step != NULL) may also carry one byte per row: 0 = the
     * row has never had a gradient, so exp_avg and exp_avg_sq are +0.0 in every column and its
     * AdamW(g = 0) updates are p *= (1 - lr wd) alone (bit for bit: the update term is -0.0); the
     * replay then moves only the parameter row (8 of its 24 bytes per element).  1 = anything
     * else.  The step sets a row's byte when it gives the row a gradient; the caller initialises
     * it (any nonzero exp_avg / exp_avg_sq in the row -> 1).  NULL = every row treated as 1. */
    uint8_t* touched;
} ttamm_table;

/* One tower: TowerEncoder (encoders.py:171-255) + its half of AdaptiveMimicMechanism
 * (adaptive_mimic.py:35-38). */
typedef struct ttamm_tower {
    ttamm_table id;        /* TowerEncoder.embedding                                   */
    ttamm_table mimic;     /* {user,item}_augmented; weight==NULL when mimic disabled  */
    const float* features; /* [id.rows, feat_ld] feature rows (zero-padded), or NULL   */
    int64_t feat_ld;       /* row stride in floats, multiple of 4                       */
    int32_t feat_dim;      /* F (unpadded)                                              */
    int32_t fusion;        /* TTAMM_FUSION_*                                            */
    int32_t n_linear;      /* Linear layers in the feature encoder; 0 with fusion !=
                              IDENTITY = the identity feature encoder (encoders.py:114-119:
                              f = the feature row, feat_dim == id.dim)                    */
    float dropout;         /* Dropout p after each hidden activation (encoders.py:132-138) */
    int32_t activation;    /* TTAMM_ACT_* of the hidden layers (encoders.py:130)          */
    ttamm_linear linear[TTAMM_MAX_LINEAR];
    ttamm_linear gate[2];  /* FeatureFusionGate.gate_network.{0,2} (encoders.py:157-162) */
    int32_t matmul_bf16;   /* 0: fp32 GEMMs (the reference).  1: "bf16 towers" (BASELINE config
                              C5): every feature-MLP / gate GEMM (forward, input and weight
                              gradients) rounds both operands to bf16 (RNE) and accumulates in
                              fp32; activations, losses, tables, weights and optimizer state stay
                              fp32.  Both towers of a step must agree.                      */
    /* matmul_bf16 towers, optional: the feature rows already rounded to bf16 (ttamm_to_bf16),
     * [id.rows, feat_bf16_ld] with feat_bf16_ld % 8 == 0.  The first feature layer's forward
     * GEMM then streams bf16 operands (same values, half the bytes) on bf16 MFMA. */
    const uint16_t* features_bf16;
    int64_t feat_bf16_ld;
    /* fp32 towers, optional: the feature rows pre-split into bf16 planes (ttamm_to_planes),
     * [id.rows, feat_planes_ld] uint16 with row r's k-tile t (features 16 t .. 16 t + 15) at
     * 48 t: hi[16], mid[16], lo[16] (hi + mid + lo == the fp32 value exactly), feat_planes_ld >=
     * 48 ceil(feat_dim / 16).  The first feature layer's forward GEMM and its weight gradient then
     * stage these planes instead of splitting the fp32 rows in every k-tile (same products, same
     * bits). */
    const uint16_t* features_planes;
    int64_t feat_planes_ld;
} ttamm_tower;

/* Optimizer hyper-parameters for one step, as the Python floats torch holds (double).
 * Derived constants (1-beta, bias corrections, step sizes) are computed on the host in
 * double precision and rounded to fp32 once, exactly as torch does
 * (adam.py:527-534, _functional.py:80-82). */
typedef struct ttamm_hparams {
    double lr, beta1, beta2, eps, weight_decay; /* dense group (Python floats)       */
    int32_t decoupled_weight_decay;             /* 1 = AdamW, 0 = Adam (L2 into grad) */
    double sparse_lr, sparse_beta1, sparse_beta2, sparse_eps; /* SparseAdam group    */
    int64_t dense_step;  /* dense step count after this step's increment (>= 1)       */
    int64_t sparse_step; /* SparseAdam per-tensor step after increment (>= 1)         */
    double lambda_mimic_user; /* loss_weights.mimic_user (training.py:722,800-801)    */
    double lambda_mimic_item; /* loss_weights.mimic_item (training.py:723,802-803)    */
    double lambda_category_alignment; /* loss_weights.category_alignment (training.py:724,805-820);
                                         used when ttamm_step_args.item_categories is set */
    double grad_clip_norm; /* gradient_clip_norm (training.py:712,824-825): > 0 scales every
                              gradient of the step by min(clip / (||g||_2 + 1e-6), 1) before the
                              optimizers, ||g|| over all parameters (clip_grad_norm_).  One-process
                              step with dense ID tables only (torch raises on the sparse
                              gradients of sparse ID tables); 0 = off */
    /* the dense group's optimizer (training.py:1311-1333): TTAMM_DENSE_ADAM = torch.optim.Adam /
     * AdamW (decoupled_weight_decay), TTAMM_DENSE_SGD = torch.optim.SGD(lr, weight_decay, momentum)
     * (sgd.py _single_tensor_sgd).  SGD keeps its momentum buffer in each dense tensor's exp_avg
     * (exp_avg_sq may alias it); with momentum == 0 both may alias the parameter itself.  The
     * deferred table replay covers SGD too: an untouched row's g = 0 step (p wd decay through the
     * momentum buffer) is replayed from the history ring with each step's SGD constants, bit for
     * bit the eager sweep's operations (no sweep at all when momentum == weight_decay == 0:
     * untouched rows do not move). */
    int32_t dense_optimizer;
    double momentum, dampening;
    int32_t nesterov;
    int32_t sgd_first_step; /* 1: the momentum buffers do not exist yet (torch: buf = grad.clone()) */
} ttamm_hparams;

#define TTAMM_DENSE_ADAM 0
#define TTAMM_DENSE_SGD 1

/* One batch of the training loop (training.py:726-736). */
typedef struct ttamm_batch {
    const int64_t* users;     /* [batch]                                              */
    const int64_t* pos_items; /* [batch]                                              */
    int64_t* neg_items;       /* [batch*num_neg]: sampler output, or caller input     */
    int64_t batch;
    int32_t num_neg;          /* negatives_per_positive                                */
    int32_t sample_negatives; /* 1 = draw on device (samplers.py:11-85), 0 = given    */
    const int64_t* pos_offsets; /* CSR of each user's positives: [num_users+1]        */
    const int64_t* pos_values;  /* sorted item ids per user                           */
    uint64_t seed;              /* RNG key (negatives + dropout)                      */
    uint64_t counter;           /* per-step RNG counter                               */
    /* Optional injected dropout keep-masks (1 = keep), one per hidden layer, row-major
     * [rows, out_features]: user tower rows = batch, item tower rows = batch*(1+num_neg)
     * ordered [positives; negatives].  NULL = draw from the RNG. */
    const uint8_t* user_keep_mask[TTAMM_MAX_LINEAR];
    const uint8_t* item_keep_mask[TTAMM_MAX_LINEAR];
} ttamm_batch;

/* Everything one fused training step touches. */
typedef struct ttamm_step_args {
    ttamm_tower user;
    ttamm_tower item;
    int32_t mimic_enabled;
    ttamm_hparams hp;
    ttamm_batch b;
    float* loss_out;      /* [5]: total, bce, mimic_user, mimic_item, category_alignment */
    double* loss_accum;   /* [2]: += total*batch, += batch  (training.py:829-831)      */
    uint32_t* status;     /* device status word (TTAMM_STATUS_* bits), OR-ed          */
    void* workspace;
    size_t workspace_bytes;
    void* timing_events[14]; /* optional hipEvent_t pairs (bench roofline), NULL = off:
                               [0],[1] around the dense-group table maintenance (eager
                               AdamW(g=0) sweep, or the deferred slice's replay kernel);
                               [2],[3] around the grouped first feature-layer forward GEMM;
                               [4],[5] around the in-batch scoring kernel (in_batch);
                               [6],[7] around the wide weight-gradient GEMM launch;
                               [8],[9] / [10],[11] around the user / item tower's deferred
                               catch-up replay kernel (on aux_stream when it is set);
                               [12],[13] around the grouped ID-row gather (one process,
                               on aux_stream; round 6)                                    */
    /* ---- row-sharded multi-GPU step (phase != TTAMM_PHASE_ALL) ----------------------
     * The same workspace must be passed to every phase of a step.                        */
    int32_t phase;                /* TTAMM_PHASE_* bits                                      */
    int64_t row_base;             /* global position of this rank's first interaction: keys
                                     the negative-sampling and dropout streams so W ranks
                                     draw exactly what one process would over the global
                                     batch                                                   */
    int64_t global_batch;         /* interactions over all ranks; losses are normalised by it
                                     and loss_out holds this rank's share (0 = batch)        */
    int64_t num_items_global;     /* sampler range (0 = item.id.rows)                        */
    const int64_t* item_rows;     /* owner: local item rows requested this step              */
    const int64_t* item_row_keys; /* owner: global request position of each requested row   */
    int64_t n_item_rows;
    int64_t item_rows_capacity;   /* workspace bound for n_item_rows                         */
    float* item_fwd_out;          /* owner:     [n_item_rows, 2*dim] (t | a)                 */
    const float* item_fwd_in;     /* requester: [batch*(1+num_neg), 2*dim] (t | a), rows
                                     ordered [positives; negatives (b-major)]               */
    float* item_bwd_out;          /* requester: [batch*(1+num_neg), 2*dim] (dT | dA)         */
    const float* item_bwd_in;     /* owner:     [n_item_rows, 2*dim] (dT | dA)               */
    float* table_sumsq;           /* sharded clipping: [1] this rank's table-row squared gradient
                                     norm (TOWERS_BWD), all-reduced by the caller before TABLES */
    float* dense_grads;           /* replicated-weight gradient arena
                                     (ttamm_dense_grad_floats floats)                        */
    /* ---- deferred exact AdamW(g = 0) on tables with last_step (see ttamm_table) ---------- */
    void* adam_history;           /* device ring: history_capacity entries of
                                     ttamm_adam_history_entry_bytes() each                  */
    int32_t history_capacity;     /* > replay_slices                                         */
    int32_t replay_slices;        /* every row is replayed at least once per replay_slices
                                     steps (bounds the lag a read has to catch up)           */
    /* ---- optional second HIP stream (NULL = everything on `stream`) ---------------------
     * The row coalesce (sort of the batch's rows) and the deferred catch-up of the rows a
     * tower reads depend only on the indices; with an aux stream they run there, overlapping
     * the feature-MLP GEMMs, and `stream` waits for them before the first table read. */
    void* aux_stream;
    /* ---- category-alignment loss (training.py:530-579, :805-820; sharded: TTAMM_PHASE_CAL_*) ----
     * item_categories: [item.id.rows] int64 category id per item, each in [0, num_categories)
     * (sharded: [num_items_global], every rank holds the global tensor)
     * (_build_item_category_tensor, training.py:582-610); NULL (or lambda 0) = no L_cal.       */
    const int64_t* item_categories;
    int64_t num_categories;
    int64_t major_category;       /* major_category_id                                       */
    /* ---- error recovery ---------------------------------------------------------------------
     * steps_applied: optional device counter, += 1 by every step that ran (status clean when it
     * began).  After a status error the host flushes the deferred tables to, and writes back
     * optimizer step counts of, the steps that ran.                                           */
    int64_t* steps_applied;
    /* ---- in-batch negatives (BASELINE configs C2 / C4).  Not reference behaviour (the reference
     * scores b.num_neg sampled negatives per positive, training.py:770-798); ttamm's definition
     * (oracle/cpu_reference.py train_step(in_batch=True)): user b is scored against every positive
     * of the global batch, S = U P^T with label 1 where the positive is b's own, followed by its
     * b.num_neg (>= 0) sampled negatives; one BCE mean over global_batch x (global_batch + num_neg)
     * logits.  S is never stored: a fused fp32-MFMA kernel forms it, its BCE and dU / dP. ---- */
    int32_t in_batch;
    float* inbatch_local;         /* sharded: [batch, dim] this rank's augmented positives        */
    const float* inbatch_items;   /* sharded: [global_batch, dim] all ranks' (all-gathered)       */
    float* inbatch_dp_all;        /* sharded: [global_batch, dim] this rank's share of dP         */
    const float* inbatch_dp;      /* sharded: [batch, dim] summed dP of this rank's positives     */
    /* ---- arithmetic of the g = 0 AdamW updates of untouched dense-group table rows (deferred
     * replay, eager sweep, ttamm_flush_tables; rows with a gradient always use IEEE ops) --------
     * TTAMM_G0_EXACT: IEEE sqrt and division — bit-identical to torch's AdamW step;
     * TTAMM_G0_FAST:  v_sqrt_f32 / v_rcp_f32 (<= 1 ulp each) and a multiply by RN(1/sqrt(bc2)):
     *                 each g = 0 update term within a few ulp of torch's, a third of the VALU work.
     * Deferred and eager stay bit-identical to each other in either mode. */
    int32_t table_g0_math;
    /* ---- sharded requester: where each request's row sits in the exchange buffers ------------
     * NULL: item_fwd_in / item_bwd_out row r is request r ([positives; negatives]).  Otherwise
     * request r's (t | a) is read from, and its (dT | dA) written to, row item_slot[r] — the
     * owner-grouped order ttamm_route_rows produced, so the all-to-alls move the buffers as
     * they are (no permutation pass). */
    const int64_t* item_slot;
    /* ---- sharded category alignment (TTAMM_PHASE_CAL_*): the caller's all-reduce buffers ------
     * cal_stats [num_categories * (dim + 1)] floats, cal_scatter [num_categories * dim * dim]
     * floats; the step zeroes and fills them between the caller's all-reduces.              */
    float* cal_stats;
    float* cal_scatter;
    /* element stride of item_rows and item_row_keys (0 = 1): the (local row, key) pairs of an
     * owner's request all-to-all are read in place (stride 2), the step stages contiguous copies */
    int64_t item_rows_ld;
    /* ---- compact exchange rows (sharded, mimic on; ttamm_exchange_compact_supported) -----------
     * NULL: every exchange row is 2*dim wide ((t | a) forward, (dT | dA) backward).  Otherwise a
     * negative request's row is dim wide — t + a forward, dT backward (its dA is dT: negatives go
     * through augment_items only, with no mimic loss, training.py:772-787) — and a positive's stays
     * (t | a) / (dT | dA): the buffers are sequences of dim-float units, a positive taking two.
     * exchange_counts = the count all-to-all's rows [2 * exchange_world, exchange_counts_ld]:
     * rows [0, world) what this rank sent to each owner, rows [world, 2 world) what it received from
     * each requester; column 0 the requests, column 2 how many of them are positives (the leading
     * ones: ttamm_route_rows with counts_ld >= 3).  Requester buffers are owner-grouped as
     * item_slot orders them, the owner's requester-grouped as item_rows arrive; each group is
     * [positives | negatives], so the all-to-alls move dim * (requests + positives) floats per
     * peer, unpermuted.  item_slot then holds each request's first unit (ttamm_route_rows with
     * counts_ld >= 3 writes them); ITEM_FWD forms the owner's with its staging. */
    const int64_t* exchange_counts;
    int64_t exchange_counts_ld;
    int32_t exchange_world;
} ttamm_step_args;

#define TTAMM_G0_EXACT 0
#define TTAMM_G0_FAST 1

/* ---------------------------------------------------------------------------------- */
/* Entry points                                                                        */
/* ---------------------------------------------------------------------------------- */

int ttamm_abi_version(void);
const char* ttamm_last_error(void);
/* 1 for a developer build (make DEV=1), which also honours the A/B, ablation and measured-slower
 * environment switches; 0 for the default library, which reads only the documented knobs
 * (INTEGRATION.md "Environment").  No reference counterpart (build introspection for tests). */
int ttamm_developer_build(void);

/* Replaces one iteration of `_train_one_epoch` (training.py:726-831): negative sampling,
 * both tower forwards, mimic augmentation + losses, dot-product scoring, BCE, backward,
 * AdamW (dense group incl. the full mimic tables) and SparseAdam (ID tables). */
size_t ttamm_train_step_workspace_size(const ttamm_step_args* args);
int ttamm_train_step(const ttamm_step_args* args, void* stream);
/* 1 when a row-sharded step with these towers may set exchange_counts (compact exchange rows):
 * mimic on and the item tower's gate on the fused kernels (gate.hip / gate16.hip), alone and
 * grouped with the user tower; 0 otherwise (the 2*dim-wide rows).  Host-only, no device work. */
int ttamm_exchange_compact_supported(const ttamm_step_args* args);

/* Size (floats) of the replicated-weight gradient arena of a sharded step: both towers'
 * feature-encoder and gate weight+bias gradients, contiguous (the all-reduce buffer). */
int64_t ttamm_dense_grad_floats(const ttamm_step_args* args);

/* Row grouping of a batch of row ids — the gradient coalescing every row-table update of the
 * step runs (torch's grad.coalesce(), _functional.py:44, and the index_add order of the
 * embedding backward, training.py:822): the unique rows, in first-occurrence order (sorted = 0)
 * or ascending (sorted = 1, table_rows <= 65536), each with its batch positions ascending.
 * Outputs: keys_out[n] / positions_out[n] (the row and batch position of each slot),
 * seg_start_out[n + 1] (row u's slots are [seg_start[u], seg_start[u + 1])), n_unique_out[1].
 * idx must hold ids in [0, table_rows).  The workspace (ttamm_coalesce_workspace_bytes) must be
 * zero-filled before its first use; every call leaves its per-row scratch zero again. */
size_t ttamm_coalesce_workspace_bytes(int64_t n, int64_t table_rows);
int ttamm_coalesce_rows(const int64_t* idx, int64_t n, int64_t table_rows, int32_t sorted, int32_t* keys_out,
                        int32_t* positions_out, int32_t* seg_start_out, int32_t* n_unique_out, void* workspace,
                        size_t workspace_bytes, void* stream);

/* ---- exact inner-product retrieval + top-k -------------------------------
 * Replaces faiss.IndexFlatIP.search + the candidate filter of _evaluate_model
 * (training.py:645-679 index build, :944-970 search and filter).  For each query q the k items
 * i with the largest <queries[q], items[i]> (fp32) that are NOT in q's blocked set, best first;
 * equal scores are ordered by item id.  Blocked sets: CSR blocked_offsets[n_queries + 1] over
 * blocked_values sorted ascending per query (both NULL: nothing blocked).  Missing results
 * (fewer than k unblocked items) are id -1 / score -inf.  dim % 8 == 0, dim <= 256, rows
 * 16-byte aligned, 1 <= k <= 192. */
size_t ttamm_retrieval_topk_workspace_size(int64_t n_queries, int64_t n_items, int32_t dim, int32_t k);
int ttamm_retrieval_topk(const float* queries, int64_t n_queries, int64_t ldq, const float* items, int64_t n_items,
                         int64_t ldi, int32_t dim, const int64_t* blocked_offsets, const int64_t* blocked_values,
                         int32_t k, float* out_scores, int64_t* out_ids, void* workspace, size_t workspace_bytes,
                         void* stream);

/* The no-FAISS branch of _evaluate_model, _retrieve_with_sampling (training.py:974-1009): query q
 * scores its candidate list — items rows cand_rows[cand_offsets[q] .. cand_offsets[q+1]), at most
 * max_candidates (<= 4096) per query — by inner product, or by cosine similarity of the
 * F.normalize'd vectors when cosine != 0 (:999-1003), and returns the k best LIST POSITIONS
 * (torch.topk(scores, k), sorted; equal scores by list position), -1 / -inf past the list. */
int ttamm_candidate_topk(const float* queries, int64_t n_queries, int64_t ldq, const float* items, int64_t n_items,
                         int64_t ldi, int32_t dim, const int64_t* cand_offsets, const int64_t* cand_rows,
                         int32_t max_candidates, int32_t cosine, int32_t k, float* out_scores, int64_t* out_positions,
                         void* stream);

/* dst[r, c] = bf16(src[r, c]) rounded to nearest even for c < cols, 0 for cols <= c < ld_dst: the
 * bf16 feature copy of a matmul_bf16 tower (ttamm_tower.features_bf16). */
int ttamm_to_bf16(const float* src, int64_t rows, int32_t cols, int64_t ld_src, uint16_t* dst, int64_t ld_dst,
                  void* stream);

/* The bf16 planes of fp32 rows (ttamm_tower.features_planes): for c < cols, x = src[r, c],
 * hi = bf16(x), mid = bf16(x - hi), lo = bf16(x - hi - mid) (round to nearest even, every
 * difference exact) at dst[r * ld_dst + 48 (c / 16) + {0, 16, 32} + c % 16]; zero for
 * cols <= c < 16 ceil(cols / 16).  ld_dst >= 48 ceil(cols / 16), a multiple of 8. */
int ttamm_to_planes(const float* src, int64_t rows, int32_t cols, int64_t ld_src, uint16_t* dst, int64_t ld_dst,
                    void* stream);

/* DataLoader(InteractionDataset(train_df), batch_size, shuffle, drop_last=False)
 * (datasets.py:12-45, training.py:260-264) over pairs resident in HBM: writes positions
 * [start, start + count) of epoch `epoch`'s order of the n pairs (users[i], items[i]) — the
 * batch of a loader is start = b * batch_size, count = min(batch_size, n - start).  shuffle = 0:
 * the stored order; otherwise pair perm(p) at position p, perm a seeded bijection of [0, n)
 * (4-round Feistel network on 2h-bit words, 4^h >= n, with cycle-walking; round keys from
 * splitmix64 of (seed, epoch), restated in oracle/data_perm.py).  Replaces the host-side
 * torch.randperm + collation of torch.utils.data. */
int ttamm_epoch_batch(const int64_t* users, const int64_t* items, int64_t n, uint64_t seed, int64_t epoch,
                      int32_t shuffle, int64_t start, int64_t count, int64_t* out_users, int64_t* out_items,
                      void* stream);

/* Owner routing of a row-sharded step (rows owned by rank id % world): the n = n0 + n1 ids
 * id0[0..n0) then id1[0..n1) are grouped by owner, stably (positions in order within an owner).
 * For every position j:  slot[j]              = its index in the grouped order,
 *                         packed[slot[j]][0]  = id_j / world (the owner's local row),
 *                         packed[slot[j]][1]  = payload ? payload[j] : (j < n0 ? key0 + j
 *                                                                     : key1 + (j - n0));
 * counts[o] = ids owned by rank o (int64[world]).  The requests of ShardedTrainStep (ids =
 * [positives; negatives], keys = global request positions) and the pair routing of its epoch
 * driver (ids = users, payload = items) — replaces a host argsort / bincount
 * (torch.argsort(owner, stable=True), ttamm/sharded.py).  1 <= world <= 1024; every id >= 0;
 * scratch: device memory of ttamm_route_scratch_bytes(n0 + n1, world) bytes.  counts[o * counts_ld]
 * (counts_ld >= 1); with status != NULL and counts_ld >= 2, counts[o * counts_ld + 1] = *status —
 * the (count, status word) rows of the sharded step's count all-to-all, written in the same launch;
 * with counts_ld >= 3, counts[o * counts_ld + 2] = how many of owner o's ids came from id0 (the
 * positives of a step's requests: ttamm_step_args.exchange_counts), and slot[j] is then position
 * j's first unit of the compact exchange layout instead of its grouped row: the owner groups in
 * order, each [its id0 ids, two units each | its id1 ids, one unit each]. */
size_t ttamm_route_scratch_bytes(int64_t n, int32_t world);
int ttamm_route_rows(const int64_t* id0, int64_t n0, const int64_t* id1, int64_t n1, const int64_t* payload,
                     int64_t key0, int64_t key1, int32_t world, int64_t* packed, int64_t* slot, int64_t* counts,
                     int64_t counts_ld, const uint32_t* status, void* scratch, size_t scratch_bytes, void* stream);

/* A HIP stream whose kernels run on `num_cus` compute units only, spread evenly over the device
 * (every (CUs / num_cus)-th CU, so every XCD keeps some): a ttamm_step_args.aux_stream for the
 * index-only prologue that overlaps the feature GEMMs without co-residing on every CU they use.
 * num_cus <= 0 or >= the device's CUs gives an unrestricted stream.  Release with
 * ttamm_stream_destroy. */
int ttamm_stream_create_cu_limited(int32_t num_cus, void** stream);
int ttamm_stream_destroy(void* stream);

/* faiss.normalize_L2 on device rows, in place (training.py:670-672 on the item matrix and
 * :954-955 on the queries when the model's similarity is cosine): row r of the [n, dim] matrix
 * with leading dim ld is scaled by 1 / sqrt(sum of its squares); rows of norm 0 are left as
 * they are.  Replaces faiss::fvec_renorm_L2 (faiss/utils/distances.cpp). */
int ttamm_normalize_rows(float* rows, int64_t n, int32_t dim, int64_t ld, void* stream);

/* Deferred AdamW(g = 0): bytes of one adam_history entry, and the flush that brings every row
 * of every dense-group table with last_step up to hp.dense_step (call before the tables or
 * their optimizer state are read outside the step: evaluation, checkpoints, epoch end). */
size_t ttamm_adam_history_entry_bytes(void);
int ttamm_flush_tables(const ttamm_step_args* args, void* stream);

/* nn.Embedding forward / AdaptiveMimicMechanism._gather_and_reshape
 * (encoders.py:222-223, adaptive_mimic.py:97-105): out[r, :] = table[idx[r], :].
 * Every row-indexed entry point below never reads outside its table: an id outside
 * [0, table_rows) yields a zero row (the Python mirror raises IndexError before the call, as
 * nn.Embedding does).  The training step reports such ids through TTAMM_STATUS_INDEX_OUT_OF_RANGE. */
int ttamm_gather_rows(const float* table, int64_t table_rows, int32_t dim, const int64_t* idx,
                      int64_t n, float* out, int64_t out_ld, void* stream);

/* TowerEncoder.forward in eval mode (encoders.py:221-255), optionally followed by
 * AdaptiveMimicMechanism.augment_* (adaptive_mimic.py:70-95) when tower->mimic.weight
 * is non-NULL and `augment` != 0.  ID (and mimic) rows are idx[r]; feature rows are
 * tower->features[feat_idx[r]] (feat_idx NULL: row r, i.e. features already gathered by the
 * caller as in training.py:741-747).  out: [n, dim]. */
size_t ttamm_tower_forward_workspace_size(const ttamm_tower* tower, int64_t n);
int ttamm_tower_forward(const ttamm_tower* tower, const int64_t* idx, const int64_t* feat_idx, int64_t n,
                        int32_t augment, float* out, void* workspace, size_t workspace_bytes,
                        void* stream);

/* TowerEncoder.forward under autograd (encoders.py:221-255): the training-mode forward keeps its
 * activations in `workspace` (ttamm_tower_train_workspace_size); ttamm_tower_train_backward, given
 * the same tower, rows, keep masks and workspace and d_out = dL/d(out) [n, dim], runs the tower's
 * backward (gate, feature-MLP dgrad chain, one grouped weight-gradient launch) into grad_arena
 * (ttamm_tower_grad_floats floats: per feature Linear weight [out, in] then bias [out], then the
 * gate's / concat projection's, each piece starting at a multiple of 64 floats) and writes the
 * ID rows' gradient per position into d_id_rows [n, dim] (nn.Embedding's sparse gradient values;
 * duplicates not summed).  d_feat_rows [n, dim]: the feature rows' gradient, identity feature
 * encoder only (FeatureFusionGate.forward on given rows).  keep_masks: NULL or one uint8
 * [n, out_features] keep mask per hidden layer (NULL entries: drawn from Philox(seed, counter)).
 * The tower's optimizer-state pointers are not read. */
size_t ttamm_tower_grad_floats(const ttamm_tower* tower);
size_t ttamm_tower_train_workspace_size(const ttamm_tower* tower, int64_t n);
int ttamm_tower_train_forward(const ttamm_tower* tower, const int64_t* idx, const int64_t* feat_idx, int64_t n,
                              const uint8_t* const* keep_masks, uint64_t seed, uint64_t counter, float* out,
                              void* workspace, size_t workspace_bytes, void* stream);
int ttamm_tower_train_backward(const ttamm_tower* tower, const int64_t* idx, const int64_t* feat_idx, int64_t n,
                               const uint8_t* const* keep_masks, const float* d_out, float* grad_arena,
                               float* d_id_rows, float* d_feat_rows, void* workspace, size_t workspace_bytes,
                               void* stream);

/* The backward of a row lookup into a dense gradient (nn.Embedding(sparse=False) / the dense
 * mimic tables, adaptive_mimic.py:97-105; F.mse_loss's input gradient with scale = 2 / numel):
 * dst[idx[r]] += (x[r] - y[r]) * scale * (*scale_dev) for y != NULL, x[r] * ... otherwise
 * (idx NULL: dst row r — an elementwise scaled difference, F.mse_loss's backward);
 * scale_dev (device float, e.g. the upstream gradient of a scalar loss) may be NULL; rows with
 * idx[r] == skip_row (padding_idx, -1 = none) are skipped.  Float atomics. */
int ttamm_scatter_add_rows(float* dst, int64_t dst_rows, int32_t dim, const int64_t* idx, int64_t n,
                           const float* x, int64_t ldx, const float* y, int64_t ldy, const float* scale_dev,
                           float scale, int64_t skip_row, void* stream);

/* AdaptiveMimicMechanism._apply_aug (adaptive_mimic.py:88-95): out = base + table[idx].
 * aug_out (optional) receives table[idx]. */
int ttamm_mimic_augment(const float* table, int64_t table_rows, int32_t dim, const int64_t* idx,
                        int64_t n, const float* base, float* out, float* aug_out, void* stream);

/* F.mse_loss(input, target) with reduction='mean' (adaptive_mimic.py:97-98): out[0] = mean. */
int ttamm_mse_loss(const float* input, const float* target, int64_t n, float* out, void* stream);

/* sample_negative_items (samplers.py:11-85) on device: out[b, j] uniform in [0, num_items)
 * and not among user b's positives (CSR over user_rows users, sorted per user; a user id outside
 * [0, user_rows) has no positives, as positives.get(user, set()) gives the reference); up to 11
 * draws per slot, then the TTAMM_STATUS_SAMPLER_EXHAUSTED bit is set in *status.  The draws of slot
 * j come from the Philox stream keyed by (seed, counter, slot_base + j): the fused step's sampler
 * for a batch whose first slot is slot_base (row_base * num_neg in a row-sharded step). */
int ttamm_sample_negatives(const int64_t* users, int64_t batch, int32_t num_neg, int64_t num_items,
                           const int64_t* pos_offsets, const int64_t* pos_values, int64_t user_rows,
                           uint64_t seed, uint64_t counter, int64_t slot_base, int64_t* out, uint32_t* status,
                           void* stream);

/* nn.Embedding's index check (encoders.py:222-223) without a lookup: sets
 * TTAMM_STATUS_INDEX_OUT_OF_RANGE in *status when an id of ids0[0..n0) lies outside [0, rows0) or
 * one of ids1[0..n1) outside [0, rows1) (ids1 may be NULL).  The row-sharded step's look-ahead
 * checks the next batch with it before that batch's request counts are exchanged. */
int ttamm_check_rows(const int64_t* ids0, int64_t n0, int64_t rows0, const int64_t* ids1, int64_t n1,
                     int64_t rows1, uint32_t* status, void* stream);

/* torch.optim.SparseAdam step on one table for already-coalesced rows
 * (_functional.py:24-84): rows[u] unique, grad [n_rows, dim]. */
int ttamm_sparse_adam_rows(float* weight, float* exp_avg, float* exp_avg_sq, int32_t dim,
                           const int64_t* rows, const float* grad, int64_t n_rows, double lr,
                           double beta1, double beta2, double eps, int64_t step, void* stream);

/* torch.optim.AdamW / Adam single-tensor step over a dense tensor (adam.py:419-547). */
int ttamm_adamw_dense(float* param, float* exp_avg, float* exp_avg_sq, const float* grad, int64_t n,
                      double lr, double beta1, double beta2, double eps, double weight_decay,
                      int32_t decoupled, int64_t step, void* stream);

/* In-batch negatives as one op (ttamm's in-batch mode, BASELINE configs C2 / C4; the scoring it
 * extends is training.py:770-798, its definition oracle/cpu_reference.py train_step(in_batch=True)):
 *   S = users . positives^T [batch, n_positives], label 1 at (b, row_base + b), 0 elsewhere;
 *   d_users = dS . positives, d_positives = dS^T . users with dS = (sigmoid(S) - Y) * inv_count;
 *   *loss_sum = sum over S of the BCE-with-logits terms (fp64 on the device).
 * Nothing batch x n_positives is stored (inbatch_x_kernel, split-bf16 MFMA).  In a row-sharded step
 * n_positives is the all-gathered global batch and row_base the rank's first global position. */
size_t ttamm_inbatch_workspace_size(int64_t batch, int64_t n_positives, int32_t dim);
int ttamm_inbatch_bce(const float* users, int64_t batch, int64_t ldu, const float* positives,
                      int64_t n_positives, int64_t ldp, int32_t dim, int64_t row_base, float inv_count,
                      float* d_users, int64_t ld_du, float* d_positives, int64_t ld_dp, double* loss_sum,
                      void* workspace, size_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* TTAMM_H */
