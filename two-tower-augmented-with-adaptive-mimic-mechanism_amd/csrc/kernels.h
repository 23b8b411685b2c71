// Internal launcher interface between the kernels (*.hip) and the step executor.
#pragma once

#include "common.h"

namespace ttamm {

// ------------------------------------------------------------------------------------
// GEMM family (gemm.hip).  fp32 in, fp32 accumulate on v_mfma_f32_32x32x2_f32.
// ------------------------------------------------------------------------------------
enum Epilogue : int {
    EPI_STORE = 0,          // C = acc (+bias)
    EPI_HIDDEN = 1,         // C = dropout(relu(acc + bias))             (encoders.py:132-138)
    EPI_GATE_HIDDEN = 2,    // C = relu(acc + bias)                        (encoders.py:158-159)
    EPI_GATE_OUT = 3,       // g = sigmoid(acc + bias); t = g*e + (1-g)*f; mimic augment
    EPI_DGRAD_RELU = 4,     // C = acc * (aux0 > 0)                        (ReLU backward)
    EPI_DGRAD_GATE_EF = 5,  // C[:, :D] = acc + dT*g ; C[:, D:] = acc + dT*(1-g)
    EPI_DGRAD_HIDDEN = 6,   // C = (aux0 > 0) ? acc * inv_keep : 0          (dropout+ReLU bwd)
};

struct GemmProblem {
    // A [M, K] row-major; row r is A + (a_idx ? a_idx[r] : r) * lda
    const float* A;
    const int64_t* a_idx;
    int64_t lda;
    // B: b_kn == 0 -> B stored [N, K] (nn.Linear weight, y = x W^T)
    //    b_kn == 1 -> B stored [K, N] (dgrad: dX = dY W)
    const float* B;
    int64_t ldb;
    int b_kn;
    int M, N, K;
    int epi;
    float* C;
    int64_t ldc;
    const float* bias;
    // epilogue operands (meaning depends on epi)
    const float* aux0;  // EPI_GATE_OUT: ef [M, 2D]; DGRAD_RELU / DGRAD_HIDDEN: activation
    const float* aux1;  // EPI_DGRAD_GATE_EF: dT [M, D]
    const float* aux2;  // EPI_DGRAD_GATE_EF: g  [M, D]
    int64_t ld_aux0, ld_aux1, ld_aux2;
    float* out1;        // EPI_GATE_OUT: g
    float* out2;        // EPI_GATE_OUT: t
    float* out3;        // EPI_GATE_OUT: a (mimic rows), may be null
    const float* table; // EPI_GATE_OUT: mimic table (may be null)
    const int64_t* idx; // EPI_GATE_OUT: rows into table
    int64_t ld_out;     // EPI_GATE_OUT: ld of g
    int64_t ld_out2;    // EPI_GATE_OUT: ld of t / a  (C = aug may be null)
    // dropout (EPI_HIDDEN / EPI_DGRAD_HIDDEN)
    float keep_prob;    // 1 - p
    float inv_keep;     // 1 / (1 - p)   (torch: noise.div_(1 - p))
    const uint8_t* keep_mask;  // optional injected [M, N]
    uint32_t rng_k0, rng_k1, rng_c2, rng_c3;
    // dropout stream key of output row r (its global interaction position, so a sharded
    // step draws the same masks as one process over the whole global batch):
    //   row_key ? row_key[r] : (r < key_split ? key_base0 + r : key_base1 + (r - key_split))
    const int64_t* row_key;
    int64_t key_base0, key_base1, key_split;
    // K-major A (weight gradient: A = X^T, rows of X indexed by k, gathered by a_idx)
    int a_kmaj;
    int a_cols;          // valid columns of X (m < a_cols)
    int a_ones_col;      // column of implicit ones (bias gradient), -1 = none
    // K-major B (weight gradient, split kernel): the blocks of M-tile 0 also sum B over their k
    // rows (bf16-rounded when bf16) and write the column sums to C row M of their split's slab —
    // the bias gradient without an implicit ones column (which cost a whole extra M-tile when
    // n_in is a multiple of the tile height: 512 + 1 = five 128-row tiles)
    int b_colsum;
    // split-K over rows: each split writes its own slab at C + split * slab_stride
    int k_split;
    int64_t slab_stride;
    int tile_begin;     // filled by the launcher
    int tiles_m, tiles_n;
    int bf16;           // 1: operands rounded to bf16 (RNE), fp32 accumulation (grouped problems agree)
    // bf16 operands already in memory (A16 / B16 non-null: the gemm_bf16 kernel, forward "NT"
    // GEMMs only): A16 rows [M, K] (gathered by a_idx), B16 = W [N, K]; lda / ldb in elements
    // (multiples of 8), K a multiple of 8.  Same epilogues as the fp32 kernel.
    const uint16_t* A16;
    const uint16_t* B16;
    // weight gradients of bf16 towers (split kernel, K-major A, XCfg::A16): A16 = the bf16 copy of X,
    // rows gathered by a_idx, lda16 elements per row (% 8 == 0, zero from a_cols on)
    int64_t lda16;
    // A pre-split into bf16 planes (split kernel, fp32 towers): row r's k-tile t (16 k) is the 96 B
    // at A3p + r * lda3 + 48 t: hi[16], mid[16], lo[16] with hi + mid + lo == the fp32 value; A keeps
    // pointing at the fp32 rows (the exact-MFMA path reads those).  lda3 in uint16 elements.
    const uint16_t* A3p;
    int64_t lda3;
    // feature-MLP activation (EPI_HIDDEN / EPI_DGRAD_HIDDEN; ttamm.h TTAMM_ACT_*, 0 = ReLU).  A
    // non-ReLU EPI_HIDDEN also writes the pre-activation to `pre` [M, ldc] and, when it draws its
    // dropout decisions, the keep bytes to `mask_out` [M, N]; its EPI_DGRAD_HIDDEN reads the
    // pre-activation as aux0 and the keep bytes as keep_mask (keep_prob < 1).
    int act;
    float* pre;
    uint8_t* mask_out;
};

constexpr int kMaxGemmProblems = 8;
struct GemmBatch {
    GemmProblem p[kMaxGemmProblems];
    int count;
    int total_tiles;
};

int launch_gemm(GemmBatch& batch, hipStream_t s);

// on-device epoch order of the interaction pairs (data.hip)
int epoch_half_bits(int64_t n);
size_t route_scratch_bytes(int64_t n, int world);
int launch_route_rows(const int64_t* id0, int64_t n0, const int64_t* id1, int64_t n1, const int64_t* payload,
                      int64_t key0, int64_t key1, int world, int64_t* packed, int64_t* slot, int64_t* counts,
                      int64_t counts_ld, const uint32_t* status, void* scratch, size_t scratch_bytes, hipStream_t s);
void epoch_round_keys(uint64_t seed, int64_t epoch, uint32_t keys[4]);
int launch_epoch_batch(const int64_t* users, const int64_t* items, int64_t n, uint64_t seed, int64_t epoch,
                       int shuffle, int64_t start, int64_t count, int64_t* out_users, int64_t* out_items,
                       hipStream_t s);
// fp32 -> bf16 (round to nearest even) rows, zero-filled from `cols` to ld_dst
int launch_to_bf16(const float* src, int64_t rows, int cols, int64_t ld_src, uint16_t* dst, int64_t ld_dst,
                   hipStream_t s);
// fp32 rows -> [rows][ceil(cols / 16)][hi, mid, lo][16] bf16 planes (ttamm.h ttamm_to_planes)
int launch_to_planes(const float* src, int64_t rows, int cols, int64_t ld_src, uint16_t* dst, int64_t ld_dst,
                     hipStream_t s);

// Weight-gradient GEMM (split-K over rows) + fixed-order reduce.
//   dW[m, n] = sum_r dY[r, m] * X[r, n] ;  db[m] = sum_r dY[r, m]
struct WgradProblem {
    const float* dY;
    int64_t ld_dy;
    const float* X;
    const int64_t* x_idx;  // gather rows of X (features) or null
    int64_t ld_x;
    const uint16_t* X3p;   // X pre-split into bf16 planes (GemmProblem::A3p layout) or null
    int64_t ld_x3;
    const uint16_t* X16;   // bf16 problems: X already rounded to bf16 (ld_x16 elements, % 8) or null
    int64_t ld_x16;
    int R, M, N;           // rows, out features, in features
    float* grad_w;         // [M, N]
    float* grad_b;         // [M] (may be null)
    float* slab;           // workspace [splits, M, N+1]
    int splits;            // chunks of rows
    int rows_per_split;
    int tile_begin;
    int tiles_m, tiles_n;
    int bf16;              // 1: operands rounded to bf16, fp32 accumulation (the batch agrees)
};
constexpr int kMaxWgradProblems = 16;
static_assert(kMaxWgradProblems >= 2 * (TTAMM_MAX_LINEAR + 2), "both towers: every Linear + the gate's two");
struct WgradBatch {
    WgradProblem p[kMaxWgradProblems];
    int count;
    int total_blocks;
};
struct WgradShape {
    int64_t R;  // rows
    int M, N;   // out features, in features
};
// weight-gradient tile class (the output tile width over m_out, the least padding):
// 0 = 128 x 96 (m_out <= 96), 1 = 128 x 192, 2 = 128 x 128, 3 = multiples of 256 (on 128 x 128
// tiles, their own split size); TTAMM_WGRAD_ALL_NARROW=1 (developer switch) puts every problem in
// class 0
constexpr int kWgradClasses = 4;
int wgrad_class(int m_out);
// rows per split-K chunk for each class of a step's weight gradients
void wgrad_rows_per_split(const WgradShape* shapes, int n, int rps[kWgradClasses]);
size_t wgrad_slab_floats(int R, int M, int N, int rows_per_split);
// ev (optional, 2 hipEvent_t): recorded around the launches of every class but the narrow one
int launch_wgrad(WgradBatch& batch, hipStream_t s, void* const* ev = nullptr);

// ------------------------------------------------------------------------------------
// Fused gate forward / backward (gate.hip): fp32 towers with D == Hg in {32, 64, 96}
// ------------------------------------------------------------------------------------
struct GateTower {
    int64_t R;
    const float* ef;     // [R, 2D] = [e | f]
    const float* G1;     // gate_network.0.weight [Hg, 2D]
    const float* c1;     // [Hg]
    const float* G2;     // gate_network.2.weight [D, Hg]
    const float* c2;     // [D]
    float* z;            // [R, Hg]
    float* g;            // [R, D]
    float* t;            // [R, ld_t]
    float* a;            // [R, ld_t] mimic rows (written when table)
    int64_t ld_t;
    const float* table;  // mimic table or null
    const int64_t* idx;  // its rows
    float* aug;          // [R, D] or null (sharded item owner)
    const float* dT;     // backward: [R, ld_dT]
    int64_t ld_dT;
    // compact exchange (sharded item owner): row r's t / dT at t / dT + u D and its a at a + u D
    // for u = xu[r] >= 0 (a positive); u < 0: a negative, whose one unit ~u holds t + a (forward)
    // and dT (backward).  Null: row r at r * ld_t / r * ld_dT.
    const int64_t* xu;
    float* dq;           // [R, D]
    float* dz;           // [R, Hg]
    float* dEF;          // [R, 2D]
    uint16_t* w16;       // bf16 towers: the weight images (gate16.hip, gate16_image_elems)
    int blocks;          // filled by the launcher
};
struct GateArgs {
    GateTower tw[2];
    int count;
    int D, HG;
    // gate16.hip operand planes: 1 = bf16 towers (operands rounded to bf16), 3 = fp32 towers
    // (split-bf16, fp32-accurate); 0 = gate.hip (fp32 MFMA)
    int planes;
    int images_ready;  // gate16: the towers' weight images were formed earlier in this step (no prep)
    int ablate;  // developer timing ablation (TTAMM_GATE_ABLATE=1: no output stores); set by launch_gate
    int direct;  // TTAMM_GATE_DIRECT_STORES=1: stores from the MFMA layout (16 rows x 64 B each); set by launch_gate
};
bool gate_fused_supported(int D, int HG);
int launch_gate(GateArgs& a, bool backward, hipStream_t s);
// gate16.hip: bf16 towers at D == Hg in {128, 256} (planes 1), fp32 towers at D == Hg == 96
// (planes 3); the per-tower bf16 weight images are formed by launch_gate16_prep (launch_gate runs
// it unless a.images_ready)
bool gate16_supported(int D, int HG, int planes);
int64_t gate16_image_elems(int D, int HG, int planes);
int launch_gate16_prep(GateArgs& a, hipStream_t s);
int launch_gate16(GateArgs& a, bool backward, hipStream_t s);

// ------------------------------------------------------------------------------------
// Row kernels (rows.hip)
// ------------------------------------------------------------------------------------
// ids outside [0, table_rows) give zero rows (never an out-of-table read)
// nn.Embedding max_norm (embedding_renorm_): each distinct row of idx[0, n) whose L2 norm exceeds
// max_norm is scaled by max_norm / (norm + 1e-7) in place; one wave per position, the first
// wave to claim a row through mark[row] = tag does it (tags unique per call, mark zeroed once)
// keys (optional): only positions with (keys[p] >= key_split) == key_phase take part (a sharded
// owner's requests: the positives' lookup, key < global batch, then the negatives')
int launch_renorm_rows(float* table, int64_t table_rows, int dim, const int64_t* idx, int64_t n, double max_norm,
                       int32_t* mark, int32_t tag, hipStream_t s, const int64_t* keys = nullptr,
                       int64_t key_split = 0, int key_phase = 0);
int launch_gather_rows(const float* table, int64_t table_rows, int dim, const int64_t* idx, int64_t n, float* out,
                       int64_t out_ld, hipStream_t s);

// Index staging (training step prologue): out[i] = in[i] if 0 <= in[i] < rows, else 0 and
// TTAMM_STATUS_INDEX_OUT_OF_RANGE is OR-ed into *status.  out == null: check only.
struct StageSeg {
    const int64_t* in;
    int64_t* out;
    int64_t n;
    int64_t rows;
    int64_t ld;  // element stride of `in` (0 = 1)
};
constexpr int kMaxStageSegs = 3;
struct StageArgs {
    StageSeg seg[kMaxStageSegs];
    int count;
    uint32_t* status;
    // compact exchange rows (ttamm.h exchange_counts), stage_rows_kernel only: the first unit of
    // each of unit_n owner rows, grouped by requester as they arrived (unit_groups groups of
    // unit_counts[g * unit_ld] rows, the first unit_counts[g * unit_ld + 2] of them positives:
    // two units each); ~unit for a negative row.  unit_out null = none.
    const int64_t* unit_counts;
    int64_t unit_ld;
    int unit_groups;
    int64_t unit_n;
    int64_t* unit_out;
};
int launch_stage_rows(const StageArgs& a, hipStream_t s);
// out = x (+ y) over [n, dim] rows (y may be null): an augmented row t + a (adaptive_mimic.py:88-95);
// with xrow, out row r reads row xrow[r] of x and y
int launch_add_rows(const float* x, int64_t ldx, const float* y, int64_t ldy, int64_t n, int dim, float* out,
                    int64_t ldo, hipStream_t s, const int64_t* xrow = nullptr);
// dst[idx[r]] += (x[r] (- y[r])) * scale (* *scale_dev), skipping rows idx[r] == skip_row and
// rows outside [0, dst_rows) (float atomics)
int launch_scatter_add_rows(float* dst, int64_t dst_rows, int dim, const int64_t* idx, int64_t n, const float* x,
                            int64_t ldx, const float* y, int64_t ldy, const float* scale_dev, float scale,
                            int64_t skip_row, hipStream_t s);

// Status bits that stop every later step (ttamm.h TTAMM_STATUS_*).
constexpr uint32_t kStatusPoison =
    TTAMM_STATUS_SAMPLER_EXHAUSTED | TTAMM_STATUS_INDEX_OUT_OF_RANGE | TTAMM_STATUS_LOOKAHEAD_MISMATCH;
__device__ __forceinline__ bool step_poisoned(const uint32_t* status) {
    return status != nullptr && (*status & kStatusPoison) != 0u;
}
// t = e (+ f); a = table[idx]; aug = t + a   (non-gated fusion)
// t = e (+ f); a = table[idx]; aug = t (+ a).  t / a rows at stride ld_ta; aug may be null.
int launch_combine(const float* e, int64_t ld_e, const float* f, int64_t ld_f, const float* table,
                   int64_t table_rows, const int64_t* idx, int64_t n, int dim, float* t, float* a, int64_t ld_ta, float* aug,
                   hipStream_t s);
// generic gated fusion: g = sigmoid(x) in place, t = g e + (1 - g) f, a = table[idx], aug = t + a
int launch_gate_mix(float* g, const float* ef, const float* table, const int64_t* idx, int64_t n, int dim, float* t,
                    float* a, int64_t ld_ta, float* aug, hipStream_t s);
int launch_pad_rows(const float* src, int64_t rows, int cols, int64_t ld_src, float* dst, int ld_dst,
                    hipStream_t s);
// the same over up to two segments in one launch (the two towers)
struct GatherSeg {
    const float* table;
    int64_t rows;
    int dim;
    const int64_t* idx;
    int64_t n;
    float* out;
    int64_t out_ld;
};
struct GatherSegs {
    GatherSeg seg[2];
    int count;
};
int launch_gather_rows_segs(const GatherSegs& g, hipStream_t s);
struct PadSeg {
    const float* src;
    int64_t rows;
    int cols;
    int64_t ld_src;
    float* dst;
    int ld_dst;
};
struct PadSegs {
    PadSeg seg[2];
    int count;
};
int launch_pad_rows_segs(const PadSegs& p, hipStream_t s);
int launch_mse(const float* x, const float* y, int64_t n, float* out, hipStream_t s);
// dq = (dT*e - dT*f) * (1-g) * g   (gate backward through the sigmoid)
int launch_gate_dq(const float* dT, int64_t ld_dT, const float* ef, const float* g, int64_t n, int dim,
                   float* dq, hipStream_t s);

struct ScoreArgs {
    int64_t B;
    int64_t Bg;             // global batch (loss normalisation), == B in a 1-process step
    int N;
    int D;
    const float* user_aug;  // [B, D]
    const float* item_aug;  // [B(1+N), ld_item] or null: t_item (+ a_item) computed in place
    const float* t_user;    // [B, D]
    const float* t_item;    // [B(1+N), ld_item]
    const float* a_user;    // [B, D] or null
    const float* a_item;    // [B(1+N), ld_item] or null
    int64_t ld_item;
    float lambda_u, lambda_i;
    int mimic;
    float* dT_user;   // [B, D]
    float* dT_item;   // [B(1+N), ld_dti]
    float* dA_user;   // [B, D]  (mimic)
    float* dA_item;   // (mimic) [B, ld_dti] positives only, or all B(1+N) rows when dA_all
    int dA_all;
    int neg_aug;      // compact exchange: negative request rows hold t + a in t_item (no a_item read)
    int64_t ld_dti;
    const int64_t* item_slot;  // or null: item request r's rows (t_item .. dA_item) are at item_slot[r]
    float* partials;  // [blocks, 3]
    int blocks;
    float inv_numel;  // 1 / logits in the BCE mean: Bg (1 + N), or Bg (Bg + N) in-batch
    // in-batch mode: the positive logit is part of the in-batch matrix; the rows' gradients
    // start from its dU / dP (ib_du [B, D], ib_dp [B, ib_ld]) and the sampled negatives add on
    const float* ib_du;
    const float* ib_dp;
    int64_t ib_ld;
};
int score_blocks(int64_t B, int D);  // [blocks, 3] partials of launch_score_loss
int launch_score_loss(const ScoreArgs& a, hipStream_t s);
// bce = (sum of the score partials + sum of ib_partials) / bce_count
int launch_loss_finalize(const float* partials, int blocks, const float* ib_partials, int ib_blocks, int64_t bce_count,
                         int64_t B, int64_t Bg, int D, float lambda_u, float lambda_i, int mimic, const float* cal,
                         float lambda_cal, float* loss_out, double* loss_accum, const uint32_t* status, hipStream_t s);

// ------------------------------------------------------------------------------------
// In-batch negatives: S = U P^T with BCE, dU, dP (inbatch.hip)
// ------------------------------------------------------------------------------------
struct InBatchArgs {
    const float* U;      // [B, ldu] augmented user rows (rows of S)
    int64_t ldu, B;
    const float* P;      // [Bc, ldp] augmented positive rows of the (global) batch (columns of S)
    int64_t ldp, Bc;
    int D;
    int64_t row_base;    // column of user 0's own positive (global batch position of the rank)
    float inv_T;         // 1 / logits in the BCE mean
    float* slab_u;       // [splits_u, B, D]
    float* slab_p;       // [splits_p, Bc, D]
    float* loss_part;    // [rblk_u * splits_u] BCE sums of the user-role blocks
    float* dU;           // [B, ld_du]  = dS P
    int64_t ld_du;
    float* dP;           // [Bc, ld_dp] = dS^T U
    int64_t ld_dp;
    // filled by inbatch_plan
    int rblk_u, rblk_p, splits_u, splits_p;
    int64_t cols_u, cols_p;
};
void inbatch_plan(int64_t B, int64_t Bc, InBatchArgs& a);
size_t inbatch_workspace_floats(int64_t B, int64_t Bc, int D, size_t* slab_u, size_t* slab_p, size_t* parts);
int launch_inbatch(InBatchArgs& a, hipStream_t s);
size_t inbatch_standalone_workspace_bytes(int64_t B, int64_t Bc, int D);
int inbatch_standalone(const float* U, int64_t B, int64_t ldu, const float* P, int64_t Bc, int64_t ldp, int D,
                       int64_t row_base, float inv_T, float* dU, int64_t ld_du, float* dP, int64_t ld_dp,
                       double* loss_sum, void* ws, size_t ws_bytes, hipStream_t s);

// ------------------------------------------------------------------------------------
// Exact inner-product retrieval + top-k (retrieval.hip)
// ------------------------------------------------------------------------------------
struct RetrievalArgs {
    const float* Q;
    int64_t ldq, nq;
    const float* X;
    int64_t ldx, ni;
    int D;
    const int64_t* boff;  // blocked items per query: CSR offsets [nq + 1] (null: none)
    const int64_t* bval;  // sorted ascending within each query
    int k;
    int parts;            // item partitions (grid.y)
    int64_t items_per_part;
    float* buf_s;         // candidate buffers [blocks, 64, 256]
    int* buf_i;
    float* part_s;        // per-partition top-k [nq, parts, k]
    int* part_i;
    int ablate;           // timing experiments only (TTAMM_RETRIEVAL_ABLATE): 1 no filter, 2 no MFMA, 4 no staging
};
size_t retrieval_workspace_bytes(int64_t nq, int64_t ni, int dim, int k);
int launch_normalize_rows(float* x, int64_t n, int dim, int64_t ld, hipStream_t s);
int launch_candidate_topk(const float* Q, int64_t nq, int64_t ldq, const float* X, int64_t ni, int64_t ldx, int dim,
                          const int64_t* coff, const int64_t* crow, int max_candidates, int cosine, int k, float* out_s,
                          int64_t* out_p, hipStream_t s);
int launch_retrieval_topk(const float* Q, int64_t nq, int64_t ldq, const float* X, int64_t ni, int64_t ldx, int dim,
                          const int64_t* boff, const int64_t* bval, int k, float* out_s, int64_t* out_i, void* ws,
                          size_t ws_bytes, hipStream_t s);

// ------------------------------------------------------------------------------------
// Coalesce + optimizers (optim.hip)
// ------------------------------------------------------------------------------------
// Grouping of a batch's row ids ("coalesce": duplicates summed in batch order, as torch's
// index_add / sparse coalesce do).  Output: slots 0..n-1 hold the positions grouped by row —
// segment u = slots [seg_start[u], seg_start[u+1]) is one row (keys_out), its positions
// ascending.  Segment order: first occurrence in the batch, or ascending row id (`sorted`, for
// small key ranges).  cnt / first / fill are per-row scratch of the table (key_range entries)
// that must be zero between calls — the call leaves them zero again.
struct CoalesceWs {
    int32_t* keys_out;   // [n]
    int32_t* vals_out;   // [n] batch position of each slot
    int32_t* vals_tmp;   // [n]
    int32_t* lead;       // [n] leader flag -> segment index of a leader position
    int32_t* lead_cnt;   // [max(n, 257)] scan scratch (tile totals)
    int32_t* seglong;    // [max(n, 257)] 1: the slot's segment is longer than a row-update piece
    int32_t* seg_start;  // [n + 1]
    int32_t* n_unique;   // [1]
    int32_t* cnt;        // [key_range] persistent, zero between calls
    int32_t* first;      // [key_range]
    int32_t* fill;       // [key_range]
    int64_t key_range;
    int sorted;          // 1: segments in ascending key order (key_range <= 65536)
};
constexpr int kCoalescePiece = 32;  // row-update piece: longer segments are summed in two levels
size_t coalesce_scratch_ints(int64_t key_range);  // per-row scratch (3 arrays)
// scratch: the cnt / first / fill arrays carved from a zeroed buffer of coalesce_scratch_ints ints
void coalesce_bind_scratch(CoalesceWs& ws, int32_t* scratch, int64_t key_range);
// group rows by index: unique rows + segment starts.  Two halves: the count (after it,
// ws.first marks every row's first position) and the grouping; launch_coalesce runs both.
int launch_coalesce_count(const int64_t* idx, int64_t n, int64_t table_rows, CoalesceWs& ws, hipStream_t s);
int launch_coalesce_group(const int64_t* idx, int64_t n, int64_t table_rows, CoalesceWs& ws, hipStream_t s);
int launch_coalesce(const int64_t* idx, int64_t n, int64_t table_rows, CoalesceWs& ws, hipStream_t s);

// ------------------------------------------------------------------------------------
// Category-alignment loss + gradient (cal.hip; training.py:530-579, :805-820)
// ------------------------------------------------------------------------------------
struct CalArgs {
    const float* x;             // augmented item rows [R, ld_x] = cat[positives; negatives]
    int64_t ld_x;
    const float* xa;            // sharded: the mimic rows (row value = x + xa); null: x is t + a
    int64_t xa_rows;            // request rows >= xa_rows read x alone (compact exchange negatives)
    const int64_t* slot;        // sharded: exchange-buffer row of request row r; null: row r
    const int64_t* idx;         // item id of row r
    const int64_t* idx1;        // sharded: item ids of rows [split, R) (the negatives); null: idx
    int64_t split;
    int64_t idx_rows;           // ids outside [0, idx_rows) read item 0's category
    float* gstats;              // sharded: [num_categories, D + 1] (sums | count), all-reduced
    const int64_t* categories;  // [items] category id (training.py:582-610)
    int64_t num_categories;
    int64_t major;              // major_category_id
    int64_t R;
    int D;
    float lambda;               // loss_weights.category_alignment
    int64_t* catrow;            // [R]
    CoalesceWs co;              // sort of the rows by category
    int nseg_max;               // min(R, num_categories)
    int32_t* pcount;            // [nseg_max] pieces per category segment
    int32_t* pstart;            // [nseg_max] exclusive scan
    float* psum;                // [pieces, D]
    float* mean;                // [nseg_max, D]
    float* pslab;               // [pieces, D, D]
    float* cov;                 // [nseg_max, D, D]; sharded: [num_categories, D, D], all-reduced
    float* part;                // [slots]: nseg_max, sharded num_categories
    int32_t* flag;              // [slots]
    float* gmajor;              // [D, D]
    float* out;                 // [2]: L_cal, compared
    float* dT;                  // item rows' dT [R, ld_d] (+= lambda dX); null: loss only
    float* dA;                  // dA of request rows < dA_rows [., ld_d] (+=), may be null
    int64_t ld_d;
    int64_t dA_rows;
};
int cal_max_pieces(int64_t R, int64_t nseg_max);
size_t cal_stats_floats(int64_t num_categories, int D);    // sharded gstats
size_t cal_scatter_floats(int64_t num_categories, int D);  // sharded cov / scatter sums
// the three stages (sharded: the caller all-reduces gstats after the first, cov after the second)
int launch_cal_local(const CalArgs& a, hipStream_t s);
int launch_cal_scatter(const CalArgs& a, hipStream_t s);
int launch_cal_finish(const CalArgs& a, hipStream_t s);
// exclusive prefix sum of n ints by one block (n up to ~1M; used for small arrays)
int launch_block_exclusive_scan(const int32_t* in, int32_t* out, int64_t n, hipStream_t s);
int launch_category_alignment(const CalArgs& a, hipStream_t s);


// Optimizer constants, derived on the host in double precision the way torch does and
// rounded to fp32 once (adam.py:419-547 single-tensor path; _functional.py:24-84).
struct AdamConsts {
    float decay;     // 1 - lr*wd                (AdamW decoupled decay)
    float w1;        // 1 - beta1                (lerp weight)
    float b2;        // beta2
    float w2;        // 1 - beta2                (addcmul value)
    float eps;
    float neg_step;  // -lr / bias_correction1
    float bc2_sqrt;  // sqrt(bias_correction2)
    float inv_bc2_sqrt;  // RN(1 / bc2_sqrt): the correctly rounded reciprocal (div_by_const)
    float wd;        // weight_decay (Adam L2 form)
    // TTAMM_G0_FAST: the step folded into the reciprocal, r = rcp(sqrt(v) * fast_ibc + fast_eps)
    // = neg_step / denom, so p = fma(m, r, p * decay) (lr = 0: fast_ibc = 0, fast_eps = +inf, r = 0)
    float fast_ibc;  // RN(1 / (sqrt(bias_correction2) * neg_step))
    float fast_eps;  // RN(eps / neg_step)
    int decoupled;
    int fast_g0;     // g = 0 updates with v_sqrt / v_rcp (ttamm.h TTAMM_G0_FAST)
    // torch.optim.SGD instead (ttamm.h TTAMM_DENSE_SGD): m holds the momentum buffer, v aliases it
    int sgd;
    float sgd_neg_lr;  // -lr
    float sgd_mom;     // momentum
    float sgd_damp1;   // 1 - dampening
    int sgd_first;     // no buffer yet: buf = grad
    int sgd_nesterov;
};
struct SparseConsts {
    float w1;        // 1 - beta1
    float w2;        // 1 - beta2
    float eps;
    float neg_step;  // -lr * sqrt(bias_correction2) / bias_correction1
};

struct RowUpdateArgs {
    int64_t n;              // rows in the tower batch (upper bound of unique count)
    int dim;
    const int32_t* n_unique;
    const int32_t* seg_start;
    const int32_t* keys;    // keys grouped by row (CoalesceWs keys_out)
    const int32_t* rows;    // tower row ids, grouped by table row (CoalesceWs vals_out)
    const int32_t* seglong; // CoalesceWs seglong: the slot's row has > kCoalescePiece contributions
    // ID table gradient source: dE[row] (ld)
    const float* dE;
    int64_t ld_dE;
    ttamm_table id;
    // mimic table gradient source: row < split_row ? dA_lo[row] : dA_hi[row]
    const float* dA_lo;
    const float* dA_hi;
    int64_t ld_dA;
    int64_t split_row;
    // compact exchange (sharded item owner, GateTower::xu): row r's mimic gradient at
    // dA_lo + xu[r] ld_dA for a positive (xu >= 0), at dA_hi + ~xu[r] ld_dA (its dT) for a negative
    const int64_t* xu;
    ttamm_table mimic;
    // per-position partial sums of the segmented reduction [n, dim]
    float* piece_e;
    float* piece_a;
    // dense-optimized tables stage their touched rows in side buffers [n, 3, dim] (p, m, v)
    float* side_id;
    float* side_mimic;
    SparseConsts sp;
    AdamConsts ad;
    int32_t dense_step;     // deferred mode (table.last_step): rows are updated in place and
                            // stamped current to this step
    const uint32_t* status; // step_poisoned(status): no write (ttamm.h TTAMM_STATUS_*)
    const float* grad_scale; // clip_grad_norm_ coefficient on the device (null: 1)
    int lanes_per_row;      // set by the launcher
};
int launch_row_update(const RowUpdateArgs& a, hipStream_t s);
// clip_grad_norm_ (training.py:824-825): sums of squares of the step's gradients into partials
// (the tables' per-row gradient sums, and the dense tensors), then the clip coefficient
// min(max_norm / (sqrt(sum) + 1e-6), 1) into *coef.  Fixed-order reductions.
int rows_sumsq_blocks(int64_t n, int dim);
int launch_rows_sumsq(const RowUpdateArgs& a, float* partials, hipStream_t s);

// ---- deferred exact AdamW(g = 0) (ttamm.h ttamm_table.last_step) ------------------------
// history[t % cap] holds the fp32 constants of dense step t; a row current to step l that is
// brought to step T replays adam_elem(g = 0) with history[l+1 .. T] — the same operations the
// eager sweep would have applied, so the bits agree.
constexpr int kMaxAdamHistory = 512;
// First kernel of a step that may write state: unless the status word is poisoned, count the
// step in *applied (may be null) and store its constants in hist[step % cap] (hist may be null).
int launch_step_begin(const uint32_t* status, int64_t* applied, AdamConsts* hist, int cap, int64_t step,
                      const AdamConsts& c, hipStream_t s);
struct ReplaySeg {
    float* p;
    float* m;
    float* v;
    int32_t* last;
    const uint8_t* touched;  // ttamm_table.touched: 0 = never given a gradient (m = v = +0), or null
    int dim;
    // rows [row_lo, row_hi), each from its own last[row] ...
    int64_t row_lo, row_hi;
    // ... or a catch-up list (list_rows != null, launch_catchup_list): list_cnt[0] rows, row r =
    // list_rows[r] replayed from target - list_lag[r] (rows grouped by lag, longest first, so the
    // threads of a wave share one trip count; `last` is not read — the build stamped it)
    const int32_t* list_rows;
    const int32_t* list_lag;
    const int32_t* list_cnt;
};
constexpr int kMaxReplaySegs = 4;
struct ReplayArgs {
    ReplaySeg seg[kMaxReplaySegs];
    int count;
    const AdamConsts* hist;
    int cap;
    int32_t target;   // replay every row up to this dense step
    int stamp;        // row ranges: write last = target afterwards; 2: atomicMax (a concurrent
                      // row update may have moved a row past target)
    int decoupled;    // AdamW (decoupled weight decay) vs Adam (L2): the optimizer's, every step
    int fast_g0;      // TTAMM_G0_FAST arithmetic
    int sgd;          // torch.optim.SGD (ttamm.h TTAMM_DENSE_SGD): sgd_elem(g = 0) per step
    const uint32_t* status;  // poisoned: no write (null for the flush)
};
// ev (optional, 2 hipEvent_t): recorded around the replay kernel itself (not the stamp)
int launch_replay(const ReplayArgs& a, hipStream_t s, void* const* ev = nullptr);

// Catch-up list of a tower batch (deferred AdamW): the rows of idx[0, n) at their first
// position (first[row] == INT_MAX - p, CoalesceWs.first after the count pass) whose
// last[0][row] < target, grouped by lag = target - last (longest lag first), and each such
// row stamped current (last[t][row] = target for the nlast tables: the dense-group tables of
// one tower are replayed, stamped and updated together, so their last arrays agree).
// cnt / fill: [cap + 1] ints, zeroed by the launcher; rows / lag: [n].
struct CatchupList {
    int32_t* cnt;   // [cap + 1]: [0] = rows listed, [b] = rows of lag b
    int32_t* fill;  // [cap + 1]
    int32_t* rows;  // [n]
    int32_t* lag;   // [n]
};
size_t catchup_list_ints(int64_t n, int cap);  // workspace of one list
void catchup_bind(CatchupList& cl, int32_t* ints, int64_t n, int cap);
int launch_catchup_list(const int64_t* idx, int64_t n, const int32_t* first, int32_t* const* last, int nlast,
                        int32_t target, int cap, const CatchupList& cl, const uint32_t* status, hipStream_t s);

// Part A of both towers' step prologue in three launches: the coalesce count of each tower's
// batch (as launch_coalesce_count; it also zeroes the tower's catch-up list counters), then —
// for towers with a list (list_cnt != null: deferred dense-group tables) — the catch-up list
// (as launch_catchup_list, cnt / fill = list_cnt[0 .. cap], list_cnt[cap + 1 .. 2 cap + 1]).
struct PrepSeg {
    const int64_t* idx;
    int64_t n;
    int32_t* cnt;    // CoalesceWs cnt / first
    int32_t* first;
    int32_t* list_cnt;  // CatchupList cnt (fill follows it) or null
    int32_t* list_rows;
    int32_t* list_lag;
    int32_t* last[2];
    int nlast;
};
struct PrepSegs {
    PrepSeg seg[2];
    int count;
    int32_t target;
    int cap;
    const uint32_t* status;
};
int launch_prepare_segs(const PrepSegs& a, hipStream_t s);

struct SweepSeg {
    float* p;
    float* m;
    float* v;
    int64_t n;  // elements
};
constexpr int kMaxSweepSegs = 4;
struct SweepArgs {
    SweepSeg seg[kMaxSweepSegs];
    int count;
    AdamConsts ad;
    const uint32_t* status;
};
// AdamW with g = 0 over whole tables (adam.py:419-547 for rows the batch did not touch)
int launch_dense_sweep(const SweepArgs& a, hipStream_t s);
// write back side-buffer rows: table[key[u]] = side[u]
int launch_side_scatter(const int32_t* n_unique, const int32_t* keys, const int32_t* seg_start,
                        const float* side, int64_t n, int dim, ttamm_table t, const uint32_t* status,
                        hipStream_t s);

struct DenseTensor {
    float* p;
    float* m;
    float* v;
    const float* g;
    int64_t n;
};
constexpr int kMaxDenseTensors = 2 * (2 * TTAMM_MAX_LINEAR + 4);  // both towers: each Linear weight + bias
struct DenseAdamArgs {
    DenseTensor t[kMaxDenseTensors];
    int count;
    AdamConsts ad;
    const uint32_t* status;
    const float* grad_scale;  // clip_grad_norm_ coefficient on the device (null: 1)
};
int launch_dense_adam(const DenseAdamArgs& a, hipStream_t s);
constexpr int kDenseSumsqBlocks = 256;
int launch_dense_sumsq(const DenseAdamArgs& a, float* partials, hipStream_t s);
int launch_clip_coef(const float* partials, int n, float max_norm, float* coef, hipStream_t s);
// *out = (float) sum of partials[0, n) in double, fixed order (one block)
int launch_sum_partials(const float* partials, int n, float* out, hipStream_t s);

int launch_sparse_adam_rows(float* w, float* m, float* v, int dim, const int64_t* rows,
                            const float* grad, int64_t n, SparseConsts sp, hipStream_t s);

float correctly_rounded_reciprocal(float c);  // RN(1/c), c > 0 normal
AdamConsts make_adam_consts(double lr, double beta1, double beta2, double eps, double wd,
                            int decoupled, int64_t step);
// torch.optim.SGD (training.py:1324-1330): first = the momentum buffers do not exist yet
AdamConsts make_sgd_consts(double lr, double wd, double momentum, double dampening, int nesterov, int first);
SparseConsts make_sparse_consts(double lr, double beta1, double beta2, double eps, int64_t step);

// ------------------------------------------------------------------------------------
// Sampler (sampler.hip)
// ------------------------------------------------------------------------------------
// slot_base: global index of this batch's first slot (row_base * num_neg) — the Philox stream key
int launch_sample_negatives(const int64_t* users, int64_t batch, int num_neg, int64_t num_items,
                            const int64_t* pos_offsets, const int64_t* pos_values, int64_t user_rows, uint64_t seed,
                            uint64_t counter, int64_t slot_base, int64_t* out, int64_t* out2, uint32_t* status,
                            hipStream_t s);  // out2: optional second copy

// The step's prologue in one launch: staging (StageArgs), the negative sampler (when num_neg > 0;
// as launch_sample_negatives, users = the RAW batch ids, range-checked against user_rows) and,
// by the last block, launch_step_begin's work.  done: a uint32 in the zeroed workspace.
// the first feature layer's weight in the layout its GEMM reads (rows padded to 16 B, or rounded
// to bf16 and padded to a multiple of 8), formed in the step prologue's launch (it changes every
// step: the dense optimizer), not in launches of their own ahead of the GEMM
struct WeightPrep {
    const float* src;
    int64_t rows;
    int cols;
    int64_t ld_src;
    void* dst;       // float (bf16 == 0) or uint16 (bf16 == 1)
    int64_t ld_dst;  // elements
    int bf16;
};
constexpr int kMaxWeightPrep = 2;
struct PrologueArgs {
    WeightPrep prep[kMaxWeightPrep];
    int n_prep;
    const int64_t* users;
    int64_t user_rows;
    int64_t batch;
    int num_neg;
    uint64_t num_items;
    const int64_t* pos_offsets;
    const int64_t* pos_values;
    uint32_t k0, k1;
    uint64_t counter;
    int64_t slot_base;
    int64_t* out;
    int64_t* out2;
    uint32_t* done;
    int64_t* applied;
    AdamConsts* hist;
    int cap;
    int64_t step;
    AdamConsts c;
};
int launch_step_prologue(const StageArgs& st, const PrologueArgs& pa, hipStream_t s);

}  // namespace ttamm
