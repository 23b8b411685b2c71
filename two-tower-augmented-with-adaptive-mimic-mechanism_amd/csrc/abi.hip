// extern "C" surface of libttamm.so (declared in include/ttamm.h).
#include <cstdio>
#include <cstring>

#include <vector>

#include <algorithm>

#include "kernels.h"

namespace ttamm {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

size_t train_step_workspace_size(const ttamm_step_args& A);
int train_step(const ttamm_step_args& A, hipStream_t s);
int64_t dense_grad_floats(const ttamm_step_args& A);
int exchange_compact_supported(const ttamm_step_args& A);
int flush_tables(const ttamm_step_args& A, hipStream_t s);
size_t tower_forward_workspace_size(const ttamm_tower& T, int64_t n);
int tower_forward_eval(const ttamm_tower& T, const int64_t* idx, const int64_t* fidx, int64_t n, int augment,
                       float* out, void* ws, size_t ws_bytes, hipStream_t s);
size_t tower_grad_floats_of(const ttamm_tower& T);
size_t tower_train_workspace_size(const ttamm_tower& T, int64_t n);
int tower_train_forward(const ttamm_tower& T, const int64_t* idx, const int64_t* fidx, int64_t n,
                        const uint8_t* const* keep_masks, uint64_t seed, uint64_t counter, float* out, void* ws,
                        size_t ws_bytes, hipStream_t s);
int tower_train_backward(const ttamm_tower& T, const int64_t* idx, const int64_t* fidx, int64_t n,
                         const uint8_t* const* keep_masks, const float* d_out, float* grad_arena, float* d_id_rows,
                         float* d_feat_rows, void* ws, size_t ws_bytes, hipStream_t s);

}  // namespace ttamm

using namespace ttamm;

#define TTAMM_API extern "C" __attribute__((visibility("default")))

TTAMM_API int ttamm_abi_version(void) { return TTAMM_ABI_VERSION; }

TTAMM_API const char* ttamm_last_error(void) { return g_last_error.c_str(); }

TTAMM_API int ttamm_developer_build(void) { return kDevKnobs ? 1 : 0; }

TTAMM_API size_t ttamm_train_step_workspace_size(const ttamm_step_args* args) {
    if (!args) return 0;
    return train_step_workspace_size(*args);
}

TTAMM_API int64_t ttamm_dense_grad_floats(const ttamm_step_args* args) {
    if (!args) return 0;
    return dense_grad_floats(*args);
}

TTAMM_API int ttamm_exchange_compact_supported(const ttamm_step_args* args) {
    return args ? exchange_compact_supported(*args) : 0;
}

TTAMM_API size_t ttamm_adam_history_entry_bytes(void) { return sizeof(AdamConsts); }

TTAMM_API int ttamm_flush_tables(const ttamm_step_args* args, void* stream) {
    if (!args) return fail(TTAMM_E_INVALID, "null step args");
    g_last_error.clear();
    return flush_tables(*args, (hipStream_t)stream);
}

TTAMM_API size_t ttamm_retrieval_topk_workspace_size(int64_t n_queries, int64_t n_items, int32_t dim, int32_t k) {
    return retrieval_workspace_bytes(n_queries, n_items, dim, k);
}

TTAMM_API int ttamm_retrieval_topk(const float* queries, int64_t n_queries, int64_t ldq, const float* items,
                                   int64_t n_items, int64_t ldi, int32_t dim, const int64_t* blocked_offsets,
                                   const int64_t* blocked_values, int32_t k, float* out_scores, int64_t* out_ids,
                                   void* workspace, size_t workspace_bytes, void* stream) {
    g_last_error.clear();
    return launch_retrieval_topk(queries, n_queries, ldq, items, n_items, ldi, dim, blocked_offsets, blocked_values, k,
                                 out_scores, out_ids, workspace, workspace_bytes, (hipStream_t)stream);
}

TTAMM_API int ttamm_candidate_topk(const float* queries, int64_t n_queries, int64_t ldq, const float* items,
                                   int64_t n_items, int64_t ldi, int32_t dim, const int64_t* cand_offsets,
                                   const int64_t* cand_rows, int32_t max_candidates, int32_t cosine, int32_t k,
                                   float* out_scores, int64_t* out_positions, void* stream) {
    g_last_error.clear();
    return launch_candidate_topk(queries, n_queries, ldq, items, n_items, ldi, dim, cand_offsets, cand_rows,
                                 max_candidates, cosine, k, out_scores, out_positions, (hipStream_t)stream);
}

TTAMM_API int ttamm_to_bf16(const float* src, int64_t rows, int32_t cols, int64_t ld_src, uint16_t* dst,
                            int64_t ld_dst, void* stream) {
    g_last_error.clear();
    return launch_to_bf16(src, rows, cols, ld_src, dst, ld_dst, (hipStream_t)stream);
}

TTAMM_API int ttamm_to_planes(const float* src, int64_t rows, int32_t cols, int64_t ld_src, uint16_t* dst,
                              int64_t ld_dst, void* stream) {
    g_last_error.clear();
    return launch_to_planes(src, rows, cols, ld_src, dst, ld_dst, (hipStream_t)stream);
}

TTAMM_API int ttamm_epoch_batch(const int64_t* users, const int64_t* items, int64_t n, uint64_t seed, int64_t epoch,
                                int32_t shuffle, int64_t start, int64_t count, int64_t* out_users, int64_t* out_items,
                                void* stream) {
    g_last_error.clear();
    return launch_epoch_batch(users, items, n, seed, epoch, shuffle, start, count, out_users, out_items,
                              (hipStream_t)stream);
}

TTAMM_API size_t ttamm_route_scratch_bytes(int64_t n, int32_t world) { return route_scratch_bytes(n, world); }

TTAMM_API int ttamm_route_rows(const int64_t* id0, int64_t n0, const int64_t* id1, int64_t n1, const int64_t* payload,
                               int64_t key0, int64_t key1, int32_t world, int64_t* packed, int64_t* slot,
                               int64_t* counts, int64_t counts_ld, const uint32_t* status, void* scratch,
                               size_t scratch_bytes, void* stream) {
    g_last_error.clear();
    return launch_route_rows(id0, n0, id1, n1, payload, key0, key1, world, packed, slot, counts, counts_ld, status,
                             scratch, scratch_bytes, (hipStream_t)stream);
}

TTAMM_API int ttamm_stream_create_cu_limited(int32_t num_cus, void** stream) {
    g_last_error.clear();
    if (!stream) return fail(TTAMM_E_INVALID, "stream: null output pointer");
    int dev = 0, cus = 0;
    TTAMM_HIP(hipGetDevice(&dev));
    TTAMM_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    hipStream_t s = nullptr;
    if (num_cus <= 0 || num_cus >= cus) {
        TTAMM_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    } else {
        std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0u);
        for (int i = 0; i < num_cus; ++i) {
            const int cu = (int)((int64_t)i * cus / num_cus);
            mask[(size_t)cu / 32] |= 1u << (cu % 32);
        }
        TTAMM_HIP(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
    }
    *stream = s;
    return TTAMM_OK;
}

TTAMM_API int ttamm_stream_destroy(void* stream) {
    g_last_error.clear();
    if (stream) TTAMM_HIP(hipStreamDestroy((hipStream_t)stream));
    return TTAMM_OK;
}

TTAMM_API int ttamm_normalize_rows(float* rows, int64_t n, int32_t dim, int64_t ld, void* stream) {
    g_last_error.clear();
    return launch_normalize_rows(rows, n, dim, ld, (hipStream_t)stream);
}

TTAMM_API int ttamm_train_step(const ttamm_step_args* args, void* stream) {
    if (!args) return fail(TTAMM_E_INVALID, "null step args");
    g_last_error.clear();
    return train_step(*args, (hipStream_t)stream);
}

TTAMM_API int ttamm_gather_rows(const float* table, int64_t table_rows, int32_t dim, const int64_t* idx, int64_t n,
                                float* out, int64_t out_ld, void* stream) {
    if (n < 0 || dim <= 0 || out_ld < dim || table_rows <= 0) return fail(TTAMM_E_INVALID, "gather_rows: bad shape");
    return launch_gather_rows(table, table_rows, dim, idx, n, out, out_ld, (hipStream_t)stream);
}

TTAMM_API size_t ttamm_tower_forward_workspace_size(const ttamm_tower* tower, int64_t n) {
    if (!tower) return 0;
    return tower_forward_workspace_size(*tower, n);
}

TTAMM_API int ttamm_tower_forward(const ttamm_tower* tower, const int64_t* idx, const int64_t* feat_idx, int64_t n,
                                  int32_t augment, float* out, void* workspace, size_t workspace_bytes, void* stream) {
    if (!tower) return fail(TTAMM_E_INVALID, "null tower");
    return tower_forward_eval(*tower, idx, feat_idx, n, augment, out, workspace, workspace_bytes, (hipStream_t)stream);
}

TTAMM_API size_t ttamm_tower_grad_floats(const ttamm_tower* tower) { return tower ? tower_grad_floats_of(*tower) : 0; }

TTAMM_API size_t ttamm_tower_train_workspace_size(const ttamm_tower* tower, int64_t n) {
    return tower ? tower_train_workspace_size(*tower, n) : 0;
}

TTAMM_API int ttamm_tower_train_forward(const ttamm_tower* tower, const int64_t* idx, const int64_t* feat_idx,
                                        int64_t n, const uint8_t* const* keep_masks, uint64_t seed, uint64_t counter,
                                        float* out, void* workspace, size_t workspace_bytes, void* stream) {
    if (!tower || (n > 0 && (!idx || !out || !workspace))) return fail(TTAMM_E_INVALID, "tower train forward: null argument");
    g_last_error.clear();
    return tower_train_forward(*tower, idx, feat_idx, n, keep_masks, seed, counter, out, workspace, workspace_bytes,
                               (hipStream_t)stream);
}

TTAMM_API int ttamm_tower_train_backward(const ttamm_tower* tower, const int64_t* idx, const int64_t* feat_idx,
                                         int64_t n, const uint8_t* const* keep_masks, const float* d_out,
                                         float* grad_arena, float* d_id_rows, float* d_feat_rows, void* workspace,
                                         size_t workspace_bytes, void* stream) {
    if (!tower || (n > 0 && (!idx || !workspace))) return fail(TTAMM_E_INVALID, "tower train backward: null argument");
    g_last_error.clear();
    return tower_train_backward(*tower, idx, feat_idx, n, keep_masks, d_out, grad_arena, d_id_rows, d_feat_rows,
                                workspace, workspace_bytes, (hipStream_t)stream);
}

TTAMM_API int ttamm_scatter_add_rows(float* dst, int64_t dst_rows, int32_t dim, const int64_t* idx, int64_t n,
                                     const float* x, int64_t ldx, const float* y, int64_t ldy, const float* scale_dev,
                                     float scale, int64_t skip_row, void* stream) {
    if (n > 0 && (!dst || !x || dim <= 0 || ldx < dim || (y && ldy < dim) || dst_rows <= 0 || (!idx && n > dst_rows)))
        return fail(TTAMM_E_INVALID, "scatter_add_rows: bad arguments");
    g_last_error.clear();
    return launch_scatter_add_rows(dst, dst_rows, dim, idx, n, x, ldx, y, ldy, scale_dev, scale, skip_row,
                                   (hipStream_t)stream);
}

TTAMM_API size_t ttamm_coalesce_workspace_bytes(int64_t n, int64_t table_rows) {
    if (n < 0 || table_rows <= 0) return 0;
    const size_t tiles = (size_t)std::max<int64_t>(n, 257);
    return sizeof(int32_t) * (coalesce_scratch_ints(table_rows) + 2 * (size_t)n + 2 * tiles);
}

TTAMM_API int ttamm_coalesce_rows(const int64_t* idx, int64_t n, int64_t table_rows, int32_t sorted, int32_t* keys_out,
                                  int32_t* positions_out, int32_t* seg_start_out, int32_t* n_unique_out,
                                  void* workspace, size_t workspace_bytes, void* stream) {
    if (n < 0 || table_rows <= 0 || !n_unique_out || !seg_start_out || (n > 0 && (!idx || !keys_out || !positions_out)) ||
        !workspace || workspace_bytes < ttamm_coalesce_workspace_bytes(n, table_rows))
        return fail(TTAMM_E_INVALID, "coalesce_rows: bad arguments");
    g_last_error.clear();
    CoalesceWs co{};
    int32_t* w = static_cast<int32_t*>(workspace);
    coalesce_bind_scratch(co, w, table_rows);
    w += coalesce_scratch_ints(table_rows);
    co.vals_tmp = w;
    w += n;
    co.lead = w;
    w += n;
    co.lead_cnt = w;
    w += std::max<int64_t>(n, 257);
    co.seglong = w;
    co.keys_out = keys_out;
    co.vals_out = positions_out;
    co.seg_start = seg_start_out;
    co.n_unique = n_unique_out;
    co.sorted = sorted ? 1 : 0;
    return launch_coalesce(idx, n, table_rows, co, (hipStream_t)stream);
}

TTAMM_API int ttamm_mimic_augment(const float* table, int64_t table_rows, int32_t dim, const int64_t* idx, int64_t n,
                                  const float* base, float* out, float* aug_out, void* stream) {
    if (n < 0 || dim <= 0 || table_rows <= 0) return fail(TTAMM_E_INVALID, "mimic_augment: bad shape");
    return launch_combine(base, dim, nullptr, 0, table, table_rows, idx, n, dim, nullptr, aug_out, dim, out, (hipStream_t)stream);
}

TTAMM_API int ttamm_mse_loss(const float* input, const float* target, int64_t n, float* out, void* stream) {
    return launch_mse(input, target, n, out, (hipStream_t)stream);
}

TTAMM_API int ttamm_sample_negatives(const int64_t* users, int64_t batch, int32_t num_neg, int64_t num_items,
                                     const int64_t* pos_offsets, const int64_t* pos_values, int64_t user_rows,
                                     uint64_t seed, uint64_t counter, int64_t slot_base, int64_t* out,
                                     uint32_t* status, void* stream) {
    g_last_error.clear();
    if (batch < 0 || (batch > 0 && (!users || !out || !status)) || (pos_offsets && user_rows <= 0))
        return fail(TTAMM_E_INVALID, "sample_negatives: bad arguments");
    return launch_sample_negatives(users, batch, num_neg, num_items, pos_offsets, pos_values, user_rows, seed, counter,
                                   slot_base, out, nullptr, status, (hipStream_t)stream);
}

TTAMM_API int ttamm_check_rows(const int64_t* ids0, int64_t n0, int64_t rows0, const int64_t* ids1, int64_t n1,
                               int64_t rows1, uint32_t* status, void* stream) {
    g_last_error.clear();
    if (!status || n0 < 0 || n1 < 0 || (n0 > 0 && !ids0) || (n1 > 0 && !ids1))
        return fail(TTAMM_E_INVALID, "check_rows: bad arguments");
    StageArgs st;
    std::memset(&st, 0, sizeof(st));
    st.status = status;
    if (n0 > 0) st.seg[st.count++] = StageSeg{ids0, nullptr, n0, rows0, 1};
    if (n1 > 0) st.seg[st.count++] = StageSeg{ids1, nullptr, n1, rows1, 1};
    return launch_stage_rows(st, (hipStream_t)stream);
}

TTAMM_API int ttamm_sparse_adam_rows(float* weight, float* exp_avg, float* exp_avg_sq, int32_t dim,
                                     const int64_t* rows, const float* grad, int64_t n_rows, double lr, double beta1,
                                     double beta2, double eps, int64_t step, void* stream) {
    if (step < 1 || dim <= 0 || n_rows < 0) return fail(TTAMM_E_INVALID, "sparse_adam_rows: bad arguments");
    const SparseConsts c = make_sparse_consts(lr, beta1, beta2, eps, step);
    return launch_sparse_adam_rows(weight, exp_avg, exp_avg_sq, dim, rows, grad, n_rows, c, (hipStream_t)stream);
}

TTAMM_API int ttamm_adamw_dense(float* param, float* exp_avg, float* exp_avg_sq, const float* grad, int64_t n,
                                double lr, double beta1, double beta2, double eps, double weight_decay,
                                int32_t decoupled, int64_t step, void* stream) {
    if (step < 1 || n < 0) return fail(TTAMM_E_INVALID, "adamw_dense: bad arguments");
    DenseAdamArgs a;
    std::memset(&a, 0, sizeof(a));
    a.count = 1;
    a.t[0] = DenseTensor{param, exp_avg, exp_avg_sq, grad, n};
    a.ad = make_adam_consts(lr, beta1, beta2, eps, weight_decay, decoupled, step);
    return launch_dense_adam(a, (hipStream_t)stream);
}

TTAMM_API size_t ttamm_inbatch_workspace_size(int64_t batch, int64_t n_positives, int32_t dim) {
    if (batch <= 0 || n_positives <= 0 || dim <= 0) return 0;
    return inbatch_standalone_workspace_bytes(batch, n_positives, dim);
}

TTAMM_API int ttamm_inbatch_bce(const float* users, int64_t batch, int64_t ldu, const float* positives,
                                int64_t n_positives, int64_t ldp, int32_t dim, int64_t row_base, float inv_count,
                                float* d_users, int64_t ld_du, float* d_positives, int64_t ld_dp, double* loss_sum,
                                void* workspace, size_t workspace_bytes, void* stream) {
    g_last_error.clear();
    return inbatch_standalone(users, batch, ldu, positives, n_positives, ldp, dim, row_base, inv_count, d_users,
                              ld_du, d_positives, ld_dp, loss_sum, workspace, workspace_bytes, (hipStream_t)stream);
}
