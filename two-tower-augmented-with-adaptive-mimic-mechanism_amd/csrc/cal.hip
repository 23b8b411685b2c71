// Category-alignment loss and its gradient:
//   _category_alignment_loss (training.py:541-579), applied at training.py:805-820 to the
//   batch's augmented item embeddings cat[positives; negatives] with weight
//   loss_weights.category_alignment.
//
//   cov(X)  = (X - mean X)^T (X - mean X) / (n - 1)                       (training.py:530-538)
//   L_cal   = sum_{c != major, n_c >= 2} ||cov_c - cov_major||_F^2 / compared   (ascending c)
//   L_cal   = 0 when the batch has <= 1 category, < 2 rows of the major category, or no
//             other category with >= 2 rows.
//   dL/dX_c = 2/(n_c - 1) * (X_c - mean) G_c,  G_c = 2 (cov_c - cov_major) / compared,
//             G_major = -sum_c G_c                     (cov is symmetric, so G + G^T = 2G)
//
// The reference loops over categories in Python with host syncs.  Here the rows are sorted by
// category (the coalesce machinery of optim.hip), each category's rows are cut into pieces of
// at most kPiece rows, and every reduction runs in a fixed order (pieces in row order,
// categories ascending), so the result is deterministic:
//   piece sums -> means -> piece centered scatter tiles (64 x 64 per block) -> covariances ->
//   per-category squared distances -> loss -> G_major -> per-row gradients added into the
//   item rows' dT (and dA for positives: the augmented embedding is t + a).
//
// Row-sharded step (slot space = category ids, CalArgs::gstats set): the global batch is the
// union of the ranks' request rows, so the statistics are global and only the rows are local:
//   CAL_STATS   local piece sums -> gstats[c] = (sum of c's rows | count)    [all-reduce]
//   CAL_SCATTER global means -> local centered scatter of c's rows -> gscat[c] [all-reduce]
//   SCORE       cov_c = gscat[c] / (n_c - 1) in place, distances, L_cal, G, and the gradients of
//               this rank's rows (global n_c and means), added into its (dT | dA) exchange rows.
// Every rank computes the same loss and G from the same all-reduced sums.
#include "kernels.h"

namespace ttamm {

namespace {

constexpr int kPiece = 256;  // rows per piece
constexpr int kTile = 64;    // covariance entries per block side
constexpr int kRowsStage = 32;

// the category segment that piece p belongs to: last u with pstart[u] <= p (u < nseg)
__device__ __forceinline__ int piece_segment(const CalArgs& A, int p, int nseg) {
    int lo = 0, hi = nseg - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (A.pstart[mid] <= p) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

__device__ __forceinline__ int total_pieces(const CalArgs& A) {
    const int last = A.nseg_max - 1;
    return A.pstart[last] + A.pcount[last];
}

// catrow[r] = category of item row r (rows [split, R) from idx1 when given; an id outside
// [0, idx_rows) — a poisoned step writes nothing — reads item 0's category)
__global__ void cal_rows_kernel(CalArgs A) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= A.R) return;
    int64_t id = A.idx1 && r >= A.split ? A.idx1[r - A.split] : A.idx[r];
    if (id < 0 || id >= A.idx_rows) id = 0;
    int64_t c = A.categories[id];
    c = c < 0 ? 0 : (c >= A.num_categories ? A.num_categories - 1 : c);
    A.catrow[r] = c;
}

// pieces per segment (0 past the unique count)
__global__ void cal_plan_kernel(CalArgs A) {
    const int u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= A.nseg_max) return;
    const int nu = A.co.n_unique[0];
    int cnt = 0;
    if (u < nu) cnt = (A.co.seg_start[u + 1] - A.co.seg_start[u] + kPiece - 1) / kPiece;
    A.pcount[u] = cnt;
}

__device__ __forceinline__ bool piece_rows(const CalArgs& A, int p, int& u, int& k0, int& k1) {
    if (p >= total_pieces(A)) return false;
    const int nu = A.co.n_unique[0];
    u = piece_segment(A, p, nu);
    k0 = A.co.seg_start[u] + (p - A.pstart[u]) * kPiece;
    k1 = min(k0 + kPiece, A.co.seg_start[u + 1]);
    return true;
}

__device__ __forceinline__ int seg_len(const CalArgs& A, int u) { return A.co.seg_start[u + 1] - A.co.seg_start[u]; }

// the category of local segment u (segment keys are the rows' categories)
__device__ __forceinline__ int64_t seg_cat(const CalArgs& A, int u) { return A.co.keys_out[A.co.seg_start[u]]; }

// slot space: local segments (one process) or category ids (sharded, gstats set)
__device__ __forceinline__ int slot_of(const CalArgs& A, int u) { return A.gstats ? (int)seg_cat(A, u) : u; }

__device__ __forceinline__ int slot_count(const CalArgs& A, int q) {
    if (A.gstats) return (int)A.gstats[(int64_t)q * (A.D + 1) + A.D];
    return q < A.co.n_unique[0] ? seg_len(A, q) : 0;
}

// the exchange-buffer row of request row j
__device__ __forceinline__ int64_t buf_row(const CalArgs& A, int64_t j) { return A.slot ? A.slot[j] : j; }

// element col of sorted row k: x (+ xa, the mimic rows of the sharded exchange buffer)
__device__ __forceinline__ float row_val(const CalArgs& A, int k, int col) {
    const int64_t j = A.co.vals_out[k];
    const int64_t o = buf_row(A, j) * A.ld_x + col;
    return A.xa && j < A.xa_rows ? A.x[o] + A.xa[o] : A.x[o];
}

// psum[p][d] = sum of the piece's rows (row order)
__global__ void cal_piece_sum_kernel(CalArgs A) {
    int u, k0, k1;
    if (!piece_rows(A, blockIdx.x, u, k0, k1)) return;
    if (!A.gstats && seg_len(A, u) < 2) return;
    for (int d = threadIdx.x; d < A.D; d += blockDim.x) {
        float s = 0.f;
        for (int k = k0; k < k1; ++k) s += row_val(A, k, d);
        A.psum[(int64_t)blockIdx.x * A.D + d] = s;
    }
}

// mean[u][d] = (sum of u's piece sums, piece order) / n_u
__global__ void cal_mean_kernel(CalArgs A) {
    const int u = blockIdx.x;
    if (u >= A.co.n_unique[0]) return;
    const int n = seg_len(A, u);
    if (n < 2) return;
    const int q0 = A.pstart[u], q1 = q0 + A.pcount[u];
    for (int d = threadIdx.x; d < A.D; d += blockDim.x) {
        float s = 0.f;
        for (int q = q0; q < q1; ++q) s += A.psum[(int64_t)q * A.D + d];
        A.mean[(int64_t)u * A.D + d] = s / (float)n;
    }
}

// sharded: gstats[c] = (sum of the segment's piece sums, piece order | row count); the buffer is
// zeroed first, categories absent here stay 0 for the all-reduce
__global__ void cal_stats_kernel(CalArgs A) {
    const int u = blockIdx.x;
    if (u >= A.co.n_unique[0]) return;
    const int q0 = A.pstart[u], q1 = q0 + A.pcount[u];
    float* g = A.gstats + seg_cat(A, u) * (A.D + 1);
    for (int d = threadIdx.x; d < A.D; d += blockDim.x) {
        float s = 0.f;
        for (int q = q0; q < q1; ++q) s += A.psum[(int64_t)q * A.D + d];
        g[d] = s;
    }
    if (threadIdx.x == 0) g[A.D] = (float)seg_len(A, u);
}

// sharded: mean[u] = the global mean of segment u's category (all-reduced gstats)
__global__ void cal_gmean_kernel(CalArgs A) {
    const int u = blockIdx.x;
    if (u >= A.co.n_unique[0]) return;
    const float* g = A.gstats + seg_cat(A, u) * (A.D + 1);
    const float n = g[A.D];
    if (n < 2.f) return;
    for (int d = threadIdx.x; d < A.D; d += blockDim.x) A.mean[(int64_t)u * A.D + d] = g[d] / n;
}

// pslab[p][i][j] = sum over the piece's rows of (x_i - mean_i)(x_j - mean_j), one 64 x 64
// tile of (i, j) per block (blockIdx.y); 256 threads x (4 x 4) entries
__global__ __launch_bounds__(256) void cal_piece_scatter_kernel(CalArgs A) {
    __shared__ float xs[kRowsStage][2 * kTile + 4];
    int u, k0, k1;
    if (!piece_rows(A, blockIdx.x, u, k0, k1)) return;
    if (slot_count(A, slot_of(A, u)) < 2) return;
    const int D = A.D;
    const int nt = (D + kTile - 1) / kTile;
    const int I0 = (blockIdx.y / nt) * kTile, J0 = (blockIdx.y % nt) * kTile;
    const int a = threadIdx.x / 16, b = threadIdx.x % 16;
    const float* mu = A.mean + (int64_t)u * D;
    float acc[4][4] = {};
    for (int kb = k0; kb < k1; kb += kRowsStage) {
        const int nr = min(kRowsStage, k1 - kb);
        __syncthreads();
        for (int e = threadIdx.x; e < kRowsStage * 2 * kTile; e += blockDim.x) {
            const int r = e / (2 * kTile), c = e % (2 * kTile);
            const int col = c < kTile ? I0 + c : J0 + (c - kTile);
            float v = 0.f;
            if (r < nr && col < D) v = row_val(A, kb + r, col) - mu[col];
            xs[r][c] = v;
        }
        __syncthreads();
        for (int r = 0; r < nr; ++r) {
            float xi[4], xj[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                xi[q] = xs[r][4 * a + q];
                xj[q] = xs[r][kTile + 4 * b + q];
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int w = 0; w < 4; ++w) acc[q][w] = fmaf(xi[q], xj[w], acc[q][w]);
        }
    }
    float* out = A.pslab + (int64_t)blockIdx.x * D * D;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const int i = I0 + 4 * a + q, j = J0 + 4 * b + w;
            if (i < D && j < D) out[(int64_t)i * D + j] = acc[q][w];
        }
}

// cov[u][e] = (sum of u's piece scatters, piece order) / (n_u - 1)
__global__ void cal_cov_kernel(CalArgs A) {
    const int u = blockIdx.y;
    if (u >= A.co.n_unique[0]) return;
    const int n = seg_len(A, u);
    if (n < 2) return;
    const int64_t DD = (int64_t)A.D * A.D;
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= DD) return;
    const int q0 = A.pstart[u], q1 = q0 + A.pcount[u];
    float s = 0.f;
    for (int q = q0; q < q1; ++q) s += A.pslab[(int64_t)q * DD + e];
    A.cov[u * DD + e] = s / (float)(n - 1);
}

// sharded: gscat[c] = sum of segment u's piece scatters (piece order); zeroed first
__global__ void cal_seg_scatter_kernel(CalArgs A) {
    const int u = blockIdx.y;
    if (u >= A.co.n_unique[0]) return;
    if (slot_count(A, slot_of(A, u)) < 2) return;
    const int64_t DD = (int64_t)A.D * A.D;
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= DD) return;
    const int q0 = A.pstart[u], q1 = q0 + A.pcount[u];
    float s = 0.f;
    for (int q = q0; q < q1; ++q) s += A.pslab[(int64_t)q * DD + e];
    A.cov[seg_cat(A, u) * DD + e] = s;
}

// sharded: cov[c] = gscat[c] / (n_c - 1) in place (all-reduced scatter sums, global counts)
__global__ void cal_cov_dense_kernel(CalArgs A) {
    const int c = blockIdx.y;
    const int n = slot_count(A, c);
    if (n < 2) return;
    const int64_t DD = (int64_t)A.D * A.D;
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= DD) return;
    A.cov[c * DD + e] = A.cov[c * DD + e] / (float)(n - 1);
}

// the slot of the major category, or -1 (keys of the unique segments are ascending)
__device__ int major_segment(const CalArgs& A) {
    if (A.gstats) return slot_count(A, (int)A.major) > 0 ? (int)A.major : -1;
    const int nu = A.co.n_unique[0];
    int lo = 0, hi = nu - 1;
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        const int64_t k = A.co.keys_out[A.co.seg_start[mid]];
        if (k == A.major) return mid;
        if (k < A.major) lo = mid + 1;
        else hi = mid - 1;
    }
    return -1;
}

// the reference's early exits (training.py:552-563): <= 1 category, < 2 major rows (with a
// single category nothing is compared either, so the sharded slot space skips that count)
__device__ bool cal_active(const CalArgs& A, int uM) {
    return (A.gstats || A.co.n_unique[0] > 1) && uM >= 0 && slot_count(A, uM) >= 2;
}

__device__ __forceinline__ int num_slots(const CalArgs& A) { return A.gstats ? (int)A.num_categories : A.nseg_max; }

// part[u] = ||cov_u - cov_major||^2 for every compared category (flag[u] = 1)
__global__ __launch_bounds__(256) void cal_dist_kernel(CalArgs A) {
    __shared__ float red[256];
    const int u = blockIdx.x;
    if (u >= num_slots(A)) return;
    const int uM = major_segment(A);
    const bool on = cal_active(A, uM) && u != uM && slot_count(A, u) >= 2;
    float s = 0.f;
    if (on) {
        const int64_t DD = (int64_t)A.D * A.D;
        const float* cu = A.cov + u * DD;
        const float* cm = A.cov + uM * DD;
        for (int64_t e = threadIdx.x; e < DD; e += blockDim.x) {
            const float d = cu[e] - cm[e];
            s += d * d;
        }
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        A.part[u] = on ? red[0] : 0.f;
        A.flag[u] = on ? 1 : 0;
    }
}

// out[0] = L_cal, out[1] = compared (categories ascending, as the reference's loop)
__global__ void cal_loss_kernel(CalArgs A) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    float loss = 0.f;
    int compared = 0;
    for (int u = 0; u < num_slots(A); ++u)
        if (A.flag[u]) {
            loss = loss + A.part[u];
            ++compared;
        }
    A.out[0] = compared ? loss / (float)compared : 0.f;
    A.out[1] = (float)compared;
}

// G_major[e] = -sum_u 2 (cov_u[e] - cov_major[e]) / compared
__global__ void cal_gmajor_kernel(CalArgs A) {
    const int64_t DD = (int64_t)A.D * A.D;
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= DD) return;
    const int compared = (int)A.out[1];
    if (compared == 0) return;
    const int uM = major_segment(A);
    const float cm = A.cov[uM * DD + e];
    const float scale = 2.0f / (float)compared;
    float g = 0.f;
    for (int u = 0; u < num_slots(A); ++u)
        if (A.flag[u]) g -= scale * (A.cov[u * DD + e] - cm);
    A.gmajor[e] = g;
}

// rows of a compared category or of the major one: dX = lambda * 2/(n-1) * (x - mean) G,
// added into dT (and dA for positive rows).  One kGradCols-column tile of G per block
// (blockIdx.y), staged in LDS with 16 centered rows at a time; 128 threads = 16 rows x 8
// groups of 4 columns.  LDS: (D * kGradCols + 16 * D) floats <= 48 KB at D = 256.
constexpr int kGradCols = 32;
__global__ __launch_bounds__(128) void cal_row_grad_kernel(CalArgs A) {
    extern __shared__ float lds[];
    int u, k0, k1;
    if (!piece_rows(A, blockIdx.x, u, k0, k1)) return;
    const int compared = (int)A.out[1];
    if (compared == 0) return;
    const int uM = major_segment(A);
    const int q = slot_of(A, u);
    if (q != uM && !A.flag[q]) return;
    const int D = A.D;
    const int64_t DD = (int64_t)D * D;
    const int J0 = blockIdx.y * kGradCols;
    float* Gs = lds;                           // [D][kGradCols]
    float* xs = lds + (int64_t)D * kGradCols;  // [16][D]
    const float scale = 2.0f / (float)compared;
    const float* cu = A.cov + q * DD;
    const float* cm = A.cov + uM * DD;
    for (int e = threadIdx.x; e < D * kGradCols; e += blockDim.x) {
        const int i = e / kGradCols, j = J0 + e % kGradCols;
        float g = 0.f;
        if (j < D) g = q == uM ? A.gmajor[(int64_t)i * D + j] : scale * (cu[(int64_t)i * D + j] - cm[(int64_t)i * D + j]);
        Gs[e] = g;
    }
    const float coef = A.lambda * (2.0f / (float)(slot_count(A, q) - 1));
    const float* mu = A.mean + (int64_t)u * D;
    const int rl = threadIdx.x / 8, cg = threadIdx.x % 8;
    for (int kb = k0; kb < k1; kb += 16) {
        const int nr = min(16, k1 - kb);
        __syncthreads();
        for (int e = threadIdx.x; e < 16 * D; e += blockDim.x) {
            const int r = e / D, c = e % D;
            xs[e] = r < nr ? row_val(A, kb + r, c) - mu[c] : 0.f;
        }
        __syncthreads();
        const int col = J0 + 4 * cg;
        if (rl < nr && col < D) {
            float o[4] = {0.f, 0.f, 0.f, 0.f};
            for (int i = 0; i < D; ++i) {
                const float xv = xs[rl * D + i];
#pragma unroll
                for (int w = 0; w < 4; ++w) o[w] = fmaf(xv, Gs[i * kGradCols + 4 * cg + w], o[w]);
            }
            const int64_t j = A.co.vals_out[kb + rl];
            const int64_t row = buf_row(A, j);
            float* dt = A.dT + row * A.ld_d + col;
#pragma unroll
            for (int w = 0; w < 4; ++w) dt[w] += coef * o[w];
            if (A.dA && j < A.dA_rows) {
                float* da = A.dA + row * A.ld_d + col;
#pragma unroll
                for (int w = 0; w < 4; ++w) da[w] += coef * o[w];
            }
        }
    }
}

inline unsigned blocks_for(int64_t n, int t = 256) { return (unsigned)ceil_div(n < 1 ? 1 : n, t); }

}  // namespace

int cal_max_pieces(int64_t R, int64_t nseg_max) { return (int)(ceil_div(R, kPiece) + nseg_max); }
size_t cal_stats_floats(int64_t num_categories, int D) { return (size_t)num_categories * (D + 1); }
size_t cal_scatter_floats(int64_t num_categories, int D) { return (size_t)num_categories * D * D; }

int launch_cal_local(const CalArgs& a, hipStream_t s) {
    TTAMM_REQUIRE(a.D % 4 == 0 && a.D <= 256, "category alignment: embedding dim must be a multiple of 4, <= 256");
    TTAMM_REQUIRE(a.R > 0 && a.nseg_max > 0 && a.nseg_max <= 65535, "category alignment: bad batch / category count");
    int rc;
    hipLaunchKernelGGL(cal_rows_kernel, dim3(blocks_for(a.R)), dim3(256), 0, s, a);
    TTAMM_LAUNCH_CHECK();
    CoalesceWs co = a.co;
    if ((rc = launch_coalesce(a.catrow, a.R, a.num_categories, co, s))) return rc;
    hipLaunchKernelGGL(cal_plan_kernel, dim3(blocks_for(a.nseg_max)), dim3(256), 0, s, a);
    TTAMM_LAUNCH_CHECK();
    if ((rc = launch_block_exclusive_scan(a.pcount, a.pstart, a.nseg_max, s))) return rc;
    const unsigned pieces = (unsigned)cal_max_pieces(a.R, a.nseg_max);
    hipLaunchKernelGGL(cal_piece_sum_kernel, dim3(pieces), dim3(256), 0, s, a);
    TTAMM_LAUNCH_CHECK();
    if (a.gstats) {
        TTAMM_HIP(hipMemsetAsync(a.gstats, 0, sizeof(float) * cal_stats_floats(a.num_categories, a.D), s));
        hipLaunchKernelGGL(cal_stats_kernel, dim3((unsigned)a.nseg_max), dim3(256), 0, s, a);
    } else {
        hipLaunchKernelGGL(cal_mean_kernel, dim3((unsigned)a.nseg_max), dim3(256), 0, s, a);
    }
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int launch_cal_scatter(const CalArgs& a, hipStream_t s) {
    const unsigned pieces = (unsigned)cal_max_pieces(a.R, a.nseg_max);
    const unsigned nt = (unsigned)ceil_div(a.D, kTile);
    const int64_t DD = (int64_t)a.D * a.D;
    if (a.gstats) {
        hipLaunchKernelGGL(cal_gmean_kernel, dim3((unsigned)a.nseg_max), dim3(256), 0, s, a);
        TTAMM_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(cal_piece_scatter_kernel, dim3(pieces, nt * nt), dim3(256), 0, s, a);
    TTAMM_LAUNCH_CHECK();
    if (a.gstats) {
        TTAMM_HIP(hipMemsetAsync(a.cov, 0, sizeof(float) * cal_scatter_floats(a.num_categories, a.D), s));
        hipLaunchKernelGGL(cal_seg_scatter_kernel, dim3(blocks_for(DD), (unsigned)a.nseg_max), dim3(256), 0, s, a);
    } else {
        hipLaunchKernelGGL(cal_cov_kernel, dim3(blocks_for(DD), (unsigned)a.nseg_max), dim3(256), 0, s, a);
    }
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int launch_cal_finish(const CalArgs& a, hipStream_t s) {
    const int64_t DD = (int64_t)a.D * a.D;
    const unsigned slots = (unsigned)(a.gstats ? a.num_categories : a.nseg_max);
    if (a.gstats) {
        hipLaunchKernelGGL(cal_cov_dense_kernel, dim3(blocks_for(DD), slots), dim3(256), 0, s, a);
        TTAMM_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(cal_dist_kernel, dim3(slots), dim3(256), 0, s, a);
    TTAMM_LAUNCH_CHECK();
    hipLaunchKernelGGL(cal_loss_kernel, dim3(1), dim3(64), 0, s, a);
    TTAMM_LAUNCH_CHECK();
    if (a.dT == nullptr) return TTAMM_OK;  // loss only
    hipLaunchKernelGGL(cal_gmajor_kernel, dim3(blocks_for(DD)), dim3(256), 0, s, a);
    TTAMM_LAUNCH_CHECK();
    const unsigned pieces = (unsigned)cal_max_pieces(a.R, a.nseg_max);
    const size_t lds = sizeof(float) * ((size_t)a.D * kGradCols + 16 * (size_t)a.D);
    hipLaunchKernelGGL(cal_row_grad_kernel, dim3(pieces, (unsigned)ceil_div(a.D, kGradCols)), dim3(128), lds, s, a);
    TTAMM_LAUNCH_CHECK();
    return TTAMM_OK;
}

int launch_category_alignment(const CalArgs& a, hipStream_t s) {
    int rc;
    if ((rc = launch_cal_local(a, s))) return rc;
    if ((rc = launch_cal_scatter(a, s))) return rc;
    return launch_cal_finish(a, s);
}

}  // namespace ttamm
