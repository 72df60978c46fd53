// Observation RunningMeanStd for VectorEnvNormObs (tianshou/env/venv_wrappers.py:65-112,
// tianshou/utils/statistics.py:69-114), kept on device.
//
// merge : batch (mean, var) from the env kernel's column partials (f64), then the Chan
//         parallel merge of RunningMeanStd.update, stored back as f32 like the reference.
// norm  : clip((x - mean) / sqrt(var + eps), +-clip) in f32, the reference's exact op order.
#include "tsrl_common.h"

namespace tsrl {
namespace {

constexpr int TPB = 256;

// Column-parallel merge.  Block = 64 columns x 16 partial lanes (1024 threads); every block
// reads the OLD count, and the last block to finish (agent-scope ticket) publishes the new
// count and re-arms the ticket, so no block can observe a half-updated count and the launch
// needs no host-side state (graph-replay safe).
constexpr int MCOLS = 64;
constexpr int MLANES = 16;

__global__ __launch_bounds__(MCOLS * MLANES) void rms_merge_kernel(
    const double* partials, int64_t nblk, int64_t dim, const uint8_t* mask, int64_t k,
    const double* batch_count, float* mean, float* var, double* count, unsigned int* ticket) {
    __shared__ double sh_s[MLANES][MCOLS];
    __shared__ double sh_ss[MLANES][MCOLS];
    __shared__ double sh_cnt[MCOLS * MLANES / kWave];
    const int tid = threadIdx.x;
    const int col = tid % MCOLS;
    const int lane = tid / MCOLS;
    // batch count (mask bytes set, or k)
    double c = 0.0;
    if (mask) {
        for (int64_t r = tid; r < k; r += MCOLS * MLANES) c += mask[r] ? 1.0 : 0.0;
    } else if (tid == 0) {
        c = (double)k;
    }
    c = wave_sum(c);
    if ((tid & (kWave - 1)) == 0) sh_cnt[tid / kWave] = c;
    const double old_count = *count;
    __syncthreads();
    double bc = 0.0;
    for (int w = 0; w < MCOLS * MLANES / kWave; ++w) bc += sh_cnt[w];
    if (batch_count) bc = *batch_count;  // e.g. summed over data-parallel ranks
    const double tot = old_count + bc;
    const int64_t d = (int64_t)blockIdx.x * MCOLS + col;
    double s0 = 0.0, s1 = 0.0, q0 = 0.0, q1 = 0.0;
    if (bc > 0.0 && d < dim) {
        int64_t b = lane;
        for (; b + MLANES < nblk; b += 2 * MLANES) {
            const double2 p0 = *reinterpret_cast<const double2*>(partials + (b * dim + d) * 2);
            const double2 p1 = *reinterpret_cast<const double2*>(
                partials + ((b + MLANES) * dim + d) * 2);
            s0 += p0.x;
            q0 += p0.y;
            s1 += p1.x;
            q1 += p1.y;
        }
        if (b < nblk) {
            const double2 p0 = *reinterpret_cast<const double2*>(partials + (b * dim + d) * 2);
            s0 += p0.x;
            q0 += p0.y;
        }
    }
    sh_s[lane][col] = s0 + s1;
    sh_ss[lane][col] = q0 + q1;
    __syncthreads();
    if (lane == 0 && bc > 0.0 && d < dim) {
        double s = 0.0, ss = 0.0;
        for (int l = 0; l < MLANES; ++l) {
            s += sh_s[l][col];
            ss += sh_ss[l][col];
        }
        const double bm = s / bc;
        double bv = ss / bc - bm * bm;
        bv = bv < 0.0 ? 0.0 : bv;
        const double m0 = (double)mean[d];
        const double v0 = (double)var[d];
        const double delta = bm - m0;
        const double new_mean = m0 + delta * bc / tot;
        const double m2 = v0 * old_count + bv * bc + delta * delta * old_count * bc / tot;
        mean[d] = (float)new_mean;
        var[d] = (float)(m2 / tot);
    }
    if (tid == 0) {
        const unsigned int t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL,
                                                      __HIP_MEMORY_SCOPE_AGENT);
        if (t == gridDim.x - 1) {  // every block has read the old count
            __hip_atomic_store(count, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// Two consecutive RunningMeanStd updates in one launch (VectorEnvNormObs.step's update over
// the step batch, then VectorEnvNormObs.reset's update over the reset rows): P1 covers k rows,
// P2 the rows counted in blk_done (blocks with none are skipped).  The state after the first
// update (rounded to f32 like the reference's stored arrays) goes to snap_mean / snap_var for
// normalising the step observations; the second update's result to mean / var / count.
#ifndef M2C
#define M2C 8  // columns per workgroup (measured 7.0 / 6.0 / 6.4 us at 16 / 8 / 4)
#endif
constexpr int M2COLS = M2C, M2LANES = 64;

__global__ __launch_bounds__(M2COLS * M2LANES) void rms_merge2_kernel(
    const double* p1, const double* p2, const double* blk_done, int64_t nblk, int64_t dim,
    int64_t k, float* mean, float* var, double* count, float* snap_mean, float* snap_var,
    unsigned int* ticket, const double* k_dev) {
    constexpr int NW = M2COLS * M2LANES / kWave;  // waves; each holds 64 / M2COLS lanes per column
    __shared__ double sh[5][NW][M2COLS];
    const int tid = threadIdx.x;
    const int col = tid % M2COLS;
    const int lane = tid / M2COLS;
    const int64_t d = (int64_t)blockIdx.x * M2COLS + col;
    const int64_t dc = d < dim ? d : dim - 1;  // in-bounds address for idle columns
    const double old_count = *count;
    // every load of the loop is independent: the P2 slots of blocks without a reset row
    // (not written this step) are read and dropped by a select instead of a branch; the
    // reset-row count rides along (each column's lanes see every block once)
    double nd = 0.0, s1 = 0.0, q1 = 0.0, s2 = 0.0, q2 = 0.0;
    for (int64_t b = lane; b < nblk; b += M2LANES) {
        const double bd = blk_done[b];
        const double2 a = *reinterpret_cast<const double2*>(p1 + (b * dim + dc) * 2);
        const double2 r = *reinterpret_cast<const double2*>(p2 + (b * dim + dc) * 2);
        nd += bd;
        s1 += a.x;
        q1 += a.y;
        s2 += bd > 0.0 ? r.x : 0.0;
        q2 += bd > 0.0 ? r.y : 0.0;
    }
    // the 4 lanes of a column inside a wave (tid bits 4-5), then the waves through LDS in
    // fixed order (one barrier instead of a 6-level LDS tree)
#pragma unroll
    for (int off = M2COLS; off < kWave; off <<= 1) {
        nd += __shfl_xor(nd, off, kWave);
        s1 += __shfl_xor(s1, off, kWave);
        q1 += __shfl_xor(q1, off, kWave);
        s2 += __shfl_xor(s2, off, kWave);
        q2 += __shfl_xor(q2, off, kWave);
    }
    const int w = tid / kWave;
    if ((tid & (kWave - 1)) < M2COLS) {
        sh[0][w][col] = nd;
        sh[1][w][col] = s1;
        sh[2][w][col] = q1;
        sh[3][w][col] = s2;
        sh[4][w][col] = q2;
    }
    __syncthreads();
    double tot2 = 0.0;
    if (tid < M2COLS) {
        double ND = 0.0, S1 = 0.0, Q1 = 0.0, S2 = 0.0, Q2 = 0.0;
        for (int v = 0; v < NW; ++v) {
            ND += sh[0][v][col];
            S1 += sh[1][v][col];
            Q1 += sh[2][v][col];
            S2 += sh[3][v][col];
            Q2 += sh[4][v][col];
        }
        const double bc1 = k_dev ? *k_dev : (double)k;
        const double tot1 = old_count + bc1;
        tot2 = tot1 + ND;
        if (d < dim) {
            double m0 = (double)mean[d], v0 = (double)var[d];
            if (bc1 > 0.0) {
                const double bm = S1 / bc1;
                double bv = Q1 / bc1 - bm * bm;
                bv = bv < 0.0 ? 0.0 : bv;
                const double delta = bm - m0;
                const double nm = m0 + delta * bc1 / tot1;
                const double m2 =
                    v0 * old_count + bv * bc1 + delta * delta * old_count * bc1 / tot1;
                m0 = (double)(float)nm;
                v0 = (double)(float)(m2 / tot1);
            }
            snap_mean[d] = (float)m0;
            snap_var[d] = (float)v0;
            if (ND > 0.0) {
                const double bm = S2 / ND;
                double bv = Q2 / ND - bm * bm;
                bv = bv < 0.0 ? 0.0 : bv;
                const double delta = bm - m0;
                const double nm = m0 + delta * ND / tot2;
                const double m2 = v0 * tot1 + bv * ND + delta * delta * tot1 * ND / tot2;
                m0 = (double)(float)nm;
                v0 = (double)(float)(m2 / tot2);
            }
            mean[d] = (float)m0;
            var[d] = (float)v0;
        }
    }
    if (tid == 0) {
        const unsigned int t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL,
                                                      __HIP_MEMORY_SCOPE_AGENT);
        if (t == gridDim.x - 1) {
            __hip_atomic_store(count, tot2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

__device__ __forceinline__ float norm1(float x, float m, float v, float eps, float clip) {
    float y = (x - m) / __builtin_sqrtf(v + eps);
    if (clip > 0.0f) y = fminf(fmaxf(y, -clip), clip);
    return y;
}

__global__ __launch_bounds__(TPB) void rms_norm_kernel(const float* x, const uint8_t* mask,
                                                       int64_t k, int64_t dim,
                                                       const float* mean, const float* var,
                                                       float eps, float clip, float* out) {
    const int64_t total = k * dim;
    for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * TPB) {
        const int64_t r = i / dim;
        if (mask && !mask[r]) continue;
        const int64_t d = i - r * dim;
        out[i] = norm1(x[i], mean[d], var[d], eps, clip);
    }
}

}  // namespace
}  // namespace tsrl

using namespace tsrl;

extern "C" int tsrl_rms_merge(const double* col_partials, int64_t nblk, int64_t dim,
                              const uint8_t* mask, int64_t k, const double* batch_count,
                              float* mean, float* var, double* count, unsigned int* ticket,
                              void* stream) {
    TSRL_CHECK_ARG(col_partials && mean && var && count && ticket && dim > 0 && nblk >= 0 &&
                       k >= 0,
                   "tsrl_rms_merge: bad arguments");
    TSRL_CHECK_ARG(((uintptr_t)col_partials & 15) == 0, "tsrl_rms_merge: partials not 16B aligned");
    if (k == 0) return 0;
    const int64_t grid = (dim + MCOLS - 1) / MCOLS;
    hipLaunchKernelGGL(rms_merge_kernel, dim3((unsigned)grid), dim3(MCOLS * MLANES), 0,
                       as_stream(stream), col_partials, nblk, dim, mask, k, batch_count, mean,
                       var, count, ticket);
    TSRL_LAUNCH_CHECK("tsrl_rms_merge");
    return 0;
}

extern "C" int tsrl_rms_merge2(const double* partials_step, const double* partials_reset,
                               const double* blk_done, int64_t nblk, int64_t dim, int64_t k,
                               float* mean, float* var, double* count, float* snap_mean,
                               float* snap_var, unsigned int* ticket, const double* k_dev,
                               void* stream) {
    TSRL_CHECK_ARG(partials_step && partials_reset && blk_done && mean && var && count &&
                       snap_mean && snap_var && ticket && dim > 0 && nblk >= 0 && k >= 0,
                   "tsrl_rms_merge2: bad arguments");
    TSRL_CHECK_ARG(aligned16(partials_step) && aligned16(partials_reset),
                   "tsrl_rms_merge2: partials not 16B aligned");
    const int64_t grid = (dim + M2COLS - 1) / M2COLS;
    hipLaunchKernelGGL(rms_merge2_kernel, dim3((unsigned)grid), dim3(M2COLS * M2LANES), 0,
                       as_stream(stream), partials_step, partials_reset, blk_done, nblk, dim, k,
                       mean, var, count, snap_mean, snap_var, ticket, k_dev);
    TSRL_LAUNCH_CHECK("tsrl_rms_merge2");
    return 0;
}

// Data-parallel form of merge2's inputs: this rank's step/reset moments folded over its
// partial blocks into one [4*dim + 2] f64 vector (sum/sumsq of the step rows, of the reset
// rows, the reset-row count and the step-row count k) -- the payload of ONE all-reduce per env step, after which
// tsrl_rms_merge2(nblk = 1) applies both global updates.
__global__ __launch_bounds__(kWave) void rms_sum_partials2_kernel(const double* p1, const double* p2,
                                                                   const double* blk_done,
                                                                   int64_t nblk, int64_t dim,
                                                                   int64_t k, double* out) {
    const int64_t d = (int64_t)blockIdx.x * kWave + threadIdx.x;
    if (d > dim) return;
    if (d == dim) {
        double nd = 0.0;
        for (int64_t b = 0; b < nblk; ++b) nd += blk_done[b];
        out[4 * dim] = nd;
        out[4 * dim + 1] = (double)k;
        return;
    }
    double s1 = 0.0, q1 = 0.0, s2 = 0.0, q2 = 0.0;
    for (int64_t b = 0; b < nblk; ++b) {
        const double2 a = *reinterpret_cast<const double2*>(p1 + (b * dim + d) * 2);
        s1 += a.x;
        q1 += a.y;
        if (blk_done[b] > 0.0) {
            const double2 r = *reinterpret_cast<const double2*>(p2 + (b * dim + d) * 2);
            s2 += r.x;
            q2 += r.y;
        }
    }
    out[2 * d] = s1;
    out[2 * d + 1] = q1;
    out[2 * dim + 2 * d] = s2;
    out[2 * dim + 2 * d + 1] = q2;
}

extern "C" int tsrl_rms_sum_partials2(const double* partials_step, const double* partials_reset,
                                      const double* blk_done, int64_t nblk, int64_t dim,
                                      int64_t k, double* out, void* stream) {
    TSRL_CHECK_ARG(partials_step && partials_reset && blk_done && out && dim > 0 && nblk >= 0,
                   "tsrl_rms_sum_partials2: bad arguments");
    const int64_t grid = (dim + 1 + kWave - 1) / kWave;
    hipLaunchKernelGGL(rms_sum_partials2_kernel, dim3((unsigned)grid), dim3(kWave), 0,
                       as_stream(stream), partials_step, partials_reset, blk_done, nblk, dim, k,
                       out);
    TSRL_LAUNCH_CHECK("tsrl_rms_sum_partials2");
    return 0;
}

extern "C" int tsrl_rms_norm_rows(const float* x, const uint8_t* mask, int64_t k, int64_t dim,
                                  const float* mean, const float* var, float eps, float clip,
                                  float* out, void* stream) {
    TSRL_CHECK_ARG(x && mean && var && out && dim > 0 && k >= 0, "tsrl_rms_norm_rows: bad args");
    if (k == 0) return 0;
    const int64_t total = k * dim;
    const int64_t grid = min((total + TPB - 1) / TPB, (int64_t)8192);
    hipLaunchKernelGGL(rms_norm_kernel, dim3((unsigned)grid), dim3(TPB), 0, as_stream(stream), x,
                       mask, k, dim, mean, var, eps, clip, out);
    TSRL_LAUNCH_CHECK("tsrl_rms_norm_rows");
    return 0;
}

// ---------------------------------------------------------------------------------------
// Exact RunningMeanStd (opt-in, VectorEnvNormObs(exact_obs_rms=True)): the reference's own f32
// arithmetic, bit for bit.  np.mean / np.var over axis 0 of a C-contiguous [k, D] f32 array
// sum each column SEQUENTIALLY in row order in f32 (the reduction axis is not the contiguous
// one, so no pairwise summation): S = x0 + x1 + ...; mean = S / k; var = sum((x - mean)^2)
// / k, every operation rounded to f32 (statistics.py:93-101).  The update then runs in f32
// with the python-int counts converted to f32 (NEP 50), in the reference's operation order
// (statistics.py:103-114).
//
// The two k-long dependent f32 add chains per column cannot be re-associated, so the kernel
// is built around them (rms_exact.h): a workgroup owns 8 columns and holds a whole span of up
// to 4096 rows of them in LDS ([column][row], 131 KB), loaded by all 8 waves with every load
// in flight at once; lanes 0-7 of wave 0 run the mean chains reading 4 rows per ds_read_b128
// (32 rows of reads in flight ahead of the adds); all waves then replace the span by
// (x - mean)^2 in place (the var chain's independent sub / mul, off the chain wave); wave 0
// runs the var chains.  The reset rows' update (the second RunningMeanStd.update of a
// Collector step: VectorEnvNormObs.reset of the finished envs, venv_wrappers.py:87-91) needs
// only the state after the first for its merge, so its two chains run on wave 1 at the same
// time as wave 0's (when its rows fit the 512-row side span).  Per row and pass the chain
// wave issues 1.25 instructions, so a 4096-row update is ~2 x 4096 x 5 cycles of chain plus
// one load latency.  Round 3's kernel (64 columns per workgroup, 128-row blocks staged one
// ahead with two barriers per block) paid a global-load latency per block: ~290 us per
// 4096 x 376 step.  Spans past 4096 rows (k > 4096: data-parallel global batches, large host
// collects) are streamed twice.
// ---------------------------------------------------------------------------------------
#include "rms_exact.h"

namespace tsrl {
namespace {

using exact::XC;
using exact::XT;
constexpr int XSPAN = 4096, XSPAN2 = 512;

// First update with b1's rows, the state after it to snap_* (when given), then b2's rows
// (when b2.x is given).  Every workgroup reads the old count first; the last to finish
// (agent-scope ticket, re-armed) publishes the new one.  Workgroup b owns columns
// [8 b, 8 b + 8).
__global__ __launch_bounds__(XT) void rms_exact_kernel(exact::Rows b1, exact::Rows b2,
                                                      int64_t dim, float* mean, float* var,
                                                      double* count, float* snap_mean,
                                                      float* snap_var, unsigned int* ticket) {
    __shared__ exact::Smem<XSPAN, XSPAN2> sm;
    const int t = threadIdx.x;
    const int64_t c0 = (int64_t)blockIdx.x * XC;
    const int64_t d = c0 + t;
    const bool own = t < XC && d < dim;
    const double cold = *count;
    float m = own ? mean[d] : 0.0f, v = own ? var[d] : 1.0f;
    float sm_ = 0.0f, sv_ = 0.0f;
    double c2 = exact::two_updates<XSPAN, XSPAN2>(b1, b2, dim, c0, cold, m, v, sm_, sv_, sm);
    if (own && snap_mean) {
        snap_mean[d] = sm_;
        snap_var[d] = sv_;
    }
    if (own) {
        mean[d] = m;
        var[d] = v;
    }
    if (t == 0) {
        const unsigned int prev = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL,
                                                         __HIP_MEMORY_SCOPE_AGENT);
        if (prev == gridDim.x - 1) {
            *count = c2;
            __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

}  // namespace
}  // namespace tsrl

extern "C" int tsrl_rms_exact_update(const float* x, const uint8_t* mask, int64_t k,
                                     const float* x2, const uint8_t* mask2, int64_t k2,
                                     int64_t dim, float* mean, float* var, double* count,
                                     float* snap_mean, float* snap_var, unsigned int* ticket,
                                     void* stream) {
    TSRL_CHECK_ARG(x && mean && var && count && ticket && dim > 0 && k >= 0 && k2 >= 0 &&
                       (snap_mean == nullptr) == (snap_var == nullptr),
                   "tsrl_rms_exact_update: bad arguments");
    const tsrl::exact::Rows b1{x, mask, k};
    const tsrl::exact::Rows b2{x2, mask2, x2 ? k2 : 0};
    const unsigned grid = (unsigned)((dim + tsrl::exact::XC - 1) / tsrl::exact::XC);
    hipLaunchKernelGGL(tsrl::rms_exact_kernel, dim3(grid), dim3(tsrl::exact::XT), 0,
                       as_stream(stream), b1, b2, dim, mean, var, count, snap_mean, snap_var,
                       ticket);
    TSRL_LAUNCH_CHECK("tsrl_rms_exact_update");
    return 0;
}

// ---------------------------------------------------------------------------------------
// tsrl_rms_exact_stats: the batch moments of one update pair alone, for the pipelined exact
// collect (collect.hip E: the next step launch merges them in its prologue).  The same f32
// arithmetic as rms_exact_kernel (sum in row order, mean = S / k, squares about the mean summed
// in row order, var = Q / k), in a form that runs on a CU BESIDE a collect-step workgroup
// (~117 KB of LDS, 190 VGPRs in its LW form): RXC = 2 columns per workgroup (128 threads), a
// span of RSPAN = 2048 rows of them in LDS ([column][row], 16 KB), loaded by LDS-DMA
// (global_load_lds_dword: one column x 64 rows per wave-instruction, a span's instructions all
// in flight -- one memory latency per span and pass), exact::chain over each column run (lanes
// 0-1 of wave 0), the squares in place (wave w: column w), the var chains; wave 1 runs the
// reset rows' two passes (row lists of RSEG = 1024 rows) while wave 0 chains.  20 KB and 128
// VGPRs per workgroup: two statistics (two steps) fit on a CU beside a step workgroup, so the
// pipeline keeps two in flight.  Workgroup b takes column pair (b % 8) * G / 8 + b / 8 (grid
// G padded to a multiple of 8): blocks b, b + 8, ... share an XCD and its L2, and neighbouring
// pairs read the same 128-B lines of every row.
// Measured (round 5, bench --exact-obs-rms, collect per 2048-step iteration; serial form 142
// ms, default obs_rms 41-42 ms): span 4096 / one statistic at a time 108-109 ms; XCD order 97;
// two at a time 110-113 (they no longer fit beside the step); span 2048 + XCD order, two at a
// time 79-80 (three: 80; span 1024: 87, three at depth 3: 80).  The first form streamed 16
// columns through a 16-stage LDS-DMA ring (16 rows per instruction): 199 us per statistic
// alone -- one DMA latency per 15 blocks -- against 38.8 us for the resident form alone.
// ---------------------------------------------------------------------------------------
namespace tsrl {
namespace {

constexpr int RXC = 2;       // columns per workgroup
constexpr int RSPAN = 2048;  // rows of a span held in LDS
constexpr int RSEG = 1024;   // reset-row flags per list segment (64 lanes x 16)

// Wave 1: the selected rows of segment [s0, s0 + n) (n <= SEG) -> list[0, cnt) in row order
// (lane l holds rows s0 + 64 j + l); returns cnt.
template <int SEG>
__device__ __forceinline__ int reset_list(const uint8_t* __restrict__ done, int64_t s0,
                                          int64_t n, int* list) {
    const int l = threadIdx.x & 63;
    int base = 0;
    // blocks of 16 x 64 rows: 16 flag loads per lane in flight, then 16 ballots
    for (int qb = 0; qb < SEG / 64; qb += 16) {
        if (64 * (int64_t)qb >= n) break;
        uint8_t f[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int64_t r = 64 * (qb + j) + l;
            f[j] = r < n ? done[s0 + r] : 0;
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint64_t m = __ballot(f[j] != 0);
            if (f[j]) list[base + (int)__popcll(m & ((1ull << l) - 1ull))] = 64 * (qb + j) + l;
            base += (int)__popcll(m);
        }
    }
    return base;
}

// Wave 1 pass over the reset rows of every segment (rebuilding the list per segment when there
// are several): lanes 0 .. NC - 1 chain their column.
template <bool SQ, int SEG, int NC>
__device__ float reset_pass(const float* __restrict__ xr, const uint8_t* __restrict__ done,
                            int64_t k, int64_t dim, int64_t col, float bm, int* list,
                            int first_cnt, int64_t* nsel) {
#pragma clang fp contract(off)
    const int l = threadIdx.x & 63;
    const bool own = l < NC && col < dim;
    float acc = 0.0f;
    int64_t tot = 0;
    for (int64_t s0 = 0; s0 < k; s0 += SEG) {
        const int64_t n = k - s0 < SEG ? k - s0 : SEG;
        const int cnt = (s0 == 0 && first_cnt >= 0) ? first_cnt
                                                    : reset_list<SEG>(done, s0, n, list);
        for (int e = 0; e < cnt; e += 16) {
            float v[16];
#pragma unroll
            for (int j = 0; j < 16; ++j)
                v[j] = (own && e + j < cnt) ? xr[(s0 + list[e + j]) * dim + col] : 0.0f;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                float y = v[j];
                if (SQ) {
                    y = y - bm;
                    y = y * y;
                }
                if (e + j < cnt) acc = acc + y;
            }
        }
        tot += cnt;
    }
    *nsel = tot;
    return acc;
}

// One LDS-DMA wave-instruction: lane l copies 4 bytes from src to LDS byte lds + 4 l (M0 set and
// restored inside the statement; lds wave-uniform).
__device__ __forceinline__ void sdma4(const void* src, uint32_t lds) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dword %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(src), "s"(lds)
        : "memory");
}

// Up to XSTEPS steps' statistics in one launch (tsrl_rms_exact_stats_n): workgroup b works on
// step b / G8, column pair of (b % G8) (G8 = the per-step grid, a multiple of 8).
constexpr int XSTEPS = 4;
struct XSteps {
    const float* x[XSTEPS];
    const float* xr[XSTEPS];
    const uint8_t* done[XSTEPS];
    float* st[XSTEPS];
    int64_t* cnts[XSTEPS];
    int g8;
};

__global__ __launch_bounds__(128) void rms_exact_stats_kernel(XSteps P, int64_t k,
                                                              int64_t dim) {
#pragma clang fp contract(off)
    __shared__ __attribute__((aligned(16))) float col[RXC][RSPAN + 4];
    __shared__ int list[RSEG];
    __shared__ float sbm[RXC];
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    const int sidx = (int)blockIdx.x / P.g8, bl = (int)blockIdx.x % P.g8;
    const float* __restrict__ x = P.x[sidx];
    const float* __restrict__ xr = P.xr[sidx];
    const uint8_t* __restrict__ done = P.done[sidx];
    float* __restrict__ st = P.st[sidx];
    int64_t* __restrict__ cnts = P.cnts[sidx];
    // XCD-aware column order (the grid is padded to a multiple of 8; pairs past the last
    // exit before any barrier)
    const int g = (bl % 8) * (P.g8 / 8) + bl / 8;
    if ((int64_t)g * RXC >= dim) return;
    const int64_t c0 = (int64_t)g * RXC;
    const int64_t mycol = c0 + w;  // the column this wave loads and squares
    const int nspan = (int)((k + RSPAN - 1) / RSPAN);
    const uint32_t lds_w = (uint32_t)(uintptr_t)&col[w][0];
    auto load_span = [&](int64_t s0, int n) {
        for (int i = 0; i < (n + 63) / 64; ++i) {
            int64_t r = s0 + 64 * i + l;
            r = r < k ? r : k - 1;
            sdma4(x + r * dim + mycol,
                  (uint32_t)__builtin_amdgcn_readfirstlane((int)(lds_w + 256u * (uint32_t)i)));
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };
    const bool chain_lane = w == 0 && l < RXC;
    const bool rs = xr && done;
    int64_t nd = 0;
    float S = 0.0f, Q = 0.0f, S2 = 0.0f, bm2 = 0.0f, bv2 = 0.0f;
    const int64_t rcol = c0 + l;  // wave 1's reset-row column (lanes 0-1)
    for (int sp = 0; sp < nspan; ++sp) {
        const int64_t s0 = (int64_t)sp * RSPAN;
        const int n = (int)min((int64_t)RSPAN, k - s0);
        load_span(s0, n);
        __syncthreads();
        if (chain_lane) S = exact::chain(&col[l][0], n, S);
        else if (w == 1 && sp == 0 && rs)
            S2 = reset_pass<false, RSEG, RXC>(xr, done, k, dim, rcol, 0.0f, list, -1, &nd);
        __syncthreads();
    }
    const float kf = (float)k;
    if (chain_lane) sbm[l] = S / kf;
    __syncthreads();
    for (int sp = 0; sp < nspan; ++sp) {
        const int64_t s0 = (int64_t)sp * RSPAN;
        const int n = (int)min((int64_t)RSPAN, k - s0);
        if (nspan > 1) {
            load_span(s0, n);
            __syncthreads();
        }
        {  // wave w: column w's run -> (x - bm)^2 in place, float4 per lane
            const float b = sbm[w];
            float* p = col[w];
            const int n4 = n & ~3;
            for (int e = 4 * l; e < n4; e += 256) {
                float4 v = *reinterpret_cast<float4*>(p + e);
                float d = v.x - b;
                v.x = d * d;
                d = v.y - b;
                v.y = d * d;
                d = v.z - b;
                v.z = d * d;
                d = v.w - b;
                v.w = d * d;
                *reinterpret_cast<float4*>(p + e) = v;
            }
            if (l < n - n4) {
                const float d = p[n4 + l] - b;
                p[n4 + l] = d * d;
            }
        }
        __syncthreads();
        if (chain_lane) Q = exact::chain(&col[l][0], n, Q);
        else if (w == 1 && sp == 0 && rs && nd > 0) {
            bm2 = S2 / (float)nd;
            int64_t nd2 = 0;
            bv2 = reset_pass<true, RSEG, RXC>(xr, done, k, dim, rcol, bm2, list, -1, &nd2) /
                  (float)nd;
        }
        __syncthreads();
    }
    if (chain_lane && c0 + l < dim) {
        st[c0 + l] = sbm[l];
        st[dim + c0 + l] = Q / kf;
    }
    if (w == 1 && l < RXC && rcol < dim) {
        st[2 * dim + rcol] = bm2;
        st[3 * dim + rcol] = bv2;
    }
    if (g == 0 && t == 0) cnts[0] = k;
    if (g == 0 && t == 64) cnts[1] = nd;
}

}  // namespace
}  // namespace tsrl

extern "C" int64_t tsrl_rms_exact_stats_bytes(int64_t dim) {
    return dim > 0 ? (16 * dim + 7) / 8 * 8 + 16 : 0;
}

extern "C" int tsrl_rms_exact_stats_max_steps(void) { return tsrl::XSTEPS; }

extern "C" int tsrl_rms_exact_stats_n(int nsteps, const float* const* x,
                                      const float* const* reset_x, const uint8_t* const* done,
                                      int64_t k, int64_t dim, void* const* stats, void* stream) {
    TSRL_CHECK_ARG(nsteps >= 1 && nsteps <= tsrl::XSTEPS && x && reset_x && done && stats &&
                       dim > 0 && dim % 4 == 0 && k >= 0,
                   "tsrl_rms_exact_stats_n: 1 <= nsteps <= %d, dim %% 4 == 0", tsrl::XSTEPS);
    tsrl::XSteps S{};
    for (int i = 0; i < nsteps; ++i) {
        TSRL_CHECK_ARG(x[i] && stats[i] && aligned16(x[i]) &&
                           (reset_x[i] == nullptr) == (done[i] == nullptr) &&
                           (reset_x[i] == nullptr || aligned16(reset_x[i])) &&
                           (reinterpret_cast<uintptr_t>(stats[i]) & 7u) == 0,
                       "tsrl_rms_exact_stats: bad arguments (16-byte aligned rows, 8-byte "
                       "aligned stats)");
        S.x[i] = x[i];
        S.xr[i] = reset_x[i];
        S.done[i] = done[i];
        S.st[i] = reinterpret_cast<float*>(stats[i]);
        S.cnts[i] = reinterpret_cast<int64_t*>(reinterpret_cast<char*>(stats[i]) +
                                               (16 * dim + 7) / 8 * 8);
    }
    S.g8 = (int)(((dim + tsrl::RXC - 1) / tsrl::RXC + 7) / 8 * 8);
    hipLaunchKernelGGL(tsrl::rms_exact_stats_kernel, dim3((unsigned)(S.g8 * nsteps)), dim3(128),
                       0, as_stream(stream), S, k, dim);
    TSRL_LAUNCH_CHECK("tsrl_rms_exact_stats");
    return 0;
}

extern "C" int tsrl_rms_exact_stats(const float* x, int64_t k, const float* reset_x,
                                    const uint8_t* done, int64_t dim, void* stats, void* stream) {
    return tsrl_rms_exact_stats_n(1, &x, &reset_x, &done, k, dim, &stats, stream);
}
