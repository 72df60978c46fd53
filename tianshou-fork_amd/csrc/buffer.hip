// Device-resident VectorReplayBuffer storage operations.
//
// add    : ReplayBufferManager.add (tianshou/data/buffer/manager.py:104-161) for one vector
//          step -- the per-env `_add_index` loop (base.py:195-214) becomes one wave per env
//          row; episode statistics live on device.  The host keeps only the index
//          arithmetic (which it can do without reading device data).  The Collector's
//          obs_next normalisation (VectorEnvNormObs) is fused into the obs_next row copy.
// gather : fancy-index row gather (Batch.__getitem__, batch.py:446-460).
#include "add_row.h"

namespace tsrl {
namespace {

constexpr int TPB = 256;
constexpr int ROWS_PER_BLOCK = TPB / kWave;  // one wave per row

__global__ __launch_bounds__(TPB) void buffer_add_kernel(tsrl_add_args a) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t r = (int64_t)blockIdx.x * ROWS_PER_BLOCK + threadIdx.x / kWave;
    const int64_t urel = a.rel_dev ? *a.rel_dev : a.uniform_rel;
    if (r < a.k) add_row(a, r, lane, urel);
    // ring cursor for the next step: written to the other slot of a ping-pong pair, so no
    // workgroup can observe it before every workgroup of this launch has read *rel_dev
    if (a.rel_next && blockIdx.x == 0 && threadIdx.x == 0) *a.rel_next = (urel + 1) % a.ring_size;
}

__global__ __launch_bounds__(TPB) void gather_rows_kernel(const char* src, int64_t src_pitch,
                                                          int64_t row_bytes,
                                                          const int64_t* idx, int64_t k,
                                                          char* dst) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t nw = (int64_t)gridDim.x * ROWS_PER_BLOCK;
    for (int64_t r = (int64_t)blockIdx.x * ROWS_PER_BLOCK + threadIdx.x / kWave; r < k;
         r += nw) {
        copy_row(src + idx[r] * src_pitch, dst + r * row_bytes, row_bytes, lane);
    }
}

// out[c] = sum_r x[r][c] over a row-major [rows, cols] f32 matrix: bias gradients (rows =
// minibatch, cols = 1..376) and the split-K partial products of the weight gradients.
// Stage kernels write per-chunk partial rows; every order is fixed (reproducible).
constexpr int SC = 64, SL = 4;
// column-tiled: block = 64 columns x 4 row lanes over rows [r0, r1)
__global__ __launch_bounds__(SC * SL) void sum_rows_tiled_kernel(const float* x, int64_t rows,
                                                                 int64_t cols, int64_t chunk,
                                                                 float* out) {
    __shared__ float sh[SL][SC];
    const int c = threadIdx.x % SC, l = threadIdx.x / SC;
    const int64_t col = (int64_t)blockIdx.x * SC + c;
    const int64_t r0 = (int64_t)blockIdx.y * chunk;
    const int64_t r1 = min(r0 + chunk, rows);
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    if (col < cols) {
        int64_t r = r0 + l;
        for (; r + 3 * SL < r1; r += 4 * SL) {
            a0 += x[r * cols + col];
            a1 += x[(r + SL) * cols + col];
            a2 += x[(r + 2 * SL) * cols + col];
            a3 += x[(r + 3 * SL) * cols + col];
        }
        for (; r < r1; r += SL) a0 += x[r * cols + col];
    }
    sh[l][c] = (a0 + a1) + (a2 + a3);
    __syncthreads();
    if (l == 0 && col < cols)
        out[(int64_t)blockIdx.y * cols + col] = (sh[0][c] + sh[1][c]) + (sh[2][c] + sh[3][c]);
}

// narrow (cols <= 256): a chunk of rows is a flat range; thread t < stride = cols*(256/cols)
// always sees column t % cols, so one scalar accumulator per thread, then an LDS fold.
__global__ __launch_bounds__(256) void sum_rows_narrow_kernel(const float* x, int64_t rows,
                                                              int64_t cols, int64_t chunk,
                                                              float* out) {
    __shared__ float sh[256];
    const int t = threadIdx.x;
    const int per = 256 / (int)cols;
    const int stride = per * (int)cols;
    const int64_t r0 = (int64_t)blockIdx.x * chunk;
    const int64_t r1 = min(r0 + chunk, rows);
    const int64_t e1 = r1 * cols;
    float a0 = 0.f, a1 = 0.f;
    if (t < stride) {
        int64_t e = r0 * cols + t;
        for (; e + stride < e1; e += 2 * (int64_t)stride) {
            a0 += x[e];
            a1 += x[e + stride];
        }
        if (e < e1) a0 += x[e];
    }
    sh[t] = a0 + a1;
    __syncthreads();
    if (t < cols) {
        float s = 0.f;
        for (int k = 0; k < per; ++k) s += sh[t + k * (int)cols];
        out[(int64_t)blockIdx.x * cols + t] = s;
    }
}

constexpr int64_t SUM_CHUNK = 1024;

int64_t sum_rows_nchunks(int64_t rows) {
    return rows <= 4 * SUM_CHUNK ? 1 : std::min<int64_t>(256, (rows + SUM_CHUNK - 1) / SUM_CHUNK);
}

int launch_sum_stage(const float* x, int64_t rows, int64_t cols, int64_t nchunks, float* out,
                     hipStream_t st) {
    const int64_t chunk = (rows + nchunks - 1) / nchunks;
    if (cols <= 256 && rows > 64) {
        hipLaunchKernelGGL(sum_rows_narrow_kernel, dim3((unsigned)nchunks), dim3(256), 0, st, x,
                           rows, cols, chunk, out);
    } else {
        hipLaunchKernelGGL(sum_rows_tiled_kernel,
                           dim3((unsigned)((cols + SC - 1) / SC), (unsigned)nchunks), dim3(SC * SL),
                           0, st, x, rows, cols, chunk, out);
    }
    TSRL_LAUNCH_CHECK("tsrl_sum_rows_f32");
    return 0;
}

}  // namespace
}  // namespace tsrl

using namespace tsrl;

__global__ void ring_advance_kernel(int64_t* rel, int64_t size) { *rel = (*rel + 1) % size; }

extern "C" int tsrl_ring_advance(int64_t* rel_dev, int64_t ring_size, void* stream) {
    TSRL_CHECK_ARG(rel_dev && ring_size > 0, "tsrl_ring_advance: bad arguments");
    hipLaunchKernelGGL(ring_advance_kernel, dim3(1), dim3(1), 0, as_stream(stream), rel_dev,
                       ring_size);
    TSRL_LAUNCH_CHECK("tsrl_ring_advance");
    return 0;
}

extern "C" int64_t tsrl_sum_rows_workspace_bytes(int64_t rows, int64_t cols) {
    const int64_t n = sum_rows_nchunks(rows);
    return n > 1 ? n * cols * (int64_t)sizeof(float) : 0;
}

extern "C" int tsrl_sum_rows_f32(const float* x, int64_t rows, int64_t cols, float* out,
                                 void* workspace, int64_t workspace_bytes, void* stream) {
    TSRL_CHECK_ARG(x && out && rows >= 0 && cols > 0, "tsrl_sum_rows_f32: bad arguments");
    hipStream_t st = as_stream(stream);
    const int64_t n = sum_rows_nchunks(rows);
    if (n == 1) return launch_sum_stage(x, rows, cols, 1, out, st);
    TSRL_CHECK_ARG(workspace && workspace_bytes >= n * cols * (int64_t)sizeof(float),
                   "tsrl_sum_rows_f32: needs %lld workspace bytes",
                   (long long)(n * cols * (int64_t)sizeof(float)));
    float* part = reinterpret_cast<float*>(workspace);
    int rc = launch_sum_stage(x, rows, cols, n, part, st);
    if (rc) return rc;
    return launch_sum_stage(part, n, cols, 1, out, st);
}

extern "C" int tsrl_buffer_add(const tsrl_add_args* a, void* stream) {
    TSRL_CHECK_ARG(a != nullptr, "tsrl_buffer_add: null args");
    TSRL_CHECK_ARG(a->k >= 0, "tsrl_buffer_add: k < 0");
    if (a->k == 0) return 0;
    TSRL_CHECK_ARG(a->offset && a->ep_rew && a->ep_len && a->ep_idx,
                   "tsrl_buffer_add: offset/episode-state pointers are required");
    TSRL_CHECK_ARG(!a->obs_next_src || a->obs_dim > 0, "tsrl_buffer_add: obs_dim must be > 0");
    TSRL_CHECK_ARG(!a->norm_mean || a->norm_var, "tsrl_buffer_add: norm_var missing");
    TSRL_CHECK_ARG(!a->rel_dev || (a->ring_size > 0 && !a->ptr),
                   "tsrl_buffer_add: rel_dev needs ring_size and ptr == NULL");
    TSRL_CHECK_ARG(!a->reset_mask || (a->reset_src && a->cur_obs),
                   "tsrl_buffer_add: reset_mask needs reset_src and cur_obs");
    TSRL_CHECK_ARG(!a->reset_mean || a->reset_var, "tsrl_buffer_add: reset_var missing");
    TSRL_CHECK_ARG(!a->rel_next || (a->rel_dev && a->rel_next != a->rel_dev),
                   "tsrl_buffer_add: rel_next needs rel_dev (a different word)");
    const int64_t grid = (a->k + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK;
    hipLaunchKernelGGL(buffer_add_kernel, dim3((unsigned)grid), dim3(TPB), 0, as_stream(stream),
                       *a);
    TSRL_LAUNCH_CHECK("tsrl_buffer_add");
    return 0;
}

extern "C" int tsrl_gather_rows_pitched(const void* src, int64_t src_pitch, int64_t row_bytes,
                                        const int64_t* idx, int64_t k, void* dst, void* stream) {
    TSRL_CHECK_ARG(k >= 0 && row_bytes > 0 && src_pitch >= row_bytes,
                   "tsrl_gather_rows: bad sizes");
    if (k == 0) return 0;
    TSRL_CHECK_ARG(src && idx && dst, "tsrl_gather_rows: null pointer");
    const int64_t grid = std::min<int64_t>((k + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK, 16384);
    hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)grid), dim3(TPB), 0, as_stream(stream),
                       (const char*)src, src_pitch, row_bytes, idx, k, (char*)dst);
    TSRL_LAUNCH_CHECK("tsrl_gather_rows");
    return 0;
}

extern "C" int tsrl_gather_rows(const void* src, int64_t row_bytes, const int64_t* idx,
                                int64_t k, void* dst, void* stream) {
    return tsrl_gather_rows_pitched(src, row_bytes, row_bytes, idx, k, dst, stream);
}
