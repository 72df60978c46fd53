// Episode-aware index stepping and frame-stack gathers of the VectorReplayBuffer.
//
// ring_step : ReplayBufferManager prev/next (tianshou/data/buffer/manager.py:259-297, the
//             numba _prev_index/_next_index; the ring arithmetic is in ring.h).
// stack     : ReplayBuffer.get(index, key, stack_num) (base.py:317-358): frame s of output row
//             r is the storage row prev^(stack_num-1-s)(idx[r]); with save_only_last_obs
//             (manager.py:127-132) the storage holds one frame per row and this rebuilds the
//             [stack_num, ...] observation (examples/atari/atari_ppo.py:183-189).  One wave
//             per (row, frame): the wave walks its prev chain (a few done[] reads that hit
//             L2) and copies the frame with 16-byte loads; the chain indices can be written
//             out for the keys that are stacked with torch gathers (info / policy).
#include "ring.h"

namespace tsrl {
namespace {

constexpr int TPB = 256;
constexpr int WPB = TPB / kWave;

__global__ __launch_bounds__(TPB) void ring_step_kernel(Ring g, const int64_t* idx, int64_t k,
                                                        int steps, int64_t* out) {
    const int64_t r = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (r >= k) return;
    int64_t i = idx[r];
    if (steps == 0) i = pmod(i, g.maxsize);
    for (int s = 0; s < steps; ++s) i = ring_prev(g, i);
    for (int s = 0; s > steps; --s) i = ring_next(g, i);
    out[r] = i;
}

__device__ __forceinline__ void copy_frame(const char* s, char* d, int64_t bytes, int lane) {
    if ((bytes & 15) == 0 && aligned16(s) && aligned16(d)) {
        const int4* s4 = reinterpret_cast<const int4*>(s);
        int4* d4 = reinterpret_cast<int4*>(d);
        for (int64_t i = lane; i < bytes / 16; i += kWave) d4[i] = s4[i];
    } else if ((bytes & 3) == 0 && (((uintptr_t)s | (uintptr_t)d) & 3) == 0) {
        const int* s4 = reinterpret_cast<const int*>(s);
        int* d4 = reinterpret_cast<int*>(d);
        for (int64_t i = lane; i < bytes / 4; i += kWave) d4[i] = s4[i];
    } else {
        for (int64_t i = lane; i < bytes; i += kWave) d[i] = s[i];
    }
}

// Output row r, frame s: wave (r * S + s) over the flattened grid.
__global__ __launch_bounds__(TPB) void stack_gather_kernel(Ring g, const char* src,
                                                           int64_t src_pitch,
                                                           int64_t frame_bytes,
                                                           const int64_t* idx, int64_t k,
                                                           int S, char* dst, int64_t* chain) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t wv = (int64_t)blockIdx.x * WPB + threadIdx.x / kWave;
    if (wv >= k * S) return;
    const int64_t r = wv / S;
    const int s = (int)(wv - r * S);
    // base.py:344-350: the newest frame is val[index] (index as given), older ones step prev
    int64_t i = pmod(idx[r], g.maxsize);
    for (int q = S - 1; q > s; --q) i = ring_prev(g, i);
    if (dst) copy_frame(src + i * src_pitch, dst + wv * frame_bytes, frame_bytes, lane);
    if (chain && lane == 0) chain[wv] = i;
}

// frames_to_f32_nhwc: [n][c][hw] u8 -> [n][hw][c] f32 through a 256-entry table (the scaled
// byte values, computed by the caller).  Vector path (c == 4, hw % 4 == 0): a thread owns
// four consecutive pixels of one row, reads one 4-byte word per channel plane (coalesced
// across lanes) and writes the 4x4 floats as four 16-byte stores (64 contiguous bytes).
__global__ __launch_bounds__(TPB) void frames_nhwc4_kernel(const uint32_t* src, uint32_t hw4,
                                                           uint32_t total, const float* lut,
                                                           float4* dst) {
    __shared__ float t[256];
    t[threadIdx.x] = lut[threadIdx.x];
    __syncthreads();
    const uint32_t i = blockIdx.x * TPB + threadIdx.x;
    if (i >= total) return;
    const uint32_t r = i / hw4, p4 = i - r * hw4;
    const uint32_t* s = src + (size_t)r * 4 * hw4 + p4;
    uint32_t w[4];
#pragma unroll
    for (int ch = 0; ch < 4; ++ch) w[ch] = s[(size_t)ch * hw4];
    float4* d = dst + (size_t)i * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int sh = 8 * j;
        d[j] = make_float4(t[(w[0] >> sh) & 0xFF], t[(w[1] >> sh) & 0xFF],
                           t[(w[2] >> sh) & 0xFF], t[(w[3] >> sh) & 0xFF]);
    }
}

__global__ __launch_bounds__(TPB) void frames_nhwc_kernel(const uint8_t* src, int64_t c,
                                                          int64_t hw, int64_t total,
                                                          const float* lut, float* dst) {
    __shared__ float t[256];
    t[threadIdx.x] = lut[threadIdx.x];
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;  // output element
    if (i >= total) return;
    const int64_t ch = i % c, rp = i / c, p = rp % hw, r = rp / hw;
    dst[i] = t[src[(r * c + ch) * hw + p]];
}

}  // namespace
}  // namespace tsrl

using namespace tsrl;

extern "C" int tsrl_frames_to_f32_nhwc(const uint8_t* src, int64_t n, int64_t c, int64_t hw,
                                       const float* lut, float* dst, void* stream) {
    TSRL_CHECK_ARG(n >= 0 && c > 0 && hw > 0, "tsrl_frames_to_f32_nhwc: bad sizes");
    if (n == 0) return 0;
    TSRL_CHECK_ARG(src && lut && dst, "tsrl_frames_to_f32_nhwc: null pointer");
    const int64_t total = n * c * hw;
    if (c == 4 && hw % 4 == 0 && (((uintptr_t)src) & 3) == 0 && aligned16(dst) &&
        total / 4 < (1ll << 32) - TPB) {
        const uint32_t t4 = (uint32_t)(total / 16);  // threads: 4 pixels x 4 channels each
        hipLaunchKernelGGL(frames_nhwc4_kernel, dim3((t4 + TPB - 1) / TPB), dim3(TPB), 0,
                           as_stream(stream), reinterpret_cast<const uint32_t*>(src),
                           (uint32_t)(hw / 4), t4, lut, reinterpret_cast<float4*>(dst));
    } else {
        const int64_t grid = (total + TPB - 1) / TPB;
        TSRL_CHECK_ARG(grid < (1ll << 31), "tsrl_frames_to_f32_nhwc: too many elements");
        hipLaunchKernelGGL(frames_nhwc_kernel, dim3((unsigned)grid), dim3(TPB), 0,
                           as_stream(stream), src, c, hw, total, lut, dst);
    }
    TSRL_LAUNCH_CHECK("tsrl_frames_to_f32_nhwc");
    return 0;
}

static int check_ring(const uint8_t* done, const int64_t* last_index, const int64_t* lengths,
                      int64_t size, int64_t num, const char* who) {
    TSRL_CHECK_ARG(done && last_index && lengths, "%s: null ring pointer", who);
    TSRL_CHECK_ARG(size > 0 && num > 0, "%s: empty ring (size %lld, num %lld)", who,
                   (long long)size, (long long)num);
    return 0;
}

extern "C" int tsrl_ring_step_index(const int64_t* idx, int64_t k, const uint8_t* done,
                                    const int64_t* last_index, const int64_t* lengths,
                                    int64_t size, int64_t num, int steps, int64_t* out,
                                    void* stream) {
    TSRL_CHECK_ARG(k >= 0, "tsrl_ring_step_index: k < 0");
    if (k == 0) return 0;
    if (int rc = check_ring(done, last_index, lengths, size, num, "tsrl_ring_step_index"))
        return rc;
    TSRL_CHECK_ARG(idx && out, "tsrl_ring_step_index: null idx/out");
    const Ring g = {done, last_index, lengths, size, size * num};
    hipLaunchKernelGGL(ring_step_kernel, dim3((unsigned)((k + TPB - 1) / TPB)), dim3(TPB), 0,
                       as_stream(stream), g, idx, k, steps, out);
    TSRL_LAUNCH_CHECK("tsrl_ring_step_index");
    return 0;
}

extern "C" int tsrl_stack_gather_pitched(const void* src, int64_t src_pitch,
                                         int64_t frame_bytes, const int64_t* idx, int64_t k,
                                         int64_t stack_num, const uint8_t* done,
                                         const int64_t* last_index, const int64_t* lengths,
                                         int64_t size, int64_t num, void* dst,
                                         int64_t* chain_out, void* stream) {
    TSRL_CHECK_ARG(k >= 0 && stack_num >= 1 && stack_num <= 1024 && frame_bytes >= 0 &&
                       src_pitch >= frame_bytes,
                   "tsrl_stack_gather: bad sizes");
    if (k == 0) return 0;
    if (int rc = check_ring(done, last_index, lengths, size, num, "tsrl_stack_gather"))
        return rc;
    TSRL_CHECK_ARG(idx && (dst || chain_out), "tsrl_stack_gather: null idx or no output");
    TSRL_CHECK_ARG(!dst || src, "tsrl_stack_gather: dst without src");
    const Ring g = {done, last_index, lengths, size, size * num};
    const int64_t waves = k * stack_num;
    const int64_t grid = (waves + WPB - 1) / WPB;
    TSRL_CHECK_ARG(grid < (1ll << 31), "tsrl_stack_gather: too many rows");
    hipLaunchKernelGGL(stack_gather_kernel, dim3((unsigned)grid), dim3(TPB), 0,
                       as_stream(stream), g, reinterpret_cast<const char*>(src), src_pitch,
                       frame_bytes, idx, k, (int)stack_num, reinterpret_cast<char*>(dst),
                       chain_out);
    TSRL_LAUNCH_CHECK("tsrl_stack_gather");
    return 0;
}

extern "C" int tsrl_stack_gather(const void* src, int64_t frame_bytes, const int64_t* idx,
                                 int64_t k, int64_t stack_num, const uint8_t* done,
                                 const int64_t* last_index, const int64_t* lengths,
                                 int64_t size, int64_t num, void* dst, int64_t* chain_out,
                                 void* stream) {
    return tsrl_stack_gather_pitched(src, frame_bytes, frame_bytes, idx, k, stack_num, done,
                                     last_index, lengths, size, num, dst, chain_out, stream);
}
