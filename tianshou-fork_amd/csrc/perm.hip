// np.random.permutation(n) of NumPy's legacy RandomState, bit-exact, with the shuffle applied
// on the device.
//
// Reference: Batch.split (tianshou/data/batch.py:896-912) draws `np.random.permutation(length)`
// from the global legacy RandomState for every PPO repeat (ppo.py:106-107).  NumPy's legacy
// permutation(n) is arange(n) + shuffle: for i = n-1 .. 1, j_i = random_interval(i) (mask the
// next tempered MT19937 word with the smallest all-ones mask >= i, reject while > i), then
// swap x[i], x[j_i].
//
// Split:
//   host   tsrl_np_shuffle_draws: the inherently sequential part, the MT19937 stream and the
//          rejection loop (advances the caller's copy of the RandomState key/pos, so the host
//          can write the state back with set_state);
//   device tsrl_shuffle_apply: the swap sequence resolved in parallel.  Step i finalises
//          position i (later steps only touch positions < i), so out[i] is the value at
//          position j_i just before step i.  Position p is only ever changed by the steps s
//          with j_s == p ("hitters" of p); with A(s) = value at position s just before step s:
//            A(s)   = A(nxt(s)) where nxt(s) = smallest hitter of s above s, else s;
//            out[t] = A(t) if j_t == t, else A(succ(t)) for the next hitter succ(t) of j_t
//                     after t, else j_t (untouched since the start);  out[0] = A(0).
//          The hitter lists come from one stable radix sort of (j_s, s); A is a pointer chase
//          along strictly increasing indices (expected length ~ ln n).
#include <hipcub/hipcub.hpp>

#include "tsrl_common.h"

namespace tsrl {
namespace {

constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr int kMtN = 624;
constexpr int kMtM = 397;

// mt19937_gen of NumPy's mt19937.c (the reference generator, Matsumoto & Nishimura 1998).
inline void mt_regen(uint32_t* k) {
    constexpr uint32_t kA = 0x9908b0dfu, kU = 0x80000000u, kL = 0x7fffffffu;
    int i = 0;
    for (; i < kMtN - kMtM; ++i) {
        const uint32_t y = (k[i] & kU) | (k[i + 1] & kL);
        k[i] = k[i + kMtM] ^ (y >> 1) ^ ((0u - (y & 1u)) & kA);
    }
    for (; i < kMtN - 1; ++i) {
        const uint32_t y = (k[i] & kU) | (k[i + 1] & kL);
        k[i] = k[i + (kMtM - kMtN)] ^ (y >> 1) ^ ((0u - (y & 1u)) & kA);
    }
    const uint32_t y = (k[kMtN - 1] & kU) | (k[0] & kL);
    k[kMtN - 1] = k[kMtM - 1] ^ (y >> 1) ^ ((0u - (y & 1u)) & kA);
}

inline uint32_t temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

__global__ void iota_keys_kernel(uint32_t* vals, int64_t m) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < m) vals[k] = (uint32_t)(k + 1);  // step s = k + 1 (steps are 1 .. n-1)
}

// Hitter lists: keys = sorted j, vals = steps in ascending order within equal j.
__global__ void hitters_kernel(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                               int64_t m, uint32_t* __restrict__ first,
                               uint32_t* __restrict__ succ) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    const uint32_t p = keys[k], s = vals[k];
    succ[s] = (k + 1 < m && keys[k + 1] == p) ? vals[k + 1] : kNone;
    if (k == 0 || keys[k - 1] != p) first[p] = s;
}

__device__ __forceinline__ uint32_t nxt(const uint32_t* __restrict__ first,
                                        const uint32_t* __restrict__ succ, uint32_t p) {
    const uint32_t f = first[p];
    return f == p ? succ[p] : f;
}

__device__ __forceinline__ uint32_t chase(const uint32_t* __restrict__ first,
                                          const uint32_t* __restrict__ succ, uint32_t a) {
    for (uint32_t q = nxt(first, succ, a); q != kNone; q = nxt(first, succ, a)) a = q;
    return a;
}

__global__ void resolve_kernel(const uint32_t* __restrict__ draws, int64_t n,
                               const uint32_t* __restrict__ first, const uint32_t* __restrict__ succ,
                               int64_t* __restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    uint32_t v;
    if (t == 0) {
        v = chase(first, succ, 0u);
    } else {
        const uint32_t j = draws[t];
        if (j == (uint32_t)t) {
            v = chase(first, succ, j);
        } else {
            const uint32_t sc = succ[t];
            v = sc == kNone ? j : chase(first, succ, sc);
        }
    }
    out[t] = (int64_t)v;
}

inline int bits_for(uint64_t x) {  // number of bits to represent values 0..x
    int b = 0;
    while (b < 64 && (x >> b) != 0) ++b;
    return b;
}

inline int64_t align256(int64_t x) { return (x + 255) & ~int64_t(255); }

struct ApplyLayout {
    int64_t keys_out, vals_in, vals_out, first, succ, temp, temp_bytes, total;
};

inline ApplyLayout apply_layout(int64_t n, size_t cub_bytes) {
    ApplyLayout L;
    const int64_t m = n > 1 ? n - 1 : 0;
    int64_t off = 0;
    L.keys_out = off; off += align256(m * 4);
    L.vals_in = off; off += align256(m * 4);
    L.vals_out = off; off += align256(m * 4);
    L.first = off; off += align256(n * 4);
    L.succ = off; off += align256(n * 4);
    L.temp = off; L.temp_bytes = (int64_t)cub_bytes; off += align256((int64_t)cub_bytes);
    L.total = off;
    return L;
}

inline size_t cub_sort_bytes(int64_t m) {
    size_t bytes = 0;
    if (m <= 0) return 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint32_t*)nullptr,
                                             (uint32_t*)nullptr, (const uint32_t*)nullptr,
                                             (uint32_t*)nullptr, (int)m, 0,
                                             bits_for((uint64_t)m), (hipStream_t)0);
    return bytes;
}

}  // namespace
}  // namespace tsrl

using namespace tsrl;

extern "C" int tsrl_np_shuffle_draws(uint32_t* key, int32_t* pos, int64_t n, uint32_t* draws) {
    TSRL_CHECK_ARG(key && pos && (draws || n <= 0), "tsrl_np_shuffle_draws: null argument");
    // n <= INT_MAX: the device side (tsrl_shuffle_apply) sorts n - 1 keys with an int count
    TSRL_CHECK_ARG(n >= 0 && n <= (int64_t)INT_MAX,
                   "tsrl_np_shuffle_draws: n=%lld outside [0, 2^31) (the shuffle's radix sort "
                   "takes an int count)", (long long)n);
    TSRL_CHECK_ARG(*pos >= 0 && *pos <= kMtN, "tsrl_np_shuffle_draws: pos=%d", (int)*pos);
    if (n == 0) return 0;
    draws[0] = 0;
    uint32_t k[kMtN], tb[kMtN];
    for (int i = 0; i < kMtN; ++i) k[i] = key[i];
    int p = *pos;
    // Branch-free consumption of the tempered stream.  Within a run of i sharing one mask
    // (i in [lo, mask]), every word is masked and written to draws[i], and i moves on only
    // when the word is accepted (<= i): a rejected word's write is overwritten by the next
    // candidate, and the loop-carried chain is one compare + subtract per word.
    uint32_t i = (uint32_t)(n - 1);
    while (i >= 1) {
        if (p == kMtN) { mt_regen(k); p = 0; }
        for (int q = p; q < kMtN; ++q) tb[q] = temper(k[q]);
        while (p < kMtN && i >= 1) {
            const uint32_t mask = 0xFFFFFFFFu >> __builtin_clz(i);
            const uint32_t lo = (mask >> 1) + 1;
            uint32_t cur = i;
            while (p < kMtN) {
                const uint32_t c = tb[p++] & mask;
                draws[cur] = c;
                cur -= (uint32_t)(c <= cur);
                if (cur < lo) break;
            }
            i = cur;
        }
    }
    for (int i = 0; i < kMtN; ++i) key[i] = k[i];
    *pos = p;
    return 0;
}

extern "C" int64_t tsrl_shuffle_apply_workspace_bytes(int64_t n) {
    if (n < 0) return -1;
    const int64_t m = n > 1 ? n - 1 : 0;
    return apply_layout(n, cub_sort_bytes(m)).total;
}

extern "C" int tsrl_shuffle_apply(const uint32_t* draws, int64_t n, int64_t* out,
                                  void* workspace, int64_t workspace_bytes, void* stream) {
    TSRL_CHECK_ARG(n >= 0 && n <= (int64_t)INT_MAX,
                   "tsrl_shuffle_apply: n=%lld outside [0, 2^31) (hipcub radix sort int count)",
                   (long long)n);
    if (n == 0) return 0;
    TSRL_CHECK_ARG(draws && out, "tsrl_shuffle_apply: null argument");
    hipStream_t s = as_stream(stream);
    const int64_t m = n - 1;
    const size_t cub_bytes = cub_sort_bytes(m);
    const ApplyLayout L = apply_layout(n, cub_bytes);
    TSRL_CHECK_ARG(workspace && workspace_bytes >= L.total,
                   "tsrl_shuffle_apply: workspace %lld < %lld bytes", (long long)workspace_bytes,
                   (long long)L.total);
    char* ws = static_cast<char*>(workspace);
    uint32_t* keys_out = reinterpret_cast<uint32_t*>(ws + L.keys_out);
    uint32_t* vals_in = reinterpret_cast<uint32_t*>(ws + L.vals_in);
    uint32_t* vals_out = reinterpret_cast<uint32_t*>(ws + L.vals_out);
    uint32_t* first = reinterpret_cast<uint32_t*>(ws + L.first);
    uint32_t* succ = reinterpret_cast<uint32_t*>(ws + L.succ);
    hipError_t e = hipMemsetAsync(first, 0xFF, (size_t)n * 4, s);
    if (e != hipSuccess) {
        set_error("tsrl_shuffle_apply: memset: %s", hipGetErrorString(e));
        return (int)e;
    }
    constexpr int kT = 256;
    if (m > 0) {
        iota_keys_kernel<<<(unsigned)((m + kT - 1) / kT), kT, 0, s>>>(vals_in, m);
        TSRL_LAUNCH_CHECK("iota_keys_kernel");
        size_t tb = cub_bytes;
        e = hipcub::DeviceRadixSort::SortPairs(ws + L.temp, tb, draws + 1, keys_out, vals_in,
                                               vals_out, (int)m, 0, bits_for((uint64_t)m), s);
        if (e != hipSuccess) {
            set_error("tsrl_shuffle_apply: radix sort: %s", hipGetErrorString(e));
            return (int)e;
        }
        hitters_kernel<<<(unsigned)((m + kT - 1) / kT), kT, 0, s>>>(keys_out, vals_out, m, first,
                                                                    succ);
        TSRL_LAUNCH_CHECK("hitters_kernel");
    }
    resolve_kernel<<<(unsigned)((n + kT - 1) / kT), kT, 0, s>>>(draws, n, first, succ, out);
    TSRL_LAUNCH_CHECK("resolve_kernel");
    return 0;
}
