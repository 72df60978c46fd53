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
// The sort is this file's own LSD radix sort (8-bit digits, ceil(bits(n-1) / 8) passes of
// histogram -> exclusive scan -> stable scatter; round 5, replacing hipcub::DeviceRadixSort).
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

// ---- stable LSD radix sort of (key, value) u32 pairs -------------------------------------
// A block owns a tile of RX_TILE consecutive pairs, visited as RX_R rounds of RX_T (pair
// r * RX_T + t of the tile is round r, thread t), so (round, thread) is the input order.
constexpr int RX_T = 256;
constexpr int RX_R = 16;
constexpr int RX_TILE = RX_T * RX_R;  // 4096 pairs
constexpr int RX_D = 256;             // 8-bit digits
constexpr int RX_NW = RX_T / kWave;
constexpr int SC_T = 1024;            // scan blocks: 4 counts per thread
constexpr int SC_SEG = 4 * SC_T;

// hist[d * nblk + b] = pairs of tile b whose digit is d (digit-major, so one exclusive scan
// of the flat array gives every (digit, tile) its output offset)
__global__ __launch_bounds__(RX_T) void radix_hist_kernel(const uint32_t* __restrict__ keys,
                                                          int64_t m, int shift, int64_t nblk,
                                                          uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[RX_D];
    const int t = threadIdx.x;
    h[t] = 0;
    __syncthreads();
    const int64_t b0 = (int64_t)blockIdx.x * RX_TILE;
    uint32_t d[RX_R];
#pragma unroll
    for (int r = 0; r < RX_R; ++r) {  // every load in flight before the counting
        const int64_t i = b0 + r * RX_T + t;
        d[r] = i < m ? (keys[i] >> shift) & (RX_D - 1) : RX_D;
    }
#pragma unroll
    for (int r = 0; r < RX_R; ++r)
        if (d[r] < RX_D) atomicAdd(&h[d[r]], 1u);
    __syncthreads();
    hist[(int64_t)t * nblk + blockIdx.x] = h[t];
}

// Exclusive scan of 1024 thread values (wave scans, then the 16 wave totals); block total
// returned to every thread.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* ws, uint32_t& total) {
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    uint32_t x = v;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, kWave);
        if (lane >= off) x += y;
    }
    if (lane == kWave - 1) ws[w] = x;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
    for (int w2 = 0; w2 < SC_T / kWave; ++w2) {
        const uint32_t s = ws[w2];
        if (w2 < w) pre += s;
        tot += s;
    }
    __syncthreads();
    total = tot;
    return pre + x - v;
}

// part[g] = sum of the counts of segment g
__global__ __launch_bounds__(SC_T) void scan_reduce_kernel(const uint32_t* __restrict__ H,
                                                           int64_t L, uint32_t* __restrict__ part) {
    __shared__ uint32_t ws[SC_T / kWave];
    const int64_t i0 = (int64_t)blockIdx.x * SC_SEG + 4 * threadIdx.x;
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) v += i0 + k < L ? H[i0 + k] : 0u;
    uint32_t tot;
    (void)block_excl_scan(v, ws, tot);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// exclusive scan of the G segment sums, in place (one block, SC_T at a time)
__global__ __launch_bounds__(SC_T) void scan_part_kernel(uint32_t* __restrict__ part, int64_t G) {
    __shared__ uint32_t ws[SC_T / kWave];
    uint32_t carry = 0;
    for (int64_t c = 0; c < G; c += SC_T) {
        const int64_t i = c + threadIdx.x;
        const uint32_t v = i < G ? part[i] : 0u;
        uint32_t tot;
        const uint32_t e = block_excl_scan(v, ws, tot);
        if (i < G) part[i] = carry + e;
        carry += tot;
    }
}

// H := exclusive prefix of H (segment g starts from part[g])
__global__ __launch_bounds__(SC_T) void scan_apply_kernel(uint32_t* __restrict__ H, int64_t L,
                                                          const uint32_t* __restrict__ part) {
    __shared__ uint32_t ws[SC_T / kWave];
    const int64_t i0 = (int64_t)blockIdx.x * SC_SEG + 4 * threadIdx.x;
    uint32_t v[4], s = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        v[k] = i0 + k < L ? H[i0 + k] : 0u;
        s += v[k];
    }
    uint32_t tot;
    uint32_t e = part[blockIdx.x] + block_excl_scan(s, ws, tot);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (i0 + k < L) H[i0 + k] = e;
        e += v[k];
    }
}

// Stable scatter of one digit pass: pair (round r, thread t) of tile b goes to
// off[d][b] + (pairs of digit d in earlier rounds of the tile) + (in this round: earlier
// waves' count of d + the lanes below with d -- a match of the 8 digit-bit ballots).
// vin == nullptr: the value is the pair's index + 1 (the shuffle's step numbers).
__global__ __launch_bounds__(RX_T) void radix_scatter_kernel(
    const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin, int64_t m, int shift,
    int64_t nblk, const uint32_t* __restrict__ off, uint32_t* __restrict__ kout,
    uint32_t* __restrict__ vout) {
    __shared__ uint32_t base[RX_D];
    __shared__ uint32_t wc[RX_NW][RX_D];
    const int t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave;
    base[t] = off[(int64_t)t * nblk + blockIdx.x];
#pragma unroll
    for (int w2 = 0; w2 < RX_NW; ++w2) wc[w2][t] = 0;
    __syncthreads();
    const int64_t b0 = (int64_t)blockIdx.x * RX_TILE;
    const uint64_t below = lane == 0 ? 0ull : (~0ull >> (kWave - lane));
    // the whole tile's pairs loaded up front (all loads in flight at once, not one memory
    // latency per round)
    uint32_t kr[RX_R], vr[RX_R];
#pragma unroll
    for (int r = 0; r < RX_R; ++r) {
        const int64_t i = b0 + r * RX_T + t;
        kr[r] = i < m ? kin[i] : 0u;
        vr[r] = i < m ? (vin ? vin[i] : (uint32_t)(i + 1)) : 0u;
    }
#pragma unroll
    for (int r = 0; r < RX_R; ++r) {
        const int64_t i = b0 + r * RX_T + t;
        const bool valid = i < m;
        const uint32_t key = kr[r];
        const uint32_t val = vr[r];
        const uint32_t d = (key >> shift) & (RX_D - 1);
        uint64_t match = __ballot(valid);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const bool bit = (d >> k) & 1u;
            const uint64_t bk = __ballot(bit);
            match &= bit ? bk : ~bk;
        }
        const uint32_t rank = (uint32_t)__popcll(match & below);
        if (valid && rank == 0) wc[w][d] = (uint32_t)__popcll(match);
        __syncthreads();
        if (valid) {
            uint32_t pre = 0;
            for (int w2 = 0; w2 < w; ++w2) pre += wc[w2][d];
            const uint32_t pos = base[d] + pre + rank;
            kout[pos] = key;
            vout[pos] = val;
        }
        __syncthreads();
        uint32_t sum = 0;
#pragma unroll
        for (int w2 = 0; w2 < RX_NW; ++w2) {
            sum += wc[w2][t];
            wc[w2][t] = 0;
        }
        base[t] += sum;
        __syncthreads();
    }
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
    int64_t keys_out, vals_out, keys_tmp, vals_tmp, first, succ, hist, part, total;
    int64_t nblk, L, G;
};

inline ApplyLayout apply_layout(int64_t n) {
    ApplyLayout L;
    const int64_t m = n > 1 ? n - 1 : 0;
    L.nblk = (m + RX_TILE - 1) / RX_TILE;
    L.L = (int64_t)RX_D * L.nblk;
    L.G = (L.L + SC_SEG - 1) / SC_SEG;
    int64_t off = 0;
    L.keys_out = off; off += align256(m * 4);
    L.vals_out = off; off += align256(m * 4);
    L.keys_tmp = off; off += align256(m * 4);
    L.vals_tmp = off; off += align256(m * 4);
    L.first = off; off += align256(n * 4);
    L.succ = off; off += align256(n * 4);
    L.hist = off; off += align256(L.L * 4);
    L.part = off; off += align256(L.G * 4);
    L.total = off;
    return L;
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
    return apply_layout(n).total;
}

extern "C" int tsrl_shuffle_apply(const uint32_t* draws, int64_t n, int64_t* out,
                                  void* workspace, int64_t workspace_bytes, void* stream) {
    TSRL_CHECK_ARG(n >= 0 && n <= (int64_t)INT_MAX,
                   "tsrl_shuffle_apply: n=%lld outside [0, 2^31) (u32 sort positions)",
                   (long long)n);
    if (n == 0) return 0;
    TSRL_CHECK_ARG(draws && out, "tsrl_shuffle_apply: null argument");
    hipStream_t s = as_stream(stream);
    const int64_t m = n - 1;
    const ApplyLayout L = apply_layout(n);
    TSRL_CHECK_ARG(workspace && workspace_bytes >= L.total,
                   "tsrl_shuffle_apply: workspace %lld < %lld bytes", (long long)workspace_bytes,
                   (long long)L.total);
    char* ws = static_cast<char*>(workspace);
    uint32_t* keys_out = reinterpret_cast<uint32_t*>(ws + L.keys_out);
    uint32_t* vals_out = reinterpret_cast<uint32_t*>(ws + L.vals_out);
    uint32_t* keys_tmp = reinterpret_cast<uint32_t*>(ws + L.keys_tmp);
    uint32_t* vals_tmp = reinterpret_cast<uint32_t*>(ws + L.vals_tmp);
    uint32_t* first = reinterpret_cast<uint32_t*>(ws + L.first);
    uint32_t* succ = reinterpret_cast<uint32_t*>(ws + L.succ);
    uint32_t* hist = reinterpret_cast<uint32_t*>(ws + L.hist);
    uint32_t* part = reinterpret_cast<uint32_t*>(ws + L.part);
    hipError_t e = hipMemsetAsync(first, 0xFF, (size_t)n * 4, s);
    if (e != hipSuccess) {
        set_error("tsrl_shuffle_apply: memset: %s", hipGetErrorString(e));
        return (int)e;
    }
    constexpr int kT = 256;
    if (m > 0) {
        // stable sort of (j_s, s), s = 1 .. n-1: ceil(bits / 8) digit passes, ping-ponging so
        // that the last pass lands in keys_out / vals_out
        const int npass = (bits_for((uint64_t)m) + 7) / 8;
        const uint32_t* kin = draws + 1;
        const uint32_t* vin = nullptr;  // pass 0: values = index + 1
        for (int ps = 0; ps < npass; ++ps) {
            const bool to_out = ((npass - 1 - ps) & 1) == 0;
            uint32_t* ko = to_out ? keys_out : keys_tmp;
            uint32_t* vo = to_out ? vals_out : vals_tmp;
            const int shift = 8 * ps;
            radix_hist_kernel<<<(unsigned)L.nblk, RX_T, 0, s>>>(kin, m, shift, L.nblk, hist);
            scan_reduce_kernel<<<(unsigned)L.G, SC_T, 0, s>>>(hist, L.L, part);
            scan_part_kernel<<<1, SC_T, 0, s>>>(part, L.G);
            scan_apply_kernel<<<(unsigned)L.G, SC_T, 0, s>>>(hist, L.L, part);
            radix_scatter_kernel<<<(unsigned)L.nblk, RX_T, 0, s>>>(kin, vin, m, shift, L.nblk,
                                                                    hist, ko, vo);
            TSRL_LAUNCH_CHECK("tsrl_shuffle_apply(radix pass)");
            kin = ko;
            vin = vo;
        }
        hitters_kernel<<<(unsigned)((m + kT - 1) / kT), kT, 0, s>>>(keys_out, vals_out, m, first,
                                                                    succ);
        TSRL_LAUNCH_CHECK("hitters_kernel");
    }
    resolve_kernel<<<(unsigned)((n + kT - 1) / kT), kT, 0, s>>>(draws, n, first, succ, out);
    TSRL_LAUNCH_CHECK("resolve_kernel");
    return 0;
}
