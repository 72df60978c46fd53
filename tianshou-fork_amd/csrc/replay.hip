// Off-policy neighbours of the on-policy path: the numba kernels of
// the n-step return and of the prioritized-replay sum tree, on device.
//
// nstep  : BasePolicy.compute_nstep_return + _nstep_return (tianshou/policy/base.py:386-440,
//          500-524).  One thread per (sampled row, target column): it walks the row's next()
//          chain (manager.py:280-297, ring.h), then runs the reference's backward Horner
//          recurrence in f64 in the reference's operation order (returns = rew + gamma *
//          returns, reset to 0 at an episode end, gammas = first end + 1), and writes
//          f64(target_q * value_mask) * gamma^gammas + returns rounded to the target dtype.
// segtree: SegmentTree (tianshou/data/utils/segtree.py:7-137), the f64 sum tree in a binary
//          heap of 2 * bound nodes (leaves at [bound, 2 * bound)).
//          set    (_setitem, :98-104): the leaves first -- with duplicate indices the LAST
//                 occurrence wins, as numpy's fancy assignment does (an atomicMax on the
//                 position per leaf picks it) -- then the parents level by level,
//                 parent = left + right, the reference's f64 sums.  One workgroup, a barrier
//                 per level (PER updates are minibatch-sized).
//          reduce (_reduce, :107-119): the reference's exact summation order, one thread.
//          prefix (_get_prefix_sum_idx, :122-137): one descent per query value; f32 query
//                 arrays keep numpy's in-place f32 rounding after every subtraction.
#include "ring.h"

namespace tsrl {
namespace {

constexpr int TPB = 256;
constexpr int SET_TPB = 1024;
constexpr int MAX_NSTEP = 64;

// Plain operators under fp contract(off): HIP's __dmul_rn / __dadd_rn are ordinary operators
// defined in a header compiled with contraction on, so a mul feeding an add through them
// still fuses into an FMA (one rounding instead of NumPy's two).
template <typename T>
__global__ __launch_bounds__(TPB) void nstep_kernel(Ring g, const double* __restrict__ rew,
                                                    const uint8_t* __restrict__ terminated,
                                                    const int64_t* __restrict__ idx,
                                                    int64_t bsz, int n_step, double gamma,
                                                    const T* __restrict__ target_q, int64_t X,
                                                    T* __restrict__ out) {
#pragma clang fp contract(off)
    const int64_t t = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (t >= bsz * X) return;
    const int64_t b = t / X;
    int64_t chain[MAX_NSTEP];
    chain[0] = pmod(idx[b], g.maxsize);
    for (int n = 1; n < n_step; ++n) chain[n] = ring_next(g, chain[n - 1]);
    // value mask of the terminal row (base.py:432): ~terminated[indices[-1]]
    const T q = target_q[t] * (T)(terminated[chain[n_step - 1]] ? 0 : 1);
    double ret = 0.0;
    int gammas = n_step;
    for (int n = n_step - 1; n >= 0; --n) {
        const int64_t now = chain[n];
        if (ring_end(g, now)) {
            gammas = n + 1;
            ret = 0.0;
        }
        ret = rew[now] + gamma * ret;  // two roundings: fp contract(off) above
    }
    double gp = 1.0;  // gamma_buffer[gammas]: repeated products, as base.py:509-511
    for (int i = 1; i <= gammas; ++i) gp = gp * gamma;
    out[t] = (T)((double)q * gp + ret);
}

// win: int32 scratch of one entry per leaf, all -1 on entry (restored on exit).
__global__ __launch_bounds__(SET_TPB) void segtree_set_kernel(double* tree, int64_t bound,
                                                             const int64_t* __restrict__ idx,
                                                             const double* __restrict__ val,
                                                             int64_t val_stride, int64_t k,
                                                             int* win) {
    const int tid = threadIdx.x;
    for (int64_t j = tid; j < k; j += SET_TPB) atomicMax(&win[idx[j]], (int)j);
    __syncthreads();
    for (int64_t j = tid; j < k; j += SET_TPB) {
        const int64_t i = idx[j];
        if (win[i] == (int)j) tree[bound + i] = val[j * val_stride];
    }
    __syncthreads();
    for (int64_t j = tid; j < k; j += SET_TPB) win[idx[j]] = -1;
    for (int lvl = 1; (bound >> lvl) >= 1; ++lvl) {
        __syncthreads();
        for (int64_t j = tid; j < k; j += SET_TPB) {
            const int64_t p = (bound + idx[j]) >> lvl;
            tree[p] = tree[2 * p] + tree[2 * p + 1];
        }
    }
}

__global__ void segtree_reduce_kernel(const double* tree, int64_t start, int64_t end,
                                      double* out) {
#pragma clang fp contract(off)
    double result = 0.0;
    while (end - start > 1) {
        if (start % 2 == 0) result += tree[start + 1];
        start /= 2;
        if (end % 2 == 1) result += tree[end - 1];
        end /= 2;
    }
    *out = result;
}

template <typename T>
__global__ __launch_bounds__(TPB) void segtree_prefix_kernel(const double* __restrict__ tree,
                                                             int64_t bound,
                                                             const T* __restrict__ value,
                                                             int64_t k, int64_t* out) {
    const int64_t j = (int64_t)blockIdx.x * TPB + threadIdx.x;
    if (j >= k) return;
    T v = value[j];
    int64_t index = 1;
    while (index < bound) {
        index *= 2;
        const double l = tree[index];
        const bool direct = l < (double)v;
        if (direct) v = (T)((double)v - l);
        index += direct;
    }
    out[j] = index - bound;
}

}  // namespace
}  // namespace tsrl

using namespace tsrl;

extern "C" int tsrl_nstep_return(const double* rew, const uint8_t* done,
                                 const uint8_t* terminated, const int64_t* last_index,
                                 const int64_t* lengths, int64_t size, int64_t num,
                                 const int64_t* idx, int64_t bsz, int64_t n_step, double gamma,
                                 const void* target_q, int64_t X, int f64, void* out,
                                 void* stream) {
    TSRL_CHECK_ARG(bsz >= 0 && X >= 1 && n_step >= 1 && n_step <= MAX_NSTEP,
                   "tsrl_nstep_return: bad sizes (1 <= n_step <= %d, X >= 1)", MAX_NSTEP);
    if (bsz == 0) return 0;
    TSRL_CHECK_ARG(rew && done && terminated && last_index && lengths && idx && target_q && out,
                   "tsrl_nstep_return: null pointer");
    TSRL_CHECK_ARG(size > 0 && num > 0, "tsrl_nstep_return: empty buffer");
    const Ring g = {done, last_index, lengths, size, size * num};
    const unsigned grid = (unsigned)((bsz * X + TPB - 1) / TPB);
    if (f64)
        hipLaunchKernelGGL(nstep_kernel<double>, dim3(grid), dim3(TPB), 0, as_stream(stream), g,
                           rew, terminated, idx, bsz, (int)n_step, gamma,
                           reinterpret_cast<const double*>(target_q), X,
                           reinterpret_cast<double*>(out));
    else
        hipLaunchKernelGGL(nstep_kernel<float>, dim3(grid), dim3(TPB), 0, as_stream(stream), g,
                           rew, terminated, idx, bsz, (int)n_step, gamma,
                           reinterpret_cast<const float*>(target_q), X,
                           reinterpret_cast<float*>(out));
    TSRL_LAUNCH_CHECK("tsrl_nstep_return");
    return 0;
}

extern "C" int tsrl_segtree_set(double* tree, int64_t bound, const int64_t* idx,
                                const double* values, int64_t value_stride, int64_t k,
                                int* win, void* stream) {
    TSRL_CHECK_ARG(bound >= 1 && (bound & (bound - 1)) == 0 && k >= 0 && k < (1ll << 31) &&
                       (value_stride == 0 || value_stride == 1),
                   "tsrl_segtree_set: bad sizes (bound a power of 2, stride 0 or 1)");
    if (k == 0) return 0;
    TSRL_CHECK_ARG(tree && idx && values && win, "tsrl_segtree_set: null pointer");
    hipLaunchKernelGGL(segtree_set_kernel, dim3(1), dim3(SET_TPB), 0, as_stream(stream), tree,
                       bound, idx, values, value_stride, k, win);
    TSRL_LAUNCH_CHECK("tsrl_segtree_set");
    return 0;
}

extern "C" int tsrl_segtree_reduce(const double* tree, int64_t bound, int64_t start,
                                   int64_t end, double* out, void* stream) {
    // any range the reference accepts: an empty or inverted one sums nothing (segtree.py:112)
    TSRL_CHECK_ARG(tree && out && bound >= 1 && start + bound - 1 >= 0 && end <= bound,
                   "tsrl_segtree_reduce: bad range");
    hipLaunchKernelGGL(segtree_reduce_kernel, dim3(1), dim3(1), 0, as_stream(stream), tree,
                       start + bound - 1, end + bound, out);
    TSRL_LAUNCH_CHECK("tsrl_segtree_reduce");
    return 0;
}

extern "C" int tsrl_segtree_prefix_idx(const double* tree, int64_t bound, const void* values,
                                       int f64, int64_t k, int64_t* out, void* stream) {
    TSRL_CHECK_ARG(bound >= 1 && (bound & (bound - 1)) == 0 && k >= 0,
                   "tsrl_segtree_prefix_idx: bad sizes");
    if (k == 0) return 0;
    TSRL_CHECK_ARG(tree && values && out, "tsrl_segtree_prefix_idx: null pointer");
    const unsigned grid = (unsigned)((k + TPB - 1) / TPB);
    if (f64)
        hipLaunchKernelGGL(segtree_prefix_kernel<double>, dim3(grid), dim3(TPB), 0,
                           as_stream(stream), tree, bound,
                           reinterpret_cast<const double*>(values), k, out);
    else
        hipLaunchKernelGGL(segtree_prefix_kernel<float>, dim3(grid), dim3(TPB), 0,
                           as_stream(stream), tree, bound,
                           reinterpret_cast<const float*>(values), k, out);
    TSRL_LAUNCH_CHECK("tsrl_segtree_prefix_idx");
    return 0;
}
