// The reference RunningMeanStd.update in its own f32 arithmetic, bit for bit, as workgroup
// device code (statistics.py:93-114; np.mean / np.var over axis 0 of a C-contiguous f32
// array: sequential f32 column sums in row order).  Used by rms.hip's rms_exact_kernel
// (tsrl_rms_exact_update).  A workgroup of XT = 512 threads owns XC = 8 consecutive columns.
//
// Data flow of one update over rows b (see rms.hip for the performance reasoning):
//   list   the rows a mask selects, in row order (one pass: 8 rows per thread, wave prefix
//          sums by shuffles, one barrier);
//   load   the selected rows' 8 columns into LDS as [column][row] runs (every load of a
//          thread in flight before its first LDS store);
//   chain  lanes 0-7 of one wave: acc = ((acc + x0) + x1) + ... over the column's run,
//          ds_read_b128 of 4 rows, the next 32 rows' reads in flight behind the adds;
//   sq     every thread: x -> (x - mean)^2 in place (float4 per lane), so the var chain is
//          the same pure add chain.
#pragma once
#include "tsrl_common.h"

namespace tsrl {
namespace exact {

constexpr int XC = 8;    // columns per workgroup
constexpr int XT = 512;  // threads per workgroup (8 waves: wave w <-> column w in `sq`)

struct Rows {
    const float* x;       // [k, dim]
    const uint8_t* mask;  // rows taken (NULL: all), in row order
    int64_t k;
};

// LDS of one workgroup: the main span (SPAN rows x 8 columns, pitch SPAN + 4 floats: a 4-bank
// skew between columns so lanes 0-7's ds_read_b128 hit distinct banks), the side span for the
// concurrent second update (SPAN2 rows), the row lists.
template <int SPAN, int SPAN2>
struct Smem {
    float col[XC][SPAN + 4];
    union {
        float col2[XC][SPAN2 + 4];  // concurrent path: the second update's rows
        int list[SPAN];             // sequential path: a masked span's row list
    };
    int list2[SPAN2];
    float bm[XC];      // the main span's batch mean (published by the chain wave)
    float bm2[XC], bv2[XC];  // the second update's batch mean / var (wave 1)
    int wsum[XT / 64];
    int nsel;
};

// Rows [s0, s0 + span) selected by mask -> list[0, min(n, cap)) in row order; returns n (the
// full count, also when it exceeds cap).  span <= 8 * XT.  Ends with a barrier.
__device__ __forceinline__ int build_list(const uint8_t* __restrict__ mask, int64_t s0, int span,
                                          int* list, int cap, int* wsum) {
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    constexpr int RPT = 8;
    const int r0 = t * RPT;
    uint32_t bits = 0;
    int cnt = 0;
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
        const int r = r0 + j;
        const bool sel = r < span && mask[s0 + r];
        bits |= (uint32_t)sel << j;
        cnt += sel;
    }
    int x = cnt;  // inclusive scan over the wave
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (l >= o) x += y;
    }
    if (l == 63) wsum[w] = x;
    __syncthreads();
    int base = 0, tot = 0;
#pragma unroll
    for (int u = 0; u < XT / 64; ++u) {
        const int ws = wsum[u];
        base += u < w ? ws : 0;
        tot += ws;
    }
    int pos = base + x - cnt;
#pragma unroll
    for (int j = 0; j < RPT; ++j)
        if ((bits >> j) & 1u) {
            if (pos < cap) list[pos] = r0 + j;
            ++pos;
        }
    __syncthreads();
    return tot;
}

// Load n rows into col[c][0, n) for columns [c0, c0 + XC): row e of the run is source row
// s0 + (list ? list[e] : e).  Wave w takes column half h = w & 1 and rows (w >> 1) * 64 + lane
// + 256 j: 64 consecutive rows per store group (conflict-free LDS stores), every load of a
// thread issued before its first store.  vec4: rows are read as two float4 per row.
template <int J, int P>
__device__ __forceinline__ void load_rows(const float* __restrict__ x, int64_t dim, int64_t c0,
                                          int64_t s0, int n, const int* list, bool vec4,
                                          float (*col)[P]) {
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    const int h = w & 1;
    const int rb = (w >> 1) * 64 + l;
    if (vec4) {
        float4 v[J];
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const int e = rb + 256 * j;
            v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (e < n) {
                const int64_t r = s0 + (list ? list[e] : e);
                v[j] = *reinterpret_cast<const float4*>(x + r * dim + c0 + 4 * h);
            }
        }
#pragma unroll
        for (int j = 0; j < J; ++j) {
            const int e = rb + 256 * j;
            if (e < n) {
                col[4 * h + 0][e] = v[j].x;
                col[4 * h + 1][e] = v[j].y;
                col[4 * h + 2][e] = v[j].z;
                col[4 * h + 3][e] = v[j].w;
            }
        }
    } else {
        // any dim / alignment: 4 scalar loads per row and half (columns past dim read 0)
#pragma unroll 4
        for (int j = 0; j < J; ++j) {
            const int e = rb + 256 * j;
            if (e >= n) break;
            const int64_t r = s0 + (list ? list[e] : e);
            float v[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int64_t c = c0 + 4 * h + q;
                v[q] = c < dim ? x[r * dim + c] : 0.0f;
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) col[4 * h + q][e] = v[q];
        }
    }
}

__device__ __forceinline__ void chain_ld(const float* p, float4 (&v)[8]) {
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(p + 4 * u);
}
__device__ __forceinline__ float chain_add(float acc, const float4 (&v)[8]) {
#pragma clang fp contract(off)
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        acc = acc + v[u].x;
        acc = acc + v[u].y;
        acc = acc + v[u].z;
        acc = acc + v[u].w;
    }
    return acc;
}
// acc = (((acc + v0) + v1) + ... + v_{n-1}) in f32 over one lane's LDS run (16-byte aligned):
// two ping-pong register blocks of 32 rows, the reads of one block issued before the 32 adds of
// the other (the scheduling barriers keep them there: without them the loop is rotated so
// that every block's reads are waited for right after their issue).
__device__ __forceinline__ float chain(const float* cp, int n, float acc) {
#pragma clang fp contract(off)
    int e = 0;
    if (n >= 64) {
        float4 A[8], B[8];
        chain_ld(cp, A);
        for (; e + 96 <= n; e += 64) {  // A holds rows [e, e + 32)
            chain_ld(cp + e + 32, B);
            __builtin_amdgcn_sched_barrier(0);
            acc = chain_add(acc, A);
            chain_ld(cp + e + 64, A);
            __builtin_amdgcn_sched_barrier(0);
            acc = chain_add(acc, B);
        }
        if (e + 64 <= n) {
            chain_ld(cp + e + 32, B);
            __builtin_amdgcn_sched_barrier(0);
            acc = chain_add(acc, A);
            acc = chain_add(acc, B);
            e += 64;
        } else {
            acc = chain_add(acc, A);
            e += 32;
        }
    }
    for (; e < n; ++e) acc = acc + cp[e];
    return acc;
}

// col[c][0, n) -> (col[c][e] - bm[c])^2 for the 8 columns, by all XT threads (wave w <->
// column w, float4 per lane).  No barrier.
template <int P>
__device__ __forceinline__ void square_dev(float (*col)[P], int n, const float* bm) {
#pragma clang fp contract(off)
    const int t = threadIdx.x, c = t >> 6, l = t & 63;
    const float b = bm[c];
    float* p = col[c];
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

// RunningMeanStd.update_from_moments (statistics.py:103-114) in f32 with the counts as f32.
__device__ __forceinline__ void merge(float& mean, float& var, double& cnt, float bm, float bv,
                                      int64_t k) {
#pragma clang fp contract(off)
    const float kf = (float)k;
    const double tot = cnt + (double)k;
    const float cf = (float)cnt, tf = (float)tot;
    const float delta = bm - mean;
    const float new_mean = mean + (delta * kf) / tf;
    const float m_a = var * cf;
    const float m_b = bv * kf;
    const float m_2 = (m_a + m_b) + (((delta * delta) * cf) * kf) / tf;
    mean = new_mean;
    var = m_2 / tf;
    cnt = tot;
}

// One update over b, sequentially span by span (any k, any mask).  mean / var / cnt of lanes
// t < XC are updated; every thread must call it.  Ends with a barrier.
template <int SPAN, int SPAN2>
__device__ void update_seq(const Rows& b, int64_t dim, int64_t c0, float& mean, float& var,
                           double& cnt, Smem<SPAN, SPAN2>& sm) {
#pragma clang fp contract(off)
    const int t = threadIdx.x;
    const bool chain_lane = t < XC;
    const bool vec4 = (dim & 3) == 0 && (reinterpret_cast<uintptr_t>(b.x) & 15) == 0 &&
                      c0 + XC <= dim;
    const bool listed = b.mask != nullptr;
    const int nspan = (int)((b.k + SPAN - 1) / SPAN);
    float S = 0.0f;
    int64_t total = 0;
    int n = 0;
    for (int sp = 0; sp < nspan; ++sp) {
        const int64_t s0 = (int64_t)sp * SPAN;
        const int span = (int)min((int64_t)SPAN, b.k - s0);
        n = listed ? build_list(b.mask, s0, span, sm.list, SPAN, sm.wsum) : span;
        load_rows<SPAN / 256>(b.x, dim, c0, s0, n, listed ? sm.list : nullptr, vec4, sm.col);
        __syncthreads();
        if (chain_lane) S = chain(&sm.col[t][0], n, S);
        total += n;
        __syncthreads();  // the next span (or the squares) overwrite the columns
    }
    if (total == 0) return;  // the reference updates only with rows (Collector resets none)
    const float kf = (float)total;
    if (chain_lane) sm.bm[t] = S / kf;
    __syncthreads();
    float Q = 0.0f;
    for (int sp = 0; sp < nspan; ++sp) {
        const int64_t s0 = (int64_t)sp * SPAN;
        const int span = (int)min((int64_t)SPAN, b.k - s0);
        if (nspan > 1) {  // the single span is still resident
            n = listed ? build_list(b.mask, s0, span, sm.list, SPAN, sm.wsum) : span;
            load_rows<SPAN / 256>(b.x, dim, c0, s0, n, listed ? sm.list : nullptr, vec4,
                                  sm.col);
            __syncthreads();
        }
        square_dev(sm.col, n, sm.bm);
        __syncthreads();
        if (chain_lane) Q = chain(&sm.col[t][0], n, Q);
        __syncthreads();
    }
    if (chain_lane) merge(mean, var, cnt, sm.bm[t], Q / kf, total);
}

// b1's update, then b2's (when b2.x): the state after b1 goes to snap_mean / snap_var.  When
// b1 is unmasked and fits one span and b2's selected rows fit the side span, b2's chains run on
// wave 1 concurrently with b1's on wave 0 (b2's batch moments do not depend on b1); otherwise
// the two updates run one after the other.  Returns the count after both (lanes t < XC hold
// mean / var / snap).
template <int SPAN, int SPAN2>
__device__ double two_updates(const Rows& b1, const Rows& b2, int64_t dim, int64_t c0,
                              double cnt, float& mean, float& var, float& snap_mean,
                              float& snap_var, Smem<SPAN, SPAN2>& sm) {
#pragma clang fp contract(off)
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    int nd = -1;
    const bool cand = b2.x && b1.mask == nullptr && b1.k <= SPAN && b2.k <= 8 * XT;
    if (cand)
        nd = b2.mask ? build_list(b2.mask, 0, (int)b2.k, sm.list2, SPAN2, sm.wsum) : (int)b2.k;
    if (!cand || nd > SPAN2) {
        update_seq(b1, dim, c0, mean, var, cnt, sm);
        snap_mean = mean;
        snap_var = var;
        if (b2.x) update_seq(b2, dim, c0, mean, var, cnt, sm);
        return cnt;
    }
    const int n1 = (int)b1.k;
    const bool vec1 = (dim & 3) == 0 && (reinterpret_cast<uintptr_t>(b1.x) & 15) == 0 &&
                      c0 + XC <= dim;
    const bool vec2 = (dim & 3) == 0 && (reinterpret_cast<uintptr_t>(b2.x) & 15) == 0 &&
                      c0 + XC <= dim;
    load_rows<SPAN / 256>(b1.x, dim, c0, 0, n1, nullptr, vec1, sm.col);
    if (nd > 0)
        load_rows<(SPAN2 + 255) / 256>(b2.x, dim, c0, 0, nd, b2.mask ? sm.list2 : nullptr, vec2,
                                       sm.col2);
    __syncthreads();
    float S1 = 0.0f;
    if (w == 0 && l < XC) {
        S1 = chain(&sm.col[l][0], n1, 0.0f);
        if (n1 > 0) sm.bm[l] = S1 / (float)n1;
    } else if (w == 1 && l < XC && nd > 0) {
        // the reset rows' two chains, entirely in this wave: the squares are written and read
        // back by the same lane (program order), so no barrier is needed
        const float kf2 = (float)nd;
        float* p = sm.col2[l];
        const float S2 = chain(p, nd, 0.0f);
        const float m2 = S2 / kf2;
        for (int e = 0; e < nd; ++e) {
            const float d = p[e] - m2;
            p[e] = d * d;
        }
        const float Q2 = chain(p, nd, 0.0f);
        sm.bm2[l] = m2;
        sm.bv2[l] = Q2 / kf2;
    }
    __syncthreads();
    if (n1 > 0) {
        square_dev(sm.col, n1, sm.bm);
        __syncthreads();
        if (w == 0 && l < XC) {
            const float Q1 = chain(&sm.col[l][0], n1, 0.0f);
            merge(mean, var, cnt, sm.bm[l], Q1 / (float)n1, n1);
        }
    }
    snap_mean = mean;
    snap_var = var;
    if (w == 0 && l < XC && nd > 0) merge(mean, var, cnt, sm.bm2[l], sm.bv2[l], nd);
    // every lane returns the count (the same arithmetic as the chain lanes')
    double c = cnt;
    if (!(w == 0 && l < XC)) {
        c = cnt + (n1 > 0 ? (double)n1 : 0.0) + (nd > 0 ? (double)nd : 0.0);
    }
    return c;
}

}  // namespace exact
}  // namespace tsrl
