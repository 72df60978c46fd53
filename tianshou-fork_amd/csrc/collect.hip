// One vector step of Collector.collect (tianshou/data/collector.py:258-361) as ONE launch, for
// the fused device path: a SyntheticVectorEnv with Box observations under VectorEnvNormObs
// (env/venv_wrappers.py:77-99, utils/statistics.py:93-114) and the MuJoCo Gaussian actor of
// utils/models.py:34-97 sampled as in pg.py:133-171.
//
// Before: four launches per step (tsrl_gauss_policy_act_rng -> tsrl_synth_box_step_reset ->
// tsrl_rms_merge2 -> tsrl_buffer_add), each a few microseconds of latency chain on 4096 rows.
// The add of step i needs the obs_rms state merged from ALL of step i's rows, so it cannot
// run in step i's launch without a grid barrier; it runs at the START of step i+1's launch
// instead (the step sequence rotated by one, "pending add"), and the caller issues the last
// step's add as a plain tsrl_buffer_add.  Per workgroup of R = 16 env rows, in order:
//   A. the pending add of step i-1 for these rows (add_row of buffer.hip: obs, act, the
//      normalised obs_next, reset rows, flags, episode statistics), the new live obs rows
//      also landing in LDS;
//   B. the actor on those rows (f32 MFMA 16x16x4: layer 1's K split over the 8 waves, layer 2
//      and the mu head over k halves / quarters, partials folded in fixed order), the noise
//      and map_action exactly as policy.hip;
//   C. the env step + auto-reset of these rows (synth.h, as env.hip's box_step_reset_kernel)
//      with the column moments of the step rows and of the reset rows;
//   D. obs_rms: the synthetic env's values are x = m 2^-23 with integer |m| <= 2^23
//      (synth.h), so the column moments are summed EXACTLY as integers by 64-bit atomics into
//      a per-step totals slot -- exact sums are independent of the summation order, so no
//      ordered fold is needed.  Bound: one row adds at most 2^46 to a column's sum of m^2, so
//      the int64 sums are exact while the rows behind one slot (k, or world * k after the
//      data-parallel all-reduce) stay <= 2^17; tsrl_collect_box_step checks k and the caller
//      checks world * k.  The slot also counts its step rows ([4D + 1], one atomic per
//      workgroup), so the merge never assumes equal env shards across ranks.
//      Totals ring (three slots, `rms_step` = i, the launch's index in its chain): launch i
//      accumulates slot i % 3, merges slot (i - 1) % 3 (the previous launch's totals) into the
//      RunningMeanStd in its prologue -- every workgroup does the merge itself, since its
//      pending add needs exactly those statistics -- and workgroup 0 zeroes slot (i + 1) % 3,
//      the slot launch i + 1 will accumulate (last read by launch i - 1, finished before
//      launch i started).  Workgroup 0 also publishes the merged state into state slot
//      (i + 1) % 2 for launch i + 1.  The first launch of a chain (i = 0) reads the caller's
//      state and relies on slots 0 and 1 being zero: a fresh (zeroed) workspace or the
//      previous chain's tsrl_collect_rms_finalize, which merges the last launch's slot and
//      clears all three.  The launch therefore ends with its env rows, with no grid-wide
//      hand-off.  With `no_moments` set (exact obs_rms) the launch computes no moments at
//      all: the caller runs tsrl_rms_exact_update on the raw step / reset rows between
//      launches, and the pending add normalises with the caller's mean / var / snapshot.
//   E. Pipelined exact obs_rms (`xpipe`, the action-independent env): the reference's f32
//      statistic needs two k-long dependent f32 add chains per column and update (~30 us at
//      4096 rows), which serialised between launches cost 3x the default collect.  The env
//      does not read the action, so its rows of step i + d are computed d launches early by a
//      "spec" env (its own counters spec_j / spec_t, started from the env's at the head of
//      each captured graph by tsrl_collect_spec_step) into a ring slot; the chains of step
//      i's rows (tsrl_rms_exact_stats, batch moments only) run on a second graph branch
//      concurrently with launches i - d + 1 .. i, and launch i + 1 merges them in its
//      prologue with update_from_moments' f32 arithmetic (rms_exact.h merge) -- the same
//      state slots as the deferred merge of D, no totals, no moments.  This launch's own env
//      phase then writes only the step's flags / reward / counters; the pending add reads the
//      ring slot's rows.
#include "add_row.h"
#include "noise.h"
#include "rms_exact.h"
#include "synth.h"

namespace tsrl {
namespace {

using synth::box_val;
using synth::env_key;
using synth::REW_SALT;
using synth::RowState;

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int R = 16;          // env rows per workgroup
constexpr int NW = 8;          // waves per workgroup
constexpr int NT = NW * 64;
constexpr int H = 64;          // actor hidden width
constexpr int AMAX = 32;
constexpr int KMAX = 512;      // observation columns handled (padded to 128)
constexpr int XP = 17;         // LDS pitch of the live-obs tile sX[col][row]
constexpr int HP = 16;         // h1 / h2 tiles [feature][row]
constexpr int WP = 68;         // W2 / W3 rows (4i + k banks: conflict-free A fragments)
// diagnostic builds only: per-workgroup s_memrealtime stamps (100 MHz) after each phase,
// stored behind the workspace (tools/collect_step_bench.py --trace)
#ifndef COLLECT_TRACE
#define COLLECT_TRACE 0
#endif
#if COLLECT_TRACE
#define TSTAMP(i) \
    if (t == 0) ws.trace[((rng_step & 15) * gridDim.x + blockIdx.x) * 8 + (i)] = __builtin_amdgcn_s_memrealtime();
// detail stamps of the prologue, in a second area of the same shape
#define TSTAMP2(i) \
    if (t == 0) ws.trace[(16 + (rng_step & 15)) * gridDim.x * 8 + blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memrealtime();
#else
#define TSTAMP(i)
#define TSTAMP2(i)
#endif

// The replay rows this step writes (obs and obs_next: 12.6 MB per 4096 x 376 step, not read
// again by this collect) leave as write-through `sc1` vector stores (inline asm, s_nop 1
// after each so the data VGPRs are read before reuse): no dirty lines for the end-of-kernel
// write-back, 23.97-24.04 vs 25.66-25.87 us per step with plain stores, two A/B rounds in one
// call (tools/collect_ab.sh, round 3).  Measured and dropped: the raw env rows (re-read by
// the next launch) write-through as well (24.13-24.21), non-temporal stores (26.2 vs 25.6),
// relaxed agent-scope 8-byte atomic stores (28.9).
// Round 5 A/B of the round-4 variants (tools/r05_ab.sh, profiles/r05_variant_ab.log), all
// three now the only form: 24.0-24.2 -> 21.5 us per step together (each alone: 24.1 / 23.6 /
// 23.4) --
//  * the env rows' counter keys, reward and flags are computed at the top of the launch by
//    the last R threads (wave 7: no merge column for D <= NT - R) while the merge's loads are
//    in flight, and the env phase only stores them;
//  * sqrt(var + eps) of both statistics is computed once per column and staged in LDS, and
//    the add divides by it (same bits as a correctly rounded square root per element);
//  * this step's stored obs rows leave LDS one column per thread over the 16 rows (no integer
//    division by D per element).
__device__ __forceinline__ void row_store4(float4* p, float4 x) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v v = {x.x, x.y, x.z, x.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void row_store1(float* p, float x) {
    asm volatile("global_store_dword %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(x) : "memory");
}

// Workgroup barrier that orders LDS only: outstanding global loads and stores stay in flight
// (__syncthreads also waits for every global store's acknowledgement and every pending load)
#define LDS_SYNC()                                                                          \
    do {                                                                                    \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                  \
        __builtin_amdgcn_s_barrier();                                                       \
        asm volatile("" ::: "memory");                                                      \
    } while (0)

__host__ __device__ inline int64_t kpad(int64_t dim) { return (dim + 127) / 128 * 128; }

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// packed[((w * SQ + sq) * 4 + ft) * 64 + lane][e] = W[16 ft + (lane & 15)][w * KW + 4 (4 sq + e)
// + (lane >> 4)] (0 beyond dim): wave w's A fragments of layer 1, one float4 load per
// (sq, ft), 1 KB contiguous per wave.
__global__ void pack_w1_kernel(const float* __restrict__ W, int64_t dim, float* __restrict__ out) {
    const int64_t Kp = kpad(dim), KW = Kp / NW, SQ = KW / 16;
    const int64_t total = (int64_t)H * Kp;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int e = (int)(i & 3);
        const int lane = (int)((i >> 2) & 63);
        const int64_t q = i >> 8;  // (w * SQ + sq) * 4 + ft
        const int ft = (int)(q & 3);
        const int64_t wsq = q >> 2, w = wsq / SQ, sq = wsq - w * SQ;
        const int64_t k = w * KW + 4 * (4 * sq + e) + (lane >> 4);
        out[i] = k < dim ? W[(int64_t)(16 * ft + (lane & 15)) * dim + k] : 0.0f;
    }
}

// Workspace: tickets, three integer-totals slots (step i of a chain accumulates slot i % 3,
// reads slot (i - 1) % 3, zeroes slot (i + 1) % 3) and two RunningMeanStd state slots (read
// i % 2, write (i + 1) % 2), the diagnostic trace.  Totals slot (int64): [0, D) sum m of the step rows per
// column, [D, 2D) sum m^2, [2D, 3D) / [3D, 4D) the same over the reset rows, [4D] reset rows.
constexpr int TOT_N = 4 * KMAX + 2;
struct RmsState {
    float mean[KMAX];
    float var[KMAX];
    double count;
    double pad[7];
};
struct Ws {
    unsigned int* tickets;  // [1] data-parallel last arriver
    long long* tot[3];
    RmsState* st[2];
    int64_t nblk;
    uint64_t* trace;
};

// tsrl_rms_exact_stats's layout: float bm1[D], bv1[D], bm2[D], bv2[D]; int64 n1, nd at byte
// offset 16 D rounded up to 8
__device__ __forceinline__ const int64_t* xstats_counts(const void* xs, int D) {
    return reinterpret_cast<const int64_t*>(reinterpret_cast<const char*>(xs) +
                                            (16 * (int64_t)D + 7) / 8 * 8);
}

// The reference's two RunningMeanStd updates of a Collector step from their batch moments, in
// f32 (statistics.py:103-114; rms_exact.h merge): (mean, var, cnt) -> snapshot after the n1
// step rows -> final after the nd reset rows.  An update with no rows changes nothing.
__device__ __forceinline__ void merge_column_x(float m, float v, double& cnt, float bm1,
                                               float bv1, int64_t n1, float bm2, float bv2,
                                               int64_t nd, float& snap_m, float& snap_v,
                                               float& fin_m, float& fin_v) {
    if (n1 > 0) exact::merge(m, v, cnt, bm1, bv1, n1);
    snap_m = m;
    snap_v = v;
    if (nd > 0) exact::merge(m, v, cnt, bm2, bv2, nd);
    fin_m = m;
    fin_v = v;
}

// The spec env's counter step of env e (the same transition as the env phase's keys, see
// the top of collect_box_step_kernel): (j, tt) after the previous step -> this step's key,
// done flag and, when done, the reset key; (j, tt) advanced.
__device__ __forceinline__ void spec_keys(uint64_t seed, int64_t ep_len, int64_t e, int64_t& j,
                                          int64_t& tt, RowState& st, RowState& sr, bool& dn) {
    tt += 1;
    st.key = env_key(seed, (uint64_t)e, j, tt);
    st.active = 1;
    sr.key = 0ull;
    sr.active = 0;
    dn = tt >= ep_len;
    if (dn) {
        j += 1;
        tt = (j == 0) ? (e % ep_len) : 0;
        sr.key = env_key(seed, (uint64_t)e, j, tt);
        sr.active = 1;
    }
}

// m such that the synthetic env value is x = m 2^-23 exactly (box_val, synth.h)
__device__ __forceinline__ int box_m(uint64_t key, int64_t d) {
    const uint64_t h = sm64(key + (uint64_t)d * synth::GOLD);
    return (int)(h >> 40) - (1 << 23);
}

__device__ __forceinline__ void atomic_add_i64(long long* p, long long v) {
    __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(p), (unsigned long long)v,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// rms.hip rms_merge2_kernel's two RunningMeanStd updates for one column from the f64 sums of
// the step rows (S1, Q1) and of the reset rows (S2, Q2): (m0, v0, count) -> snapshot after the
// k step rows -> state after the nd reset rows.
__device__ __forceinline__ void merge_column_f(double m0, double v0, double old_count, double k,
                                               double S1, double Q1, double nd, double S2,
                                               double Q2, float& snap_m, float& snap_v,
                                               float& fin_m, float& fin_v) {
#pragma clang fp contract(off)
    const double tot1 = old_count + k, tot2 = tot1 + nd;
    if (k > 0.0) {
        const double bm = S1 / k;
        double bv = Q1 / k - bm * bm;
        bv = bv < 0.0 ? 0.0 : bv;
        const double delta = bm - m0;
        const double nm = m0 + delta * k / tot1;
        const double m2 = v0 * old_count + bv * k + delta * delta * old_count * k / tot1;
        m0 = (double)(float)nm;
        v0 = (double)(float)(m2 / tot1);
    }
    snap_m = (float)m0;
    snap_v = (float)v0;
    if (nd > 0.0) {
        const double bm = S2 / nd;
        double bv = Q2 / nd - bm * bm;
        bv = bv < 0.0 ? 0.0 : bv;
        const double delta = bm - m0;
        const double nm = m0 + delta * nd / tot2;
        const double m2 = v0 * tot1 + bv * nd + delta * delta * tot1 * nd / tot2;
        m0 = (double)(float)nm;
        v0 = (double)(float)(m2 / tot2);
    }
    fin_m = (float)m0;
    fin_v = (float)v0;
}

// The same from exact integer moments of the quantised synthetic env (x = m 2^-23: the sums
// scale exactly into f64).
__device__ __forceinline__ void merge_column(double m0, double v0, double old_count, double k,
                                             long long s1i, long long q1i, double nd,
                                             long long s2i, long long q2i, float& snap_m,
                                             float& snap_v, float& fin_m, float& fin_v) {
#pragma clang fp contract(off)
    merge_column_f(m0, v0, old_count, k, (double)s1i * 0x1p-23, (double)q1i * 0x1p-46, nd,
                   (double)s2i * 0x1p-23, (double)q2i * 0x1p-46, snap_m, snap_v, fin_m, fin_v);
}

// A totals-slot entry: int64 for the quantised env, f64 (sums and counts) for the
// action-coupled env (CPL)
template <bool CPL>
__device__ __forceinline__ double slot_f(const long long* p, int i) {
    return CPL ? reinterpret_cast<const double*>(p)[i] : (double)p[i];
}

// SQC = kpad(dim) / 128: the 128-column groups of an observation row (a compile-time bound, so
// the layer-1 weight fragments and the prefetched rows take only the registers dim needs).
// CPL: the action-coupled env (a.act_coef != 0, synth.h coupled_val): the env phase runs
// AFTER the actor on this launch's actions, and the obs_rms moments are f64 sums (atomic f64
// adds: the values are not 2^-23-quantised), the counts f64 too (one all-reducible f64 slot).
template <int SQC, bool CPL, bool LW>
__global__ __launch_bounds__(NT, 1) void collect_box_step_kernel(tsrl_collect_args a, Ws ws) {
#pragma clang fp contract(off)
    __shared__ float sX[KMAX * XP];
    __shared__ float sW2[H * WP], sW3[AMAX * WP];
    __shared__ float red[NW * 16 * 64];
    __shared__ float sH1[H * HP], sH2[H * HP];
    __shared__ float sb1[H], sb2[H], sb3[AMAX], ssig[AMAX], slo[AMAX], shi[AMAX];
    __shared__ float seps[R][AMAX + 1];
    __shared__ RowState rs[R], rr[R];
    __shared__ float sAr[CPL ? R : 1][AMAX + 1];  // CPL: this workgroup's remapped actions
    __shared__ int s_nd;
    // the rows' reward, flags (term | trunc << 1 | done << 2) and new episode counters,
    // stored to HBM by the env phase
    __shared__ double s_rew[R];
    __shared__ int s_flg[R];
    __shared__ int64_t s_jn[R], s_tn[R];
    __shared__ float* s_row[R];  // this step's stored obs row of each env (obs_dst + pitch)
    // xpipe: the spec env's keys of step i + d (E)
    __shared__ RowState xs_rs[R], xs_rr[R];
    __shared__ int xs_nd;
    // deferred obs_rms merge: the statistics after the previous step's step rows (obs_next
    // normalisation) and after its reset rows (reset rows, state)
    __shared__ __attribute__((aligned(16))) float sSnapM[KMAX], sSnapV[KMAX], sFinM[KMAX],
        sFinV[KMAX];
    // sqrt(var + eps) of both statistics, once per column (the add divides by them: the
    // correctly rounded square root is ~20 VALU, per element before)
    __shared__ __attribute__((aligned(16))) float sSnapS[KMAX], sFinS[KMAX];
    const int t = threadIdx.x;
    const int w = t >> 6, l = t & 63;
    const int64_t k = a.k;
    const int D = (int)a.dim;
    const int A = (int)a.act_dim;
    const int64_t r0 = (int64_t)blockIdx.x * R;
    const int nrows = (int)min((int64_t)R, k - r0);
    const int Kp = (int)kpad(D), KW = Kp / NW, SQ = KW / 16;
    const int64_t rng_step = a.rng_ctr ? *a.rng_ctr : 0;
    // this step's ring position of the pending add (first load: nothing waits behind it)
    const int64_t urel = a.add.k > 0 ? (a.add.rel_dev ? *a.add.rel_dev : a.add.uniform_rel) : 0;
#if COLLECT_TRACE
    if (t == 0) {
        unsigned xcc, hwid;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
        ws.trace[((rng_step & 15) * gridDim.x + blockIdx.x) * 8 + 4] = 0;
        ws.trace[((rng_step & 15) * gridDim.x + blockIdx.x) * 8 + 5] = 0;
        ws.trace[((rng_step & 15) * gridDim.x + blockIdx.x) * 8 + 6] = xcc;
        ws.trace[((rng_step & 15) * gridDim.x + blockIdx.x) * 8 + 7] = hwid;
    }
#endif
    TSTAMP(0)

    // ---- deferred obs_rms merge of the previous step (see D) ----------------------------------
    const bool xp = a.xpipe != 0;               // pipelined exact obs_rms (E)
    const bool defer = !a.no_moments && !xp;    // the integer-totals chain (D)
    const int step = a.rms_step;  // index of this launch in its chain of deferred steps
    const int par = step & 1;
    const int tcur = step % 3, tprev = (step + 2) % 3, tnext = (step + 1) % 3;
    const bool merge = (defer || xp) && step > 0;
    tsrl_add_args ad = a.add;
    // A1 (merge chain): every load of the pending add (raw rows, reset flag, act row, flags
    // and episode counters) and of the merge is issued first; they are consumed after the
    // merge, so one memory latency covers all of them.  32 lanes per row, float4 pieces
    // q = lane + 32 j of the row.
    constexpr int AQ = SQC;  // float4 pieces per lane: ceil(dim / 128) = SQC
    const int arw = t >> 5, aln = t & 31;
    const int nq = D >> 2;
    const int act_n = (int)(ad.act_row_bytes >> 2);
    const bool fast = merge && ad.k > 0 && !ad.ids && (D & 3) == 0 && ad.obs_next_src && ad.obs_next_dst &&
                      ad.norm_mean && ad.reset_mean && ad.reset_src && ad.reset_mask &&
                      !ad.obs_src && !ad.obs_next_src_raw && ad.act_src && ad.act_dst &&
                      (ad.act_row_bytes & 3) == 0 && act_n <= 32 &&
                      aligned16(ad.obs_next_src) && aligned16(ad.obs_next_dst) &&
                      aligned16(ad.reset_src);
    // the episode counters of the key rows, loaded before anything else
    constexpr int KT0 = NT - R;
    const int ki = t - KT0;
    const bool krow = ki >= 0 && ki < nrows;
    int64_t kj = 0, kt = 0, koff = 0;
    if (krow) {
        kj = a.ep_j[r0 + ki];
        kt = a.ep_t[r0 + ki];
        koff = a.obs_offset[r0 + ki];
    }
    // xpipe: the spec env's counters of these rows (the R threads before the key threads)
    const int si = t - (KT0 - R);
    const bool sgrp = xp && a.spec_raw && si >= 0 && si < R;
    const bool srow = sgrp && si < nrows;
    int64_t sj = 0, stt = 0;
    if (srow) {
        sj = a.spec_j[r0 + si];
        stt = a.spec_t[r0 + si];
    }
    const int64_t ar = r0 + arw;
    const bool arow = fast && arw < nrows;
    float4 axs[AQ], axr[AQ];
    uint8_t amask = 0;
    float aact = 0.0f;
    int64_t aptr_ld = 0;
    RowTail atail;
    if (arow) {
        amask = ad.reset_mask[ar];  // first: waiting for it below waits for nothing later
        const float4* s4 = reinterpret_cast<const float4*>(ad.obs_next_src + ar * D);
#pragma unroll
        for (int j = 0; j < AQ; ++j) {
            const int q = aln + 32 * j;
            axs[j] = s4[q < nq ? q : 0];
        }
        if (aln < act_n) aact = reinterpret_cast<const float*>(ad.act_src)[ar * act_n + aln];
        // the row's storage position (every lane: it addresses the lane's stores); the ring
        // position urel is added at A2, so no load here waits for it
        aptr_ld = ad.ptr ? ad.ptr[ar] : ad.offset[ar];
        if (aln == 0) atail.load(ad, ar, ar);
    }
    TSTAMP2(0)
    float mm0 = 0.f, mv0 = 0.f;
    long long ms1 = 0, mq1 = 0, ms2 = 0, mq2 = 0;  // raw slot words (int64 or f64 bits)
    double mcount = 0.0, mnd = 0.0, mk = 0.0;
    float xb1 = 0.f, xv1 = 0.f, xb2 = 0.f, xv2 = 0.f;  // xpipe: the previous step's batch moments
    int64_t xn1 = 0, xnd = 0;
    if (merge && xp) {
        const RmsState* sin = ws.st[par];
        const int64_t* xc = xstats_counts(a.xstats, D);
        const float* xf = reinterpret_cast<const float*>(a.xstats);
        mcount = sin->count;
        xn1 = xc[0];
        xnd = xc[1];
        if (t < D) {
            mm0 = sin->mean[t];
            mv0 = sin->var[t];
            xb1 = xf[t];
            xv1 = xf[D + t];
            xb2 = xf[2 * D + t];
            xv2 = xf[3 * D + t];
        }
    } else if (merge) {
        const RmsState* sin = ws.st[par];
        const long long* tp = ws.tot[tprev];
        mcount = sin->count;
        mnd = slot_f<CPL>(tp, 4 * D);
        mk = slot_f<CPL>(tp, 4 * D + 1);
        if (t < D) {  // D <= KMAX = NT: one column per thread
            mm0 = sin->mean[t];
            mv0 = sin->var[t];
            ms1 = tp[t];
            mq1 = tp[D + t];
            ms2 = tp[2 * D + t];
            mq2 = tp[3 * D + t];
        }
    }
    TSTAMP2(1)
    // the reset rows of envs that finished (their flag has arrived with the other loads)
    if (arow && amask) {
        const float4* r4 = reinterpret_cast<const float4*>(ad.reset_src + ar * D);
#pragma unroll
        for (int j = 0; j < AQ; ++j) {
            const int q = aln + 32 * j;
            axr[j] = r4[q < nq ? q : 0];
        }
    }
    TSTAMP2(2)
    if (ki >= 0) {
        // this step's counter keys (env.hip box_step_reset_kernel): every read the env phase
        // needs from them goes to LDS; the HBM stores wait for the env phase (the pending add
        // still reads the previous step's flags and counters of these rows)
        RowState st = {0ull, 0}, sr = {0ull, 0};
        bool dn = false;
        if (krow) {
            const int64_t e = r0 + ki;
            int64_t j = kj;
            int64_t tt = kt + 1;
            st.key = env_key(a.env_seed, (uint64_t)e, j, tt);
            st.active = 1;
            const uint64_t h = sm64(st.key ^ REW_SALT);
            s_rew[ki] = (double)(h >> 40) * 0x1p-24;
            dn = tt >= a.ep_len;
            s_flg[ki] = (dn && (e % 2 == 0) ? 1 : 0) | (dn && (e % 2 == 1) ? 2 : 0) | (dn ? 4 : 0);
            if (dn) {
                j += 1;
                tt = (j == 0) ? (e % a.ep_len) : 0;
                sr.key = env_key(a.env_seed, (uint64_t)e, j, tt);
                sr.active = 1;
            }
            s_jn[ki] = j;
            s_tn[ki] = tt;
        }
        rs[ki] = st;
        rr[ki] = sr;
        const uint64_t dm = __ballot(dn);
        if (ki == 0) s_nd = __popcll(dm);
        if (krow) {
            // this step's stored obs row of the env (see the store loop after the add); with a
            // pending add, block 0 advances the device cursor concurrently, so the position
            // is the add's own (urel) plus one, the ring's uniform next
            const int64_t uo = a.add.k > 0
                                   ? (urel + 1) % a.add.ring_size
                                   : (a.obs_rel_dev ? *a.obs_rel_dev : a.obs_uniform_rel);
            s_row[ki] = a.obs_dst + (koff + uo) * (a.obs_pitch ? a.obs_pitch : D);
        }
    }
    if (sgrp) {
        // xpipe: the spec env's step (i + d) of these rows; its counters and done flags go to
        // HBM now (nothing else in this launch reads them), its rows in the env phase
        RowState st = {0ull, 0}, sr = {0ull, 0};
        bool dn = false;
        if (srow) {
            const int64_t e = r0 + si;
            spec_keys(a.env_seed, a.ep_len, e, sj, stt, st, sr, dn);
            a.spec_j[e] = sj;
            a.spec_t[e] = stt;
            a.spec_done[e] = (uint8_t)dn;
        }
        xs_rs[si] = st;
        xs_rr[si] = sr;
        const uint64_t dm = __ballot(dn);
        if (si == 0) xs_nd = __popcll(dm);
    }
    double xcnt = mcount;  // xpipe: the count after the merge
    if (merge) {
        // the step rows behind the totals (counted in the slot: k, or the sum of every
        // rank's k when the slot was all-reduced)
        const double kp = mk;
        if (t < D) {
            if (xp)
                merge_column_x(mm0, mv0, xcnt, xb1, xv1, xn1, xb2, xv2, xnd, sSnapM[t],
                               sSnapV[t], sFinM[t], sFinV[t]);
            else if (CPL)
                merge_column_f((double)mm0, (double)mv0, mcount, kp, __longlong_as_double(ms1),
                               __longlong_as_double(mq1), mnd, __longlong_as_double(ms2),
                               __longlong_as_double(mq2), sSnapM[t], sSnapV[t], sFinM[t],
                               sFinV[t]);
            else
                merge_column((double)mm0, (double)mv0, mcount, kp, ms1, mq1, mnd, ms2, mq2,
                             sSnapM[t], sSnapV[t], sFinM[t], sFinV[t]);
            sSnapS[t] = __builtin_sqrtf(sSnapV[t] + ad.norm_eps);
            sFinS[t] = __builtin_sqrtf(sFinV[t] + ad.norm_eps);
        }
        TSTAMP2(3)
        LDS_SYNC();
        TSTAMP2(4)
        if (blockIdx.x == 0) {
            RmsState* so = ws.st[par ^ 1];
            if (t < D) {
                so->mean[t] = sFinM[t];
                so->var[t] = sFinV[t];
            }
            if (t == 0) so->count = xp ? xcnt : mcount + kp + mnd;
            if (defer) {
                // the slot the next launch accumulates: read by the launch before this one
                long long* tz = ws.tot[tnext];
                for (int i = t; i < 4 * D + 2; i += NT) tz[i] = 0;
            }
        }
        // the add reads the statistics from LDS, with sqrt(var + eps) per column
        // (add_row<true>)
        if (ad.norm_mean) {
            ad.norm_mean = sSnapM;
            ad.norm_var = sSnapS;
        }
        if (ad.reset_mean) {
            ad.reset_mean = sFinM;
            ad.reset_var = sFinS;
        }
    } else if ((defer || xp) && blockIdx.x == 0) {
        // first step of a chain: the caller's state seeds the state slot (slot 1 of the
        // totals ring is zero: tsrl_collect_rms_finalize cleared the ring)
        RmsState* so = ws.st[par ^ 1];
        for (int d = t; d < D; d += NT) {
            so->mean[d] = a.mean[d];
            so->var[d] = a.var[d];
        }
        if (t == 0) so->count = *a.count;
    }
    if (!merge && ad.k > 0 && (ad.norm_mean || ad.reset_mean)) {
        // statistics of a launch without the deferred merge (exact obs_rms, a chain's first
        // step): staged into LDS with sqrt(var + eps) per column, as the merge leaves them
        for (int d = t; d < D; d += NT) {
            if (ad.norm_mean) {
                sSnapM[d] = ad.norm_mean[d];
                sSnapS[d] = __builtin_sqrtf(ad.norm_var[d] + ad.norm_eps);
            }
            if (ad.reset_mean) {
                sFinM[d] = ad.reset_mean[d];
                sFinS[d] = __builtin_sqrtf(ad.reset_var[d] + ad.norm_eps);
            }
        }
        LDS_SYNC();
        if (ad.norm_mean) {
            ad.norm_mean = sSnapM;
            ad.norm_var = sSnapS;
        }
        if (ad.reset_mean) {
            ad.reset_mean = sFinM;
            ad.reset_var = sFinS;
        }
    }

    // actor weights: issued after every load the add and the merge wait for (vmcnt retires
    // in order, so a wait for an earlier load would also wait for these), in flight during
    // the add and the env step
    float4 w2r[2], w3r;
#pragma unroll
    for (int j = 0; j < 2; ++j) w2r[j] = reinterpret_cast<const float4*>(a.w2)[t + NT * j];
    w3r = reinterpret_cast<const float4*>(a.w3)[t < A * 16 ? t : 0];
    float vb1 = 0.f, vb2 = 0.f, vb3 = 0.f, vls = 0.f, vlo = -1.f, vhi = 1.f;
    if (t < H) {
        vb1 = a.b1[t];
        vb2 = a.b2[t];
    }
    if (t < A) {
        vb3 = a.b3[t];
        vls = a.log_std[t];
        if (a.low) {
            vlo = a.low[t];
            vhi = a.high[t];
        }
    }

    // layer-1 weight fragments of this wave (SQ == SQC): independent of the add phase, so
    // their latency hides behind it.  LW (the pipelined exact kernels, E): issued after the
    // add instead -- held across it they take the kernel to 241 VGPRs, two waves per SIMD
    // then fill the register file, and the concurrent tsrl_rms_exact_stats workgroup (128
    // VGPRs) finds no room on the CU; issued late, 190.  The default keeps the early issue:
    // 22.5 vs 23.8 us per step (tools/collect_ab.sh, two rounds).
    float4 wall[SQC][4];
    const float4* wp = reinterpret_cast<const float4*>(a.w1p) + (int64_t)w * SQ * 4 * 64 + l;
    if constexpr (!LW) {
#pragma unroll
        for (int sq = 0; sq < SQC; ++sq)
#pragma unroll
            for (int ft = 0; ft < 4; ++ft) wall[sq][ft] = wp[(sq * 4 + ft) * 64];
    }
    TSTAMP(4)
    // ---- A. pending add of the previous step -> buffer rows + live obs (HBM and sX) ---------
    if (ad.k > 0) {
        if (fast) {
            // A2: normalise the prefetched rows: obs_next with the statistics after the step
            // rows, the live obs of a reset env with those after the reset rows (add_row)
            if (arow) {
                const int64_t aptr = ad.ptr ? aptr_ld : aptr_ld + urel;
                float4* dst = reinterpret_cast<float4*>(
                    ad.obs_next_dst + aptr * (ad.obs_dst_pitch ? ad.obs_dst_pitch / 4 : D));
                const float clip = ad.norm_clip;
#pragma unroll
                for (int j = 0; j < AQ; ++j) {
                    const int q = aln + 32 * j;
                    if (q >= nq) break;
#define NRM(x_, m_, s_) norm1s(x_, m_, s_, clip)
                    const float* const sv = sSnapS;
                    const float* const fv = sFinS;
                    const float4 m = *reinterpret_cast<const float4*>(&sSnapM[4 * q]);
                    const float4 v = *reinterpret_cast<const float4*>(&sv[4 * q]);
                    float4 x = axs[j];
                    x.x = NRM(x.x, m.x, v.x);
                    x.y = NRM(x.y, m.y, v.y);
                    x.z = NRM(x.z, m.z, v.z);
                    x.w = NRM(x.w, m.w, v.w);
                    row_store4(&dst[q], x);
                    if (amask) {
                        const float4 mr = *reinterpret_cast<const float4*>(&sFinM[4 * q]);
                        const float4 vr = *reinterpret_cast<const float4*>(&fv[4 * q]);
                        x = axr[j];
                        x.x = NRM(x.x, mr.x, vr.x);
                        x.y = NRM(x.y, mr.y, vr.y);
                        x.z = NRM(x.z, mr.z, vr.z);
                        x.w = NRM(x.w, mr.w, vr.w);
                    }
#undef NRM
                    float* lx = sX + arw;
                    lx[(4 * q) * XP] = x.x;
                    lx[(4 * q + 1) * XP] = x.y;
                    lx[(4 * q + 2) * XP] = x.z;
                    lx[(4 * q + 3) * XP] = x.w;
                }
                if (aln < act_n) reinterpret_cast<float*>(ad.act_dst)[aptr * act_n + aln] = aact;
                if (aln == 0) atail.apply(ad, ar, urel, ar, aptr);
            }
        } else {
            // 32 lanes per row: all 16 rows' loads in flight at once
            if (arw < nrows)
                add_row<true>(ad, r0 + arw, aln, urel, sX + arw, XP, 32, false);
        }
        if (a.add.rel_next && blockIdx.x == 0 && t == 0)
            *a.add.rel_next = (urel + 1) % a.add.ring_size;
    } else if ((D & 3) == 0) {
        for (int i = t; i < nrows * nq; i += NT) {
            const int rw = i / nq, q = i - rw * nq;
            const float4 x = reinterpret_cast<const float4*>(a.cur + (r0 + rw) * D)[q];
            sX[(4 * q) * XP + rw] = x.x;
            sX[(4 * q + 1) * XP + rw] = x.y;
            sX[(4 * q + 2) * XP + rw] = x.z;
            sX[(4 * q + 3) * XP + rw] = x.w;
        }
    } else {
        // rows of D % 4 != 0 columns (e.g. config 2's D = 17): not 16-byte aligned
        for (int i = t; i < nrows * D; i += NT) {
            const int rw = i / D, c = i - rw * D;
            sX[c * XP + rw] = a.cur[(r0 + rw) * D + c];
        }
    }
    if constexpr (LW) {
#pragma unroll
        for (int sq = 0; sq < SQC; ++sq)
#pragma unroll
            for (int ft = 0; ft < 4; ++ft) wall[sq][ft] = wp[(sq * 4 + ft) * 64];
    }
    TSTAMP(1)
    // zero padding: columns [D, Kp) and rows past the last env of a partial tile
    for (int i = t; i < (Kp - D) * R; i += NT) sX[(D + i / R) * XP + (i % R)] = 0.0f;
    if (nrows < R)
        for (int i = t; i < D * (R - nrows); i += NT) {
            const int c = i / (R - nrows), rw = nrows + i % (R - nrows);
            sX[c * XP + rw] = 0.0f;
        }
    // noise of this workgroup's rows: thread -> (row, pair of action dims)
    if (a.sample && t < R * 16) {
        const int er = t >> 4, pr = t & 15, a0 = 2 * pr;
        float2 z = make_float2(0.f, 0.f);
        if (er < nrows && a0 < A) z = counter_normal2(a.act_seed, rng_step, r0 + er, pr);
        seps[er][a0] = z.x;
        seps[er][a0 + 1] = z.y;
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int e = 4 * (t + NT * j), rw = e >> 6, col = e & 63;
        float* d = sW2 + rw * WP + col;
        d[0] = w2r[j].x;
        d[1] = w2r[j].y;
        d[2] = w2r[j].z;
        d[3] = w2r[j].w;
    }
    {
        const int e = 4 * t, rw = e >> 6, col = e & 63;
        if (rw < AMAX) {
            const bool ok = rw < A;
            float* d = sW3 + rw * WP + col;
            d[0] = ok ? w3r.x : 0.f;
            d[1] = ok ? w3r.y : 0.f;
            d[2] = ok ? w3r.z : 0.f;
            d[3] = ok ? w3r.w : 0.f;
        }
    }
    if (t < H) {
        sb1[t] = vb1;
        sb2[t] = vb2;
    }
    if (t < AMAX) {
        sb3[t] = vb3;
        ssig[t] = t < A ? expf(vls) : 1.0f;
        slo[t] = vlo;
        shi[t] = vhi;
    }
    if (a.rng_next && blockIdx.x == 0 && t == 0) *a.rng_next = rng_step + 1;
    LDS_SYNC();
    // this step's stored obs rows (ReplayBuffer obs of step i = the live obs the actor sees):
    // written here from LDS, so the add of step i (next launch / flush) copies nothing and the
    // live obs never round-trips through HBM between fused steps (their row pointers came
    // from the top of the launch)
    // one column per thread (D <= NT), the rows in turn: no index division, coalesced rows
    if (t < D)
        for (int rw = 0; rw < nrows; ++rw) row_store1(s_row[rw] + t, sX[t * XP + rw]);
    // ---- C. env step + auto-reset of these rows (env.hip box_step_reset_kernel) -------------
    // The quantised synthetic env's transition does not read the action, so its step runs
    // before the actor: its obs_rms atomics drain while the actor computes.  (Round 5,
    // measured and dropped: the env's hashes / raw-row stores / atomics issued in pieces under
    // the actor's three MFMA chains instead -- 23.3-24.0 vs 21.3 us per step, two A/B rounds:
    // the pieces outlast the chains they hide under and every stage barrier then waits for
    // them.)  The
    // action-coupled env (CPL) steps after the actor, on the actions in sAr.  Phase A of
    // this launch has consumed the previous step's env rows of this workgroup (the barrier
    // above).
    auto env_phase = [&]() {
        if (t < nrows) {
            // keys, reward and flags came from the top of the launch (LDS)
            const int64_t r = r0 + t;
            const int f = s_flg[t];
            a.rew[r] = s_rew[t];
            a.term[r] = (uint8_t)(f & 1);
            a.trunc[r] = (uint8_t)((f >> 1) & 1);
            a.done[r] = (uint8_t)((f >> 2) & 1);
            if (f & 4) a.ep_j[r] = s_jn[t];
            a.ep_t[r] = s_tn[t];
        }
        if (xp) {
            // E: this step's rows were computed d launches ago; the spec env's rows of step
            // i + d (one column per thread) go to the ring slot for tsrl_rms_exact_stats and
            // the pending add of launch i + d + 1
            if (a.spec_raw && t < D) {
                const int d = t;
                for (int r = 0; r < nrows; ++r)
                    a.spec_raw[(r0 + r) * D + d] = (float)box_m(xs_rs[r].key, d) * 0x1p-23f;
                if (xs_nd > 0)
                    for (int r = 0; r < nrows; ++r)
                        if (xs_rr[r].active)
                            a.spec_reset_raw[(r0 + r) * D + d] =
                                (float)box_m(xs_rr[r].key, d) * 0x1p-23f;
            }
            return;
        }
        const int nd = s_nd;
        long long* tc = ws.tot[tcur];
        if (CPL) {
            // the coupled env: f64 column moments of the step rows (their values read the
            // actions) and of the reset rows, atomic f64 adds into the f64 slot
            double fs1 = 0.0, fq1 = 0.0, fs2 = 0.0, fq2 = 0.0;
            if (t < D) {
                const int d = t, ad = d % A;
                for (int r = 0; r < nrows; ++r) {
                    const float x = synth::coupled_val(rs[r].key, d, sAr[r][ad], a.act_coef);
                    a.raw[(r0 + r) * D + d] = x;
                    fs1 += (double)x;
                    fq1 += (double)x * (double)x;
                }
                if (nd > 0)
                    for (int r = 0; r < nrows; ++r) {
                        if (!rr[r].active) continue;
                        const float x = box_val(rr[r].key, d);
                        a.reset_raw[(r0 + r) * D + d] = x;
                        fs2 += (double)x;
                        fq2 += (double)x * (double)x;
                    }
            }
            if (defer) {
                double* tcd = reinterpret_cast<double*>(tc);
                auto fadd = [](double* p, double v) {
                    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                };
                if (t < D) {
                    fadd(tcd + t, fs1);
                    fadd(tcd + D + t, fq1);
                    if (nd > 0) {
                        fadd(tcd + 2 * D + t, fs2);
                        fadd(tcd + 3 * D + t, fq2);
                    }
                }
                if (t == 0) {
                    if (nd > 0) fadd(tcd + 4 * D, (double)nd);
                    fadd(tcd + 4 * D + 1, (double)nrows);
                }
            }
            return;
        }
        // this thread's column (D <= KMAX = NT): its exact integer moments, added to the totals
        // slot by atomics
        long long cs1 = 0, cq1 = 0, cs2 = 0, cq2 = 0;
        if (t < D) {
            const int d = t;
            for (int r = 0; r < nrows; ++r) {
                const int m = box_m(rs[r].key, d);
                a.raw[(r0 + r) * D + d] = (float)m * 0x1p-23f;  // == box_val(key, d), exactly
                cs1 += m;
                cq1 += (long long)m * m;
            }
            if (nd > 0)
                for (int r = 0; r < nrows; ++r) {
                    if (!rr[r].active) continue;
                    const int m = box_m(rr[r].key, d);
                    a.reset_raw[(r0 + r) * D + d] = (float)m * 0x1p-23f;
                    cs2 += m;
                    cq2 += (long long)m * m;
                }
        }
        if (defer) {
            if (t < D) {
                atomic_add_i64(tc + t, cs1);
                atomic_add_i64(tc + D + t, cq1);
                if (nd > 0) {
                    atomic_add_i64(tc + 2 * D + t, cs2);
                    atomic_add_i64(tc + 3 * D + t, cq2);
                }
            }
            if (t == 0) {
                if (nd > 0) atomic_add_i64(tc + 4 * D, nd);
                atomic_add_i64(tc + 4 * D + 1, nrows);
            }
        }
    };
    if (!CPL) env_phase();
    TSTAMP(2)

    // ---- B. actor: layer 1 (wave w: k in [w KW, (w+1) KW), all 64 features) -----------------
    {
        f32x4 acc[4];
#pragma unroll
        for (int ft = 0; ft < 4; ++ft) acc[ft] = f32x4{0.f, 0.f, 0.f, 0.f};
        const float* xb = sX + (w * KW + (l >> 4)) * XP + (l & 15);
#pragma unroll
        for (int sq = 0; sq < SQC; ++sq) {
            const float* xs = xb + 16 * sq * XP;
            const float b0 = xs[0], b1 = xs[4 * XP], b2 = xs[8 * XP], b3 = xs[12 * XP];
#pragma unroll
            for (int ft = 0; ft < 4; ++ft) {
                acc[ft] = mfma4(wall[sq][ft].x, b0, acc[ft]);
                acc[ft] = mfma4(wall[sq][ft].y, b1, acc[ft]);
                acc[ft] = mfma4(wall[sq][ft].z, b2, acc[ft]);
                acc[ft] = mfma4(wall[sq][ft].w, b3, acc[ft]);
            }
        }
        // red[w][ft][r][lane]
#pragma unroll
        for (int ft = 0; ft < 4; ++ft)
#pragma unroll
            for (int r = 0; r < 4; ++r) red[((w * 4 + ft) * 4 + r) * 64 + l] = acc[ft][r];
    }
    LDS_SYNC();
    TSTAMP2(5)
    // h1 = tanh(sum over the 8 waves in order + b1) -> sH1[f][row]
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int i = t + NT * j;  // (ft, r, lane)
        const int ln = i & 63, r = (i >> 6) & 3, ft = i >> 8;
        float z = red[i];
#pragma unroll
        for (int v = 1; v < NW; ++v) z += red[v * 16 * 64 + i];
        const int f = 16 * ft + 4 * (ln >> 4) + r;
        sH1[f * HP + (ln & 15)] = tanh_nb(z + sb1[f]);
    }
    LDS_SYNC();
    TSTAMP2(6)
    // layer 2: wave w -> feature tile w & 3 over k half w >> 2 (8 steps of 4)
    {
        const int ft = w & 3, kh = w >> 2;
        f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
        const float* wa = sW2 + (16 * ft + (l & 15)) * WP + 32 * kh + (l >> 4);
        const float* hb = sH1 + (32 * kh + (l >> 4)) * HP + (l & 15);
#pragma unroll
        for (int s = 0; s < 8; ++s) z = mfma4(wa[4 * s], hb[4 * s * HP], z);
#pragma unroll
        for (int r = 0; r < 4; ++r) red[(w * 4 + r) * 64 + l] = z[r];
    }
    LDS_SYNC();
    // h2 = tanh(half 0 + half 1 + b2) -> sH2
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int i = t + NT * j;  // (ft, r, lane) of 4 x 4 x 64
        const int ln = i & 63, r = (i >> 6) & 3, ft = i >> 8;
        const float z = red[(ft * 4 + r) * 64 + ln] + red[((ft + 4) * 4 + r) * 64 + ln];
        const int f = 16 * ft + 4 * (ln >> 4) + r;
        sH2[f * HP + (ln & 15)] = tanh_nb(z + sb2[f]);
    }
    LDS_SYNC();
    // mu head: wave w -> action tile w & 1 over k quarter w >> 1 (4 steps of 4)
    {
        const int at = w & 1, kq = w >> 1;
        f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
        const float* wa = sW3 + (16 * at + (l & 15)) * WP + 16 * kq + (l >> 4);
        const float* hb = sH2 + (16 * kq + (l >> 4)) * HP + (l & 15);
#pragma unroll
        for (int s = 0; s < 4; ++s) z = mfma4(wa[4 * s], hb[4 * s * HP], z);
#pragma unroll
        for (int r = 0; r < 4; ++r) red[(w * 4 + r) * 64 + l] = z[r];
    }
    LDS_SYNC();
    TSTAMP2(7)
    // mu = sum of the 4 quarters + b3; act = randn * sigma + mu; map_action -> act_remap
    {
        const int ln = t & 63, r = (t >> 6) & 3, at = t >> 8;  // 2 x 4 x 64 = 512 threads
        const int a_ = 16 * at + 4 * (ln >> 4) + r, rw = ln & 15;
        if (a_ < A && rw < nrows) {
            float mu = red[(at * 4 + r) * 64 + ln];
#pragma unroll
            for (int kq = 1; kq < 4; ++kq) mu += red[((at + 2 * kq) * 4 + r) * 64 + ln];
            const float m = mu + sb3[a_];
            float x = m;
            if (a.sample) x = seps[rw][a_] * ssig[a_] + m;  // contract(off): two roundings
            const int64_t row = r0 + rw;
            a.act[row * A + a_] = x;
            float y = x;
            if (a.bound_method == 1) y = y < -1.0f ? -1.0f : (y > 1.0f ? 1.0f : y);
            else if (a.bound_method == 2) y = tanh_nb(y);
            if (a.low) {
                const float lo = slo[a_], hi = shi[a_];
                y = lo + (hi - lo) * (y + 1.0f) / 2.0f;
            }
            a.act_remap[row * A + a_] = y;
            if (CPL) sAr[rw][a_] = y;
        }
    }
    if (CPL) {
        LDS_SYNC();  // sAr complete
        env_phase();
    }

    TSTAMP(3)
}

// tsrl_collect_rms_finalize: the last deferred step's totals merged into the caller's state
// (mean / var / count and the snapshot after its step rows), the totals slot re-zeroed.
__global__ __launch_bounds__(NT) void rms_finalize_kernel(tsrl_collect_args a, Ws ws) {
#pragma clang fp contract(off)
    const int t = threadIdx.x;
    const int D = (int)a.dim;
    const int step = a.rms_step;  // the chain's last launch
    const RmsState* sin = ws.st[(step + 1) & 1];  // the state the last launch published
    long long* tp = ws.tot[step % 3];
    const bool cpl = a.act_coef != 0.0f;  // the action-coupled env's f64 slot
    const double old_count = sin->count;
    const double nd = cpl ? slot_f<true>(tp, 4 * D) : slot_f<false>(tp, 4 * D);
    const double kp = cpl ? slot_f<true>(tp, 4 * D + 1) : slot_f<false>(tp, 4 * D + 1);
    for (int d = t; d < D; d += NT) {
        float sm, sv, fm, fv;
        if (cpl)
            merge_column_f((double)sin->mean[d], (double)sin->var[d], old_count, kp,
                           __longlong_as_double(tp[d]), __longlong_as_double(tp[D + d]), nd,
                           __longlong_as_double(tp[2 * D + d]),
                           __longlong_as_double(tp[3 * D + d]), sm, sv, fm, fv);
        else
            merge_column((double)sin->mean[d], (double)sin->var[d], old_count, kp, tp[d],
                         tp[D + d], nd, tp[2 * D + d], tp[3 * D + d], sm, sv, fm, fv);
        a.snap_mean[d] = sm;
        a.snap_var[d] = sv;
        a.mean[d] = fm;
        a.var[d] = fv;
    }
    __syncthreads();  // every thread has read the totals
    for (int j = 0; j < 3; ++j)
        for (int i = t; i < 4 * D + 2; i += NT) ws.tot[j][i] = 0;
    if (t == 0) *a.count = old_count + kp + nd;
}

// tsrl_collect_spec_step: the spec env step alone (E) -- the head of a pipelined chain computes
// the rows of its first d steps with it.  Workgroup = R env rows, one column per thread.
__global__ __launch_bounds__(NT) void spec_step_kernel(tsrl_collect_args a, int init) {
    __shared__ RowState rs[R], rr[R];
    __shared__ int s_nd;
    const int t = threadIdx.x;
    const int D = (int)a.dim;
    const int64_t r0 = (int64_t)blockIdx.x * R;
    const int nrows = (int)min((int64_t)R, a.k - r0);
    if (t < R) {
        RowState st = {0ull, 0}, sr = {0ull, 0};
        bool dn = false;
        if (t < nrows) {
            const int64_t e = r0 + t;
            int64_t j = init ? a.ep_j[e] : a.spec_j[e];
            int64_t tt = init ? a.ep_t[e] : a.spec_t[e];
            spec_keys(a.env_seed, a.ep_len, e, j, tt, st, sr, dn);
            a.spec_j[e] = j;
            a.spec_t[e] = tt;
            a.spec_done[e] = (uint8_t)dn;
        }
        rs[t] = st;
        rr[t] = sr;
        const uint64_t dm = __ballot(dn);
        if (t == 0) s_nd = __popcll(dm);
    }
    __syncthreads();
    if (t < D) {
        for (int r = 0; r < nrows; ++r)
            a.spec_raw[(r0 + r) * D + t] = (float)box_m(rs[r].key, t) * 0x1p-23f;
        if (s_nd > 0)
            for (int r = 0; r < nrows; ++r)
                if (rr[r].active)
                    a.spec_reset_raw[(r0 + r) * D + t] = (float)box_m(rr[r].key, t) * 0x1p-23f;
    }
}

// tsrl_collect_xpipe_finalize: the pipelined chain's last step -- its batch moments (xstats)
// merged into the state its launch published -> the caller's mean / var / count and the
// snapshot after its step rows.
__global__ __launch_bounds__(NT) void xpipe_finalize_kernel(tsrl_collect_args a, Ws ws) {
#pragma clang fp contract(off)
    const int t = threadIdx.x;
    const int D = (int)a.dim;
    const RmsState* sin = ws.st[(a.rms_step + 1) & 1];
    const int64_t* xc = xstats_counts(a.xstats, D);
    const float* xf = reinterpret_cast<const float*>(a.xstats);
    const int64_t n1 = xc[0], nd = xc[1];
    double cnt = sin->count;
    for (int d = t; d < D; d += NT) {
        cnt = sin->count;
        float sm, sv, fm, fv;
        merge_column_x(sin->mean[d], sin->var[d], cnt, xf[d], xf[D + d], n1, xf[2 * D + d],
                       xf[3 * D + d], nd, sm, sv, fm, fv);
        a.snap_mean[d] = sm;
        a.snap_var[d] = sv;
        a.mean[d] = fm;
        a.var[d] = fv;
    }
    if (t == 0) *a.count = cnt;
}

inline int64_t nblk_for(int64_t k) { return (k + R - 1) / R; }
constexpr int64_t TICKET_BYTES = 256;
constexpr int64_t TOT_BYTES = (TOT_N * 8 + 255) / 256 * 256;
constexpr int64_t ST_BYTES = (sizeof(RmsState) + 255) / 256 * 256;
inline int64_t trace_bytes(int64_t k) { return COLLECT_TRACE ? 2 * 16 * nblk_for(k) * 64 : 0; }

Ws make_ws(const tsrl_collect_args* a) {
    Ws ws;
    ws.nblk = nblk_for(a->k);
    char* base = reinterpret_cast<char*>(a->workspace);
    ws.tickets = reinterpret_cast<unsigned int*>(base);
    for (int i = 0; i < 3; ++i)
        ws.tot[i] = reinterpret_cast<long long*>(base + TICKET_BYTES + i * TOT_BYTES);
    for (int i = 0; i < 2; ++i)
        ws.st[i] = reinterpret_cast<RmsState*>(base + TICKET_BYTES + 3 * TOT_BYTES + i * ST_BYTES);
    ws.trace = reinterpret_cast<uint64_t*>(base + TICKET_BYTES + 3 * TOT_BYTES + 2 * ST_BYTES);
    return ws;
}

}  // namespace
}  // namespace tsrl

using namespace tsrl;

extern "C" int64_t tsrl_collect_pack_floats(int64_t dim) { return dim > 0 ? H * kpad(dim) : 0; }

extern "C" int tsrl_collect_pack_w1(const float* W, int64_t dim, float* packed, void* stream) {
    TSRL_CHECK_ARG(W && packed && dim > 0 && dim <= KMAX, "tsrl_collect_pack_w1: bad arguments");
    const int64_t total = tsrl_collect_pack_floats(dim);
    const unsigned grid = (unsigned)std::min<int64_t>((total + 255) / 256, 1024);
    hipLaunchKernelGGL(pack_w1_kernel, dim3(grid), dim3(256), 0, as_stream(stream), W, dim, packed);
    TSRL_LAUNCH_CHECK("tsrl_collect_pack_w1");
    return 0;
}

extern "C" int64_t tsrl_collect_workspace_bytes(int64_t k, int64_t dim) {
    if (k <= 0 || dim <= 0) return 0;
    return TICKET_BYTES + 3 * TOT_BYTES + 2 * ST_BYTES + trace_bytes(k);
}

extern "C" int tsrl_collect_box_step(const tsrl_collect_args* a, void* stream) {
    TSRL_CHECK_ARG(a != nullptr, "tsrl_collect_box_step: null args");
    const int64_t k = a->k, D = a->dim;
    TSRL_CHECK_ARG(k > 0 && D > 0 && D <= KMAX,
                   "tsrl_collect_box_step: need k > 0 and 0 < dim <= %d", KMAX);
    TSRL_CHECK_ARG(a->act_dim > 0 && a->act_dim <= AMAX && a->bound_method >= 0 &&
                       a->bound_method <= 2,
                   "tsrl_collect_box_step: 0 < act_dim <= %d, bound_method 0..2", AMAX);
    TSRL_CHECK_ARG(a->obs_dst && a->obs_offset && (a->obs_rel_dev || a->obs_uniform_rel >= 0),
                   "tsrl_collect_box_step: obs_dst / obs_offset / this step's ring position");
    TSRL_CHECK_ARG(a->obs_pitch == 0 || a->obs_pitch >= D, "tsrl_collect_box_step: obs_pitch < dim");
    TSRL_CHECK_ARG(a->add.k == 0 || a->add.obs_dst_pitch % 16 == 0,
                   "tsrl_collect_box_step: add.obs_dst_pitch must keep rows 16-byte aligned");
    TSRL_CHECK_ARG(a->cur && a->w1p && a->b1 && a->w2 && a->b2 && a->w3 && a->b3 && a->log_std &&
                       a->act && a->act_remap && a->ep_j && a->ep_t && a->raw && a->reset_raw &&
                       a->rew && a->term && a->trunc && a->done && a->workspace && a->mean &&
                       a->var && a->count && (a->no_moments || (a->snap_mean && a->snap_var)),
                   "tsrl_collect_box_step: null pointer");
    // w1p / workspace are this library's layouts; w2 and w3 (and cur when dim % 4 == 0) are
    // read with 16-byte loads at 4-byte alignment (parameters may be views into a flat
    // parameter buffer); rows of dim % 4 != 0 take the scalar paths (add_row's generic loop)
    TSRL_CHECK_ARG(aligned16(a->w1p) && aligned16(a->workspace) &&
                       ((reinterpret_cast<uintptr_t>(a->cur) | reinterpret_cast<uintptr_t>(a->w2) |
                         reinterpret_cast<uintptr_t>(a->w3)) & 3u) == 0,
                   "tsrl_collect_box_step: w1p / workspace must be 16-byte aligned, cur / w2 / w3 "
                   "4-byte aligned");
    TSRL_CHECK_ARG((a->low == nullptr) == (a->high == nullptr), "tsrl_collect_box_step: low/high");
    TSRL_CHECK_ARG(!a->sample || (a->rng_ctr && a->rng_next && a->rng_ctr != a->rng_next),
                   "tsrl_collect_box_step: sampling needs the rng counter pair");
    TSRL_CHECK_ARG(a->ep_len > 0, "tsrl_collect_box_step: ep_len <= 0");
    const tsrl_add_args& ad = a->add;
    if (ad.k != 0) {
        // the pending add runs row for row with this launch's env rows: same rows, identity
        // ids, f32 live-obs rows of dim columns, the live obs as cur_obs (its new rows are
        // the policy input)
        TSRL_CHECK_ARG(ad.k == k && ad.ids == nullptr && ad.obs_next_src && ad.cur_obs == a->cur &&
                           ad.obs_dim == D && ad.offset && ad.ep_rew && ad.ep_len && ad.ep_idx,
                       "tsrl_collect_box_step: pending add must cover the same k rows "
                       "(ids NULL, cur_obs == cur, obs_dim == dim)");
        TSRL_CHECK_ARG(!ad.rel_dev || (ad.ring_size > 0 && !ad.ptr),
                       "tsrl_collect_box_step: add.rel_dev needs ring_size and ptr == NULL");
        TSRL_CHECK_ARG(!ad.rel_next || (ad.rel_dev && ad.rel_next != ad.rel_dev),
                       "tsrl_collect_box_step: add.rel_next needs rel_dev (a different word)");
        TSRL_CHECK_ARG(!ad.reset_mask || ad.reset_src, "tsrl_collect_box_step: add reset_src");
        TSRL_CHECK_ARG(!ad.obs_src, "tsrl_collect_box_step: the pending add copies no obs (the "
                                    "launch that produced it stored them)");
    }
    if (a->xpipe) {
        TSRL_CHECK_ARG(a->act_coef == 0.0f && !a->no_moments && (a->rms_step == 0 || a->xstats),
                       "tsrl_collect_box_step: xpipe needs the action-independent env, "
                       "no_moments = 0 and, past a chain's first launch, xstats");
        TSRL_CHECK_ARG(!a->spec_raw || (a->spec_j && a->spec_t && a->spec_reset_raw && a->spec_done),
                       "tsrl_collect_box_step: xpipe spec rows need spec_j / spec_t / "
                       "spec_reset_raw / spec_done");
        TSRL_CHECK_ARG(!a->xstats || (reinterpret_cast<uintptr_t>(a->xstats) & 7u) == 0,
                       "tsrl_collect_box_step: xstats must be 8-byte aligned");
    }
    // one row adds <= 2^46 to a column's int64 sum of m^2: exact for <= 2^17 rows per slot (the
    // data-parallel caller also checks world * k); the coupled env's f64 slot has no such bound
    TSRL_CHECK_ARG(a->act_coef != 0.0f || k <= (int64_t)1 << 17,
                   "tsrl_collect_box_step: k <= 2^17 (exact int64 moments)");
    const Ws ws = make_ws(a);
    tsrl_collect_args p = *a;
    p.act_seed = sm64(a->act_seed);
    p.env_seed = sm64(a->env_seed);
#define TSRL_COLLECT_LAUNCH(SQ, CP, LW)                                                     \
    hipLaunchKernelGGL((collect_box_step_kernel<SQ, CP, LW>), dim3((unsigned)ws.nblk), dim3(NT), \
                       0, as_stream(stream), p, ws)
#define TSRL_COLLECT_SQ(SQ)                                                                 \
    if (cpl) TSRL_COLLECT_LAUNCH(SQ, true, false);                                          \
    else if (a->xpipe) TSRL_COLLECT_LAUNCH(SQ, false, true);                                \
    else TSRL_COLLECT_LAUNCH(SQ, false, false);
    const bool cpl = a->act_coef != 0.0f;
    switch (kpad(D) / 128) {
        case 1: TSRL_COLLECT_SQ(1) break;
        case 2: TSRL_COLLECT_SQ(2) break;
        case 3: TSRL_COLLECT_SQ(3) break;
        default: TSRL_COLLECT_SQ(4) break;
    }
#undef TSRL_COLLECT_SQ
#undef TSRL_COLLECT_LAUNCH
    TSRL_LAUNCH_CHECK("tsrl_collect_box_step");
    return 0;
}

extern "C" int64_t tsrl_collect_totals_offset(int64_t step) {
    return TICKET_BYTES + (step % 3) * TOT_BYTES;
}

extern "C" int tsrl_collect_spec_step(const tsrl_collect_args* a, int init, void* stream) {
    TSRL_CHECK_ARG(a != nullptr && a->k > 0 && a->dim > 0 && a->dim <= KMAX && a->ep_len > 0 &&
                       a->spec_j && a->spec_t && a->spec_raw && a->spec_reset_raw &&
                       a->spec_done && (!init || (a->ep_j && a->ep_t)),
                   "tsrl_collect_spec_step: bad arguments");
    tsrl_collect_args p = *a;
    p.env_seed = sm64(a->env_seed);  // as tsrl_collect_box_step passes it
    hipLaunchKernelGGL(spec_step_kernel, dim3((unsigned)nblk_for(a->k)), dim3(NT), 0,
                       as_stream(stream), p, init);
    TSRL_LAUNCH_CHECK("tsrl_collect_spec_step");
    return 0;
}

extern "C" int tsrl_collect_xpipe_finalize(const tsrl_collect_args* a, void* stream) {
    TSRL_CHECK_ARG(a != nullptr && a->workspace && a->mean && a->var && a->count &&
                       a->snap_mean && a->snap_var && a->xstats && a->k > 0 && a->dim > 0 &&
                       a->dim <= KMAX && (reinterpret_cast<uintptr_t>(a->xstats) & 7u) == 0,
                   "tsrl_collect_xpipe_finalize: bad arguments");
    hipLaunchKernelGGL(xpipe_finalize_kernel, dim3(1), dim3(NT), 0, as_stream(stream), *a,
                       make_ws(a));
    TSRL_LAUNCH_CHECK("tsrl_collect_xpipe_finalize");
    return 0;
}

extern "C" int tsrl_collect_rms_finalize(const tsrl_collect_args* a, void* stream) {
    TSRL_CHECK_ARG(a != nullptr && a->workspace && a->mean && a->var && a->count &&
                       a->snap_mean && a->snap_var && a->k > 0 && a->dim > 0 && a->dim <= KMAX,
                   "tsrl_collect_rms_finalize: bad arguments");
    hipLaunchKernelGGL(rms_finalize_kernel, dim3(1), dim3(NT), 0, as_stream(stream), *a,
                       make_ws(a));
    TSRL_LAUNCH_CHECK("tsrl_collect_rms_finalize");
    return 0;
}
