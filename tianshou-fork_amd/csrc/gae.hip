// GAE reverse scan for gfx950.
//
// Replaces tianshou/policy/base.py:337-384 (compute_episodic_return) + :453-497 (_gae_return).
// The reference recurrence  adv_i = delta_i + c_i * adv_{i+1},  c_i = (1 - end_i) * gamma*lambda,
// is an affine map x -> delta_i + c_i x per element.  A workgroup owns a range of the flat
// batch whose last element closes an episode (the VectorReplayBuffer sample(0) layout), so
// ranges are independent and the whole scan is ONE pass over HBM:
//   * each thread loads 8 consecutive transitions (16-byte vector loads),
//   * composes its 8 maps locally (f64),
//   * a wave-level Hillis-Steele suffix scan of affine maps (64 lanes, __shfl_down) plus a
//     4-entry LDS combine across the workgroup gives every thread its carry-in,
//   * the thread then re-runs the reference's exact sequential recurrence over its 8
//     elements from that carry (so only the carry at a thread boundary is re-associated).
// All f64 arithmetic is done without FMA contraction (`fp contract(off)`), matching the
// reference's separately-rounded NumPy/Python operations.
// Algorithmic traffic: 26 B/transition (rew f64, v_s f32, v_s_ f32, term u8, trunc u8,
// adv f32, ret f32).
#include <hip/hip_ext.h>

#include "tsrl_common.h"

#pragma clang fp contract(off)

namespace tsrl {
namespace {

constexpr int TPB = 256;
constexpr int EPT = 8;
constexpr int TILE = TPB * EPT;  // 2048 transitions per tile
constexpr int NWAVE = TPB / kWave;

struct Aff {
    double a, b;  // x -> a + b * x
};

__device__ __forceinline__ Aff compose(Aff f, Aff g) {  // f o g
    Aff r;
    r.a = f.a + f.b * g.a;
    r.b = f.b * g.b;
    return r;
}

struct GaeArgs {
    const float* vs;
    const float* vn;
    const double* vs64;  // mode 2: f64 value inputs
    const double* vn64;
    const double* rew;
    const uint8_t* term;
    const uint8_t* trunc;
    const uint8_t* extra;
    int64_t n;
    int64_t row_len;
    double gamma;
    float g32;
    double gl;
    const double* scale;  // non-null: rew_norm f64 value path
    float* adv;
    float* ret;
    double* adv64;
    double* ret64;
    double* partials;  // [nblocks][3]
};

struct Elems {
    double d[EPT];    // delta
    double vsd[EPT];  // v_s as used for returns (f64)
    uint32_t endb;    // bit k: end flag (c_k = 0)
    uint32_t validb;  // bit k: element inside [tb, te)
};

template <bool F64V, typename VT>
__device__ __forceinline__ void make_elem(const GaeArgs& p, int k, int64_t i, double rew,
                                          VT vs, VT vn, uint8_t tm, uint8_t tr,
                                          uint8_t ex, bool forced, double scale, Elems& e) {
    const bool te = tm != 0;
    const bool en = te || (tr != 0) || (ex != 0) || forced;
    if (F64V) {
        double vs64 = (double)vs * scale;
        double vn64 = (double)vn * scale;
        vn64 = vn64 * (te ? 0.0 : 1.0);
        e.d[k] = (rew + vn64 * p.gamma) - vs64;
        e.vsd[k] = vs64;
    } else {
        float vnm = (float)vn * (te ? 0.0f : 1.0f);
        float t = vnm * p.g32;
        e.d[k] = (rew + (double)t) - (double)vs;
        e.vsd[k] = (double)vs;
    }
    if (en) e.endb |= 1u << k;
    e.validb |= 1u << k;
}

template <bool F64V, bool VEC>
__device__ __forceinline__ void load_elems(const GaeArgs& p, int64_t base, int64_t lim,
                                           double scale, Elems& e) {
    e.endb = 0;
    e.validb = 0;
    int64_t rem = 0;
    if (p.row_len > 0) rem = (base + 1) % p.row_len;
    if (VEC) {
        const double2* r2 = reinterpret_cast<const double2*>(p.rew + base);
        const float4* s4 = reinterpret_cast<const float4*>(p.vs + base);
        const float4* n4 = reinterpret_cast<const float4*>(p.vn + base);
        double2 r[4] = {r2[0], r2[1], r2[2], r2[3]};
        float4 s[2] = {s4[0], s4[1]};
        float4 nv[2] = {n4[0], n4[1]};
        uint2 tm = *reinterpret_cast<const uint2*>(p.term + base);
        uint2 tr = *reinterpret_cast<const uint2*>(p.trunc + base);
        uint2 ex = make_uint2(0u, 0u);
        if (p.extra) ex = *reinterpret_cast<const uint2*>(p.extra + base);
        const double rv[8] = {r[0].x, r[0].y, r[1].x, r[1].y, r[2].x, r[2].y, r[3].x, r[3].y};
        const float sv[8] = {s[0].x, s[0].y, s[0].z, s[0].w, s[1].x, s[1].y, s[1].z, s[1].w};
        const float nvv[8] = {nv[0].x, nv[0].y, nv[0].z, nv[0].w,
                              nv[1].x, nv[1].y, nv[1].z, nv[1].w};
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            const uint32_t wt = k < 4 ? tm.x : tm.y;
            const uint32_t wr = k < 4 ? tr.x : tr.y;
            const uint32_t wx = k < 4 ? ex.x : ex.y;
            const int sh = (k & 3) * 8;
            bool forced = false;
            if (p.row_len > 0) {
                forced = rem == 0;
                rem = (rem + 1 == p.row_len) ? 0 : rem + 1;
            }
            make_elem<F64V, float>(p, k, base + k, rv[k], sv[k], nvv[k], (uint8_t)(wt >> sh),
                            (uint8_t)(wr >> sh), (uint8_t)(wx >> sh), forced, scale, e);
        }
    } else {
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            const int64_t i = base + k;
            bool forced = false;
            if (p.row_len > 0) {
                forced = rem == 0;
                rem = (rem + 1 == p.row_len) ? 0 : rem + 1;
            }
            if (i < lim) {
                if (p.vs64)
                    make_elem<F64V, double>(p, k, i, p.rew[i], p.vs64[i], p.vn64[i], p.term[i],
                                            p.trunc[i], p.extra ? p.extra[i] : (uint8_t)0,
                                            forced, scale, e);
                else
                    make_elem<F64V, float>(p, k, i, p.rew[i], p.vs[i], p.vn[i], p.term[i],
                                           p.trunc[i], p.extra ? p.extra[i] : (uint8_t)0,
                                           forced, scale, e);
            } else {
                e.d[k] = 0.0;
                e.vsd[k] = 0.0;
            }
        }
    }
}

// Composition of this thread's element maps: m_0 o m_1 o ... o m_7.
__device__ __forceinline__ Aff local_map(const Elems& e, double gl) {
    Aff m = {0.0, 1.0};
#pragma unroll
    for (int k = EPT - 1; k >= 0; --k) {
        if (e.validb & (1u << k)) {
            const double c = (e.endb & (1u << k)) ? 0.0 : gl;
            m.a = e.d[k] + c * m.a;
            m.b = c * m.b;
        }
    }
    return m;
}

struct ScanOut {
    Aff excl;   // composition of all later threads' maps in this tile
    Aff total;  // composition of the whole tile
};

// Exclusive suffix scan of affine maps over the 256 threads of the tile.
__device__ __forceinline__ ScanOut block_suffix_scan(Aff m, Aff* lds) {
    const int lane = threadIdx.x & (kWave - 1);
    const int w = threadIdx.x / kWave;
    Aff s = m;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
        Aff o;
        o.a = __shfl_down(s.a, off, kWave);
        o.b = __shfl_down(s.b, off, kWave);
        if (lane + off < kWave) s = compose(s, o);
    }
    Aff e;
    e.a = __shfl_down(s.a, 1, kWave);
    e.b = __shfl_down(s.b, 1, kWave);
    if (lane == kWave - 1) e = Aff{0.0, 1.0};
    if (lane == 0) lds[w] = s;
    __syncthreads();
    Aff z = {0.0, 1.0};
    Aff tot = {0.0, 1.0};
#pragma unroll
    for (int w2 = NWAVE - 1; w2 >= 0; --w2) {
        const Aff W = lds[w2];
        if (w2 > w) z = compose(W, z);
        tot = compose(W, tot);
    }
    ScanOut o;
    o.excl = compose(e, z);
    o.total = tot;
    return o;
}

struct Welford {
    double n, mean, m2;
};

__device__ __forceinline__ Welford chan(Welford x, Welford y) {
    if (y.n == 0.0) return x;
    if (x.n == 0.0) return y;
    Welford r;
    r.n = x.n + y.n;
    const double delta = y.mean - x.mean;
    r.mean = x.mean + delta * y.n / r.n;
    r.m2 = x.m2 + y.m2 + delta * delta * x.n * y.n / r.n;
    return r;
}

// Block-wide Chan merge (fixed tree order -> deterministic); result valid in thread 0.
__device__ Welford block_welford(Welford v, double* sh /*[3*TPB]*/) {
    const int t = threadIdx.x;
    sh[3 * t] = v.n;
    sh[3 * t + 1] = v.mean;
    sh[3 * t + 2] = v.m2;
    __syncthreads();
    for (int s = TPB / 2; s > 0; s >>= 1) {
        if (t < s) {
            Welford a = {sh[3 * t], sh[3 * t + 1], sh[3 * t + 2]};
            Welford b = {sh[3 * (t + s)], sh[3 * (t + s) + 1], sh[3 * (t + s) + 2]};
            Welford c = chan(a, b);
            sh[3 * t] = c.n;
            sh[3 * t + 1] = c.mean;
            sh[3 * t + 2] = c.m2;
        }
        __syncthreads();
    }
    Welford r = {sh[0], sh[1], sh[2]};
    __syncthreads();
    return r;
}

// Block-wide Chan merge with wave shuffles (xor butterfly inside each wave, then the 4 wave
// results folded in wave order by thread 0): fixed order -> deterministic; result valid in
// thread 0.  `sh` holds NWAVE entries.
__device__ __forceinline__ Welford block_welford_fast(Welford v, Welford* sh) {
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) {
        Welford o;
        o.n = __shfl_xor(v.n, off, kWave);
        o.mean = __shfl_xor(v.mean, off, kWave);
        o.m2 = __shfl_xor(v.m2, off, kWave);
        v = chan(v, o);
    }
    const int w = threadIdx.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == 0) sh[w] = v;
    __syncthreads();
    Welford r = sh[0];
#pragma unroll
    for (int i = 1; i < NWAVE; ++i) r = chan(r, sh[i]);
    return r;
}

// Chan merge of two partials with equal power-of-two counts (every lane of a full tile holds
// 8 returns, so every butterfly level merges equal counts): delta*n/(2n) = delta*0.5 and
// delta^2*n*n/(2n) = delta^2*(n/2) are exact scalings, so this is chan() bit for bit without
// its two f64 divisions.
__device__ __forceinline__ Welford chan_eq(Welford x, Welford y) {
    Welford r;
    r.n = x.n + y.n;
    const double delta = y.mean - x.mean;
    r.mean = x.mean + delta * 0.5;
    r.m2 = x.m2 + y.m2 + delta * delta * (x.n * 0.5);
    return r;
}

// block_welford_fast for a full tile (all 256 lanes hold EPT returns): butterfly inside each
// wave, then the 4 wave results as a pairwise tree ((w0,w1),(w2,w3)).  Result in thread 0.
__device__ __forceinline__ Welford block_welford_full(Welford v, Welford* sh) {
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) {
        Welford o;
        o.n = __shfl_xor(v.n, off, kWave);
        o.mean = __shfl_xor(v.mean, off, kWave);
        o.m2 = __shfl_xor(v.m2, off, kWave);
        v = chan_eq(v, o);
    }
    const int w = threadIdx.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == 0) sh[w] = v;
    __syncthreads();
    static_assert(NWAVE == 4, "pairwise wave fold assumes 4 waves");
    return chan_eq(chan_eq(sh[0], sh[1]), chan_eq(sh[2], sh[3]));
}

// a / b, correctly rounded, from y = RN(1/b): q0 = RN(a*y) is faithful, and one correction
// with the exact fma residual a - q0*b rounds to RN(a/b) (Markstein) -- 3 operations instead
// of the ~10 of a full f64 division, for the rew_norm `returns / sqrt(var + eps)`
// (a2c.py:110-111).  Non-finite quotients pass through.
__device__ __forceinline__ double div_by(double a, double b, double y) {
    const double q0 = a * y;
    const double r = __builtin_fma(-q0, b, a);
    return __builtin_isfinite(r) ? __builtin_fma(r, y, q0) : q0;
}

// One tile [tb, te) with carry-in `carry` (= adv at te, 0 beyond a segment end).
// Returns the carry for the tile to its left (adv at tb).
template <bool F64V, bool VEC>
__device__ double gae_tile(const GaeArgs& p, int64_t tb, int64_t te, double carry,
                           double scale, Aff* lds, double* wsh, Welford* acc) {
    const int64_t base = tb + (int64_t)threadIdx.x * EPT;
    Elems e;
    load_elems<F64V, VEC>(p, base, te, scale, e);
    const Aff m = local_map(e, p.gl);
    const ScanOut so = block_suffix_scan(m, lds);
    const double x = so.excl.a + so.excl.b * carry;
    const double carry_out = so.total.a + so.total.b * carry;

    double g = x;
    const double rscale = 1.0 / scale;
    double adv[EPT], ret[EPT];
#pragma unroll
    for (int k = EPT - 1; k >= 0; --k) {
        if (e.validb & (1u << k)) {
            const double c = (e.endb & (1u << k)) ? 0.0 : p.gl;
            g = e.d[k] + c * g;
        }
        adv[k] = g;
        ret[k] = g + e.vsd[k];
    }
    if (VEC) {
        if (p.adv) {
            float4* o = reinterpret_cast<float4*>(p.adv + base);
            o[0] = make_float4((float)adv[0], (float)adv[1], (float)adv[2], (float)adv[3]);
            o[1] = make_float4((float)adv[4], (float)adv[5], (float)adv[6], (float)adv[7]);
        }
        if (p.ret) {
            float r[EPT];
#pragma unroll
            for (int k = 0; k < EPT; ++k)
                r[k] = F64V ? (float)div_by(ret[k], scale, rscale) : (float)ret[k];
            float4* o = reinterpret_cast<float4*>(p.ret + base);
            o[0] = make_float4(r[0], r[1], r[2], r[3]);
            o[1] = make_float4(r[4], r[5], r[6], r[7]);
        }
        if (p.adv64) {
            double2* o = reinterpret_cast<double2*>(p.adv64 + base);
#pragma unroll
            for (int k = 0; k < 4; ++k) o[k] = make_double2(adv[2 * k], adv[2 * k + 1]);
        }
        if (p.ret64) {
            double2* o = reinterpret_cast<double2*>(p.ret64 + base);
#pragma unroll
            for (int k = 0; k < 4; ++k) o[k] = make_double2(ret[2 * k], ret[2 * k + 1]);
        }
    } else {
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            if (e.validb & (1u << k)) {
                const int64_t i = base + k;
                if (p.adv) p.adv[i] = (float)adv[k];
                if (p.ret) p.ret[i] = F64V ? (float)div_by(ret[k], scale, rscale) : (float)ret[k];
                if (p.adv64) p.adv64[i] = adv[k];
                if (p.ret64) p.ret64[i] = ret[k];
            }
        }
    }
    if (F64V && p.partials) {
        Welford w = {0.0, 0.0, 0.0};
        double s = 0.0;
        int cnt = 0;
#pragma unroll
        for (int k = 0; k < EPT; ++k)
            if (e.validb & (1u << k)) { s += ret[k]; ++cnt; }
        if (cnt) {
            w.n = (double)cnt;
            w.mean = s / w.n;
#pragma unroll
            for (int k = 0; k < EPT; ++k)
                if (e.validb & (1u << k)) { const double dv = ret[k] - w.mean; w.m2 += dv * dv; }
        }
        Welford t = VEC ? block_welford_full(w, reinterpret_cast<Welford*>(wsh))
                        : block_welford_fast(w, reinterpret_cast<Welford*>(wsh));
        if (threadIdx.x == 0) *acc = chan(t, *acc);
    }
    __syncthreads();  // lds reuse by the next tile
    return carry_out;
}

__device__ __forceinline__ double load_scale(const GaeArgs& p) {
    return p.scale ? *p.scale : 1.0;
}

// LDS staging for one full, aligned tile (the sample(0) row layout at every row_len that is
// a multiple of 8).  rew (f64) and v_s_ arrive with fully coalesced 16-byte loads (lane l of
// a wave reads vector l: one 1 KB span per instruction, instead of the 4 KB / 2 KB spans a
// thread-owns-8-elements load touches) and are redistributed through LDS; after the scan the
// same regions carry adv and ret (f32) back out as coalesced stores.  v_s and the u8 flags
// keep per-thread loads (32 B and 8 B per lane).
// (Round 5, measured and dropped: rew loaded per thread, 8 consecutive values, instead of
// staged -- a 16 instead of 24 KB stage; 47.6-47.8 vs 47.6-48.1 us by events at 4096 x 2048,
// two A/B rounds: no change, the kernel is VGPR-limited to 4 workgroups per CU either way.)
struct Stage {
    double rew[TILE];  // rew; after the scan, ret as f32 in the first half
    float vn[TILE];    // v_s_; after the scan, adv as f32
};

template <bool F64V>
__device__ double gae_tile_staged(const GaeArgs& p, int64_t tb, double carry, double scale,
                                  Stage& st, Aff* lds, double* wsh, Welford* acc) {
    const int t = threadIdx.x;
    {
        const double2* r2 = reinterpret_cast<const double2*>(p.rew + tb);
        const float4* n4 = reinterpret_cast<const float4*>(p.vn + tb);
        double2 r[4];
        float4 nv[2];
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = r2[t + TPB * j];
#pragma unroll
        for (int j = 0; j < 2; ++j) nv[j] = n4[t + TPB * j];
        double2* sr = reinterpret_cast<double2*>(st.rew);
        float4* sn = reinterpret_cast<float4*>(st.vn);
#pragma unroll
        for (int j = 0; j < 4; ++j) sr[t + TPB * j] = r[j];
#pragma unroll
        for (int j = 0; j < 2; ++j) sn[t + TPB * j] = nv[j];
    }
    const int64_t base = tb + (int64_t)t * EPT;
    const float4* s4 = reinterpret_cast<const float4*>(p.vs + base);
    const float4 s0 = s4[0], s1 = s4[1];
    const uint2 tm = *reinterpret_cast<const uint2*>(p.term + base);
    const uint2 tr = *reinterpret_cast<const uint2*>(p.trunc + base);
    uint2 ex = make_uint2(0u, 0u);
    if (p.extra) ex = *reinterpret_cast<const uint2*>(p.extra + base);
    __syncthreads();

    const float sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    Elems e;
    e.endb = 0;
    e.validb = 0;
    {
        const double2* sr = reinterpret_cast<const double2*>(st.rew + t * EPT);
        const float4* sn = reinterpret_cast<const float4*>(st.vn + t * EPT);
        const double2 r0 = sr[0], r1 = sr[1], r2 = sr[2], r3 = sr[3];
        const float4 n0 = sn[0], n1 = sn[1];
        const double rv[8] = {r0.x, r0.y, r1.x, r1.y, r2.x, r2.y, r3.x, r3.y};
        const float nvv[8] = {n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, n1.z, n1.w};
        int64_t rem = p.row_len > 0 ? (base + 1) % p.row_len : 0;
#pragma unroll
        for (int k = 0; k < EPT; ++k) {
            const uint32_t wt = k < 4 ? tm.x : tm.y;
            const uint32_t wr = k < 4 ? tr.x : tr.y;
            const uint32_t wx = k < 4 ? ex.x : ex.y;
            const int sh = (k & 3) * 8;
            bool forced = false;
            if (p.row_len > 0) {
                forced = rem == 0;
                rem = (rem + 1 == p.row_len) ? 0 : rem + 1;
            }
            make_elem<F64V, float>(p, k, base + k, rv[k], sv[k], nvv[k], (uint8_t)(wt >> sh),
                                   (uint8_t)(wr >> sh), (uint8_t)(wx >> sh), forced, scale, e);
        }
    }
    const Aff m = local_map(e, p.gl);
    // The scan's barrier orders every thread's LDS reads above before the writes below.
    const ScanOut so = block_suffix_scan(m, lds);
    const double x = so.excl.a + so.excl.b * carry;
    const double carry_out = so.total.a + so.total.b * carry;

    double g = x;
    const double rscale = 1.0 / scale;
    double ret[EPT];
    float* sadv = st.vn + t * EPT;
    float* sret = reinterpret_cast<float*>(st.rew) + t * EPT;
#pragma unroll
    for (int k = EPT - 1; k >= 0; --k) {
        const double c = (e.endb & (1u << k)) ? 0.0 : p.gl;
        g = e.d[k] + c * g;
        sadv[k] = (float)g;
        // v_s for the return is re-derived from the f32 input (as make_elem does) rather
        // than kept in e.vsd: 16 fewer live VGPRs across the scan.
        ret[k] = g + (F64V ? (double)sv[k] * scale : (double)sv[k]);
        sret[k] = F64V ? (float)div_by(ret[k], scale, rscale) : (float)ret[k];
    }
    if (F64V && p.partials) {
        Welford w;
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < EPT; ++k) s += ret[k];
        w.n = (double)EPT;
        w.mean = s / w.n;
        w.m2 = 0.0;
#pragma unroll
        for (int k = 0; k < EPT; ++k) { const double dv = ret[k] - w.mean; w.m2 += dv * dv; }
        // block_welford_fast's barrier also publishes the f32 adv/ret written above.
        Welford tw = block_welford_full(w, reinterpret_cast<Welford*>(wsh));
        if (threadIdx.x == 0) *acc = chan(tw, *acc);
    } else {
        __syncthreads();
    }
    {
        const float4* sn = reinterpret_cast<const float4*>(st.vn);
        const float4* sr = reinterpret_cast<const float4*>(st.rew);
        if (p.adv) {
            float4* o = reinterpret_cast<float4*>(p.adv + tb);
#pragma unroll
            for (int j = 0; j < 2; ++j) o[t + TPB * j] = sn[t + TPB * j];
        }
        if (p.ret) {
            float4* o = reinterpret_cast<float4*>(p.ret + tb);
#pragma unroll
            for (int j = 0; j < 2; ++j) o[t + TPB * j] = sr[t + TPB * j];
        }
    }
    __syncthreads();  // LDS reuse by the next tile
    return carry_out;
}

// Fast path: block b owns [b*range_len, min((b+1)*range_len, n)), independent of others.
template <bool F64V>
__global__ __launch_bounds__(TPB) void gae_rows_kernel(GaeArgs p, int64_t range_len,
                                                       int vec_ok) {
    __shared__ Aff lds[NWAVE];
    __shared__ double wsh[F64V ? 3 * NWAVE : 1];
    const int64_t s = (int64_t)blockIdx.x * range_len;
    const int64_t e = min(s + range_len, p.n);
    const double scale = load_scale(p);
    const int64_t ntiles = (e - s + TILE - 1) / TILE;
    double carry = 0.0;
    Welford acc = {0.0, 0.0, 0.0};
    for (int64_t t = ntiles - 1; t >= 0; --t) {
        const int64_t tb = s + t * TILE;
        const int64_t te = min(tb + TILE, e);
        const bool vec = vec_ok && (te - tb == TILE) && ((tb & 7) == 0);
        if (vec)
            carry = gae_tile<F64V, true>(p, tb, te, carry, scale, lds, wsh, &acc);
        else
            carry = gae_tile<F64V, false>(p, tb, te, carry, scale, lds, wsh, &acc);
    }
    if (F64V && p.partials && threadIdx.x == 0) {
        p.partials[3 * blockIdx.x + 0] = acc.n;
        p.partials[3 * blockIdx.x + 1] = acc.mean;
        p.partials[3 * blockIdx.x + 2] = acc.m2;
    }
}

// Staged variant of gae_rows_kernel for the layout bench / process_fn produce: rows of
// row_len % TILE == 0 transitions, n % row_len == 0, 16-byte aligned f32 outputs only.
template <bool F64V>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(4, 8))) void gae_rows_staged_kernel(GaeArgs p, int64_t range_len) {
    __shared__ Aff lds[NWAVE];
    __shared__ double wsh[F64V ? 3 * NWAVE : 1];
    __shared__ Stage st;
    const int64_t s = (int64_t)blockIdx.x * range_len;
    const double scale = load_scale(p);
    double carry = 0.0;
    Welford acc = {0.0, 0.0, 0.0};
    for (int64_t tb = s + range_len - TILE; tb >= s; tb -= TILE)
        carry = gae_tile_staged<F64V>(p, tb, carry, scale, st, lds, wsh, &acc);
    if (F64V && p.partials && threadIdx.x == 0) {
        p.partials[3 * blockIdx.x + 0] = acc.n;
        p.partials[3 * blockIdx.x + 1] = acc.mean;
        p.partials[3 * blockIdx.x + 2] = acc.m2;
    }
}

// General path, phase 1: per-tile aggregate map.
template <bool F64V>
__global__ __launch_bounds__(TPB) void gae_tile_agg_kernel(GaeArgs p, double* agg) {
    __shared__ Aff lds[NWAVE];
    const int64_t tb = (int64_t)blockIdx.x * TILE;
    const int64_t te = min(tb + TILE, p.n);
    const double scale = load_scale(p);
    Elems e;
    load_elems<F64V, false>(p, tb + (int64_t)threadIdx.x * EPT, te, scale, e);
    const Aff m = local_map(e, p.gl);
    const ScanOut so = block_suffix_scan(m, lds);
    if (threadIdx.x == 0) {
        agg[2 * blockIdx.x] = so.total.a;
        agg[2 * blockIdx.x + 1] = so.total.b;
    }
}

// General path, phase 2: carry[t] = (T_{t+1} o ... o T_{G-1})(0), one workgroup.
__global__ __launch_bounds__(TPB) void gae_carry_kernel(const double* agg, int64_t g,
                                                         double* carry) {
    __shared__ Aff lds[NWAVE];
    const int64_t per = (g + TPB - 1) / TPB;
    const int64_t lo = min((int64_t)threadIdx.x * per, g);
    const int64_t hi = min(lo + per, g);
    Aff m = {0.0, 1.0};
    for (int64_t t = hi - 1; t >= lo; --t) m = compose(Aff{agg[2 * t], agg[2 * t + 1]}, m);
    const ScanOut so = block_suffix_scan(m, lds);
    double x = so.excl.a;  // carry into tile hi-1's right neighbour chain (x = value at hi)
    for (int64_t t = hi - 1; t >= lo; --t) {
        carry[t] = x;
        x = agg[2 * t] + agg[2 * t + 1] * x;
    }
}

// General path, phase 3.
template <bool F64V>
__global__ __launch_bounds__(TPB) void gae_tile_apply_kernel(GaeArgs p, const double* carry,
                                                             int vec_ok) {
    __shared__ Aff lds[NWAVE];
    __shared__ double wsh[F64V ? 3 * TPB : 1];
    const int64_t tb = (int64_t)blockIdx.x * TILE;
    const int64_t te = min(tb + TILE, p.n);
    const double scale = load_scale(p);
    Welford acc = {0.0, 0.0, 0.0};
    if (vec_ok && te - tb == TILE)
        gae_tile<F64V, true>(p, tb, te, carry[blockIdx.x], scale, lds, wsh, &acc);
    else
        gae_tile<F64V, false>(p, tb, te, carry[blockIdx.x], scale, lds, wsh, &acc);
    if (F64V && p.partials && threadIdx.x == 0) {
        p.partials[3 * blockIdx.x + 0] = acc.n;
        p.partials[3 * blockIdx.x + 1] = acc.mean;
        p.partials[3 * blockIdx.x + 2] = acc.m2;
    }
}

__global__ __launch_bounds__(TPB) void ret_rms_update_kernel(const double* partials,
                                                             int64_t nparts, double* rms) {
    __shared__ double wsh[3 * TPB];
    Welford w = {0.0, 0.0, 0.0};
    const int64_t per = (nparts + TPB - 1) / TPB;
    const int64_t lo = min((int64_t)threadIdx.x * per, nparts);
    const int64_t hi = min(lo + per, nparts);
    for (int64_t i = lo; i < hi; ++i)
        w = chan(w, Welford{partials[3 * i], partials[3 * i + 1], partials[3 * i + 2]});
    const Welford b = block_welford(w, wsh);
    if (threadIdx.x == 0 && b.n > 0.0) {
        // RunningMeanStd.update (statistics.py:93-114) with batch (mean, var = M2/n, n).
        const double mean = rms[0], var = rms[1], count = rms[2];
        const double bm = b.mean, bv = b.m2 / b.n, bc = b.n;
        const double delta = bm - mean;
        const double tot = count + bc;
        const double new_mean = mean + delta * bc / tot;
        const double m_a = var * count;
        const double m_b = bv * bc;
        const double m_2 = m_a + m_b + delta * delta * count * bc / tot;
        rms[0] = new_mean;
        rms[1] = m_2 / tot;
        rms[2] = tot;
    }
}

int64_t range_len_for(int64_t row_len) {
    if (row_len >= TILE) return row_len;
    const int64_t rows = TILE / row_len;
    return rows * row_len;
}

}  // namespace
}  // namespace tsrl

using namespace tsrl;

extern "C" int64_t tsrl_gae_workspace_bytes(int64_t n, int64_t row_len) {
    if (row_len > 0 || n <= 0) return 0;
    const int64_t g = (n + TILE - 1) / TILE;
    return g * 3 * (int64_t)sizeof(double);
}

extern "C" int64_t tsrl_gae_num_partials(int64_t n, int64_t row_len) {
    if (n <= 0) return 0;
    if (row_len > 0) {
        const int64_t r = range_len_for(row_len);
        return (n + r - 1) / r;
    }
    return (n + TILE - 1) / TILE;
}

// tsrl_gae_time_next: HIP events the NEXT row-path tsrl_gae launch of this host thread
// records its kernel's start / stop into (bench.py's roofline: the kernel's own duration on
// its launch stream, not an event pair around the launch, which also holds the dispatch)
namespace {
thread_local hipEvent_t g_time_start = nullptr, g_time_stop = nullptr;
}

extern "C" int tsrl_gae_time_next(void* start_event, void* stop_event) {
    TSRL_CHECK_ARG((start_event == nullptr) == (stop_event == nullptr),
                   "tsrl_gae_time_next: both events or neither");
    g_time_start = reinterpret_cast<hipEvent_t>(start_event);
    g_time_stop = reinterpret_cast<hipEvent_t>(stop_event);
    return 0;
}

extern "C" int tsrl_gae(const float* v_s, const float* v_s_next, const double* rew,
                        const uint8_t* terminated, const uint8_t* truncated,
                        const uint8_t* end_extra, int64_t n, int64_t row_len,
                        const double* value_scale, double gamma, double gae_lambda,
                        float* adv_out, float* ret_out, double* adv64_out, double* ret64_out,
                        double* ret_partials, void* workspace, int64_t workspace_bytes,
                        void* stream) {
    // tsrl_gae_time_next's events belong to THIS call whichever path runs (or returns
    // early): taken and cleared before anything can return, so they never reach a later,
    // unrelated launch (e.g. one inside a graph capture)
    hipEvent_t t0 = g_time_start, t1 = g_time_stop;
    g_time_start = g_time_stop = nullptr;
    TSRL_CHECK_ARG(n >= 0, "tsrl_gae: n < 0");
    if (n == 0) return 0;
    TSRL_CHECK_ARG(v_s && v_s_next && rew && terminated && truncated,
                   "tsrl_gae: null input pointer");
    TSRL_CHECK_ARG(row_len >= 0, "tsrl_gae: row_len < 0");
    TSRL_CHECK_ARG(!ret_partials || value_scale,
                   "tsrl_gae: ret_partials requires value_scale (rew_norm path)");
    GaeArgs p = {};
    p.vs = v_s;
    p.vn = v_s_next;
    p.rew = rew;
    p.term = terminated;
    p.trunc = truncated;
    p.extra = end_extra;
    p.n = n;
    p.row_len = row_len;
    p.gamma = gamma;
    p.g32 = (float)gamma;
    p.gl = gamma * gae_lambda;
    p.scale = value_scale;
    p.adv = adv_out;
    p.ret = ret_out;
    p.adv64 = adv64_out;
    p.ret64 = ret64_out;
    p.partials = ret_partials;
    const int vec_ok = aligned16(v_s) && aligned16(v_s_next) && aligned16(rew) &&
                       ((uintptr_t)terminated % 8 == 0) && ((uintptr_t)truncated % 8 == 0) &&
                       (!end_extra || (uintptr_t)end_extra % 8 == 0) &&
                       (!adv_out || aligned16(adv_out)) && (!ret_out || aligned16(ret_out)) &&
                       (!adv64_out || aligned16(adv64_out)) &&
                       (!ret64_out || aligned16(ret64_out));
    hipStream_t s = as_stream(stream);
    const bool f64v = value_scale != nullptr;
    if (row_len > 0) {
        const int64_t r = range_len_for(row_len);
        const int64_t grid = (n + r - 1) / r;
        TSRL_CHECK_ARG(grid < (1ll << 31), "tsrl_gae: too many ranges");
        const bool staged = vec_ok && !adv64_out && !ret64_out && r % TILE == 0 &&
                            n % r == 0 && !getenv("TSRL_GAE_UNSTAGED");
        // tsrl_gae_time_next: the launch's own start / stop timestamps (hipExtLaunchKernel);
        // the general path below launches three kernels and records none
        if (staged) {
            if (f64v)
                hipExtLaunchKernelGGL(gae_rows_staged_kernel<true>, dim3((unsigned)grid),
                                      dim3(TPB), 0, s, t0, t1, 0, p, r);
            else
                hipExtLaunchKernelGGL(gae_rows_staged_kernel<false>, dim3((unsigned)grid),
                                      dim3(TPB), 0, s, t0, t1, 0, p, r);
            TSRL_LAUNCH_CHECK("tsrl_gae(rows, staged)");
            return 0;
        }
        if (f64v)
            hipExtLaunchKernelGGL(gae_rows_kernel<true>, dim3((unsigned)grid), dim3(TPB), 0, s,
                                  t0, t1, 0, p, r, vec_ok);
        else
            hipExtLaunchKernelGGL(gae_rows_kernel<false>, dim3((unsigned)grid), dim3(TPB), 0, s,
                                  t0, t1, 0, p, r, vec_ok);
        TSRL_LAUNCH_CHECK("tsrl_gae(rows)");
        return 0;
    }
    const int64_t g = (n + TILE - 1) / TILE;
    TSRL_CHECK_ARG(workspace && workspace_bytes >= tsrl_gae_workspace_bytes(n, 0),
                   "tsrl_gae: general path needs %lld workspace bytes",
                   (long long)tsrl_gae_workspace_bytes(n, 0));
    TSRL_CHECK_ARG(g < (1ll << 31), "tsrl_gae: too many tiles");
    double* agg = reinterpret_cast<double*>(workspace);
    double* carry = agg + 2 * g;
    if (f64v)
        hipLaunchKernelGGL(gae_tile_agg_kernel<true>, dim3((unsigned)g), dim3(TPB), 0, s, p, agg);
    else
        hipLaunchKernelGGL(gae_tile_agg_kernel<false>, dim3((unsigned)g), dim3(TPB), 0, s, p, agg);
    TSRL_LAUNCH_CHECK("tsrl_gae(agg)");
    hipLaunchKernelGGL(gae_carry_kernel, dim3(1), dim3(TPB), 0, s, agg, g, carry);
    TSRL_LAUNCH_CHECK("tsrl_gae(carry)");
    if (f64v)
        hipLaunchKernelGGL(gae_tile_apply_kernel<true>, dim3((unsigned)g), dim3(TPB), 0, s, p,
                           carry, vec_ok);
    else
        hipLaunchKernelGGL(gae_tile_apply_kernel<false>, dim3((unsigned)g), dim3(TPB), 0, s, p,
                           carry, vec_ok);
    TSRL_LAUNCH_CHECK("tsrl_gae(apply)");
    return 0;
}

extern "C" int tsrl_gae_f64v(const double* v_s, const double* v_s_next, const double* rew,
                             const uint8_t* terminated, const uint8_t* truncated,
                             const uint8_t* end_extra, int64_t n, int64_t row_len,
                             double gamma, double gae_lambda, double* adv64_out,
                             double* ret64_out, void* workspace, int64_t workspace_bytes,
                             void* stream) {
    TSRL_CHECK_ARG(n >= 0, "tsrl_gae_f64v: n < 0");
    if (n == 0) return 0;
    TSRL_CHECK_ARG(v_s && v_s_next && rew && terminated && truncated,
                   "tsrl_gae_f64v: null input pointer");
    GaeArgs p = {};
    p.vs64 = v_s;
    p.vn64 = v_s_next;
    p.rew = rew;
    p.term = terminated;
    p.trunc = truncated;
    p.extra = end_extra;
    p.n = n;
    p.row_len = row_len;
    p.gamma = gamma;
    p.g32 = (float)gamma;
    p.gl = gamma * gae_lambda;
    p.adv64 = adv64_out;
    p.ret64 = ret64_out;
    hipStream_t s = as_stream(stream);
    // f64 inputs always take the scalar-load path (vec_ok = 0); mode F64V with scale 1.0
    if (row_len > 0) {
        const int64_t r = range_len_for(row_len);
        const int64_t grid = (n + r - 1) / r;
        hipLaunchKernelGGL(gae_rows_kernel<true>, dim3((unsigned)grid), dim3(TPB), 0, s, p, r, 0);
        TSRL_LAUNCH_CHECK("tsrl_gae_f64v(rows)");
        return 0;
    }
    const int64_t g = (n + TILE - 1) / TILE;
    TSRL_CHECK_ARG(workspace && workspace_bytes >= tsrl_gae_workspace_bytes(n, 0),
                   "tsrl_gae_f64v: general path needs workspace");
    double* agg = reinterpret_cast<double*>(workspace);
    double* carry = agg + 2 * g;
    hipLaunchKernelGGL(gae_tile_agg_kernel<true>, dim3((unsigned)g), dim3(TPB), 0, s, p, agg);
    TSRL_LAUNCH_CHECK("tsrl_gae_f64v(agg)");
    hipLaunchKernelGGL(gae_carry_kernel, dim3(1), dim3(TPB), 0, s, agg, g, carry);
    TSRL_LAUNCH_CHECK("tsrl_gae_f64v(carry)");
    hipLaunchKernelGGL(gae_tile_apply_kernel<true>, dim3((unsigned)g), dim3(TPB), 0, s, p, carry,
                       0);
    TSRL_LAUNCH_CHECK("tsrl_gae_f64v(apply)");
    return 0;
}

extern "C" int tsrl_ret_rms_update(const double* partials, int64_t nparts, double* rms,
                                   void* stream) {
    TSRL_CHECK_ARG(partials && rms && nparts >= 0, "tsrl_ret_rms_update: bad arguments");
    if (nparts == 0) return 0;
    hipLaunchKernelGGL(ret_rms_update_kernel, dim3(1), dim3(TPB), 0, as_stream(stream),
                       partials, nparts, rms);
    TSRL_LAUNCH_CHECK("tsrl_ret_rms_update");
    return 0;
}
