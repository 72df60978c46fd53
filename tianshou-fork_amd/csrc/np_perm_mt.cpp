// NumPy's legacy np.random.permutation draws (tsrl_np_shuffle_draws, csrc/perm.hip) for LARGE n,
// computed by several host threads -- the draws the data-parallel PPO split of the GLOBAL batch
// needs (tianshou/data/batch.py:896-912 over world x n rows) without the
// O(world x n) single-thread cost.
//
// The output is bit-identical to the sequential loop (and so to NumPy): the same draws, the same
// final RandomState (key, pos).  Two parts of the sequential loop are parallelised:
//
// 1. The MT19937 stream.  The untempered words obey x_{k+624} = x_{k+397} ^ f(x_k, x_{k+1}), a
//    linear recurrence whose state (the upper bit of x_k and x_{k+1..k+623}) evolves by a map T of
//    minimal polynomial phi (degree 19937, found once by Berlekamp-Massey).  Every bit of the word
//    sequence satisfies phi's scalar recurrence, so with p = x^J mod phi,
//        x_{a+J+k} = XOR_{i : p_i = 1} x_{a+i+k}
//    ("jump ahead", Haramoto et al. 2008): the window 624 words ahead of chunk c's first output is
//    an XOR of shifted windows of one extended sequence, and each thread generates its chunk from
//    its own window.  (Word 0 of a jumped window can differ from the true one in its low 31 bits,
//    which are not part of the state; it is never an output of that chunk and only its top bit
//    feeds the recurrence.)
// 2. The masked rejection consumption (for i = n-1 .. 1: draw until (y & mask(i)) <= i).  The
//    stream is cut into chunks of CL words; chunk c's starting i is guessed from the exact
//    expectation of the death process (E[i + 1] falls by the factor m / (m + 1) per word under
//    mask m) and every word is classified for ALL starts within +-EW of the guess: certainly
//    accepted, certainly rejected, or uncertain (its value lies in the band the start
//    uncertainty allows).  A sequential walk then resolves only the uncertain words with the
//    exact start (~2 EW / m of the words), and a last parallel pass writes the draws chunk by
//    chunk from the exact starts.  A chunk whose exact start falls outside its window, or whose
//    band meets a mask change, is walked word by word (exact, just slower).
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>
#include <chrono>
#include <cstdio>
#include <cstdlib>

#include "tsrl_common.h"

namespace tsrl {
namespace npmt {

constexpr int NW = 624, MM = 397, DEG = 19937;
constexpr int PW = (DEG + 63) / 64;  // words of a polynomial of degree < DEG (312)
constexpr uint32_t MATA = 0x9908b0dfu, UPPER = 0x80000000u, LOWER = 0x7fffffffu;

inline uint32_t temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

// s[624 .. 624 + len) from the window s[0 .. 624).  Word k + 624 reads words k, k + 1 and
// k + 397, so the 224 words of a block depend only on earlier blocks: the inner loop vectorises.
inline void extend(uint32_t* __restrict__ s, size_t len) {
    constexpr size_t BLK = 224;
    size_t k0 = 0;
    for (; k0 + BLK <= len; k0 += BLK) {
        const uint32_t* __restrict__ a = s + k0;
        const uint32_t* __restrict__ b = s + k0 + MM;
        uint32_t* __restrict__ o = s + k0 + NW;
#pragma clang loop vectorize(enable)
        for (size_t k = 0; k < BLK; ++k) {
            const uint32_t y = (a[k] & UPPER) | (a[k + 1] & LOWER);
            o[k] = b[k] ^ (y >> 1) ^ ((0u - (y & 1u)) & MATA);
        }
    }
    for (size_t k = k0; k < len; ++k) {
        const uint32_t y = (s[k] & UPPER) | (s[k + 1] & LOWER);
        s[k + NW] = s[k + MM] ^ (y >> 1) ^ ((0u - (y & 1u)) & MATA);
    }
}

// out[0 .. len) = the 624 + len words after the window w[0 .. 624), written in place (len >= 624).
inline void gen_after(const uint32_t* w, uint32_t* __restrict__ out, size_t len) {
    auto f = [](uint32_t a, uint32_t b, uint32_t c) {
        const uint32_t y = (a & UPPER) | (b & LOWER);
        return c ^ (y >> 1) ^ ((0u - (y & 1u)) & MATA);
    };
    for (int k = 0; k < NW; ++k)
        out[k] = f(w[k], k + 1 < NW ? w[k + 1] : out[0], k + MM < NW ? w[k + MM] : out[k + MM - NW]);
    constexpr size_t BLK = 224;
    size_t k0 = NW;
    for (; k0 + BLK <= len; k0 += BLK) {
        const uint32_t* __restrict__ a = out + k0 - NW;
        const uint32_t* __restrict__ b = out + k0 - NW + MM;
        uint32_t* __restrict__ o = out + k0;
#pragma clang loop vectorize(enable)
        for (size_t k = 0; k < BLK; ++k) o[k] = f(a[k], a[k + 1], b[k]);
    }
    for (size_t k = k0; k < len; ++k) out[k] = f(out[k - NW], out[k - NW + 1], out[k - NW + MM]);
}

// ---- GF(2)[x] arithmetic -------------------------------------------------------------------
typedef std::vector<uint64_t> Poly;

inline bool getbit(const uint64_t* a, int64_t i) { return (a[i >> 6] >> (i & 63)) & 1; }

// a ^= b << sh (b has nb words, a is large enough)
inline void xor_shifted(uint64_t* a, const uint64_t* b, int nb, int64_t sh) {
    const int64_t ws = sh >> 6;
    const int bs = (int)(sh & 63);
    if (bs == 0) {
        for (int i = 0; i < nb; ++i) a[ws + i] ^= b[i];
    } else {
        uint64_t carry = 0;
        for (int i = 0; i < nb; ++i) {
            a[ws + i] ^= (b[i] << bs) | carry;
            carry = b[i] >> (64 - bs);
        }
        a[ws + nb] ^= carry;
    }
}

__attribute__((target("pclmul,sse2"))) inline void clmul64(uint64_t a, uint64_t b, uint64_t& lo,
                                                            uint64_t& hi) {
    typedef long long v2di __attribute__((vector_size(16)));
    const v2di va = {(long long)a, 0}, vb = {(long long)b, 0};
    const v2di r = __builtin_ia32_pclmulqdq128(va, vb, 0x00);
    lo = (uint64_t)r[0];
    hi = (uint64_t)r[1];
}

inline void clmul64_soft(uint64_t a, uint64_t b, uint64_t& lo, uint64_t& hi) {
    lo = hi = 0;
    for (int i = 0; i < 64; ++i)
        if ((b >> i) & 1) {
            lo ^= a << i;
            if (i) hi ^= a >> (64 - i);
        }
}

struct Field {
    Poly phi;  // PW + 1 words, degree DEG
    bool have_clmul = false;

    // r (2 PW words) -> r mod phi (first PW words valid, degree < DEG)
    void reduce(uint64_t* r) const {
        for (int64_t i = 2 * (int64_t)PW * 64 - 1; i >= DEG; --i)
            if (getbit(r, i)) xor_shifted(r, phi.data(), PW + 1, i - DEG);
    }
    Poly mulmod(const Poly& a, const Poly& b) const {
        std::vector<uint64_t> r(2 * PW + 2, 0);
        for (int i = 0; i < PW; ++i) {
            if (!a[i]) continue;
            for (int j = 0; j < PW; ++j) {
                uint64_t lo, hi;
                if (have_clmul) clmul64(a[i], b[j], lo, hi);
                else clmul64_soft(a[i], b[j], lo, hi);
                r[i + j] ^= lo;
                r[i + j + 1] ^= hi;
            }
        }
        reduce(r.data());
        return Poly(r.begin(), r.begin() + PW);
    }
};

// Minimal polynomial of bit 0 of the MT19937 word sequence (Berlekamp-Massey over GF(2)).
Poly find_phi() {
    const int64_t nbits = 2 * (int64_t)DEG + 64;
    std::vector<uint32_t> s(NW + nbits + 8);
    // init_genrand(5489) (the reference generator's default seed): any state works
    s[0] = 5489u;
    for (int i = 1; i < NW; ++i) s[i] = 1812433253u * (s[i - 1] ^ (s[i - 1] >> 30)) + i;
    extend(s.data(), nbits + 8);
    // bit sequence b_n = bit 0 of x_{n+1} (x_0's low bits are not part of the state)
    std::vector<uint8_t> b(nbits);
    for (int64_t n = 0; n < nbits; ++n) b[n] = s[n + 1] & 1u;
    // byte-level BM: O(N^2) but one-time (N ~ 40k)
    std::vector<uint8_t> C(nbits + 1, 0), B(nbits + 1, 0), T;
    C[0] = B[0] = 1;
    int64_t L = 0, m = -1;
    for (int64_t n = 0; n < nbits; ++n) {
        uint8_t d = b[n];
        for (int64_t i = 1; i <= L; ++i) d ^= C[i] & b[n - i];
        if (!d) continue;
        T = C;
        const int64_t sh = n - m;
        for (int64_t i = 0; i + sh <= nbits; ++i) C[i + sh] ^= B[i];
        if (2 * L <= n) {
            L = n + 1 - L;
            m = n;
            B = T;
        }
    }
    // connection polynomial C(x) = 1 + c1 x + ... + cL x^L; the characteristic polynomial of
    // the recurrence is its reciprocal x^L C(1/x)
    Poly phi(PW + 1, 0);
    if (L != DEG) return Poly();  // not the full period polynomial (never for MT19937)
    for (int64_t i = 0; i <= L; ++i)
        if (C[i]) phi[(L - i) >> 6] |= 1ull << ((L - i) & 63);
    return phi;
}

struct JumpTable {
    std::mutex mu;
    Field f;
    bool ready = false;
    int64_t J = 0;
    std::vector<Poly> pc;  // pc[c] = x^(cJ) mod phi

    const Poly& get(int64_t c) {
        std::lock_guard<std::mutex> g(mu);
        while ((int64_t)pc.size() <= c) pc.push_back(f.mulmod(pc.back(), pc[1]));
        return pc[c];
    }
    bool init(int64_t j_log2) {
        std::lock_guard<std::mutex> g(mu);
        if (ready) return true;
        f.have_clmul = __builtin_cpu_supports("pclmul");
        f.phi = find_phi();
        if (f.phi.empty()) return false;
        // x^(2^j_log2) mod phi by repeated squaring of x
        Poly p(PW, 0);
        p[0] = 2;  // x
        for (int k = 0; k < j_log2; ++k) p = f.mulmod(p, p);
        J = (int64_t)1 << j_log2;
        Poly one(PW, 0);
        one[0] = 1;
        pc.push_back(one);
        pc.push_back(p);
        ready = true;
        return true;
    }
};

JumpTable g_jump;

// Stream buffers kept across calls (no zero-fill, pages faulted in once): the draws of every
// repeat of an update have the same size.
struct Buffers {
    std::mutex mu;
    std::unique_ptr<uint32_t[]> X, Y;
    int64_t nx = 0, ny = 0;
    // 1/16 headroom: the stream length of one n varies by a few thousand words per call
    uint32_t* x(int64_t n) {
        if (n > nx) X.reset(new uint32_t[(size_t)(nx = n + n / 16)]);
        return X.get();
    }
    uint32_t* y(int64_t n) {
        if (n > ny) Y.reset(new uint32_t[(size_t)(ny = n + n / 16)]);
        return Y.get();
    }
};
Buffers g_buf;
constexpr int JLOG = 22;  // 4 Mi words per generation chunk

// Window 624 words ahead: out[k] = XOR_{i: p_i} E[i + k], k < 624 (E: >= DEG - 1 + 624 words).
void apply_jump(const Poly& p, const uint32_t* E, uint32_t* out) {
    uint32_t acc[NW];
    memset(acc, 0, sizeof(acc));
    for (int w = 0; w < PW; ++w) {
        uint64_t bits = p[w];
        while (bits) {
            const int i = 64 * w + __builtin_ctzll(bits);
            bits &= bits - 1;
            const uint32_t* src = E + i;
            for (int k = 0; k < NW; ++k) acc[k] ^= src[k];
        }
    }
    memcpy(out, acc, sizeof(acc));
}

// ---- the parallel draws ------------------------------------------------------------------------
inline uint32_t mask_of(uint32_t i) { return 0xFFFFFFFFu >> __builtin_clz(i); }

struct ChunkInfo {
    int64_t w0, w1;        // word range [w0, w1) of the stream
    double guess;          // guessed i at w0
    bool seq;              // walk word by word
    int64_t cert_acc;      // certainly accepted words (window mode)
    std::vector<int32_t> unc;     // uncertain words (local index)
    std::vector<int32_t> unc_acc; // certainly accepted words before each uncertain one
    int64_t start = -1;    // exact i at w0 (phase 2)
};

}  // namespace npmt
}  // namespace tsrl

using namespace tsrl::npmt;

// Threads: nthreads <= 0 -> hardware concurrency (at most 32).
extern "C" int tsrl_np_shuffle_draws_mt(uint32_t* key, int32_t* pos, int64_t n, uint32_t* draws,
                                        int nthreads) {
    TSRL_CHECK_ARG(key && pos && (draws || n <= 0), "tsrl_np_shuffle_draws_mt: null argument");
    TSRL_CHECK_ARG(n >= 0 && n <= (int64_t)INT_MAX,
                   "tsrl_np_shuffle_draws_mt: n=%lld outside [0, 2^31)", (long long)n);
    TSRL_CHECK_ARG(*pos >= 0 && *pos <= NW, "tsrl_np_shuffle_draws_mt: pos=%d", (int)*pos);
    if (n < ((int64_t)1 << 21)) return tsrl_np_shuffle_draws(key, pos, n, draws);
    if (!g_jump.init(JLOG)) return tsrl_np_shuffle_draws(key, pos, n, draws);
    const bool timing = getenv("TSRL_PERM_TIMING") != nullptr;
    auto now = [] { return std::chrono::duration<double>(
                        std::chrono::steady_clock::now().time_since_epoch()).count(); };
    double tm[8];
    tm[0] = now();
    int T = nthreads > 0 ? nthreads : (int)std::thread::hardware_concurrency();
    T = std::max(1, std::min(T, 32));
    draws[0] = 0;
    const int p0 = *pos;
    const int64_t J = g_jump.J;
    // expected words: sum over i of (mask(i) + 1) / (i + 1), plus a wide margin (the sd is
    // ~sqrt of the rejections, a few thousand at 2^26)
    double expect = 0.0;
    for (int64_t hi = n - 1; hi >= 1;) {
        const uint32_t m = mask_of((uint32_t)hi);
        const int64_t lo = (int64_t)(m >> 1) + 1;
        // sum_{i=lo}^{hi} (m+1)/(i+1)
        expect += (double)(m + 1.0) * (std::log((hi + 1.5) / (lo + 0.5)));
        hi = lo - 1;
    }
    int64_t W = (int64_t)(expect * 1.01) + (1 << 20);
    // stream words: prefix = key[p0 .. 624), then x_{t+624 ..} generated in chunks of J
    const int64_t pre = NW - p0;
    int64_t nchunk = (W - pre + J - 1) / J;
    if (nchunk < 1) nchunk = 1;
    W = pre + nchunk * J;
    std::lock_guard<std::mutex> buf_guard(g_buf.mu);
    uint32_t* X = g_buf.x(nchunk * J);  // untempered x_{t+624+i}
    uint32_t* Y = g_buf.y(W);           // tempered stream
    // extended sequence of the base window for the jumps
    std::vector<uint32_t> E(NW + DEG + NW);
    memcpy(E.data(), key, NW * 4);
    extend(E.data(), DEG + NW);
    for (int64_t c = 0; c <= nchunk; ++c) (void)g_jump.get(c);  // polys (cached, one-time)
    tm[1] = now();
    {
        std::atomic<int64_t> next(0);
        auto gen = [&]() {
            uint32_t win[NW];
            for (int64_t c; (c = next.fetch_add(1)) < nchunk;) {
                if (c == 0) memcpy(win, key, NW * 4);
                else apply_jump(g_jump.get(c), E.data(), win);
                uint32_t* x = X + c * J;
                gen_after(win, x, (size_t)J);
                uint32_t* y = Y + pre + c * J;
                for (int64_t u = 0; u < J; ++u) y[u] = temper(x[u]);
            }
        };
        std::vector<std::thread> th;
        for (int k = 0; k < T; ++k) th.emplace_back(gen);
        for (auto& t : th) t.join();
    }
    for (int64_t u = 0; u < pre; ++u) Y[u] = temper(key[p0 + u]);
    tm[2] = now();

    // ---- acceptance: chunks of CL words with guessed starts ----------------------------------
    const int64_t CL = 1 << 16;
    // start uncertainty of the window classification: the exact start drifts from the
    // expectation like a random walk (sd ~ sqrt(words / 4)); 8 sd + 2048 at each chunk
    auto ew_of = [](int64_t w0) { return 2048.0 + 8.0 * std::sqrt(0.25 * (double)w0); };
    const int64_t nc = (W + CL - 1) / CL;
    std::vector<ChunkInfo> ch((size_t)nc);
    {
        // exact expectation of the death process: E[i + 1] *= m / (m + 1) per word under mask m
        double g = (double)(n - 1);
        for (int64_t c = 0; c < nc; ++c) {
            ChunkInfo& k = ch[c];
            k.w0 = c * CL;
            k.w1 = std::min(W, k.w0 + CL);
            k.guess = g;
            int64_t left = k.w1 - k.w0;
            while (left > 0 && g >= 1.0) {
                const uint32_t m = mask_of((uint32_t)std::max(1.0, std::floor(g)));
                const double lo = (double)(m >> 1) + 1.0;
                const double q = (double)m / ((double)m + 1.0);
                // words until E[i] reaches the mask's lower bound
                const double need = std::log((lo - 0.5 + 1.0) / (g + 1.0)) / std::log(q);
                const double step = std::min((double)left, std::max(1.0, need));
                g = (g + 1.0) * std::pow(q, step) - 1.0;
                left -= (int64_t)step;
                if (step >= need) g = std::min(g, lo - 1.0);
            }
        }
    }
    // phase 1 (parallel): classification for starts in [guess - EW, guess + EW]
    auto classify = [&](ChunkInfo& k) {
        const double EW = ew_of(k.w0);
        const int64_t gl = (int64_t)std::floor(k.guess - EW), gh = (int64_t)std::ceil(k.guess + EW);
        if (gl < 2 || gh > (int64_t)UINT32_MAX) {
            k.seq = true;
            return;
        }
        const uint32_t mhi = mask_of((uint32_t)gh);
        const int64_t mlo = (int64_t)(mhi >> 1) + 1;  // the band must stay at or above it
        const int64_t floor_i = std::max<int64_t>(2, mlo);
        int64_t acc_lo = 0, unc = 0;  // certain accepts / uncertain words so far
        k.seq = false;
        k.cert_acc = 0;
        const uint32_t* y = Y + k.w0;
        const int64_t len = k.w1 - k.w0;
        // blocks of 64 words classified against one band that holds for every word of the block
        // (at most 64 more accepts or uncertain words inside it): branch-free, vectorisable
        for (int64_t j0 = 0; j0 < len; j0 += 64) {
            const int nb = (int)std::min<int64_t>(64, len - j0);
            const int64_t imin = gl - (acc_lo + unc) - 64, imax = gh - acc_lo;
            if (imin < floor_i) {
                k.seq = true;  // the band meets a mask change (or the end): walk it exactly
                k.unc.clear();
                k.unc_acc.clear();
                return;
            }
            uint64_t acc_bits = 0, unc_bits = 0;
            for (int q = 0; q < nb; ++q) {
                const int64_t v = (int64_t)(y[j0 + q] & mhi);
                acc_bits |= (uint64_t)(v <= imin) << q;
                unc_bits |= (uint64_t)((v > imin) & (v <= imax)) << q;
            }
            while (__builtin_expect(unc_bits != 0, 0)) {
                const int q = __builtin_ctzll(unc_bits);
                unc_bits &= unc_bits - 1;
                k.unc.push_back((int32_t)(j0 + q));
                k.unc_acc.push_back(
                    (int32_t)(acc_lo + __builtin_popcountll(acc_bits & ((1ull << q) - 1))));
                ++unc;
            }
            acc_lo += __builtin_popcountll(acc_bits);
        }
        k.cert_acc = acc_lo;
    };
    {
        std::atomic<int64_t> next(0);
        auto work = [&]() {
            for (int64_t c; (c = next.fetch_add(1)) < nc;) classify(ch[c]);
        };
        std::vector<std::thread> th;
        for (int k = 0; k < T; ++k) th.emplace_back(work);
        for (auto& t : th) t.join();
    }
    tm[3] = now();
    // phase 2 (sequential): exact chunk starts
    int64_t cur = n - 1;
    int64_t used = -1;  // words consumed
    int64_t n_miss = 0;
    double max_dev = 0.0;
    for (int64_t c = 0; c < nc && used < 0; ++c) {
        ChunkInfo& k = ch[c];
        k.start = cur;
        const double EW = ew_of(k.w0);
        const bool in_win = !k.seq && (double)cur >= std::floor(k.guess - EW) &&
                            (double)cur <= std::ceil(k.guess + EW);
        if (!k.seq && !in_win) ++n_miss;
        if (!k.seq) max_dev = std::max(max_dev, std::fabs((double)cur - k.guess));
        if (in_win) {
            int64_t accu = 0;
            for (size_t u = 0; u < k.unc.size(); ++u) {
                const int64_t i = cur - ((int64_t)k.unc_acc[u] + accu);
                const uint32_t v = Y[k.w0 + k.unc[u]] & mask_of((uint32_t)i);
                accu += (int64_t)v <= i;
            }
            cur -= k.cert_acc + accu;
            continue;
        }
        // walk the chunk word by word (also detects the end of the draws)
        k.seq = true;
        for (int64_t w = k.w0; w < k.w1; ++w) {
            const uint32_t v = Y[w] & mask_of((uint32_t)cur);
            cur -= (int64_t)(v <= (uint32_t)cur);
            if (cur == 0) {
                used = w + 1;
                break;
            }
        }
    }
    if (used < 0) {
        tsrl::set_error("tsrl_np_shuffle_draws_mt: stream of %lld words exhausted (n=%lld)",
                  (long long)W, (long long)n);
        return (int)hipErrorUnknown;
    }
    tm[4] = now();
    // phase 3 (parallel): the draws of every chunk from its exact start (cur is exact at each
    // chunk start up to the last one, which ends at i = 0)
    std::vector<uint32_t> first_v((size_t)nc, 0);
    {
        std::atomic<int64_t> next(0);
        auto work = [&]() {
            for (int64_t c; (c = next.fetch_add(1)) < nc;) {
                const ChunkInfo& k = ch[c];
                if (k.start < 1) continue;
                int64_t i = k.start;
                const int64_t w1 = std::min(k.w1, used);
                // only accepted words are written: a chunk's trailing rejections for the next
                // chunk's first i must not race with that chunk's accepted draw
                // branch-free like the sequential loop (every word written at the current i, a
                // rejected word overwritten by the next candidate); the next chunk's first draw
                // index may receive this chunk's trailing rejections: first_v repairs it below
                uint32_t m = mask_of((uint32_t)i), mlo = (m >> 1) + 1;
                uint32_t ui = (uint32_t)i;
                bool first = true;
                for (int64_t w = k.w0; w < w1; ++w) {
                    const uint32_t v = Y[w] & m;
                    draws[ui] = v;
                    const uint32_t acc = v <= ui;
                    if (first && acc) {
                        first_v[c] = v;
                        first = false;
                    }
                    ui -= acc;
                    if (__builtin_expect(ui < mlo, 0)) {
                        if (ui < 1) break;
                        m >>= 1;
                        mlo = (m >> 1) + 1;
                    }
                }
            }
        };
        std::vector<std::thread> th;
        for (int k = 0; k < T; ++k) th.emplace_back(work);
        for (auto& t : th) t.join();
    }
    // chunk c's first accepted draw lands at draws[start_c], where chunk c - 1's trailing
    // rejected words also wrote: restore it (chunks in order; a chunk that accepts nothing
    // leaves start unchanged for the next, whose own first_v then rules)
    for (int64_t c = 0; c < nc; ++c)
        if (ch[c].start >= 1 && ch[c].w0 < used) {
            // only if this chunk accepted at least once (else the next chunk starts at the same i)
            const int64_t nxt = c + 1 < nc ? ch[c + 1].start : 0;
            if (nxt < ch[c].start || c + 1 == nc) draws[ch[c].start] = first_v[c];
        }
    tm[5] = now();
    if (timing) {
        int64_t nseq = 0, nunc = 0;
        for (const auto& k : ch) {
            nseq += k.seq;
            nunc += (int64_t)k.unc.size();
        }
        fprintf(stderr, "np_perm_mt n=%lld W=%lld T=%d: polys %.1f ms, stream %.1f ms, classify "
                "%.1f ms, walk %.1f ms (seq chunks %lld / %lld, uncertain %lld, window misses %lld, "
                "max start deviation %.0f), draws %.1f ms\n",
                (long long)n, (long long)W, T, 1e3 * (tm[1] - tm[0]), 1e3 * (tm[2] - tm[1]),
                1e3 * (tm[3] - tm[2]), 1e3 * (tm[4] - tm[3]), (long long)nseq, (long long)nc,
                (long long)nunc, (long long)n_miss, max_dev, 1e3 * (tm[5] - tm[4]));
    }
    // final state: the block holding the last consumed word (NumPy twists lazily: pos in 1..624)
    const int64_t arel = (int64_t)p0 + used - 1;  // index of the last word relative to key[0]
    const int64_t blk = arel / NW;
    if (blk > 0) memcpy(key, X + (blk - 1) * NW, NW * 4);
    *pos = (int32_t)(arel - blk * NW + 1);
    return 0;
}
