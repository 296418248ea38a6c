// CPython 3.10 random.Random restated for the sampler: the MT19937 core of
// Modules/_randommodule.c (genrand_uint32, init_genrand, init_by_array) plus
// the Lib/random.py pieces the reference calls — _randbelow_with_getrandbits,
// sample() (both branches) and choice().  The reference's sampling semantics
// are *defined* by these (models.py:281-282 random.sample, :178 random.choice),
// so the state here is word-for-word interchangeable with random.getstate().
#pragma once

#include <immintrin.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#ifndef GS_SELECT_SMALL
#define GS_SELECT_SMALL 1
#endif

namespace gs {

struct MT19937 {
    static constexpr int N = 624;
    static constexpr int M = 397;
    uint32_t mt[N];
    int index = N + 1;

    void init_genrand(uint32_t s) {
        ext = false;
        mt[0] = s;
        for (int i = 1; i < N; ++i)
            mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + static_cast<uint32_t>(i);
        index = N;
    }

    // random.seed(int): init_by_array over the 32-bit words of abs(seed).
    void init_by_array(const uint32_t* key, size_t len) {
        init_genrand(19650218u);
        size_t i = 1, j = 0;
        size_t k = (N > len ? N : len);
        for (; k; --k) {
            mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] +
                    static_cast<uint32_t>(j);
            ++i;
            ++j;
            if (i >= static_cast<size_t>(N)) {
                mt[0] = mt[N - 1];
                i = 1;
            }
            if (j >= len) j = 0;
        }
        for (k = N - 1; k; --k) {
            mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) -
                    static_cast<uint32_t>(i);
            ++i;
            if (i >= static_cast<size_t>(N)) {
                mt[0] = mt[N - 1];
                i = 1;
            }
        }
        mt[0] = 0x80000000u;
        index = N;
    }

    // Output words of the current block, tempered once per block (the block's
    // raw state stays in mt[], exactly what random.getstate() exposes).
    // out[N .. N + kExt): the next block's first words, valid while `ext`
    // (extend()), so a fast path can read across the block end; mt[] and the
    // stream position stay CPython's (settle() twists once they are consumed).
    static constexpr int kExt = 32;
    alignas(64) uint32_t out[N + kExt];
    bool ext = false;

    static inline uint32_t temper(uint32_t y) {
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= (y >> 18);
        return y;
    }

    // Recompute out[] from mt[] (after setstate and every twist): the
    // tempering of 8 words per AVX2 instruction sequence.
    void refresh() {
        const __m256i b = _mm256_set1_epi32(static_cast<int32_t>(0x9d2c5680u));
        const __m256i c = _mm256_set1_epi32(static_cast<int32_t>(0xefc60000u));
        static_assert(N % 8 == 0, "whole vectors");
        for (int i = 0; i < N; i += 8) {
            __m256i y = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(mt + i));
            y = _mm256_xor_si256(y, _mm256_srli_epi32(y, 11));
            y = _mm256_xor_si256(y, _mm256_and_si256(_mm256_slli_epi32(y, 7), b));
            y = _mm256_xor_si256(y, _mm256_and_si256(_mm256_slli_epi32(y, 15), c));
            y = _mm256_xor_si256(y, _mm256_srli_epi32(y, 18));
            _mm256_store_si256(reinterpret_cast<__m256i*>(out + i), y);
        }
        ext = false;
    }

    // The next block's first kExt tempered words from the current mt[]
    // (new mt[kk] = mt[kk + M] ^ twist(mt[kk], mt[kk + 1]) for kk < N - M),
    // mt[] untouched: twist() later produces the same words.
    void extend() {
        constexpr uint32_t A = 0x9908b0dfu;
        for (int kk = 0; kk < kExt; ++kk) {
            const uint32_t y = (mt[kk] & 0x80000000u) | (mt[kk + 1] & 0x7fffffffu);
            out[N + kk] = temper(mt[kk + M] ^ (y >> 1) ^ ((0u - (y & 1u)) & A));
        }
        ext = true;
    }

    // After a fast path consumed words past the block end: the twist that
    // genrand_uint32 would have done, the position carried into the new block
    // (index == N stays as is: CPython twists lazily on the next draw).
    void settle() {
        if (index > N) {
            const int over = index - N;
            twist();
            index = over;
        }
    }

    // genrand_uint32's block regeneration, eight words per AVX2 step: the
    // recurrence distances (1 ahead, 397 ahead, then 227 behind) all exceed
    // or precede the 8-word vector, so each vector reads only words that are
    // final for this twist (old mt[kk + 1 ..], new mt[kk - 227 ..]).
    static inline __m256i twist8(__m256i cur, __m256i nxt, __m256i far) {
        const __m256i up = _mm256_set1_epi32(static_cast<int32_t>(0x80000000u));
        const __m256i lo = _mm256_set1_epi32(0x7fffffff);
        const __m256i a = _mm256_set1_epi32(static_cast<int32_t>(0x9908b0dfu));
        const __m256i one = _mm256_set1_epi32(1);
        const __m256i y = _mm256_or_si256(_mm256_and_si256(cur, up), _mm256_and_si256(nxt, lo));
        const __m256i mag = _mm256_and_si256(_mm256_cmpeq_epi32(_mm256_and_si256(y, one), one), a);
        return _mm256_xor_si256(_mm256_xor_si256(far, _mm256_srli_epi32(y, 1)), mag);
    }
    static inline uint32_t twist1(uint32_t cur, uint32_t nxt, uint32_t far) {
        constexpr uint32_t A = 0x9908b0dfu;
        const uint32_t y = (cur & 0x80000000u) | (nxt & 0x7fffffffu);
        return far ^ (y >> 1) ^ ((0u - (y & 1u)) & A);
    }
    void twist() {
        auto ld = [&](int i) { return _mm256_loadu_si256(reinterpret_cast<const __m256i*>(mt + i)); };
        int kk = 0;
        for (; kk + 8 <= N - M; kk += 8)  // 0 .. 223
            _mm256_storeu_si256(reinterpret_cast<__m256i*>(mt + kk), twist8(ld(kk), ld(kk + 1), ld(kk + M)));
        for (; kk < N - M; ++kk) mt[kk] = twist1(mt[kk], mt[kk + 1], mt[kk + M]);
        for (; kk + 8 <= N - 1; kk += 8)  // 227 .. 618
            _mm256_storeu_si256(reinterpret_cast<__m256i*>(mt + kk),
                                twist8(ld(kk), ld(kk + 1), ld(kk + (M - N))));
        for (; kk < N - 1; ++kk) mt[kk] = twist1(mt[kk], mt[kk + 1], mt[kk + (M - N)]);
        mt[N - 1] = twist1(mt[N - 1], mt[0], mt[M - 1]);
        refresh();
        index = 0;
    }

    inline uint32_t next() {
        if (index >= N) twist();
        return out[index++];
    }

    // getrandbits(k) for 1 <= k <= 32 (the fast path of _random_Random_getrandbits).
    inline uint32_t getrandbits(int k) { return next() >> (32 - k); }

    // Random._randbelow_with_getrandbits(n): k = n.bit_length(); reject r >= n.
    // n == 1 still consumes words (k = 1) — the randbelow(1) quirk.
    inline uint32_t randbelow(uint64_t n) {
        if (n == 0) return 0;
        const int k = 64 - __builtin_clzll(n);
        uint32_t r = getrandbits(k);
        while (r >= n) r = getrandbits(k);
        return r;
    }
};

// random.sample(): `setsize` decides between the list-pool and the
// selected-set branch (Lib/random.py, 3.10).
inline int64_t sample_setsize(int64_t k) {
    int64_t setsize = 21;
    if (k > 5) {
        const double e = std::ceil(std::log(static_cast<double>(k * 3)) / std::log(4.0));
        int64_t p = 1;
        for (int64_t t = 0; t < static_cast<int64_t>(e); ++t) p *= 4;
        setsize += p;
    }
    return setsize;
}

// The selected-set branch for k <= 32, eight stream words at a time.  A
// word is a repeat exactly when it equals an already selected value or an
// earlier in-range word of the same call (an earlier in-range word was either
// selected or itself a repeat of a selected value), so the freshness of the
// eight words of a chunk follows from comparisons alone, without a
// data-dependent branch per word.  The first (k - cnt) fresh words are taken,
// and the stream advances by exactly the words up to the last one taken —
// the same consumption as redrawing word by word.  Near the end of a block
// (fewer than 8 words left) words are taken one at a time through next().
template <class OutT>
inline void select_chunked(MT19937& rng, int64_t n, int64_t k, OutT* out) {
    const int sh = 32 - (64 - __builtin_clzll(static_cast<uint64_t>(n)));
    const __m128i shv = _mm_cvtsi32_si128(sh);
    const __m256i nv = _mm256_set1_epi32(static_cast<int32_t>(n));
    alignas(32) int32_t sel[32];
    const __m256i none = _mm256_set1_epi32(-1);
    for (int q = 0; q < 4; ++q) _mm256_store_si256(reinterpret_cast<__m256i*>(sel) + q, none);
    int32_t cnt = 0;
    while (cnt < k) {
        if (rng.index + 8 <= MT19937::N) {
            const __m256i w = _mm256_srl_epi32(
                _mm256_loadu_si256(reinterpret_cast<const __m256i*>(rng.out + rng.index)), shv);
            const int inr = _mm256_movemask_ps(_mm256_castsi256_ps(_mm256_cmpgt_epi32(nv, w)));
            const __m256i s0 = _mm256_load_si256(reinterpret_cast<const __m256i*>(sel));
            const __m256i s1 = _mm256_load_si256(reinterpret_cast<const __m256i*>(sel) + 1);
            const __m256i s2 = _mm256_load_si256(reinterpret_cast<const __m256i*>(sel) + 2);
            const __m256i s3 = _mm256_load_si256(reinterpret_cast<const __m256i*>(sel) + 3);
            uint32_t fresh = 0;
#pragma GCC unroll 8
            for (int i = 0; i < 8; ++i) {
                const __m256i b = _mm256_permutevar8x32_epi32(w, _mm256_set1_epi32(i));
                const int earlier = _mm256_movemask_ps(_mm256_castsi256_ps(_mm256_cmpeq_epi32(b, w))) & inr &
                                    ((1 << i) - 1);
                const __m256i h = _mm256_or_si256(_mm256_or_si256(_mm256_cmpeq_epi32(b, s0), _mm256_cmpeq_epi32(b, s1)),
                                                  _mm256_or_si256(_mm256_cmpeq_epi32(b, s2), _mm256_cmpeq_epi32(b, s3)));
                const uint32_t ok = ((inr >> i) & 1) & (earlier == 0) & _mm256_testz_si256(h, h);
                fresh |= ok << i;
            }
            const int need = static_cast<int>(k) - cnt;
            int consumed = 8;
            if (__builtin_popcount(fresh) >= need) {
                const int last = __builtin_ctz(_pdep_u32(1u << (need - 1), fresh));
                consumed = last + 1;
                fresh &= (2u << last) - 1;
            }
            alignas(32) int32_t wv[8];
            _mm256_store_si256(reinterpret_cast<__m256i*>(wv), w);
            while (fresh) {
                const int i = __builtin_ctz(fresh);
                sel[cnt] = wv[i];
                out[cnt] = static_cast<OutT>(wv[i]);
                ++cnt;
                fresh &= fresh - 1;
            }
            rng.index += consumed;
        } else {
            const uint32_t r = rng.next() >> sh;
            bool ok = r < static_cast<uint32_t>(n);
            for (int32_t t = 0; t < cnt; ++t) ok &= sel[t] != static_cast<int32_t>(r);
            sel[cnt] = ok ? static_cast<int32_t>(r) : -1;
            out[cnt] = static_cast<OutT>(r);  // kept only when fresh
            cnt += ok;
        }
    }
}

// Selected-set branch, common case for k <= 16: the k selected values are
// the first k in-range words of the next 32 whenever those k values are
// pairwise distinct (no word of the call is then a repeat).  The in-range
// test is one vector compare per 8 words, the k values are compacted in
// stream order and checked for a repeat with in-register rotations.  Returns
// false, having consumed nothing, when fewer than k of the 32 words are in
// range, a repeat occurs, or the block has fewer than 32 words left; the
// caller then runs the general scan from the same stream position.
// Left-packing permutations of an 8-lane vector: row m lists the lanes whose
// bit is set in m, in lane order (the rest 0).
struct PackLut {
    int32_t idx[256][8];
};
constexpr PackLut make_pack_lut() {
    PackLut t{};
    for (int m = 0; m < 256; ++m) {
        int j = 0;
        for (int i = 0; i < 8; ++i)
            if ((m >> i) & 1) t.idx[m][j++] = i;
        for (; j < 8; ++j) t.idx[m][j] = 0;
    }
    return t;
}
alignas(32) inline constexpr PackLut kPackLut = make_pack_lut();

template <class OutT>
inline bool select_fast16(MT19937& rng, int64_t n, int64_t k, OutT* out) {
    static_assert(MT19937::kExt >= 32, "the fast path reads 32 words");
    if (rng.index >= MT19937::N) rng.twist();  // genrand_uint32's lazy twist, before the first word
    if (rng.index + 32 > MT19937::N && !rng.ext) rng.extend();  // words across the block end
    const int sh = 32 - (64 - __builtin_clzll(static_cast<uint64_t>(n)));
    const __m128i shv = _mm_cvtsi32_si128(sh);
    const __m256i nv = _mm256_set1_epi32(static_cast<int32_t>(n));
    const __m256i* src = reinterpret_cast<const __m256i*>(rng.out + rng.index);
    __m256i v[4];
    uint32_t inr = 0;
#pragma GCC unroll 4
    for (int q = 0; q < 4; ++q) {
        v[q] = _mm256_srl_epi32(_mm256_loadu_si256(src + q), shv);
        inr |= static_cast<uint32_t>(_mm256_movemask_ps(_mm256_castsi256_ps(_mm256_cmpgt_epi32(nv, v[q])))) << (8 * q);
    }
    if (__builtin_popcount(inr) < k) return false;
    // The in-range values in stream order, left-packed 8 lanes at a time (a
    // table permutation per chunk: no per-value dependency chain); only the
    // first k are used.
    alignas(32) int32_t c[40];
    int at = 0;
#pragma GCC unroll 4
    for (int q = 0; q < 4; ++q) {
        const uint32_t m = (inr >> (8 * q)) & 0xFFu;
        const __m256i perm = _mm256_load_si256(reinterpret_cast<const __m256i*>(kPackLut.idx[m]));
        _mm256_storeu_si256(reinterpret_cast<__m256i*>(c + at), _mm256_permutevar8x32_epi32(v[q], perm));
        at += __builtin_popcount(m);
    }
    const int last = __builtin_ctz(_pdep_u32(1u << (k - 1), inr));  // the k-th in-range word
    // lanes past k padded with distinct negatives (never equal to a value)
    const __m256i kv = _mm256_set1_epi32(static_cast<int32_t>(k));
    const __m256i a = _mm256_blendv_epi8(
        _mm256_setr_epi32(-1, -2, -3, -4, -5, -6, -7, -8), _mm256_load_si256(reinterpret_cast<const __m256i*>(c)),
        _mm256_cmpgt_epi32(kv, _mm256_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7)));
    const __m256i b = _mm256_blendv_epi8(
        _mm256_setr_epi32(-9, -10, -11, -12, -13, -14, -15, -16), _mm256_load_si256(reinterpret_cast<const __m256i*>(c) + 1),
        _mm256_cmpgt_epi32(kv, _mm256_setr_epi32(8, 9, 10, 11, 12, 13, 14, 15)));
    __m256i dup = _mm256_setzero_si256();
#pragma GCC unroll 4
    for (int r = 1; r <= 4; ++r) {  // rotations 1..4 cover every pair inside a vector
        const __m256i rot = _mm256_setr_epi32(r & 7, (r + 1) & 7, (r + 2) & 7, (r + 3) & 7, (r + 4) & 7,
                                              (r + 5) & 7, (r + 6) & 7, (r + 7) & 7);
        dup = _mm256_or_si256(dup, _mm256_cmpeq_epi32(a, _mm256_permutevar8x32_epi32(a, rot)));
        if (k > 8) dup = _mm256_or_si256(dup, _mm256_cmpeq_epi32(b, _mm256_permutevar8x32_epi32(b, rot)));
    }
    if (k > 8) {
#pragma GCC unroll 8
        for (int r = 0; r < 8; ++r) {  // every pair across the two vectors
            const __m256i rot = _mm256_setr_epi32(r & 7, (r + 1) & 7, (r + 2) & 7, (r + 3) & 7, (r + 4) & 7,
                                                  (r + 5) & 7, (r + 6) & 7, (r + 7) & 7);
            dup = _mm256_or_si256(dup, _mm256_cmpeq_epi32(a, _mm256_permutevar8x32_epi32(b, rot)));
        }
    }
    if (!_mm256_testz_si256(dup, dup)) {
        // A repeat among the first k in-range values: the picks are the first
        // k values of the packed in-range run that repeat no earlier pick (a
        // value repeating an earlier in-range word repeats a pick), and the
        // stream advances past the word of the k-th.  Fewer than k such values
        // in the 32 words: the general scan from the same position.
        int32_t sel[16];
        int cnt = 0, idx = 0;
        for (; idx < at && cnt < k; ++idx) {
            const int32_t v = c[idx];
            bool fresh = true;
            for (int t = 0; t < cnt; ++t) fresh &= sel[t] != v;
            sel[cnt] = v;
            cnt += fresh;
        }
        if (cnt < k) return false;
        for (int i = 0; i < k; ++i) out[i] = static_cast<OutT>(sel[i]);
        rng.index += __builtin_ctz(_pdep_u32(1u << (idx - 1), inr)) + 1;
        rng.settle();
        return true;
    }
    for (int i = 0; i < k; ++i) out[i] = static_cast<OutT>(c[i]);
    rng.index += last + 1;
    rng.settle();
    return true;
}

// Pool branch: the draws' word consumption first (each randbelow(n - i)
// takes words until one is below n - i; a rejected word just advances the
// stream), as one loop over words whose only unpredictable decision is a
// counter increment, then the pool swaps (result[i] = pool[j];
// pool[j] = pool[n-i-1]).  Requires k <= 32 and the draws to fit in the
// current block (checked: otherwise false, nothing consumed).
template <class OutT>
inline bool pool_fast(MT19937& rng, int64_t n, int64_t k, OutT* out, int32_t* pool) {
    constexpr int kMaxWords = 96;  // enough for k <= 32 at rejection rates < 1/2, else fall back
    int idx = rng.index;
    const int end = std::min(MT19937::N, idx + kMaxWords);
    uint32_t r[32];
    int i = 0;
    const uint32_t nn = static_cast<uint32_t>(n);
    const int sh0 = __builtin_clz(nn);  // 32 - bit_length(n)
    if (__builtin_clz(nn - static_cast<uint32_t>(k - 1)) == sh0) {
        // every n - i has n's bit length: one shift for all words
        while (i < k && idx < end) {
            const uint32_t v = rng.out[idx++] >> sh0;
            r[i] = v;
            i += v < nn - static_cast<uint32_t>(i);
        }
    } else {
        while (i < k && idx < end) {
            const uint32_t mlim = nn - static_cast<uint32_t>(i);
            const uint32_t v = rng.out[idx++] >> __builtin_clz(mlim);
            r[i] = v;
            i += v < mlim;
        }
    }
    if (i < k) return false;
    rng.index = idx;
    for (int64_t t = 0; t < n; ++t) pool[t] = static_cast<int32_t>(t);
    for (int64_t q = 0; q < k; ++q) {
        const uint32_t j = r[q];
        out[q] = static_cast<OutT>(pool[j]);
        pool[j] = pool[n - q - 1];
    }
    return true;
}

// Pool branch for k <= 16 from a 32-word window: the accepted word of draw i
// is the first word at or after the previous draw's whose top bits,
// (w >> clz(n - i)), fall below n - i.  Each draw's accept mask over the 32
// words is a few vector shifts and compares, independent of the other draws,
// so the only serial chain left is one tzcnt per draw (the per-word loop of
// pool_fast carries i -> bound -> shift -> compare through every word).
// Returns false, having consumed nothing, when the 32 words run out.
template <class OutT>
inline bool pool_fast_window(MT19937& rng, int64_t n, int64_t k, OutT* out, int32_t* pool) {
    static_assert(MT19937::kExt >= 32, "the window reads 32 words");
    if (k > 16) return false;
    if (rng.index >= MT19937::N) rng.twist();
    if (rng.index + 32 > MT19937::N && !rng.ext) rng.extend();
    const uint32_t nn = static_cast<uint32_t>(n);
    const uint32_t* wp = rng.out + rng.index;
    __m256i w[4];
#pragma GCC unroll 4
    for (int q = 0; q < 4; ++q) w[q] = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(wp) + q);
    uint32_t r[16];
    uint64_t p = 0;  // words consumed so far
    for (int i = 0; i < k; ++i) {
        const uint32_t m = nn - static_cast<uint32_t>(i);
        const int sh = __builtin_clz(m);
        const __m128i shv = _mm_cvtsi32_si128(sh);
        const __m256i mv = _mm256_set1_epi32(static_cast<int32_t>(m));
        uint32_t acc = 0;
#pragma GCC unroll 4
        for (int q = 0; q < 4; ++q)  // w >> sh < m, as signed: both below 2^31 (sh >= 1)
            acc |= static_cast<uint32_t>(_mm256_movemask_ps(_mm256_castsi256_ps(
                       _mm256_cmpgt_epi32(mv, _mm256_srl_epi32(w[q], shv)))))
                   << (8 * q);
        const uint64_t live = static_cast<uint64_t>(acc) & (~uint64_t(0) << p);
        if (!live) return false;
        const int j = __builtin_ctzll(live);
        r[i] = wp[j] >> sh;
        p = static_cast<uint64_t>(j) + 1;
    }
    for (int64_t t = 0; t < n; ++t) pool[t] = static_cast<int32_t>(t);
    for (int64_t q = 0; q < k; ++q) {
        const uint32_t j = r[q];
        out[q] = static_cast<OutT>(pool[j]);
        pool[j] = pool[n - q - 1];
    }
    rng.index += static_cast<int>(p);
    rng.settle();
    return true;
}

// random.sample(population, k) expressed on positions 0..n-1 of the
// population: writes the k chosen positions in result order.  `pool` must
// hold setsize entries.  Requires 0 <= k <= n.
template <class OutT>
inline void sample_positions(MT19937& rng, int64_t n, int64_t k, int64_t setsize, OutT* out,
                             int32_t* pool) {
    if (n <= setsize) {
        if (GS_SELECT_SMALL && k <= 16 && n < (int64_t(1) << 31) && pool_fast_window(rng, n, k, out, pool)) return;
        if (GS_SELECT_SMALL && k <= 32 && pool_fast(rng, n, k, out, pool)) return;
        // pool branch: pool = list(population); j = randbelow(n-i);
        // result[i] = pool[j]; pool[j] = pool[n-i-1]   (positions stand in
        // for the population items).
        for (int64_t t = 0; t < n; ++t) pool[t] = static_cast<int32_t>(t);
        for (int64_t i = 0; i < k; ++i) {
            const int64_t j = rng.randbelow(static_cast<uint64_t>(n - i));
            out[i] = static_cast<OutT>(pool[j]);
            pool[j] = pool[n - i - 1];
        }
    } else if (GS_SELECT_SMALL && k <= 32 && n < (int64_t(1) << 31)) {
        if (k <= 16 && select_fast16(rng, n, k, out)) return;
        select_chunked(rng, n, k, out);
    } else if (n <= (int64_t(1) << 24)) {
        // selected-set branch for larger k (extend_nodes' num_neg = 100 over
        // far lists of ~10^4): the selected values in a thread-local bitmap
        // (cleared through out[] afterwards) instead of a scan of all of them
        // per word — the same words consumed, the same values in order.
        thread_local std::vector<uint64_t> seen;
        const size_t words = static_cast<size_t>((n + 63) >> 6);
        if (seen.size() < words) seen.resize(words, 0);
        const int sh = 32 - (64 - __builtin_clzll(static_cast<uint64_t>(n)));
        int64_t cnt = 0;
        while (cnt < k) {
            const uint32_t r = rng.next() >> sh;
            if (static_cast<int64_t>(r) < n) {
                uint64_t& w = seen[r >> 6];
                const uint64_t bit = uint64_t(1) << (r & 63);
                if (!(w & bit)) {
                    w |= bit;
                    out[cnt++] = static_cast<OutT>(r);
                }
            }
        }
        for (int64_t t = 0; t < k; ++t) seen[static_cast<size_t>(out[t]) >> 6] = 0;
    } else {
        // selected-set branch: j = randbelow(n), redrawn while j in selected.
        // Both a rejected word (r >= n) and a repeat are simply skipped, so
        // the result is the stream's accepted-and-new values in order; the
        // scan below keeps that exact word consumption without a
        // data-dependent branch per word.
        const int sh = 32 - (64 - __builtin_clzll(static_cast<uint64_t>(n)));
        int64_t cnt = 0;
        while (cnt < k) {
            const uint32_t r = rng.next() >> sh;
            bool fresh = static_cast<uint64_t>(r) < static_cast<uint64_t>(n);
            for (int64_t t = 0; t < cnt; ++t) fresh &= static_cast<int64_t>(out[t]) != static_cast<int64_t>(r);
            out[cnt] = static_cast<OutT>(r);  // kept only when fresh
            cnt += fresh;
        }
    }
}

}  // namespace gs
