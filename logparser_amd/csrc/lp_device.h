// Per-line hot path of the logparser reference, written once for the GPU
// (gfx950 kernel in kernels.hip; every function is __host__ __device__ so the
// test-only CPU emulation in tests/ can run the identical source).
//
// One thread owns one line.  Phase 1 matches the LogFormat and runs the
// token / timestamp / first-line stages; phase 2 (after a wave-aggregated
// arena allocation) runs the URI and query-string stages that produce bytes
// that are not substrings of the line.
//
// Any input the device cannot prove it handles exactly returns FALLBACK
// (status 2): the caller hands that line to the reference Java dissector.
#pragma once
#include <cstddef>
#include <type_traits>
#include <utility>

#include "lp_program.h"

namespace lp {

enum : int { ST_OK = 0, ST_BAD = 1, ST_FALLBACK = 2,
             ST_REDO = 3 };  // (kernel-internal, never stored: the line needs the backtracking DFS, which
                             // the one-pass chunk kernel leaves to the queued-line kernel; phase1<..., DFS = false>)

// Profiling build only (-DLP_PROFILE): wave timestamps at fixed points,
// stored per wave (the waves of blocks [PROF_W0, PROF_W0 + PROF_WAVES)),
// no atomics: the host averages the cycles between consecutive points.
#if defined(LP_PROFILE) && defined(__HIP__)
static __device__ unsigned long long g_prof[PROF_WAVES * PROF_POINTS];  // one per kernel translation unit
#endif
#if defined(LP_PROFILE) && defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ void lp_prof_mark(int k) {
    const unsigned long long t = clock64();
    const unsigned w = blockIdx.x - PROF_W0;
    const uint64_t act = __ballot(1);
    if (w < (unsigned)PROF_WAVES && (int)threadIdx.x % 64 == (int)__builtin_ctzll(act))
        __builtin_nontemporal_store(t, &g_prof[w * PROF_POINTS + k]);
}
// accumulating points (inside loops): slot k += cycles since the lane's last LP_PACC
__device__ __forceinline__ void lp_prof_acc(int k, unsigned long long& t0) {
    const unsigned long long t = clock64();
    const unsigned w = blockIdx.x - PROF_W0;
    const uint64_t act = __ballot(1);
    if (w < (unsigned)PROF_WAVES && (int)threadIdx.x % 64 == (int)__builtin_ctzll(act))
        g_prof[w * PROF_POINTS + k] += t - t0;
    t0 = t;
}
#define LP_PROF(k) lp_prof_mark(k)
#define LP_PT_DECL unsigned long long lp_pt = clock64();
#define LP_PACC(k) lp_prof_acc(k, lp_pt)
#else
#define LP_PROF(k)
#define LP_PT_DECL
#define LP_PACC(k)
#endif
// element i of the first-leaf match: its cycles accumulate in slot 64 + i
#if defined(LP_PROFILE) && defined(__HIP_DEVICE_COMPILE__)
#define LP_PROF_EL_BEGIN() unsigned long long lp_el_t = clock64();
#define LP_PROF_EL_END(i) if ((i) < 32) lp_prof_acc(64 + (i), lp_el_t);
#else
#define LP_PROF_EL_BEGIN()
#define LP_PROF_EL_END(i)
#endif

// ----------------------------------------------------------- byte classes
__host__ __device__ LP_INLINE bool is_ws(uint32_t c) { return c == ' ' || (c >= 9 && c <= 13); }      // \s
__host__ __device__ LP_INLINE bool is_digit(uint32_t c) { return c - '0' < 10u; }
__host__ __device__ LP_INLINE bool is_hex(uint32_t c) { return is_digit(c) || ((c | 32u) - 'a') < 6u; }
__host__ __device__ LP_INLINE bool is_alpha(uint32_t c) { return ((c | 32u) - 'a') < 26u; }
__host__ __device__ LP_INLINE bool is_alnum(uint32_t c) { return is_alpha(c) || is_digit(c); }
__host__ __device__ LP_INLINE uint32_t hexv(uint32_t c) { return c <= '9' ? c - '0' : (c | 32u) - 'a' + 10; }
// bytes of the UTF-8 char whose lead byte is c (lines are validated first)
__host__ __device__ LP_INLINE int utf8_len(uint32_t c) { return c < 0x80 ? 1 : c < 0xE0 ? 2 : c < 0xF0 ? 3 : 4; }
// chars commons-httpclient URIUtil.encode escapes with the HttpUriDissector
// "badUriChars" set (HttpUriDissector.java:111-120): control, space, unwise
// {}|\^[]` and <>"  (ASCII only; non-ASCII lines never reach this point)
__host__ __device__ LP_INLINE bool uri_needs_encode(uint32_t c) {
    // bit c of the 128-bit set {0x00-0x20, " < > [ \ ] ^ ` { | } 0x7F}
    constexpr uint64_t LO = 0x5000000500000000ull | 0x1FFFFFFFFull;  // 0x00-0x20, '"' (0x22), '<' (0x3C), '>' (0x3E)
    constexpr uint64_t HI = 0xB800000178000000ull;                   // [ \ ] ^ (0x5B-0x5E), ` (0x60), { | } (0x7B-0x7D), 0x7F
    return c >= 0x80 || (((c < 64 ? LO : HI) >> (c & 63)) & 1u);
}

// -------------------------------------------------------------- matcher
// A line's bytes: b is a 4-byte aligned base (the wave's LDS window in the
// kernel, or the input buffer), the line starts at byte o of it.  Byte reads
// and aligned word reads (for the 4-bytes-at-a-time scanners below) go
// through the same base, so one source serves LDS and HBM.
// aligned 32-bit loads (global/plain pointer, and LDS in the kernel)
__host__ __device__ LP_INLINE uint32_t load_word(const uint8_t* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return *reinterpret_cast<const uint32_t*>(__builtin_assume_aligned(p, 4));
#else
    uint32_t v;
    __builtin_memcpy(&v, p, 4);
    return v;
#endif
}
#if defined(__HIP__)
typedef const __attribute__((address_space(3))) uint8_t* lds_bytes;
typedef const __attribute__((address_space(3))) uint32_t* lds_words;
__device__ LP_INLINE uint32_t load_word(lds_bytes p) { return *(lds_words)p; }
#endif
#if defined(__HIP_DEVICE_COMPILE__) && defined(LP_KERNEL_TU)
__device__ LP_INLINE uint32_t load_word(const LP_G uint8_t* p) {
    return *reinterpret_cast<const LP_G uint32_t*>(__builtin_assume_aligned(p, 4));
}
#endif

// ---- byte-class bitmasks (1 bit per byte, one 64-bit word per 64 bytes),
// built once per LDS window by the staging pass of a kernel, so the per-line
// scanners walk 64 bytes per step instead of 4.  The parse kernels' windows
// carry two planes (NPL = 2): P0 = QUOTE ('"'), P1 = WS (the bytes <= 0x20:
// exactly ' ' and TAB inside a line the guard passes, whose other control
// bytes send it to FALLBACK before any scanner runs); the planes of 64-byte
// block w are the 16 bytes at 16 w (one 128-bit LDS read).  The URI kernel's
// compact buffer carries the one UEV plane (NPL = 1).  Phase 1 never asks
// for UEV, the URI stages never for QUOTE / WS.
enum : int {
    MC_QUOTE = 0,  // '"'
    MC_UEV = 1,    // URI events: % # & ? ; + and the bytes URIUtil.encode escapes (not '=', not A-Z)
    MC_WS = 2,     // \s of a line that passed the guard: ' ' and TAB
    MC_N = 2       // bit planes
};
__host__ __device__ LP_INLINE uint64_t mask_load(const uint64_t* p) { return *p; }
#if defined(__HIP__)
typedef const __attribute__((address_space(3))) uint64_t* lds_u64;
__device__ LP_INLINE uint64_t mask_load(lds_u64 p) { return *p; }
#endif
struct NoMasks {};

// NPL = 2: the two planes of the parse kernel's window (QUOTE, WS, UEV);
// NPL = 1: one UEV plane only (the URI kernel's compact buffer: only the URI
// scanners run on it, and they only ask for MC_UEV)
template <typename Ptr, typename MPtr = NoMasks, int NPL = 2>
struct LineT {
    Ptr b;
    uint32_t o;
    int n;
    MPtr m = MPtr{};       // planes of the 64-byte block w of b: m[NPL w .. NPL w + NPL)
    static constexpr bool has_masks = !std::is_same<MPtr, NoMasks>::value;
    static constexpr bool in_arena = false;  // positions are line offsets
    __host__ __device__ LP_INLINE uint32_t operator[](int i) const { return b[o + i]; }
    // aligned 32-bit word w of the base (little-endian: byte k at bits 8k..8k+7)
    __host__ __device__ LP_INLINE uint32_t word(uint32_t w) const { return load_word(b + 4 * w); }
    // word w if it still holds bytes of the line, else 0 (look-ahead reads
    // never leave the line's words)
    __host__ __device__ LP_INLINE uint32_t word_or0(uint32_t w) const {
        return 4 * w < o + (uint32_t)n ? load_word(b + 4 * w) : 0u;
    }
    __host__ __device__ LP_INLINE uint64_t mask(int c, uint32_t w) const {
        if constexpr (NPL == 1) {
            return mask_load(m + w);  // c == MC_UEV (the only class of a one-plane line)
        } else {
            return mask_load(m + 2 * w + (c == MC_QUOTE ? 0 : 1));  // QUOTE / WS (no UEV plane, see above)
        }
    }
};
using Line = LineT<const uint8_t*>;
using MLine = LineT<const uint8_t*, const uint64_t*>;
using ULine = LineT<const uint8_t*, const uint64_t*, 1>;

// A URI source held in the line's arena region (a decoded query value that a
// type remapping dissects again): position q is region byte rb + q, and the
// refs made from positions are region refs.
template <typename Ptr>
struct ArenaLineT : LineT<Ptr> {
    uint32_t rb;
    static constexpr bool in_arena = true;
};

// the ref of [x, x + n) of the source viewed by L
template <typename LN>
__host__ __device__ LP_INLINE uint64_t src_ref(const LN& L, int x, int n) {
    if constexpr (LN::in_arena) return mkref(L.rb + (uint32_t)x, (uint32_t)n, true);
    else return mkref((uint32_t)x, (uint32_t)n, false);
}

// ---- SWAR byte classes on a 32-bit word: bit 8k+7 set when byte k is in
// the class (exact, no false positives from carries).
namespace swar {
constexpr uint32_t ONES = 0x01010101u, HI = 0x80808080u, LO7 = 0x7F7F7F7Fu;
__host__ __device__ LP_INLINE uint32_t eq(uint32_t w, uint32_t c) {
    const uint32_t x = w ^ (c * ONES);
    return ~(((x & LO7) + LO7) | x | LO7);
}
// bytes >= n / < n (1 <= n <= 0x80; bytes >= 0x80 count as >= n)
__host__ __device__ LP_INLINE uint32_t ge(uint32_t w, uint32_t n) { return (((w & LO7) + (0x80u - n) * ONES) | w) & HI; }
__host__ __device__ LP_INLINE uint32_t lt(uint32_t w, uint32_t n) { return ~ge(w, n) & HI; }
__host__ __device__ LP_INLINE uint32_t ws(uint32_t w) { return eq(w, ' ') | (ge(w, 9) & lt(w, 14)); }  // \s
__host__ __device__ LP_INLINE uint32_t digit(uint32_t w) { return ge(w, '0') & lt(w, '9' + 1); }
__host__ __device__ LP_INLINE uint32_t hex(uint32_t w) {
    const uint32_t l = w | 0x20202020u;
    return digit(w) | (ge(l, 'a') & lt(l, 'g') & ~(w & HI));
}
__host__ __device__ LP_INLINE uint32_t upper(uint32_t w) { return ge(w, 'A') & lt(w, 'Z' + 1); }
// not printable ASCII and not TAB: the fast-path guard
__host__ __device__ LP_INLINE uint32_t guard_bad(uint32_t w) { return (lt(w, 0x20) & ~eq(w, '\t')) | ge(w, 0x7F); }
// controls other than TAB, and DEL: never on the fast path (bytes >= 0x80
// are, in valid UTF-8 outside the URI stages)
__host__ __device__ LP_INLINE uint32_t guard_ctl(uint32_t w) { return (lt(w, 0x20) & ~eq(w, '\t')) | eq(w, 0x7F); }
// URIUtil "badUriChars" (see uri_needs_encode below), ASCII part
__host__ __device__ LP_INLINE uint32_t needs_encode(uint32_t w) {
    return lt(w, 0x21) | ge(w, 0x7F) | (ge(w, '{') & lt(w, '~')) | (ge(w, '[') & lt(w, '_')) | eq(w, '`') |
           eq(w, '<') | eq(w, '>') | eq(w, '"');
}
__host__ __device__ LP_INLINE int first(uint32_t m) {
#if defined(__HIP_DEVICE_COMPILE__)
    return (int)(__builtin_ctz(m) >> 3);
#else
    return (int)(__builtin_ctz(m) >> 3);
#endif
}
__host__ __device__ LP_INLINE int last(uint32_t m) { return (int)((31 - __builtin_clz(m)) >> 3); }
__host__ __device__ LP_INLINE int count(uint32_t m) { return __builtin_popcount(m); }
}  // namespace swar

// ---- byte classes through two nibble look-up tables (the SIMD "shuffle"
// classifier): class bits(b) = LO[b & 15] & HI[b >> 4], one v_perm_b32 per
// 8-entry table half.  Bits (rectangles hi-nibble set x lo-nibble set):
// 0 hi 2 x lo 0 (' '), 1 hi 0 x lo {9,A,D} (TAB, LF, CR), 2 hi 2 x lo 2 ('"'),
// 3 hi 2 x lo {3,5,6,B} (# % & +), 4 hi 3 x lo {B,C,E,F} (; < > ?),
// 5 hi {5,7} x lo {B,C,D} ([ \ ] { | }), 6 hi 5 x lo E (^), 7 hi 6 x lo 0 (`).
// QUOTE = bit 2, UEV = any bit: the URI event bytes % # & ? ; + and every
// byte URIUtil.encode escapes (upper-case letters are not events: the query
// stage finds a name's upper-case bytes itself, query_piece).  LF and CR
// share TAB's class (\s); inside a line they never occur (they end it), so
// they only matter to the staging guard, which reads class bit 1 as "a
// control byte the guard allows" (guard16).

namespace bcls {
constexpr uint32_t LO0 = 0x08040081u, LO1 = 0x00080800u;  // LO[0..3], LO[4..7]
constexpr uint32_t LO2 = 0x38020200u, LO3 = 0x10502230u;  // LO[8..11], LO[12..15]
constexpr uint32_t HI0 = 0x100D0002u, HI1 = 0x20806000u;  // HI[0..3], HI[4..7]
// v_perm_b32: byte i of the result = byte sel_i (0..7) of (s0:s1), s1 low
__host__ __device__ LP_INLINE uint32_t perm(uint32_t s0, uint32_t s1, uint32_t sel) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_perm(s0, s1, sel);
#else
    const uint64_t v = ((uint64_t)s0 << 32) | s1;
    uint32_t r = 0;
    for (int i = 0; i < 4; ++i) r |= (uint32_t)((v >> (8 * ((sel >> (8 * i)) & 7))) & 0xFFu) << (8 * i);
    return r;
#endif
}
// class bits of the 4 bytes of w; bytes >= 0x80 (UTF-8) get bit 3 only: a
// URI event (URIUtil leaves them raw, the URI stage sends them to FALLBACK),
// neither '"' nor \s
__host__ __device__ LP_INLINE uint32_t bits(uint32_t w) {
    const uint32_t s = w & 0x07070707u;
    const uint32_t p1 = perm(LO1, LO0, s), p2 = perm(LO3, LO2, s);
    const uint32_t m8 = ((w >> 3) & 0x01010101u) * 0xFFu;
    const uint32_t rl = (p2 & m8) | (p1 & ~m8);
    const uint32_t hb = ((w >> 7) & 0x01010101u) * 0xFFu;
    return (rl & perm(HI1, HI0, (w >> 4) & 0x07070707u) & ~hb) | (hb & 0x08080808u);
}
// java.net.URI authority bytes: a second table pair whose class is the
// bytes outside L_SERVER and L_REG_NAME (controls, space, " # % & / < > ? @
// [ \ ] ^ ` { | } DEL; rectangles hi x lo of the nibbles, one bit each)
constexpr uint32_t NA_LO0 = 0x0303010Bu, NA_LO1 = 0x01030301u, NA_LO2 = 0x11010101u, NA_LO3 = 0x47251115u;
constexpr uint32_t NA_HI0 = 0x04020101u, NA_HI1 = 0x50083008u;
__host__ __device__ LP_INLINE uint32_t nonauth_bits(uint32_t w) {
    const uint32_t s = w & 0x07070707u;
    const uint32_t p1 = perm(NA_LO1, NA_LO0, s), p2 = perm(NA_LO3, NA_LO2, s);
    const uint32_t m8 = ((w >> 3) & 0x01010101u) * 0xFFu;
    return ((p2 & m8) | (p1 & ~m8)) & perm(NA_HI1, NA_HI0, (w >> 4) & 0x07070707u);
}
// bytes with bit 7 set -> 4-bit mask (byte k -> bit k)
__host__ __device__ LP_INLINE uint32_t nib(uint32_t hb) { return (((hb >> 7) * 0x204081u) >> 21) & 15u; }
__host__ __device__ LP_INLINE uint32_t uev_hb(uint32_t r) { return (((r & swar::LO7) + swar::LO7) | r) & swar::HI; }
// 16 bytes (4 little-endian words) -> the 16-bit UEV mask (the URI kernel's one plane)
__host__ __device__ LP_INLINE uint32_t pack16(uint32_t h0, uint32_t h1, uint32_t h2, uint32_t h3);
__host__ __device__ LP_INLINE uint32_t classify16u(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
    return pack16(uev_hb(bits(w0)), uev_hb(bits(w1)), uev_hb(bits(w2)), uev_hb(bits(w3)));
}
// The parse kernels' staging classifier (SWAR on the 4 little-endian words
// of 16 bytes): p0 = QUOTE, p1 = WS (bytes <= 0x20) as 16-bit masks, lf /
// other = the '\n' bytes / the control bytes other than '\n' (TAB, '\r',
// ...: rare; the caller resolves them), bad |= the bytes >= 0x7F.  The
// high-bit-per-byte masks are packed with v_dot4_u32_u8 (bytes 0x80 or 0
// times the bit weights 1, 2, 4, 8): two per 8 mask bits.
__host__ __device__ LP_INLINE uint32_t pack16(uint32_t h0, uint32_t h1, uint32_t h2, uint32_t h3) {
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t lo = __builtin_amdgcn_udot4(h1, 0x80402010u, __builtin_amdgcn_udot4(h0, 0x08040201u, 0u, false), false);
    const uint32_t hi = __builtin_amdgcn_udot4(h3, 0x80402010u, __builtin_amdgcn_udot4(h2, 0x08040201u, 0u, false), false);
    return (lo >> 7) | (hi << 1);  // lo, hi = 0x80 x (8-bit mask)
#else
    return nib(h0) | (nib(h1) << 4) | (nib(h2) << 8) | (nib(h3) << 12);
#endif
}
__host__ __device__ LP_INLINE void classify16p(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t& p0,
                                               uint32_t& p1, uint32_t& bad, uint32_t& lf, uint32_t& other) {
    const uint32_t w[4] = {w0, w1, w2, w3};
    uint32_t q[4], le[4], l[4], o = 0, hi = 0;
    LP_UNROLL for (int k = 0; k < 4; ++k) {
        const uint32_t lo7 = w[k] & swar::LO7;
        le[k] = ~((lo7 + 0x5F5F5F5Fu) | w[k]) & swar::HI;         // bytes <= 0x20
        const uint32_t lt = ~((lo7 + 0x60606060u) | w[k]) & swar::HI;  // bytes < 0x20
        hi |= ((lo7 + 0x01010101u) | w[k]) & swar::HI;             // bytes >= 0x7F
        q[k] = swar::eq(w[k], '"');
        l[k] = swar::eq(w[k], '\n');
        o |= lt & ~l[k];
    }
    p0 = pack16(q[0], q[1], q[2], q[3]);
    p1 = pack16(le[0], le[1], le[2], le[3]);
    lf = pack16(l[0], l[1], l[2], l[3]);
    bad |= hi;
    other = o;
}
// the guard of 16 bytes holding control bytes other than '\n' (classify16p's
// `other`): the controls other than TAB / LF / CR, and the '\r' mask
__host__ __device__ LP_INLINE void classify16c(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t& bad,
                                               uint32_t& cr) {
    const uint32_t w[4] = {w0, w1, w2, w3};
    uint32_t c[4];
    LP_UNROLL for (int k = 0; k < 4; ++k) {
        const uint32_t lt = ~(((w[k] & swar::LO7) + 0x60606060u) | w[k]) & swar::HI;
        c[k] = swar::eq(w[k], '\r');
        bad |= lt & ~(c[k] | swar::eq(w[k], '\n') | swar::eq(w[k], '\t'));
    }
    cr = pack16(c[0], c[1], c[2], c[3]);
}
// mask class whose members are exactly the byte c, -1 none
__host__ __device__ LP_INLINE int class_of(uint32_t c) { return c == '"' ? (int)MC_QUOTE : -1; }
}  // namespace bcls

// Host builder of the class masks of buf[0, n) (n a multiple of 64), the same
// computation the kernel's staging pass does; used by the test-only CPU
// emulation.  masks: 2 x n / 64 words (the planes of each 64-byte block).
inline void build_masks(const uint8_t* buf, uint32_t n, uint64_t* masks) {
    for (uint32_t i = 0; i < MC_N * (n / 64); ++i) masks[i] = 0;
    for (uint32_t k = 0; 16 * k < n; ++k) {
        uint32_t w[4];
        for (int j = 0; j < 4; ++j) __builtin_memcpy(&w[j], buf + 16 * k + 4 * j, 4);
        uint32_t a, b, bad = 0, lf, other;
        bcls::classify16p(w[0], w[1], w[2], w[3], a, b, bad, lf, other);
        const int sh = 16 * (k & 3);
        masks[2 * (k >> 2)] |= (uint64_t)a << sh;
        masks[2 * (k >> 2) + 1] |= (uint64_t)b << sh;
    }
}

// The UEV plane alone (the URI kernel's compact buffer): 1 x n / 64 words.
inline void build_uev_plane(const uint8_t* buf, uint32_t n, uint64_t* plane) {
    for (uint32_t i = 0; i < n / 64; ++i) plane[i] = 0;
    for (uint32_t k = 0; 16 * k < n; ++k) {
        uint32_t w[4];
        for (int j = 0; j < 4; ++j) __builtin_memcpy(&w[j], buf + 16 * k + 4 * j, 4);
        plane[k >> 2] |= (uint64_t)bcls::classify16u(w[0], w[1], w[2], w[3]) << (16 * (k & 3));
    }
}

__host__ __device__ LP_INLINE int ctz64(uint64_t m) { return __builtin_ctzll(m); }
__host__ __device__ LP_INLINE int msb64(uint64_t m) { return 63 - __builtin_clzll(m); }
__host__ __device__ LP_INLINE int popc64(uint64_t m) { return __builtin_popcountll(m); }

// First position in [from, to) whose byte is in class F, else `to`.
template <typename LN, typename F>
__host__ __device__ LP_INLINE int find_fwd(const LN& L, int from, int to, F cls) {
    if (from >= to) return to;
    const uint32_t A = L.o + (uint32_t)from, E = L.o + (uint32_t)to;
    uint32_t W = A >> 2;
    uint32_t m = cls(L.word(W)) & (swar::HI << (8 * (A & 3)));
    for (;;) {
        if (m) {
            const uint32_t p = (W << 2) + (uint32_t)swar::first(m);
            return p < E ? (int)(p - L.o) : to;
        }
        ++W;
        if ((W << 2) >= E) return to;
        m = cls(L.word(W));
    }
}
// Last position in [lo, hi] whose byte is in class F, else -1.
template <typename LN, typename F>
__host__ __device__ LP_INLINE int find_bwd(const LN& L, int hi, int lo, F cls) {
    if (hi < lo) return -1;
    const uint32_t A = L.o + (uint32_t)hi, S = L.o + (uint32_t)lo;
    uint32_t W = A >> 2;
    uint32_t m = cls(L.word(W)) & (swar::HI >> (8 * (3 - (A & 3))));
    for (;;) {
        if (m) {
            const uint32_t p = (W << 2) + (uint32_t)swar::last(m);
            return p >= S ? (int)(p - L.o) : -1;
        }
        if ((W << 2) <= S) return -1;
        --W;
        m = cls(L.word(W));
    }
}
// Number of bytes in [a, b) in class F.
template <typename LN, typename F>
__host__ __device__ LP_INLINE uint32_t count_in(const LN& L, int a, int b, F cls) {
    if (a >= b) return 0;
    const uint32_t A = L.o + (uint32_t)a, E = L.o + (uint32_t)b;
    const uint32_t W0 = A >> 2, W1 = (E - 1) >> 2;
    uint32_t c = 0;
    for (uint32_t W = W0; W <= W1; ++W) {
        uint32_t m = cls(L.word(W));
        if (W == W0) m &= swar::HI << (8 * (A & 3));
        if (W == W1) m &= swar::HI >> (8 * (3 - ((E - 1) & 3)));
        c += (uint32_t)swar::count(m);
    }
    return c;
}

// ---- scanners over the class masks (lines staged with masks)
// First position in [from, to) in mask class c, else `to`.
template <typename LN>
__host__ __device__ LP_INLINE int mfind_fwd(const LN& L, int c, int from, int to) {
    if (from >= to) return to;
    const uint32_t A = L.o + (uint32_t)from, E = L.o + (uint32_t)to;
    uint32_t W = A >> 6;
    uint64_t m = L.mask(c, W) & (~0ull << (A & 63));
    for (;;) {
        if (m) {
            const uint32_t p = (W << 6) + (uint32_t)ctz64(m);
            return p < E ? (int)(p - L.o) : to;
        }
        ++W;
        if ((W << 6) >= E) return to;
        m = L.mask(c, W);
    }
}
// Last position in [lo, hi] in mask class c, else -1.
template <typename LN>
__host__ __device__ LP_INLINE int mfind_bwd(const LN& L, int c, int hi, int lo) {
    if (hi < lo) return -1;
    const uint32_t A = L.o + (uint32_t)hi, S = L.o + (uint32_t)lo;
    uint32_t W = A >> 6;
    uint64_t m = L.mask(c, W) & (~0ull >> (63 - (A & 63)));
    for (;;) {
        if (m) {
            const uint32_t p = (W << 6) + (uint32_t)msb64(m);
            return p >= S ? (int)(p - L.o) : -1;
        }
        if ((W << 6) <= S) return -1;
        --W;
        m = L.mask(c, W);
    }
}

// Calls f(q, c) for every position q in [a, b) whose byte c is a URI event
// byte (MC_UEV: % # & ? ; + and the URIUtil-escaped bytes), in order,
// until f returns false.  Returns false when f stopped the walk.  Lines with
// masks walk 64 bytes per step and read the next event's byte before f runs
// on the current one (its LDS latency overlaps f); others classify 4 bytes
// per step with the same nibble tables.
template <typename LN, typename F>
__host__ __device__ LP_INLINE bool for_uev(const LN& L, int a, int b, F&& f) {
    if (a >= b) return true;
    const uint32_t A = L.o + (uint32_t)a, E = L.o + (uint32_t)b;
    if constexpr (LN::has_masks) {
        const uint32_t W1 = (E - 1) >> 6;
        const uint64_t last = ~0ull >> (63 - ((E - 1) & 63));
        uint32_t W = A >> 6;
        uint64_t m = L.mask(MC_UEV, W) & (~0ull << (A & 63));
        if (W == W1) m &= last;
        auto next = [&](int& q) {
            while (!m) {
                if (++W > W1) return false;
                m = L.mask(MC_UEV, W);
                if (W == W1) m &= last;
            }
            q = (int)((W << 6) + (uint32_t)ctz64(m) - L.o);
            m &= m - 1;
            return true;
        };
        int q;
        if (!next(q)) return true;
        uint32_t c = L[q];
        for (;;) {
            int q2 = 0;
            const bool more = next(q2);
            const uint32_t c2 = more ? L[q2] : 0u;
            if (!f(q, c)) return false;
            if (!more) return true;
            q = q2;
            c = c2;
        }
    } else {
        const uint32_t W0 = A >> 2, W1 = (E - 1) >> 2;
        for (uint32_t W = W0; W <= W1; ++W) {
            const uint32_t w = L.word(W);
            uint32_t m = bcls::uev_hb(bcls::bits(w));
            if (W == W0) m &= swar::HI << (8 * (A & 3));
            if (W == W1) m &= swar::HI >> (8 * (3 - ((E - 1) & 3)));
            while (m) {
                const int k = swar::first(m);
                m &= m - 1;
                if (!f((int)((W << 2) + (uint32_t)k - L.o), (w >> (8 * k)) & 0xFFu)) return false;
            }
        }
    }
    return true;
}

// for_uev with the event's byte and the two after it: f(q, w), w = the 4
// bytes at q (little-endian, bytes past the line's last word read as 0).
template <typename LN, typename F>
__host__ __device__ LP_INLINE bool for_uev_w(const LN& L, int a, int b, F&& f) {
    if (a >= b) return true;
    const uint32_t A = L.o + (uint32_t)a, E = L.o + (uint32_t)b;
    if constexpr (LN::has_masks) {
        const uint32_t W1 = (E - 1) >> 6;
        const uint64_t last = ~0ull >> (63 - ((E - 1) & 63));
        uint32_t W = A >> 6;
        uint64_t m = L.mask(MC_UEV, W) & (~0ull << (A & 63));
        if (W == W1) m &= last;
        auto next = [&](int& q) {
            while (!m) {
                if (++W > W1) return false;
                m = L.mask(MC_UEV, W);
                if (W == W1) m &= last;
            }
            q = (int)((W << 6) + (uint32_t)ctz64(m) - L.o);
            m &= m - 1;
            return true;
        };
        int q;
        if (!next(q)) return true;
        uint32_t w = load_u32_at(L, q);
        for (;;) {
            int q2 = 0;
            const bool more = next(q2);
            const uint32_t w2 = more ? load_u32_at(L, q2) : 0u;
            if (!f(q, w)) return false;
            if (!more) return true;
            q = q2;
            w = w2;
        }
    } else {
        return for_uev(L, a, b, [&](int q, uint32_t) { return f(q, load_u32_at(L, q)); });
    }
}

// Number of URI event bytes in [a, b).
template <typename LN>
__host__ __device__ LP_INLINE uint32_t count_uev(const LN& L, int a, int b) {
    if (a >= b) return 0;
    const uint32_t A = L.o + (uint32_t)a, E = L.o + (uint32_t)b;
    uint32_t c = 0;
    if constexpr (LN::has_masks) {
        const uint32_t W0 = A >> 6, W1 = (E - 1) >> 6;
        for (uint32_t W = W0; W <= W1; ++W) {
            uint64_t m = L.mask(MC_UEV, W);
            if (W == W0) m &= ~0ull << (A & 63);
            if (W == W1) m &= ~0ull >> (63 - ((E - 1) & 63));
            c += (uint32_t)popc64(m);
        }
    } else {
        const uint32_t W0 = A >> 2, W1 = (E - 1) >> 2;
        for (uint32_t W = W0; W <= W1; ++W) {
            uint32_t m = bcls::uev_hb(bcls::bits(L.word(W)));
            if (W == W0) m &= swar::HI << (8 * (A & 3));
            if (W == W1) m &= swar::HI >> (8 * (3 - ((E - 1) & 3)));
            c += (uint32_t)swar::count(m);
        }
    }
    return c;
}

// First \s in [from, to), else `to` (lines with masks: the WS class).
template <typename LN>
__host__ __device__ LP_INLINE int find_ws(const LN& L, int from, int to) {
    if constexpr (LN::has_masks) return mfind_fwd(L, MC_WS, from, to);
    else return find_fwd(L, from, to, [](uint32_t w) { return swar::ws(w); });
}

// The 4 bytes at line position p as one little-endian word (bytes past the
// line's last word read as 0).
template <typename LN>
__host__ __device__ LP_INLINE uint32_t load_u32_at(const LN& L, int p) {
    const uint32_t A = L.o + (uint32_t)p;
    const uint32_t w0 = L.word(A >> 2), w1 = L.word_or0((A >> 2) + 1);
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbyte(w1, w0, A & 3);
#else
    return (uint32_t)((((uint64_t)w1 << 32) | w0) >> (8 * (A & 3)));
#endif
}

// 28 bytes from line position p (p + 26 <= n) in 7 little-endian words.
struct Bytes28 {
    uint32_t v[7];
    __host__ __device__ LP_INLINE uint32_t operator[](int k) const { return (v[k >> 2] >> (8 * (k & 3))) & 0xFFu; }
};
template <typename LN>
__host__ __device__ LP_INLINE Bytes28 load28(const LN& L, int p) {
    const uint32_t A = L.o + (uint32_t)p, W = A >> 2, s = A & 3;
    uint32_t w[8];
    LP_UNROLL for (int j = 0; j < 7; ++j) w[j] = L.word(W + j);
    w[7] = L.word_or0(W + 7);
    Bytes28 r;
    LP_UNROLL for (int j = 0; j < 7; ++j) {
#if defined(__HIP_DEVICE_COMPILE__)
        r.v[j] = __builtin_amdgcn_alignbyte(w[j + 1], w[j], s);
#else
        r.v[j] = (uint32_t)((((uint64_t)w[j + 1] << 32) | w[j]) >> (8 * s));
#endif
    }
    return r;
}

// Small per-line array kept in registers: every element access in the source
// uses a compile-time index (fold expressions), and a data-dependent index is
// a compare-and-select chain, so the array is promoted to registers before
// any pass could turn it into a dynamically indexed scratch-memory array.
template <int N>
struct RegArr {
    static constexpr int size = N;
#if defined(__HIP_DEVICE_COMPILE__)
    // a vector value: an element write with a wave-uniform index is one
    // VGPR-indexed move (s_set_gpr_idx), not a branch or a select chain
    typedef uint32_t vec_t __attribute__((ext_vector_type(N)));
    vec_t v;
#else
    uint32_t v[N];
#endif
    template <size_t... J>
    __host__ __device__ LP_INLINE uint32_t get_(int k, std::index_sequence<J...>) const {
        uint32_t r = 0;
        ((r = ((int)J == k) ? v[J] : r), ...);
        return r;
    }
    template <size_t... J>
    __host__ __device__ LP_INLINE void set_(int k, uint32_t x, std::index_sequence<J...>) {
        ((v[J] = ((int)J == k) ? x : v[J]), ...);
    }
    template <typename F, size_t... J>
    __host__ __device__ LP_INLINE void each_(F&& f, std::index_sequence<J...>) const {
        (f((int)J, v[J]), ...);
    }
    __host__ __device__ LP_INLINE uint32_t get(int k) const { return get_(k, std::make_index_sequence<N>{}); }
    // get with a wave-uniform index 0 <= k < N: one indexed register read
    __host__ __device__ LP_INLINE uint32_t get_u(int k) const { return v[k]; }
    // set with a wave-uniform index: one indexed register write on the device
    // (the select chain of set() rewrites every element).  A lane-varying k
    // is still correct but compiles to a waterfall loop: index by a lane's own
    // stage (e.g. the SLOT URI instances' u) with set() / get()
    __host__ __device__ LP_INLINE void set_u(int k, uint32_t x) {
        if ((unsigned)k < (unsigned)N) v[k] = x;
    }
    __host__ __device__ LP_INLINE void set(int k, uint32_t x) { set_(k, x, std::make_index_sequence<N>{}); }
    __host__ __device__ LP_INLINE void fill(uint32_t x) { set_all(x, std::make_index_sequence<N>{}); }
    template <size_t... J>
    __host__ __device__ LP_INLINE void set_all(uint32_t x, std::index_sequence<J...>) { ((v[J] = x), ...); }
    // f(index, value) for every element, in index order
    template <typename F>
    __host__ __device__ LP_INLINE void each(F&& f) const { each_(f, std::make_index_sequence<N>{}); }
};

// Literal of element e (its own for EK_LIT, the following one for tokens)
// at pos.  Literals of up to 4 bytes compare against e.lit4 (no Program
// memory reads inside the scanners).
template <typename LN>
__host__ __device__ LP_INLINE bool lit_at(const Program& P, const LN& L, int pos, const ElemV& e) {
    const int len = e.lit_len;
    if (pos + len > L.n) return false;
    if (len <= 4) {
        const uint32_t keep = len == 4 ? 0xFFFFFFFFu : ((1u << (8 * len)) - 1u);
        return ((load_u32_at(L, pos) ^ e.lit4) & keep) == 0;
    }
    for (int k = 0; k < len; ++k)
        if (L[pos + k] != P.lit_byte(e.lit_off + k)) return false;
    return true;
}

template <typename LN>
__host__ __device__ LP_INLINE bool time_us_ok(const LN& L, int p) {
    if (p + 26 > L.n) return false;
    const Bytes28 c = load28(L, p);
    if (!(c[0] >= '0' && c[0] <= '3') || !is_digit(c[1]) || c[2] != '/') return false;
    if (!is_alpha(c[3]) || !is_alpha(c[4]) || !is_alpha(c[5]) || c[6] != '/') return false;
    if (!(c[7] >= '1' && c[7] <= '9') || !is_digit(c[8]) || !is_digit(c[9]) || !is_digit(c[10]) || c[11] != ':') return false;
    if (!is_digit(c[12]) || !is_digit(c[13]) || c[14] != ':' || !is_digit(c[15]) || !is_digit(c[16]) || c[17] != ':') return false;
    if (!is_digit(c[18]) || !is_digit(c[19]) || c[20] != ' ') return false;
    if (!(c[21] == '+' || c[21] == '|' || c[21] == '-')) return false;   // [\+|\-]
    return is_digit(c[22]) && is_digit(c[23]) && is_digit(c[24]) && is_digit(c[25]);
}

// The highest-priority IPv4 alternative of FORMAT_IPV4
// (TokenParser.java:43-46) when every octet is taken whole: returns end or -1.
template <typename LN>
__host__ __device__ LP_INLINE int ipv4_first(const LN& L, int p) {
    int q = p;
    for (int o = 0; o < 4; ++o) {
        int a = q;
        while (q < L.n && q - a < 4 && is_digit(L[q])) ++q;
        int nd = q - a;
        if (nd < 1 || nd > 3) return -1;
        if (nd == 3) {
            uint32_t d1 = L[a], v = (L[a] - '0') * 100 + (L[a + 1] - '0') * 10 + (L[a + 2] - '0');
            // 25[0-5] | 2[0-4][0-9] | [01][0-9][0-9] take three digits
            if (!(d1 == '0' || d1 == '1' || (v >= 200 && v <= 255))) return -1;
        }
        if (q < L.n && is_digit(L[q])) return -1;
        if (o < 3) {
            if (q >= L.n || L[q] != '.') return -1;
            ++q;
        }
    }
    return q;
}

// Position of the k-th byte c (k >= 1) counted from the end of the line
// within [lo, n), or -1.
template <typename LN>
__host__ __device__ LP_INLINE int kth_from_end(const LN& L, uint32_t c, int k, int lo) {
    if constexpr (LN::has_masks) {
        if (c == '"') {  // exact class: count set bits of the QUOTE mask backwards
            if (L.n - 1 < lo) return -1;
            const uint32_t A = L.o + (uint32_t)L.n - 1, S = L.o + (uint32_t)lo;
            uint32_t W = A >> 6;
            uint64_t m = L.mask(MC_QUOTE, W) & (~0ull >> (63 - (A & 63)));
            for (;;) {
                if (W == (S >> 6)) m &= ~0ull << (S & 63);
                const int pc = popc64(m);
                if (pc >= k) {
                    for (int j = 1; j < k; ++j) m ^= 1ull << msb64(m);
                    return (int)((W << 6) + (uint32_t)msb64(m) - L.o);
                }
                k -= pc;
                if ((W << 6) <= S) return -1;
                --W;
                m = L.mask(MC_QUOTE, W);
            }
        }
    }
    int q = L.n - 1;
    for (;;) {
        q = find_bwd(L, q, lo, [c](uint32_t w) { return swar::eq(w, c); });
        if (q < 0 || --k == 0) return q;
        --q;
    }
}

// Candidate starts of e's following literal: positions of its first byte,
// through the mask class holding that byte (e.acls) when the line has masks.
template <typename LN>
__host__ __device__ LP_INLINE int anchor_bwd(const LN& L, const ElemV& e, int hi, int lo) {
    const uint32_t c0 = e.lit4 & 0xFFu;
    if constexpr (LN::has_masks) {
        if (e.acls >= 0) {
            return mfind_bwd(L, e.acls, hi, lo);  // exact class
        }
    }
    return find_bwd(L, hi, lo, [c0](uint32_t w) { return swar::eq(w, c0); });
}
template <typename LN>
__host__ __device__ LP_INLINE int anchor_fwd(const LN& L, const ElemV& e, int lo, int to) {
    const uint32_t c0 = e.lit4 & 0xFFu;
    if constexpr (LN::has_masks) {
        if (e.acls >= 0) {
            return mfind_fwd(L, e.acls, lo, to);  // exact class
        }
    }
    return find_fwd(L, lo, to, [c0](uint32_t w) { return swar::eq(w, c0); });
}

// Occurrence of e's following literal: the last one starting in [lo, hi]
// (greedy order) or the first one starting in [lo, hi] (lazy order); -1 none.
template <typename LN>
__host__ __device__ LP_INLINE int lit_last(const Program& P, const LN& L, const ElemV& e, int hi, int lo) {
    for (int q = hi;;) {
        q = anchor_bwd(L, e, q, lo);
        if (q < 0) return -1;
        if (lit_at(P, L, q, e)) return q;
        --q;
    }
}
template <typename LN>
__host__ __device__ LP_INLINE int lit_first(const Program& P, const LN& L, const ElemV& e, int lo, int hi) {
    for (int q = lo;;) {
        q = anchor_fwd(L, e, q, hi + 1);
        if (q > hi) return -1;
        if (lit_at(P, L, q, e)) return q;
        ++q;
    }
}

// lit_last out of line, for the candidate enumerators of elements that only
// some programs have (a literal-aware [^\s]* / NGINX "$request"): inlined,
// its code reshapes the register allocation of every program's kernel
template <typename LN>
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __noinline__
#else
inline
#endif
int lit_last_call(const Program& P, const LN& L, const ElemV& e, int hi, int lo) {
    return lit_last(P, L, e, hi, lo);
}

// End of the digit run starting at p (p if none).
template <typename LN>
__host__ __device__ LP_INLINE int digits_end(const LN& L, int p) {
    return find_fwd(L, p, L.n, [](uint32_t w) { return ~swar::digit(w) & swar::HI; });
}

// [0-9]+\.[0-9]+ at p: end (the fraction greedy, maximal), -1 none, -2 when
// a run is longer than 18 digits (Long.parseLong of the SECOND_MILLIS
// converters could overflow: a runtime exception of the reference).
template <typename LN>
__host__ __device__ LP_INLINE int decimal_at(const LN& L, int p) {
    const int d = digits_end(L, p);
    if (d == p || d >= L.n || L[d] != '.') return -1;
    const int r = digits_end(L, d + 1);
    if (r == d + 1) return -1;
    if (d - p > 18 || r - d - 1 > 18) return -2;
    return r;
}

// UpstreamModule.upstreamListOf(X) = X(?: *, *X(?: *: *X)?)* at p: the
// first candidate in java.util.regex order (every X, star iteration and
// optional group taken as far as it goes), -1 none, -2 FALLBACK.  Lists
// whose ',' or ':' is not followed by ' ' would not split into clean items
// in UpstreamListDissector (split(", ") / split(": ")): FALLBACK.
template <typename LN>
__host__ __device__ LP_INLINE int uplist_at(const LN& L, int p, bool dec) {
    auto X = [&](int q) { return dec ? decimal_at(L, q) : (digits_end(L, q) > q ? digits_end(L, q) : -1); };
    auto spaces = [&](int q) { while (q < L.n && L[q] == ' ') ++q; return q; };
    int e = X(p);
    if (e < 0) return e;
    for (;;) {
        int q = spaces(e);
        if (q >= L.n || L[q] != ',') break;
        const int e2 = X(spaces(q + 1));
        if (e2 == -2) return -2;
        if (e2 < 0) break;
        e = e2;
        q = spaces(e);
        if (q < L.n && L[q] == ':') {
            const int e3 = X(spaces(q + 1));
            if (e3 == -2) return -2;
            if (e3 >= 0) e = e3;
        }
    }
    for (int q = p; q < e; ++q) {
        const uint32_t c = L[q];
        if ((c == ',' || c == ':') && (q + 1 >= e || L[q + 1] != ' ')) return -2;
    }
    return e;
}

// uplist_at on the 32 bytes at p read into registers at once (one aligned
// word load per 4 bytes, all in flight together) and classified into bit
// masks (digits, '.', ',', ':', ' '): the runs and separators are found with
// bit scans instead of one dependent LDS read per byte (the first-leaf
// candidate of $upstream_response_time was config 4's costliest element,
// 17 K cycles per wave).  The same steps and results as uplist_at; a list
// still going at the 32nd byte before the line ends: uplist_at decides.
template <typename LN>
__host__ __device__ LP_INLINE int uplist_at_regs(const LN& L, int p, bool dec) {
    constexpr int UNK = -3;
    const int avail = L.n - p;  // bytes to the line end
    const bool open = avail > 32;  // the line goes on past the registers
    const uint32_t A = L.o + (uint32_t)p, W0 = A >> 2, sh = A & 3;
    uint32_t x[9];
    LP_UNROLL for (int j = 0; j < 9; ++j) x[j] = L.word_or0(W0 + (uint32_t)j);
    uint32_t dg = 0, dot = 0, com = 0, col = 0, sp = 0;
    LP_UNROLL for (int j = 0; j < 8; ++j) {
#if defined(__HIP_DEVICE_COMPILE__)
        const uint32_t v = __builtin_amdgcn_alignbyte(x[j + 1], x[j], sh);
#else
        const uint32_t v = (uint32_t)((((uint64_t)x[j + 1] << 32) | x[j]) >> (8 * sh));
#endif
        dg |= bcls::nib(swar::digit(v)) << (4 * j);
        dot |= bcls::nib(swar::eq(v, '.')) << (4 * j);
        com |= bcls::nib(swar::eq(v, ',')) << (4 * j);
        col |= bcls::nib(swar::eq(v, ':')) << (4 * j);
        sp |= bcls::nib(swar::eq(v, ' ')) << (4 * j);
    }
    const uint32_t in = avail >= 32 ? ~0u : avail <= 0 ? 0u : (1u << avail) - 1u;  // bytes inside the line
    dg &= in; dot &= in; com &= in; col &= in; sp &= in;
    auto bit = [](uint32_t m, int q) { return q < 32 && ((m >> q) & 1u); };
    // the first position >= q (q <= 32) not in m: the end of a run
    auto run = [&](uint32_t m, int q) -> int {
        const int r = q + (int)__builtin_ctzll(~((uint64_t)m >> q));
        return r >= 32 && open ? UNK : r;
    };
    auto X = [&](int q) -> int {  // decimal_at / the digit run at q (relative)
        if (q >= 32) return open ? UNK : -1;
        const int d = run(dg, q);
        if (d == UNK) return UNK;
        if (!dec) return d > q ? d : -1;
        if (d == q || d >= avail || !bit(dot, d)) return -1;
        const int r = run(dg, d + 1);
        if (r == UNK) return UNK;
        if (r == d + 1) return -1;
        if (d - q > 18 || r - d - 1 > 18) return -2;
        return r;
    };
    auto spaces = [&](int q) -> int { return q >= 32 ? (open ? UNK : q) : run(sp, q); };
    int e = X(0);
    if (e == UNK) return UNK;
    if (e < 0) return e;
    for (;;) {
        int q = spaces(e);
        if (q == UNK) return UNK;
        if (q >= avail || !bit(com, q)) break;
        const int s = spaces(q + 1);
        if (s == UNK) return UNK;
        const int e2 = X(s);
        if (e2 == UNK) return UNK;
        if (e2 == -2) return -2;
        if (e2 < 0) break;
        e = e2;
        q = spaces(e);
        if (q == UNK) return UNK;
        if (q < avail && bit(col, q)) {
            const int s3 = spaces(q + 1);
            if (s3 == UNK) return UNK;
            const int e3 = X(s3);
            if (e3 == UNK) return UNK;
            if (e3 == -2) return -2;
            if (e3 >= 0) e = e3;
        }
    }
    // a ',' / ':' not followed by ' ' inside the list (e <= 32 here)
    const uint32_t sep = (com | col) & (e >= 32 ? ~0u : (1u << e) - 1u);
    if ((sep & ~(sp >> 1)) || (e > 0 && bit(sep, e - 1))) return -2;
    return p + e;
}

template <typename LN>
__host__ __device__ LP_INLINE int uplist_at_r(const LN& L, int p, bool dec) {
    const int r = uplist_at_regs(L, p, dec);
    return r == -3 ? uplist_at(L, p, dec) : r;
}

// The largest item end of the list at p that is < cur (-1 none).  The list
// was accepted by uplist_at, so its items split cleanly.
template <typename LN>
__host__ __device__ LP_INLINE int uplist_prev_end(const LN& L, int p, int cur, bool dec) {
    auto X = [&](int q) { return dec ? decimal_at(L, q) : (digits_end(L, q) > q ? digits_end(L, q) : -1); };
    auto spaces = [&](int q) { while (q < L.n && L[q] == ' ') ++q; return q; };
    int e = X(p), best = -1;
    while (e >= 0 && e < cur) {
        best = e;
        int q = spaces(e);
        if (q >= L.n || (L[q] != ',' && L[q] != ':')) break;
        e = X(spaces(q + 1));
    }
    return best;
}

// EK_UPLIST_NS, UpstreamModule.upstreamListOf(FORMAT_NO_SPACE_STRING)
// (nginxmodules/UpstreamModule.java:42-44, 139-199): X(?: *, *X(?: *: *X)?)*
// with X = [^\s]*.  X also eats ',' and ':', so the regex's ends in priority
// order are not simple; instead every end of it from p is found (an NFA over
// the positions) and kept if the next literal (or the line end) follows.  A
// single such end is exact whatever the priority order (the others fail at
// the literal); several -> FALLBACK.  Also FALLBACK: a server piece of the
// value that UpstreamListDissector would split into no parts (a piece of
// ": " pairs: ArrayIndexOutOfBoundsException in the reference).
template <typename LN>
__host__ __device__ LP_INLINE int uplist_ns_end(const Program& P, const ElemV& e, const LN& L, int p) {
    // state bits: X0 1 (the first X), X1 2 (X after S), X2 4 (X after C),
    // S_pre 8, S_post 16 (implies X1), C_pre 32, C_post 64 (implies X2)
    constexpr uint32_t XS = 1 | 2 | 4 | 16 | 64;
    uint32_t s = 1;
    int found = -1;
    for (int q = p;; ++q) {
        if (s & XS) {
            const bool ok = e.last ? q == L.n : (!e.nlit || lit_at(P, L, q, e));
            if (ok) {
                if (found >= 0 || (!e.nlit && !e.last)) return -2;
                found = q;
            }
        }
        if (q >= L.n || !s) break;
        const uint32_t c = L[q];
        uint32_t t = 0;
        if (c == ' ') {
            t = (s & XS ? 8u : 0u) | (s & (2 | 16 | 32) ? 32u : 0u) | (s & 8) | (s & 16) | (s & 64);
        } else if (!is_ws(c)) {
            t = (s & 1) | (s & (2 | 16) ? 2u : 0u) | (s & (4 | 64) ? 4u : 0u);
            if (c == ',' && (s & (XS | 8))) t |= 16;
            if (c == ':' && (s & (2 | 16 | 32))) t |= 64;
        }
        s = t;
    }
    if (found < 0) return -1;
    for (int q = p; q + 1 < found; ++q)  // ": " opening a server piece
        if (L[q] == ':' && L[q + 1] == ' ' && (q == p || (q >= p + 2 && L[q - 2] == ',' && L[q - 1] == ' '))) return -2;
    return found;
}

// First candidate end of element e at position p (exact leftmost-first
// order), -1 = none, -2 = FALLBACK.  '.' runs to the end of the line: the
// fast-path guard already rejected every line terminator.
// SIMPLE: an instance for programs whose elements are all literals,
// [^\s]*, the number kinds, .* / .*? and TIME_US (the Apache common /
// combined family): the other kinds' code is left out of it (-2, never
// reached: the host picks the instance from the program).
template <bool LA = true, bool SIMPLE = false, typename LN>
__host__ __device__ LP_INLINE int cand_first(const Program& P, const ElemV& e, const LN& L, int p) {
    switch (e.kind) {
    case EK_NOSPACE: {
        // [^\s]* gives its ends longest first (cand_next: one shorter); when a
        // shorter end can meet the following literal (not det: the literal
        // starts with a non-space byte, e.g. the '"' of a quoted NGINX
        // field), the longest end that the literal follows is the first that
        // can succeed
        const int q = find_ws(L, p, L.n);
        if (!LA || e.det || e.last || !e.nlit) return q;
        return lit_last_call(P, L, e, q, p);
    }
    case EK_NUMBER: { int q = find_fwd(L, p, L.n, [](uint32_t w) { return ~swar::digit(w) & swar::HI; }); return q > p ? q : -1; }
    case EK_CLFNUMBER: {
        int q = find_fwd(L, p, L.n, [](uint32_t w) { return ~swar::digit(w) & swar::HI; });
        if (q > p) return q;
        return (p < L.n && L[p] == '-') ? p + 1 : -1;
    }
    case EK_HEXNUMBER: { int q = find_fwd(L, p, L.n, [](uint32_t w) { return ~swar::hex(w) & swar::HI; }); return q > p ? q : -1; }
    case EK_CLFHEXNUMBER: {
        int q = find_fwd(L, p, L.n, [](uint32_t w) { return ~swar::hex(w) & swar::HI; });
        if (q > p) return q;
        return (p < L.n && L[p] == '-') ? p + 1 : -1;
    }
    case EK_NONZERO: {
        if (p >= L.n || !(L[p] >= '1' && L[p] <= '9')) return -1;
        return find_fwd(L, p + 1, L.n, [](uint32_t w) { return ~swar::digit(w) & swar::HI; });
    }
    case EK_ANY_GREEDY: {
        if (e.last) return L.n;
        if (!e.nlit) return L.n;
        // candidates past the need-th copy of the literal's first byte from
        // the end cannot be followed by the rest of the format
        const int hi = e.need > 1 ? kth_from_end(L, e.lit4 & 0xFFu, e.need, p) : L.n - 1;
        return hi < 0 ? -1 : lit_last(P, L, e, hi, p);
    }
    case EK_ANY_LAZY: {
        if (e.last) return L.n;
        if (!e.nlit) return p;
        return lit_first(P, L, e, p, L.n - 1);
    }
    case EK_TIME_US: return time_us_ok(L, p) ? p + 26 : -1;
    case EK_CLF_IP:
    case EK_IP: {
        if constexpr (SIMPLE) return -2;
        int q = ipv4_first(L, p);
        if (q >= 0) return q;
        // IPv6 alternative can only match empty at '-' (no hex/':'), so '-'
        // is exact when the following literal cannot start at p.
        if (e.kind == EK_CLF_IP && p < L.n && L[p] == '-' && e.nlit && (e.lit4 & 0xFFu) != '-') return p + 1;
        return -2;  // resolved by match_line (ip_resolve)
    }
    case EK_ANYCHAR: if constexpr (SIMPLE) return -2; else return p < L.n ? p + utf8_len(L[p]) : -1;  // '.': one char (the guard rejected line terminators)
    case EK_DECIMAL: if constexpr (SIMPLE) return -2; else return decimal_at(L, p);
    case EK_MSEC: {
        if constexpr (SIMPLE) return -2;
        const int d = digits_end(L, p);
        if (d == p || d + 4 > L.n || L[d] != '.' || !is_digit(L[d + 1]) || !is_digit(L[d + 2]) || !is_digit(L[d + 3]))
            return -1;
        return d - p > 18 ? -2 : d + 4;
    }
    case EK_NOSPACE3: {
        if constexpr (SIMPLE) return -2;
        // only the maximal first and second runs can be followed by ' '; the
        // third run's ends come longest first (cand_next: one shorter), and
        // with a following literal the first that the literal follows is the
        // first that can succeed (NGINX "$request": the longest end takes the
        // closing '"' too and fails at the literal '" ')
        const int q1 = find_ws(L, p, L.n);
        if (q1 >= L.n || L[q1] != ' ') return -1;
        const int q2 = find_ws(L, q1 + 1, L.n);
        if (q2 >= L.n || L[q2] != ' ') return -1;
        const int q3 = find_ws(L, q2 + 1, L.n);
        if (!LA || e.last || !e.nlit) return q3;
        return lit_last_call(P, L, e, q3, q2 + 1);
    }
    case EK_UPLIST_DEC: if constexpr (SIMPLE) return -2; else return uplist_at_r(L, p, true);
    case EK_UPLIST_NUM: if constexpr (SIMPLE) return -2; else return uplist_at_r(L, p, false);
    case EK_UPLIST_NS: if constexpr (SIMPLE) return -2; else return uplist_ns_end(P, e, L, p);
    case EK_CACHE_STATUS: {
        if constexpr (SIMPLE) return -2;
        // the alternatives in order; their first letters differ, so at most
        // one matches at p (the element has a single candidate)
        const char* alt[7] = {"MISS", "BYPASS", "EXPIRED", "STALE", "UPDATING", "REVALIDATED", "HIT"};
        for (int k = 0; k < 7; ++k) {
            int q = 0;
            while (alt[k][q] && p + q < L.n && L[p + q] == (uint32_t)(uint8_t)alt[k][q]) ++q;
            if (!alt[k][q]) return p + q;
        }
        return -1;
    }
    case EK_TIME_ISO: {  // [1-9]ddd-[01]d-[0-3]dTdd:dd:dd[+|-]dd:dd
        if constexpr (SIMPLE) return -2;
        if (p + 25 > L.n) return -1;
        const uint32_t c0 = L[p], s = L[p + 19];
        bool ok = c0 >= '1' && c0 <= '9' && L[p + 4] == '-' && L[p + 7] == '-' && L[p + 10] == 'T' &&
                  L[p + 13] == ':' && L[p + 16] == ':' && L[p + 22] == ':' && (s == '+' || s == '|' || s == '-') &&
                  L[p + 5] <= '1' && L[p + 8] <= '3';
        const int dg[] = {1, 2, 3, 5, 6, 8, 9, 11, 12, 14, 15, 17, 18, 20, 21, 23, 24};
        for (int k = 0; k < 17 && ok; ++k) ok = is_digit(L[p + dg[k]]);
        return ok ? p + 25 : -1;
    }
    case EK_BINIP: {
        if constexpr (SIMPLE) return -2;
        if (p + 16 > L.n) return -1;
        for (int k = p; k < p + 16; k += 4)
            if (L[k] != '\\' || L[k + 1] != 'x' || !is_hex(L[k + 2]) || !is_hex(L[k + 3])) return -1;
        return p + 16;
    }
    }
    return -2;
}

// Could another alternative of FORMAT_IP (TokenParser.java:43-51) at p end
// somewhere other than cur and be followed by the rest of the format (its
// next literal, or '$')?  Every IPv4 end is also an end of the IPv6 branch
// ":?(?:H{1,4}(?::|.)?){0,8}(?::|::)?(?:H{1,4}(?::|.)?){0,8}" (digits are
// hex, '.' matches the dots), so the reachable ends of that branch are
// simulated as bit sets over the <= 83 bytes it can span.
// ip_alt_ends: the same ends as a bit set (bit k = end p + k); returns
// whether there is any.
// 128-bit set in two registers (no arrays: dynamically indexed arrays go to
// scratch memory on the GPU)
struct Set128 {
    uint64_t lo = 0, hi = 0;
    __host__ __device__ LP_INLINE void add(int k) {
        if (k < 64) lo |= 1ull << k;
        else if (k < 128) hi |= 1ull << (k - 64);
    }
    __host__ __device__ LP_INLINE bool any() const { return (lo | hi) != 0; }
    // f(k) for every member k, ascending
    template <typename F>
    __host__ __device__ LP_INLINE void each(F&& f) const {
        for (uint64_t m = lo; m; m &= m - 1) f(__builtin_ctzll(m));
        for (uint64_t m = hi; m; m &= m - 1) f(64 + __builtin_ctzll(m));
    }
};

template <typename LN>
__host__ __device__ LP_INLINE bool ip_alt_ends(const Program& P, const LN& L, const ElemV& e, int p, int cur,
                                               Set128& ends) {
    constexpr int W = 96;
    auto hexat = [&](int q) {
        if (q >= L.n) return false;
        const uint32_t c = L[q];
        return (c - '0' < 10u) || ((c | 32u) - 'a' < 6u);
    };
    Set128 cur_set;
    cur_set.add(0);
    if (p < L.n && L[p] == ':') cur_set.add(1);
    // one (H{1,4}(?::|.)?) group from every position of m, up to 8 times
    auto groups = [&](Set128 m, Set128& acc) {
        for (int it = 0; it < 8; ++it) {
            Set128 nx;
            m.each([&](int k) {
                for (int h = 1; h <= 4 && hexat(p + k + h - 1); ++h) {
                    if (k + h < W) nx.add(k + h);
                    if (p + k + h < L.n) {  // (?::|.): any char but a line terminator (1-4 UTF-8 bytes)
                        const int cl = utf8_len(L[p + k + h]);
                        if (k + h + cl < W) nx.add(k + h + cl);
                    }
                }
            });
            if (!nx.any()) break;
            acc.lo |= nx.lo;
            acc.hi |= nx.hi;
            m = nx;
        }
    };
    Set128 all = cur_set;
    groups(cur_set, all);
    Set128 mid = all;
    all.each([&](int k) {
        if (p + k >= L.n || L[p + k] != ':') return;
        if (k + 1 < W) mid.add(k + 1);
        if (p + k + 1 < L.n && L[p + k + 1] == ':' && k + 2 < W) mid.add(k + 2);
    });
    Set128 fin = mid;
    groups(mid, fin);
    bool any = false;
    ends = Set128{};
    fin.each([&](int k) {
        if (p + k == cur || p + k > L.n) return;
        if (e.last ? p + k == L.n : (!e.nlit || lit_at(P, L, p + k, e))) { ends.add(k); any = true; }
    });
    return any;
}

template <typename LN>
__host__ __device__ LP_INLINE bool ip_alt_end_possible(const Program& P, const LN& L, const ElemV& e, int p, int cur) {
    Set128 ends;
    return ip_alt_ends(P, L, e, p, cur, ends);
}

// Next candidate after 'cur' (same priority order).  SIMPLE: see cand_first.
template <bool SIMPLE = false, typename LN>
__host__ __device__ LP_INLINE int cand_next(const Program& P, const ElemV& e, const LN& L, int p, int cur) {
    switch (e.kind) {
    case EK_NOSPACE: return cur - 1 >= p ? cur - 1 : -1;
    case EK_NUMBER: case EK_HEXNUMBER: case EK_NONZERO: return cur - 1 >= p + 1 ? cur - 1 : -1;
    case EK_CLFNUMBER: case EK_CLFHEXNUMBER:
        if (L[p] == '-') return -1;
        return cur - 1 >= p + 1 ? cur - 1 : -1;
    case EK_ANY_GREEDY:
        if (e.last) return -1;
        if (!e.nlit) return cur - 1 >= p ? cur - 1 : -1;
        return lit_last(P, L, e, cur - 1, p);
    case EK_ANY_LAZY: {
        if (e.last) return -1;
        if (!e.nlit) return cur + 1 <= L.n ? cur + 1 : -1;
        return lit_first(P, L, e, cur + 1, L.n - 1);
    }
    case EK_TIME_US: return -1;
    case EK_CLF_IP: case EK_IP:
        if constexpr (SIMPLE) return -2;
        if (L[p] == '-') return -1;
        // shorter IPv4 / IPv6 alternatives: exact only when none of them can
        // be followed by the rest of the format
        return ip_alt_end_possible(P, L, e, p, cur) ? -2 : -1;
    case EK_ANYCHAR: case EK_MSEC: case EK_UPLIST_NS: case EK_BINIP: case EK_TIME_ISO: case EK_CACHE_STATUS:
        return -1;
    case EK_DECIMAL: {  // a shorter fraction
        if constexpr (SIMPLE) return -2;
        const int d = digits_end(L, p);
        return cur - 1 >= d + 2 ? cur - 1 : -1;
    }
    case EK_NOSPACE3: {  // a shorter third run
        if constexpr (SIMPLE) return -2;
        const int q2 = find_ws(L, find_ws(L, p, L.n) + 1, L.n);
        return cur - 1 >= q2 + 1 ? cur - 1 : -1;
    }
    case EK_UPLIST_DEC: case EK_UPLIST_NUM: {
        if constexpr (SIMPLE) return -2;
        // Backtracking into X(?: *, *X(?: *: *X)?)* yields, in priority order,
        // every shorter end: fewer digits in an item's last run (followed by
        // a digit) and fewer items (item ends, descending).  Followed by the
        // end of the line or a literal that does not start with a digit, only
        // the item ends can succeed.
        if (e.last) return -1;
        if (!e.nlit || is_digit(e.lit4 & 0xFFu)) return -2;
        return uplist_prev_end(L, p, cur, e.kind == EK_UPLIST_DEC);
    }
    }
    return -2;
}

struct NoCapsDfs {
    __host__ __device__ LP_INLINE void set(int, uint32_t) {}
};

// Backtracking match of "^" elems "$" with java.util.regex priority
// semantics.  caps = spans of the captured tokens.  stk: P.max_stack entries.
// elems: the ne elements of one LogFormat.
// elems: the program's element table (the kernel passes an LDS copy).
//
// An IP token whose other alternatives could end elsewhere (cand_* = -2:
// the IPv6 branch of FORMAT_IP, TokenParser.java:43-52, and FORMAT_CLF_IP's
// '-') is resolved exactly when none of those ends lets the rest of the
// format match: a nested DFS over the remaining elements from each such end
// (stack entries above the caller's; Nested = no further nesting).  Then the
// token has no further candidate (-1); otherwise the line is FALLBACK, as
// the priority order among the IPv6 branch's ends is not modelled.
template <bool Nested = false, bool SIMPLE = false, typename LN, typename EL, typename Caps, typename Stk>
__host__ __device__ LP_INLINE int match_line(const Program& P, const EL& elems, int ne, const LN& L, Caps& caps,
                                             Stk stk, int pos0 = 0, int sp0 = 0) {
    int i = 0, pos = pos0, sp = sp0;
    int steps = 0;
    const int budget = 16 * L.n + 256;
    // -1 when no alternative end of the IP element j at p (other than cur)
    // completes the match, -2 otherwise
    auto ip_resolve = [&](int j, int p, int cur, int spn) -> int {
        if constexpr (Nested || SIMPLE) {
            return -2;
        } else {
            const ElemV e = load_elem(elems + j);
            if (e.kind != EK_IP && e.kind != EK_CLF_IP) return -2;
            Set128 ends;
            ip_alt_ends(P, L, e, p, cur, ends);
            if (e.kind == EK_CLF_IP && p < L.n && L[p] == '-' && p + 1 != cur) ends.add(1);  // the '-' alternative
            NoCapsDfs nc;
            bool hit = false;
            ends.each([&](int k) {
                if (!hit && match_line<true, SIMPLE>(P, elems + j + 1, ne - j - 1, L, nc, stk, p + k, spn) != ST_BAD) hit = true;
            });
            return hit ? -2 : -1;
        }
    };
    for (;;) {
        if (++steps > budget) return ST_FALLBACK;
        bool ok;
        if (i == ne) {
            if (pos == L.n) return ST_OK;
            ok = false;
        } else {
            const ElemV e = load_elem(elems + i);
            if (e.kind == EK_LIT) {
                ok = lit_at(P, L, pos, e);
                if (ok) { pos += e.lit_len; ++i; continue; }
            } else {
                int c = cand_first<true, SIMPLE>(P, e, L, pos);
                if (c == -2) c = ip_resolve(i, pos, -1, sp);
                if (c == -2) return ST_FALLBACK;
                ok = c >= 0;
                if (ok) {
                    if (e.cap >= 0) caps.set(e.cap, mkspan(pos, c));
                    if (!e.det) {
                        if (sp >= P.max_stack) return ST_FALLBACK;  // cannot happen: one entry per non-det element
                        stk[sp++] = (uint32_t)i | ((uint32_t)pos << 6) | ((uint32_t)c << 19);
                    }
                    pos = c;
                    ++i;
                    continue;
                }
            }
        }
        // backtrack to the most recent choice point with another candidate
        for (;;) {
            if (sp == sp0) return ST_BAD;
            uint32_t top = stk[sp - 1];
            int j = top & 63, p = (top >> 6) & 8191, cur = (top >> 19) & 8191;
            const ElemV e = load_elem(elems + j);
            int c = cand_next<SIMPLE>(P, e, L, p, cur);
            if (c == -2) c = ip_resolve(j, p, cur, sp);
            if (c == -2) return ST_FALLBACK;
            if (c >= 0) {
                stk[sp - 1] = (uint32_t)j | ((uint32_t)p << 6) | ((uint32_t)c << 19);
                if (e.cap >= 0) caps.set(e.cap, mkspan(p, c));
                pos = c;
                i = j + 1;
                break;
            }
            --sp;
        }
    }
}

// The first leaf of match_line's DFS (every element's first candidate) for
// a one-format program, elements read from the Program with a uniform
// index.  true: the line matches along that leaf (then it is the DFS's
// result: its first complete match); false: decide with match_line.
template <bool LA = true, bool SIMPLE = false, typename LN, typename Caps>
__host__ __device__ LP_INLINE bool match_first_leaf(const Program& P, const LN& L, Caps& caps) {
    int pos = 0;
    bool ok = true;
    const int ne = P.n_elems;
    for (int i = 0; i < ne; ++i) {
        LP_PROF_EL_BEGIN();
        const ElemV e = load_elem(P.elems + i);
        if (e.kind == EK_LIT) {
            ok = ok && lit_at(P, L, pos, e);
            pos += e.lit_len;
        } else if (ok) {
            const int c = cand_first<LA, SIMPLE>(P, e, L, pos);
            ok = c >= 0;
            if (e.cap >= 0) caps.set_u(e.cap, mkspan(pos, c));  // e.cap is uniform
            pos = ok ? c : pos;
        }
        LP_PROF_EL_END(i);
    }
    return ok && pos == L.n;
}

// The same first leaf for a lane of a several-format program: the lane's
// own format's elements (LDS in the kernel, a lane-dependent index), caps
// set by a select chain.  false also when an element needs the DFS's
// resolution (-2): match_line decides.
template <typename LN, typename EL, typename Caps>
__host__ __device__ LP_INLINE bool match_first_leaf_lane(const Program& P, const EL& elems, int ne, const LN& L,
                                                         Caps& caps) {
    int pos = 0;
    for (int i = 0; i < ne; ++i) {
        const ElemV e = load_elem(elems + i);
        if (e.kind == EK_LIT) {
            if (!lit_at(P, L, pos, e)) return false;
            pos += e.lit_len;
        } else {
            const int c = cand_first(P, e, L, pos);
            if (c < 0) return false;
            if (e.cap >= 0) caps.set(e.cap, mkspan(pos, c));
            pos = c;
        }
    }
    return pos == L.n;
}

struct NoCaps {
    __host__ __device__ LP_INLINE void set(int, uint32_t) {}
};

// '"' bytes of the line (aligned words of the base, SWAR compare)
template <typename LN>
__host__ __device__ LP_INLINE int count_quotes(const LN& L) {
    if (L.n <= 0) return 0;
    const uint32_t a = L.o, b = L.o + (uint32_t)L.n - 1;
    int cnt = 0;
    if constexpr (LN::has_masks) {
        {  // popcount of the QUOTE mask, 64 bytes per step
            for (uint32_t W = a >> 6; W <= b >> 6; ++W) {
                uint64_t m = L.mask(MC_QUOTE, W);
                if (W == a >> 6) m &= ~0ull << (a & 63);
                if (W == b >> 6) m &= ~0ull >> (63 - (b & 63));
                cnt += popc64(m);
            }
            return cnt;
        }
    }
    for (uint32_t w = a >> 2; w <= b >> 2; ++w) {
        uint32_t m = swar::eq(L.word(w), '"');
        if (w == a >> 2) m &= 0xFFFFFFFFu << (8 * (a & 3));
        if (w == b >> 2) m &= 0xFFFFFFFFu >> (8 * (3 - (b & 3)));
        cnt += __builtin_popcount(m);
    }
    return cnt;
}

// Necessary conditions for format elems to match the whole line, checked
// from its end: trailing literals and '.' elements at their fixed places,
// then the last byte of the token before them in its class.  false = the
// format cannot match (exact), so the routing pass skips its DFS.
template <typename LN, typename EL>
__host__ __device__ LP_INLINE bool fmt_tail_ok(const Program& P, const EL& elems, int ne, const LN& L) {
    int q = L.n;
    for (int i = ne - 1; i >= 0; --i) {
        const ElemV e = load_elem(elems + i);
        if (e.kind == EK_LIT) {
            q -= e.lit_len;
            if (q < 0 || !lit_at(P, L, q, e)) return false;
            continue;
        }
        if (e.kind == EK_ANYCHAR) {
            if (--q < 0) return false;
            continue;
        }
        const uint32_t c = q > 0 ? L[q - 1] : 0u;
        switch (e.kind) {
        case EK_NUMBER: case EK_NONZERO: case EK_DECIMAL: case EK_MSEC: case EK_TIME_US:
        case EK_UPLIST_DEC: case EK_UPLIST_NUM:
            return q > 0 && is_digit(c);
        case EK_CLFNUMBER: return q > 0 && (is_digit(c) || c == '-');
        case EK_HEXNUMBER: return q > 0 && is_hex(c);
        case EK_CLFHEXNUMBER: return q > 0 && (is_hex(c) || c == '-');
        default: return true;
        }
    }
    return q == 0;
}

// The line as the reference sees it after Hadoop's Text -> String decode:
// no controls but TAB (a line never holds its terminators), no DEL, and any
// bytes >= 0x80 are strict UTF-8 (else the decoder's U+FFFD replacements
// would change the values) other than U+0085, U+2028 and U+2029, which
// java.util.regex '.' does not match.  Lines with such bytes go to FALLBACK.
template <typename LN>
__host__ __device__ LP_INLINE bool line_text_ok(const LN& L) {
    if (find_fwd(L, 0, L.n, [](uint32_t w) { return swar::guard_ctl(w); }) < L.n) return false;
    int i = find_fwd(L, 0, L.n, [](uint32_t w) { return w & swar::HI; });
    while (i < L.n) {
        const uint32_t c = L[i];
        if (c < 0x80) { ++i; continue; }
        int need;
        uint32_t cp;
        if (c >= 0xC2 && c <= 0xDF) { need = 1; cp = c & 0x1F; }
        else if (c >= 0xE0 && c <= 0xEF) { need = 2; cp = c & 0x0F; }
        else if (c >= 0xF0 && c <= 0xF4) { need = 3; cp = c & 0x07; }
        else return false;
        if (i + need >= L.n) return false;
        for (int r = 1; r <= need; ++r) {
            const uint32_t d = L[i + r];
            if ((d & 0xC0) != 0x80) return false;
            cp = (cp << 6) | (d & 0x3F);
        }
        if (need == 2 && (cp < 0x800 || (cp >= 0xD800 && cp <= 0xDFFF))) return false;
        if (need == 3 && (cp < 0x10000 || cp > 0x10FFFF)) return false;
        if (cp == 0x85 || cp == 0x2028 || cp == 0x2029) return false;
        i += need + 1;
    }
    return true;
}

// The match word of a line for sticky routing: bit f = format f matches,
// bit 8+f = undecided on the device (FALLBACK).  Formats whose literal '"'
// count or line tail rule them out skip the DFS.
// DFS = false (the one-pass chunk kernel of several-format programs): a
// format whose first leaf fails and that the prefilters do not rule out sets
// `redo` instead of running the backtracking DFS (the line is then queued:
// k_route_ovf computes its word with the DFS).
// caps (the one-pass chunk kernel): the spans of the first format whose first
// leaf matches (phase1<..., PRE> then starts from them instead of matching
// that format again).
template <bool DFS = true, typename LN, typename EL, typename Stk, typename Caps = NoCaps>
__host__ __device__ LP_INLINE uint32_t fmt_match_word(const Program& P, const EL& elems, const LN& L, Stk stk,
                                                      bool clean, bool* redo = nullptr, Caps* caps = nullptr) {
    const uint32_t all = (1u << P.n_fmt) - 1u;
    if (L.n > MAX_LINE) return all << 8;
    if (!clean && !line_text_ok(L)) return all << 8;
    uint32_t m = 0;
    NoCaps nc;
    const int quotes = count_quotes(L);
    for (int f = 0; f < P.n_fmt; ++f) {
        const int e0 = P.fmt_elem0[f], ne = P.fmt_elem0[f + 1] - e0;
        if (quotes < P.fmt_quotes[f] || !fmt_tail_ok(P, elems + e0, ne, L)) continue;
        // the DFS's first leaf decides most lines of the format (exact: its
        // first complete match); the backtracking DFS the rest
        if constexpr (!std::is_same<Caps, NoCaps>::value) {
            if (!(m & 0xFFu)) {  // no format matched yet: capture this one's spans
                caps->fill(0);
                if (match_first_leaf_lane(P, elems + e0, ne, L, *caps)) {
                    m |= 1u << f;
                    continue;
                }
            } else if (match_first_leaf_lane(P, elems + e0, ne, L, nc)) {
                m |= 1u << f;
                continue;
            }
        } else if (match_first_leaf_lane(P, elems + e0, ne, L, nc)) {
            m |= 1u << f;
            continue;
        }
        if constexpr (DFS) {
            const int st = match_line(P, elems + e0, ne, L, nc, stk);
            m |= st == ST_OK ? (1u << f) : st == ST_FALLBACK ? (256u << f) : 0u;
        } else {
            *redo = true;
        }
    }
    return m;
}

// ------------------------------------------------- sticky format routing
// HttpdLogFormatDissector.dissect (hp/HttpdLogFormatDissector.java:173-204):
// the active format (initially format 0) is tried first; when it does not
// match, the formats are tried in order and the first that matches becomes
// active; when none matches the line fails and the active format stays.
// Which formats match a line is known per line (m: bit f = format f matches,
// bit 8+f = the device could not decide format f), so the active format of
// line i is a left fold of per-line transition functions over the states
// 0..n_fmt-1 and FMT_UNKNOWN -- an associative scan.  A table holds the
// result for state s in nibble s.
__host__ __device__ LP_INLINE uint64_t fmt_table(uint32_t m, int nf) {
    const uint32_t c = m & 0xFFu, u = (m >> 8) & 0xFFu;
    int first = -1;  // -1: no format matches (state kept)
    for (int f = nf - 1; f >= 0; --f) {
        if ((c >> f) & 1u) first = f;
        else if ((u >> f) & 1u) first = FMT_UNKNOWN;
    }
    uint64_t t = ~0ull;  // unused states -> FMT_UNKNOWN
    int common = -2;
    for (int s = 0; s < nf; ++s) {
        const int r = ((c >> s) & 1u) ? s : ((u >> s) & 1u) ? (int)FMT_UNKNOWN : first < 0 ? s : first;
        t = (t & ~(15ull << (4 * s))) | ((uint64_t)r << (4 * s));
        common = common == -2 ? r : common == r ? r : (int)FMT_UNKNOWN;
    }
    // from an undecided state: decided only when every state leads to the same format
    const int ru = common < 0 ? (int)FMT_UNKNOWN : common;
    return (t & ~(15ull << 60)) | ((uint64_t)ru << 60);
}
__host__ __device__ LP_INLINE uint32_t fmt_apply(uint64_t t, uint32_t s) { return (uint32_t)(t >> (4 * s)) & 15u; }
// b after a
__host__ __device__ LP_INLINE uint64_t fmt_compose(uint64_t a, uint64_t b) {
    uint64_t r = 0;
    for (int s = 0; s < 16; ++s) r |= (uint64_t)fmt_apply(b, fmt_apply(a, (uint32_t)s)) << (4 * s);
    return r;
}
// ------------------------------------------------------------- calendar
// Proleptic Gregorian, 32-bit arithmetic: every year the formats admit is
// in [0, 10000) ([1-9][0-9]{3}, plus/minus one day), so day numbers fit in
// int32 and the divisions are unsigned divisions by constants.
__host__ __device__ LP_INLINE int32_t days_from_civil(int32_t y, int m, int d) {
    y -= m <= 2;
    const uint32_t era = (uint32_t)y / 400u;
    const uint32_t yoe = (uint32_t)y - era * 400u;
    const uint32_t doy = (153u * (uint32_t)(m + (m > 2 ? -3 : 9)) + 2u) / 5u + (uint32_t)d - 1u;
    const uint32_t doe = yoe * 365u + yoe / 4u - yoe / 100u + doy;
    return (int32_t)(era * 146097u + doe) - 719468;
}
__host__ __device__ LP_INLINE void civil_from_days(int32_t days, int32_t& y, int& m, int& d) {
    const uint32_t z = (uint32_t)(days + 719468);
    const uint32_t era = z / 146097u;
    const uint32_t doe = z - era * 146097u;
    const uint32_t yoe = (doe - doe / 1460u + doe / 36524u - doe / 146096u) / 365u;
    const uint32_t doy = doe - (365u * yoe + yoe / 4u - yoe / 100u);
    const uint32_t mp = (5u * doy + 2u) / 153u;
    d = (int)(doy - (153u * mp + 2u) / 5u + 1u);
    m = (int)(mp < 10u ? mp + 3u : mp - 9u);
    y = (int32_t)(yoe + era * 400u) + (m <= 2);
}
__host__ __device__ LP_INLINE bool leap(int32_t y) { return (y % 4 == 0 && y % 100 != 0) || y % 400 == 0; }
__host__ __device__ LP_INLINE int month_len(int32_t y, int m) {
    if (m == 2) return leap(y) ? 29 : 28;
    return (m == 4 || m == 6 || m == 9 || m == 11) ? 30 : 31;
}
// ISO day of week, Mon = 1 (day 0 = 1970-01-01 is a Thursday)
__host__ __device__ LP_INLINE int iso_dow(int32_t days) { return (int)((uint32_t)(days + 719468 + 2) % 7u) + 1; }
// WeekFields.ISO (== WeekFields.of(Locale.UK)): week-based-year and week of
// the date with day number `days` in year y
__host__ __device__ LP_INLINE void iso_week(int32_t y, int32_t days, int32_t& wy, int& wk) {
    const int32_t jan1 = days_from_civil(y, 1, 1);
    const int wd = iso_dow(days);
    const int doy = (int)(days - jan1) + 1;
    const int w = (doy - wd + 10) / 7;
    const int jwd = iso_dow(jan1);
    if (w < 1) {
        const int32_t py = y - 1;
        const int pjwd = iso_dow(jan1 - (leap(py) ? 366 : 365));
        wy = py;
        wk = (pjwd == 4 || (pjwd == 3 && leap(py))) ? 53 : 52;
        return;
    }
    const int weeks = (jwd == 4 || (jwd == 3 && leap(y))) ? 53 : 52;
    if (w > weeks) { wy = y + 1; wk = 1; return; }
    wy = y;
    wk = w;
}

// Packed local ("as parsed") and UTC calendar fields and epoch seconds of a
// resolved local date-time (day number `days`) at offset `off` seconds.
__host__ __device__ LP_INLINE void time_fields(int32_t y, int m, int d, int hh, int mi, int ss, int off, int32_t days,
                                               int64_t& epoch_s, uint64_t& local, uint64_t& utc) {
    const int sod = hh * 3600 + mi * 60 + ss;
    epoch_s = (int64_t)days * 86400 + sod - off;
    int32_t wy;
    int wk;
    iso_week(y, days, wy, wk);
    local = pack_cal((uint32_t)y, m, d, hh, mi, ss, (uint32_t)wy, wk);
    // UTC: the same date unless the offset moves the time across midnight
    int t = sod - off;
    int32_t ud = days;
    if (t < 0) { t += 86400; --ud; }
    else if (t >= 86400) { t -= 86400; ++ud; }
    if (ud != days) {
        civil_from_days(ud, y, m, d);
        iso_week(y, ud, wy, wk);
    }
    utc = pack_cal((uint32_t)y, m, d, (uint32_t)(t / 3600), (uint32_t)(t % 3600 / 60), (uint32_t)(t % 60),
                   (uint32_t)wy, wk);
}

// DateTimeFormatter "dd/MMM/yyyy:HH:mm:ss ZZ", parseCaseInsensitive,
// Locale.UK, ResolverStyle.SMART (TimeStampDissector.java:46,100-109,418):
// day 1..31 clamped to the month length, 24:00:00 = next day 00:00:00,
// offset sign+HHMM (each <= 59) with |offset| <= 18:00.
template <typename LN>
__host__ __device__ LP_INLINE bool parse_apache_time(const LN& L, int a, int64_t& epoch_s, uint64_t& local, uint64_t& utc) {
    const Bytes28 c = load28(L, a);
    int day = (c[0] - '0') * 10 + (c[1] - '0');
    // month name: case-insensitive against the 12 UK short names
    uint32_t m3 = ((uint32_t)(c[3] | 32) << 16) | ((uint32_t)(c[4] | 32) << 8) | (uint32_t)(c[5] | 32);
    int month = 0;
    const uint32_t names[12] = {0x6a616e, 0x666562, 0x6d6172, 0x617072, 0x6d6179, 0x6a756e,
                                0x6a756c, 0x617567, 0x736570, 0x6f6374, 0x6e6f76, 0x646563};
    for (int k = 0; k < 12; ++k) if (names[k] == m3) month = k + 1;
    if (!month) return false;
    int hh = (c[12] - '0') * 10 + (c[13] - '0');
    int mi = (c[15] - '0') * 10 + (c[16] - '0');
    int ss = (c[18] - '0') * 10 + (c[19] - '0');
    int off;
    if (c[21] == '+' && c[22] == '0' && c[23] == '0' && c[24] == '0' && c[25] == '0') off = 0;
    else {
        if (c[21] == '|') return false;
        int oh = (c[22] - '0') * 10 + (c[23] - '0'), om = (c[24] - '0') * 10 + (c[25] - '0');
        if (oh > 59 || om > 59) return false;
        off = (c[21] == '-' ? -1 : 1) * (oh * 3600 + om * 60);
    }
    if (off > 64800 || off < -64800) return false;
    if (day < 1 || day > 31) return false;
    const int32_t year = (int32_t)((c[7] - '0') * 1000 + (c[8] - '0') * 100 + (c[9] - '0') * 10 + (c[10] - '0'));
    int ml = month_len(year, month);
    if (day > ml) day = ml;
    if (mi > 59) return false;
    int d = day, m = month;
    int32_t y = year;
    int32_t days = days_from_civil(y, m, d);
    if (hh == 24 && mi == 0 && ss == 0) {
        hh = 0;
        ++days;
        civil_from_days(days, y, m, d);
    } else if (hh > 23 || ss > 59) {
        return false;
    }
    time_fields(y, m, d, hh, mi, ss, off, days, epoch_s, local, utc);
    return true;
}

// TimeStampDissector("TIME.ISO8601", "yyyy-MM-dd'T'HH:mm:ssXXX")
// (hp/HttpdLoglineParser.java:110, TimeStampDissector.java:100-108) on the
// 25 bytes at a (the token kind proved the digit / separator layout):
// SMART resolution as parse_apache_time, numeric month 1..12, offset
// "+HH:MM" (numbers <= 59, total within +-18:00; '|' fails).
template <typename LN>
__host__ __device__ LP_INLINE bool parse_iso_time(const LN& L, int a, int64_t& epoch_s, uint64_t& local, uint64_t& utc) {
    const Bytes28 c = load28(L, a);
    auto d2 = [&](int k) { return (int)(c[k] - '0') * 10 + (int)(c[k + 1] - '0'); };
    const int32_t year = (int32_t)((c[0] - '0') * 1000 + (c[1] - '0') * 100 + (c[2] - '0') * 10 + (c[3] - '0'));
    int month = d2(5), day = d2(8), hh = d2(11), mi = d2(14), ss = d2(17);
    if (c[19] == '|') return false;
    const int oh = d2(20), om = d2(23);
    if (oh > 59 || om > 59) return false;
    const int off = (c[19] == '-' ? -1 : 1) * (oh * 3600 + om * 60);
    if (off > 64800 || off < -64800) return false;
    if (month < 1 || month > 12 || day < 1 || day > 31) return false;
    const int ml = month_len(year, month);
    if (day > ml) day = ml;
    if (mi > 59) return false;
    int32_t y = year;
    int32_t days = days_from_civil(y, month, day);
    if (hh == 24 && mi == 0 && ss == 0) {
        hh = 0;
        ++days;
        civil_from_days(days, y, month, day);
    } else if (hh > 23 || ss > 59) {
        return false;
    }
    time_fields(y, month, day, hh, mi, ss, off, days, epoch_s, local, utc);
    return true;
}

// WeekFields (java.time.temporal.WeekFields.ComputedDayOfField) of the date
// with day number `days` in year y: first day of week sow (1 Monday .. 7
// Sunday), minimal days mind in week 1.
__host__ __device__ LP_INLINE int wf_start_offset(int day, int ldow, int mind) {
    const int week_start = ((day - ldow) % 7 + 7) % 7;
    return week_start + 1 > mind ? 7 - week_start : -week_start;
}
__host__ __device__ LP_INLINE int wf_week(int offset, int day) { return (7 + offset + (day - 1)) / 7; }
__host__ __device__ LP_INLINE int wf_week_of_year(int32_t y, int32_t days, int sow, int mind) {
    const int doy = (int)(days - days_from_civil(y, 1, 1)) + 1;
    const int ldow = ((iso_dow(days) - sow) % 7 + 7) % 7 + 1;
    return wf_week(wf_start_offset(doy, ldow, mind), doy);
}
__host__ __device__ LP_INLINE int32_t wf_week_based_year(int32_t y, int32_t days, int sow, int mind) {
    const int doy = (int)(days - days_from_civil(y, 1, 1)) + 1;
    const int ldow = ((iso_dow(days) - sow) % 7 + 7) % 7 + 1;
    const int offset = wf_start_offset(doy, ldow, mind);
    const int week = wf_week(offset, doy);
    if (week == 0) return y - 1;
    if (week >= wf_week(offset, (leap(y) ? 366 : 365) + mind)) return y + 1;
    return y;
}

// Text of a strftime text element (default locale en_US, JDK 8 data),
// lower-case, packed little-endian: months / days of week short and full,
// "am" / "pm" (AMPM_OF_DAY SHORT is "AM" / "PM"; parsing is case-insensitive).
// The texts are compile-time constants (a constexpr table per kind, folded
// into immediates where the entry is known): no per-call string walk -- the
// earlier version packed each entry from its C string with one dependent
// byte load per character, ~45 K cycles per wave for config 3's %b.
constexpr uint64_t strf_pk8(const char* t) {
    uint64_t v = 0;
    for (int q = 0; q < 8 && t[q]; ++q) v |= (uint64_t)(uint8_t)t[q] << (8 * q);
    return v;
}
constexpr int strf_len(const char* t) {
    int n = 0;
    while (t[n]) ++n;
    return n;
}
__host__ __device__ LP_INLINE int strf_text(int table, int k, uint64_t& lo, uint32_t& hi) {
#define LP_STRF_MON "january", "february", "march", "april", "may", "june", "july", "august", "september", "october", \
                    "november", "december"
#define LP_STRF_DOW "monday", "tuesday", "wednesday", "thursday", "friday", "saturday", "sunday"
    constexpr const char* mon[12] = {LP_STRF_MON};
    constexpr const char* dow[7] = {LP_STRF_DOW};
    constexpr uint64_t mon_lo[12] = {strf_pk8(mon[0]), strf_pk8(mon[1]), strf_pk8(mon[2]), strf_pk8(mon[3]),
                                     strf_pk8(mon[4]), strf_pk8(mon[5]), strf_pk8(mon[6]), strf_pk8(mon[7]),
                                     strf_pk8(mon[8]), strf_pk8(mon[9]), strf_pk8(mon[10]), strf_pk8(mon[11])};
    constexpr uint8_t mon_n[12] = {(uint8_t)strf_len(mon[0]), (uint8_t)strf_len(mon[1]), (uint8_t)strf_len(mon[2]),
                                   (uint8_t)strf_len(mon[3]), (uint8_t)strf_len(mon[4]), (uint8_t)strf_len(mon[5]),
                                   (uint8_t)strf_len(mon[6]), (uint8_t)strf_len(mon[7]), (uint8_t)strf_len(mon[8]),
                                   (uint8_t)strf_len(mon[9]), (uint8_t)strf_len(mon[10]), (uint8_t)strf_len(mon[11])};
    constexpr uint64_t dow_lo[7] = {strf_pk8(dow[0]), strf_pk8(dow[1]), strf_pk8(dow[2]), strf_pk8(dow[3]),
                                    strf_pk8(dow[4]), strf_pk8(dow[5]), strf_pk8(dow[6])};
    constexpr uint8_t dow_n[7] = {(uint8_t)strf_len(dow[0]), (uint8_t)strf_len(dow[1]), (uint8_t)strf_len(dow[2]),
                                  (uint8_t)strf_len(dow[3]), (uint8_t)strf_len(dow[4]), (uint8_t)strf_len(dow[5]),
                                  (uint8_t)strf_len(dow[6])};
#undef LP_STRF_MON
#undef LP_STRF_DOW
    hi = 0;
    switch (table) {
    case ST_MON_SHORT: lo = mon_lo[k] & 0xFFFFFFull; return 3;  // "Jan" .. "Dec"
    case ST_MON_FULL: lo = mon_lo[k]; if (mon_n[k] > 8) hi = 'r'; return mon_n[k];  // "september"
    case ST_DOW_SHORT: lo = dow_lo[k] & 0xFFFFFFull; return 3;  // "Mon" .. "Sun"
    case ST_DOW_FULL: lo = dow_lo[k]; if (dow_n[k] > 8) hi = 'y'; return dow_n[k];  // "wednesday"
    default: lo = k ? 0x6D70ull : 0x6D61ull; return 2;  // "pm" / "am"
    }
}

// The element loop of parse_strf_time for a layout of fixed-width elements
// (T.fixed_w: literals, fixed-width numbers, the 3-letter month / day names,
// AM / PM, "+HHMM"; e.g. %d/%b/%Y %T) on a value of exactly that width and
// all ASCII, from the host's plan of the layout (T.fx_*, plan.cpp
// strf_compile): the value's bytes are read once into registers (one aligned
// word load per 4 bytes, all in flight together); the literals and the digit
// positions are checked for all 32 bytes at once with the plan's byte masks;
// then each field takes its bytes at its fixed offset (a wave-uniform
// indexed register read) -- no per-element dispatch over T.op.  Every check
// the general loop makes on this subset fails it with ST_BAD, so checking
// them all at once decides the same status; the plan exists only when no
// field is given twice (the "must agree" check stays with the general loop).
// -1: not applicable, the general loop decides.
template <typename LN>
__host__ __device__ LP_INLINE int strf_fixed(const TimeStage& T, const LN& L, int a, int b, RegArr<SF_NFIELDS>& fv,
                                             uint32_t& has) {
    const int W = T.fixed_w;
    if (T.fx_n <= 0 || b - a != W) return -1;
    const uint32_t A = L.o + (uint32_t)a, W0 = A >> 2, sh = A & 3;
    uint32_t w[9];
    LP_UNROLL for (int j = 0; j < 9; ++j) w[j] = L.word_or0(W0 + (uint32_t)j);
    RegArr<8> v;
    uint32_t hi = 0, bad = 0;
    LP_UNROLL for (int j = 0; j < 8; ++j) {
#if defined(__HIP_DEVICE_COMPILE__)
        const uint32_t x = __builtin_amdgcn_alignbyte(w[j + 1], w[j], sh);
#else
        const uint32_t x = (uint32_t)((((uint64_t)w[j + 1] << 32) | w[j]) >> (8 * sh));
#endif
        v.v[j] = x;
        const int r = W - 4 * j;  // the value's bytes in this word
        hi |= r >= 4 ? (x & swar::HI) : r > 0 ? (x & swar::HI & ((1u << (8 * r)) - 1u)) : 0u;
        // CharLiteralPrinterParser (case-insensitive) at the literal bytes
        bad |= ((x | T.fx_fold[j]) ^ T.fx_lit[j]) & T.fx_litm[j];
        // '0'..'9' at the digit bytes (ASCII: no carry leaves a byte)
        const uint32_t t = x ^ 0x30303030u;
        bad |= (t | (t + 0x06060606u)) & 0xF0F0F0F0u & T.fx_dig[j];
    }
    if (hi) return -1;  // non-ASCII: the general loop (its text elements fall back)
    if (bad) return ST_BAD;
    for (int k = 0; k < T.fx_n; ++k) {
        const uint32_t f = T.fx_f[k];
        const int off = (int)(f & 0xFF), width = (int)((f >> 8) & 0xFF), field = (int)((f >> 16) & 0xFF);
        const uint32_t code = f >> 24;
        // the field's bytes [off, off + 8) (off is wave-uniform)
        const int wi = off >> 2, bs = 8 * (off & 3);
        const uint64_t w01 = (uint64_t)v.get_u(wi) | (uint64_t)(wi + 1 < 8 ? v.get_u(wi + 1) : 0u) << 32;
        const uint32_t w2 = wi + 2 < 8 ? v.get_u(wi + 2) : 0u;
        const uint64_t u = bs ? (w01 >> bs) | ((uint64_t)w2 << (64 - bs)) : w01;
        uint32_t val = 0;
        switch (code & 0xF) {
        case FX_NUM: case FX_RED2:  // fixed width, NOT_NEGATIVE (digits checked above); reduced: base 2000
            for (int q = 0; q < width; ++q) val = val * 10 + (uint32_t)((u >> (8 * q)) & 0xF);
            if ((code & 0xF) == FX_RED2) val += 2000;
            break;
        case FX_TEXT: {  // TextPrinterParser: every entry of these tables has the same length
            const uint32_t tb = code >> 4;
            int best = -1;
            if (tb == ST_MON_SHORT || tb == ST_DOW_SHORT) {
                const uint32_t tlo = (uint32_t)u | 0x202020u;
                if (tb == ST_MON_SHORT) {
                    LP_UNROLL for (int t = 0; t < 12; ++t) {
                        uint64_t elo; uint32_t ehi;
                        strf_text(ST_MON_SHORT, t, elo, ehi);
                        if (best < 0 && ((tlo ^ (uint32_t)elo) & 0xFFFFFFu) == 0) best = t;
                    }
                } else {
                    LP_UNROLL for (int t = 0; t < 7; ++t) {
                        uint64_t elo; uint32_t ehi;
                        strf_text(ST_DOW_SHORT, t, elo, ehi);
                        if (best < 0 && ((tlo ^ (uint32_t)elo) & 0xFFFFFFu) == 0) best = t;
                    }
                }
                if (best < 0) return ST_BAD;
                val = (uint32_t)best + 1;
            } else {  // AM / PM
                const uint32_t tlo = ((uint32_t)u | 0x2020u) & 0xFFFFu;
                if (tlo == 0x6D61u) val = 0;       // "am"
                else if (tlo == 0x6D70u) val = 1;  // "pm"
                else return ST_BAD;
            }
            break;
        }
        default: {  // FX_OFF, appendOffset("+HHMM", "+0000") (digits checked above)
            const uint32_t sg = (uint32_t)u & 0xFF;
            if (sg != '+' && sg != '-') return ST_BAD;
            const int oh = (int)((u >> 8) & 0xF) * 10 + (int)((u >> 16) & 0xF);
            const int om = (int)((u >> 24) & 0xF) * 10 + (int)((u >> 32) & 0xF);
            if (oh > 59 || om > 59) return ST_BAD;
            val = (uint32_t)((sg == '-' ? -1 : 1) * (oh * 3600 + om * 60));
            break;
        }
        }
        fv.set_u(field, val);
    }
    has |= T.fx_has;
    return ST_OK;
}

// StrfTimeStampDissector (hp/dissectors/StrfTimeStampDissector.java:44-70)
// on the value [a, b): DateTimeFormatter.parse(text, ZonedDateTime::from)
// with the elements of T (parseCaseInsensitive, strict), then JDK 8's
// java.time.format.Parsed.resolve under ResolverStyle.SMART: instant seconds
// (at the parsed zone, else the formatter's UTC, else the offset) -> date +
// second-of-day; IsoChronology.resolveDate (YEAR + MONTH + DAY with the
// month-length clamp, else YEAR + DAY_OF_YEAR); resolveTimeFields
// (CLOCK_HOUR_OF_DAY 0..24, CLOCK_HOUR_OF_AMPM 0..12 with AMPM_OF_DAY,
// second-of-day, each with updateCheckConflict); WeekFields.ISO.dayOfWeek()
// replacing DAY_OF_WEEK; resolveTimeLenient (defaulted minute / second /
// nano, 24:00 end of day); crossCheck of every field left against the date
// and time.  A field parsed twice must agree (DateTimeParseContext).
// Returns ST_OK, ST_BAD (DateTimeParseException) or ST_FALLBACK (outside the
// restated subset: non-ASCII text, zone names other than UTC / GMT, signs,
// 19-digit numbers, week-based dates, years outside 1..9999).  The oracle's
// strf_parse restates the same steps independently.
template <typename LN>
__host__ __device__ LP_INLINE int parse_strf_time(const TimeStage& T, const LN& L, int a, int b, int64_t& epoch_ms,
                                                  uint64_t& local, uint64_t& utc, uint32_t& nanos) {
    RegArr<SF_NFIELDS> fv;  // field values (SF_INSTANT: low word; high word in inst_hi)
    fv.fill(0);
    uint32_t has = 0, inst_hi = 0;
    bool zone_utc = false;
    int pos = a;
    auto low = [](uint32_t c) { return c | 0x20u; };  // safe fold against lower-case ASCII letters
#if defined(LP_NO_STRF_FIXED)
    const int fx = -1;
#else
    const int fx = strf_fixed(T, L, a, b, fv, has);
#endif
    LP_PROF(14);
    if (fx == ST_BAD) return ST_BAD;
    if (fx == ST_OK) pos = b;
    for (int k = 0; k < T.n_ops && fx < 0; ++k) {
        const uint32_t op = T.op[k];
        const int kind = (int)(op & 0xFF), field = (int)((op >> 8) & 0xFF), width = (int)((op >> 16) & 0xFF);
        const uint32_t arg = op >> 24;
        uint32_t v = 0;
        switch (kind) {
        case SE_LIT: {  // CharLiteralPrinterParser, case-insensitive
            if (pos >= b) return ST_BAD;
            const uint32_t c = L[pos];
            const bool eq = c == arg || ((arg | 0x20u) - 'a' < 26u && low(c) == (arg | 0x20u));
            if (!eq) return c >= 0x80 ? ST_FALLBACK : ST_BAD;
            ++pos;
            continue;
        }
        case SE_NUM: case SE_RED2: {  // fixed width, NOT_NEGATIVE; reduced: base 2000
            if (pos + width > b) return ST_BAD;
            for (int q = 0; q < width; ++q) {
                const uint32_t d = L[pos + q] - '0';
                if (d > 9) return ST_BAD;
                v = v * 10 + d;
            }
            pos += width;
            if (kind == SE_RED2) v += 2000;
            break;
        }
        case SE_NUMV: {  // 1..19 digits (INSTANT_SECONDS, week-of-year)
            if (pos < b && (L[pos] == '+' || L[pos] == '-')) return ST_FALLBACK;
            uint64_t w = 0;
            int q = pos;
            while (q < b && q - pos < 19 && L[q] - '0' < 10u) { w = w * 10 + (L[q] - '0'); ++q; }
            if (q == pos) return ST_BAD;
            if (q - pos >= 19 || w > 0xFFFFFFFFFFull) return ST_FALLBACK;  // beyond the restated range
            pos = q;
            if (field == SF_INSTANT) {
                const uint32_t hi = (uint32_t)(w >> 32);
                if (((has >> SF_INSTANT) & 1u) && (fv.get(SF_INSTANT) != (uint32_t)w || inst_hi != hi)) return ST_BAD;
                inst_hi = hi;
            }
            v = (uint32_t)w;
            if (field != SF_INSTANT && w > 0x7FFFFFFFull) return ST_FALLBACK;
            break;
        }
        case SE_PAD2: {  // PadPrinterParserDecorator(2, ' '): spaces, then digits to the end
            if (pos + 2 > b) return ST_BAD;
            int q = pos;
            while (q < pos + 2 && L[q] == ' ') ++q;
            if (q < pos + 2 && (L[q] == '+' || L[q] == '-')) return ST_FALLBACK;
            if (q == pos + 2) return ST_BAD;
            for (int r = q; r < pos + 2; ++r) {
                const uint32_t d = L[r] - '0';
                if (d > 9) return ST_BAD;
                v = v * 10 + d;
            }
            pos += 2;
            break;
        }
        case SE_TEXT: {  // TextPrinterParser: the longest entry that matches
            uint64_t tlo = 0;
            uint32_t thi = 0;
            for (int q = 0; q < 9 && pos + q < b; ++q) {
                const uint32_t c = L[pos + q];
                // java's case-insensitive charEquals folds a few non-ASCII
                // letters to ASCII ones (U+017F, U+0131, U+0130, U+212A)
                if (c >= 0x80) return ST_FALLBACK;
                if (q < 8) tlo |= (uint64_t)low(c) << (8 * q);
                else thi = low(c);
            }
            const int nt = arg == ST_MON_SHORT || arg == ST_MON_FULL ? 12 : arg == ST_AMPM_UP || arg == ST_AMPM_LOW ? 2 : 7;
            int best = -1, blen = 0;
            for (int t = 0; t < nt; ++t) {
                uint64_t elo;
                uint32_t ehi;
                const int n = strf_text(arg, t, elo, ehi);
                if (pos + n > b || n <= blen) continue;
                const uint64_t m = n >= 8 ? ~0ull : (1ull << (8 * n)) - 1;
                if (((tlo ^ elo) & m) == 0 && (n <= 8 || (thi & 0xFFu) == ehi)) { best = t; blen = n; }
            }
            if (best < 0) return ST_BAD;
            pos += blen;
            v = arg == ST_AMPM_UP || arg == ST_AMPM_LOW ? (uint32_t)best : (uint32_t)best + 1;
            break;
        }
        case SE_OFF: {  // appendOffset("+HHMM", "+0000")
            if (pos + 5 > b) return ST_BAD;
            const uint32_t sg = L[pos];
            int off = 0;
            if (!(sg == '+' && L[pos + 1] == '0' && L[pos + 2] == '0' && L[pos + 3] == '0' && L[pos + 4] == '0')) {
                if (sg != '+' && sg != '-') return ST_BAD;
                for (int q = 1; q <= 4; ++q) if (L[pos + q] - '0' > 9u) return ST_BAD;
                const int oh = (int)(L[pos + 1] - '0') * 10 + (int)(L[pos + 2] - '0');
                const int om = (int)(L[pos + 3] - '0') * 10 + (int)(L[pos + 4] - '0');
                if (oh > 59 || om > 59) return ST_BAD;
                off = (sg == '-' ? -1 : 1) * (oh * 3600 + om * 60);
            }
            pos += 5;
            v = (uint32_t)off;
            break;
        }
        case SE_ZONE: {  // appendZoneText(SHORT): "UTC" / "GMT" not followed by an offset
            if (pos + 3 > b) return ST_FALLBACK;
            const uint32_t c0 = low(L[pos]), c1 = low(L[pos + 1]), c2 = low(L[pos + 2]);
            const bool ok = (c0 == 'u' && c1 == 't' && c2 == 'c') || (c0 == 'g' && c1 == 'm' && c2 == 't');
            if (!ok || (pos + 3 < b && (L[pos + 3] == '+' || L[pos + 3] == '-'))) return ST_FALLBACK;
            pos += 3;
            zone_utc = true;
            continue;
        }
        default: return ST_FALLBACK;
        }
        // DateTimeParseContext.setParsedField: a field parsed twice must agree
        if (((has >> field) & 1u) && fv.get(field) != v) return ST_BAD;
        has |= 1u << field;
        fv.set_u(field, v);
    }
    if (pos != b) return ST_BAD;  // text left over
    auto H = [&](int f) { return ((has >> f) & 1u) != 0; };
    auto V = [&](int f) { return (int32_t)fv.get(f); };
    // ---- Parsed.resolve (JDK 8), SMART
    bool have_date = false, have_time = false, plus_day = false;
    int32_t dy = 0;
    int dm = 0, dd = 0;
    int64_t sod = -1;
    if (H(SF_INSTANT)) {  // resolveInstantFields
        int64_t off;
        if (zone_utc || !T.zone) off = 0;
        else if (H(SF_OFFSET)) off = V(SF_OFFSET);
        else return ST_FALLBACK;
        if (off > 64800 || off < -64800) return ST_BAD;
        const int64_t inst = (int64_t)(((uint64_t)inst_hi << 32) | fv.get(SF_INSTANT));
        if (inst > 253402300799ll) return ST_FALLBACK;  // past year 9999
        const int64_t t = inst + off;
        const int64_t days = t >= 0 ? t / 86400 : -((-t + 86399) / 86400);
        civil_from_days((int32_t)days, dy, dm, dd);
        sod = t - days * 86400;
        have_date = true;
    }
    if (H(SF_YEAR) && ((H(SF_MONTH) && H(SF_DOM)) || H(SF_DOY))) {  // IsoChronology.resolveDate
        const int32_t y = V(SF_YEAR);
        int32_t ry;
        int rm, rd;
        if (H(SF_MONTH) && H(SF_DOM)) {  // resolveYMD
            const int mo = V(SF_MONTH);
            int dom = V(SF_DOM);
            if (mo < 1 || mo > 12 || dom < 1 || dom > 31) return ST_BAD;
            if (y < 1 || y > 9999) return ST_FALLBACK;
            const int ml = month_len(y, mo);
            if (dom > ml) dom = ml;
            ry = y; rm = mo; rd = dom;
            has &= ~((1u << SF_MONTH) | (1u << SF_DOM));
        } else {  // resolveYD
            const int doy = V(SF_DOY);
            if (doy < 1 || doy > 366) return ST_BAD;
            if (y < 1 || y > 9999) return ST_FALLBACK;
            if (doy == 366 && !leap(y)) return ST_BAD;
            civil_from_days(days_from_civil(y, 1, 1) + doy - 1, ry, rm, rd);
            has &= ~(1u << SF_DOY);
        }
        has &= ~(1u << SF_YEAR);
        if (have_date && (ry != dy || rm != dm || rd != dd)) return ST_BAD;  // updateCheckConflict(date)
        dy = ry; dm = rm; dd = rd;
        have_date = true;
    }
    if (H(SF_WOY) && H(SF_YEAR)) return ST_FALLBACK;  // WeekFields.resolveWoY builds the date
    int32_t hod = H(SF_HOD) ? V(SF_HOD) : -1, hap = -1;
    if (H(SF_CHOD)) {  // SMART: 0..24, 24 -> 0
        const int32_t ch = V(SF_CHOD);
        if (ch != 0 && (ch < 1 || ch > 24)) return ST_BAD;
        const int32_t h = ch == 24 ? 0 : ch;
        if (hod >= 0 && hod != h) return ST_BAD;
        hod = h;
    }
    if (H(SF_CHAP)) {  // SMART: 0..12, 12 -> 0
        const int32_t ch = V(SF_CHAP);
        if (ch != 0 && (ch < 1 || ch > 12)) return ST_BAD;
        hap = ch == 12 ? 0 : ch;
    }
    bool ampm_used = false;
    if (H(SF_AMPM) && hap >= 0) {
        const int32_t h = V(SF_AMPM) * 12 + hap;
        if (hod >= 0 && hod != h) return ST_BAD;
        hod = h;
        ampm_used = true;
    }
    int32_t moh = H(SF_MIN) ? V(SF_MIN) : -1, som = H(SF_SEC) ? V(SF_SEC) : -1;
    if (sod >= 0) {  // SECOND_OF_DAY -> HOUR_OF_DAY, MINUTE_OF_HOUR, SECOND_OF_MINUTE
        const int32_t h = (int32_t)(sod / 3600), mi = (int32_t)(sod / 60 % 60), se = (int32_t)(sod % 60);
        if ((hod >= 0 && hod != h) || (moh >= 0 && moh != mi) || (som >= 0 && som != se)) return ST_BAD;
        hod = h; moh = mi; som = se;
    }
    int32_t dow = H(SF_DOW) ? V(SF_DOW) : 0;
    if (H(SF_ISODOW)) {  // WeekFields.ISO.dayOfWeek() replaces DAY_OF_WEEK
        if (V(SF_ISODOW) < 1 || V(SF_ISODOW) > 7) return ST_BAD;
        dow = V(SF_ISODOW);
    }
    if (H(SF_MILLI) && H(SF_MICRO)) return ST_FALLBACK;
    int32_t nos = H(SF_MILLI) ? V(SF_MILLI) * 1000000 : H(SF_MICRO) ? V(SF_MICRO) * 1000 : -1;
    int th = 0, tmi = 0, tse = 0;
    if (hod >= 0 && !((moh < 0 && (som >= 0 || nos >= 0)) || (moh >= 0 && som < 0 && nos >= 0))) {
        const int32_t m2 = moh < 0 ? 0 : moh, s2 = som < 0 ? 0 : som, n2 = nos < 0 ? 0 : nos;
        if (m2 > 59) return ST_BAD;  // resolveTime: minute, then 24:00 end of day, then hour / second
        if (hod == 24 && m2 == 0 && s2 == 0 && n2 == 0) { th = 0; plus_day = true; }
        else if (hod > 23 || s2 > 59) return ST_BAD;
        else th = hod;
        tmi = m2;
        tse = s2;
        nos = n2;
        have_time = true;
    }
    if (!have_date || !have_time) return ST_BAD;  // LocalDateTime.from
    int32_t days = days_from_civil(dy, dm, dd);
    if (plus_day) civil_from_days(++days, dy, dm, dd);
    // crossCheck
    if (dow && dow != iso_dow(days)) return ST_BAD;
    if (H(SF_DOY) && V(SF_DOY) != (int32_t)(days - days_from_civil(dy, 1, 1)) + 1) return ST_BAD;
    if (H(SF_WOY) && V(SF_WOY) != wf_week_of_year(dy, days, 1, 4)) return ST_BAD;
    if (H(SF_WBY) && V(SF_WBY) != wf_week_based_year(dy, days, 7, 1)) return ST_BAD;
    if (H(SF_AMPM) && !ampm_used && V(SF_AMPM) != th / 12) return ST_BAD;
    if (hap >= 0 && !ampm_used && hap != th % 12) return ST_BAD;
    if ((H(SF_MONTH) && V(SF_MONTH) != dm) || (H(SF_DOM) && V(SF_DOM) != dd) || (H(SF_YEAR) && V(SF_YEAR) != dy))
        return ST_BAD;
    int off = 0;  // ZonedDateTime.from: the offset (ZoneOffset.ofTotalSeconds)
    if (!zone_utc && T.zone) {
        if (!H(SF_OFFSET)) return ST_BAD;
        off = V(SF_OFFSET);
        if (off > 64800 || off < -64800) return ST_BAD;
    }
    if (dy < 1 || dy > 9999) return ST_FALLBACK;
    LP_PROF(15);
    int64_t es;
    time_fields(dy, dm, dd, th, tmi, tse, off, days, es, local, utc);
    LP_PROF(16);
    epoch_ms = es * 1000 + (int64_t)(nos / 1000000);
    nanos = (uint32_t)nos;
    return ST_OK;
}

// ----------------------------------------------------------- per-line state
struct LineOut {
    int status;
    int fmt;  // the LogFormat the line was routed to
    RegArr<MAX_TOK> caps;
    uint32_t tok_flags;
    RegArr<MAX_FL> fl_kind, fl_method, fl_uri, fl_proto;
    // time stage t's results (bit t of tdone: delivered), written with the
    // row by write_line (the chunked kernel knows the line's number only
    // after phase 1)
    uint32_t tdone;
    RegArr<MAX_TIME> ep_lo, ep_hi, lo_lo, lo_hi, ut_lo, ut_hi, nano;
    uint32_t hist;  // run-histogram word of an OK line (hist_word)
    uint32_t smdone;  // SECOND_MILLIS stage s delivered (bit s)
    RegArr<MAX_SECMS> sm_lo, sm_hi;
    uint32_t bipdone;  // BinaryIP stage b delivered (bit b)
    RegArr<MAX_BINIP> bip;
};

// A line's URI stages (the URI kernel): per query stage the piece table
// (arena region offset) and its pending pieces.  NQ: query stages the
// kernel instance handles (the registers it keeps)
template <int NQ>
struct UriOutT {
    int status = ST_OK;
    RegArr<NQ> qlist, qpend;
};
using UriOut = UriOutT<MAX_QUERY>;

// Last ' ' in [lo, hi], else -1 (lines with masks: the WS class, skipping TABs).
template <typename LN>
__host__ __device__ LP_INLINE int find_space_bwd(const LN& L, int hi, int lo) {
    if constexpr (LN::has_masks) {
        int q = mfind_bwd(L, MC_WS, hi, lo);
        while (q >= 0 && L[q] != ' ') q = mfind_bwd(L, MC_WS, q - 1, lo);
        return q;
    } else {
        return find_bwd(L, hi, lo, [](uint32_t w) { return swar::eq(w, ' '); });
    }
}

template <typename LN>
__host__ __device__ LP_INLINE bool prefix_at(const LN& L, int a, int b, const char* lit) {
    int k = 0;
    for (; lit[k]; ++k)
        if (a + k >= b || L[a + k] != (uint8_t)lit[k]) return false;
    return true;
}
template <typename LN>
__host__ __device__ LP_INLINE bool value_is_header_name(const LN& L, int a, int b) {
    return (b - a == 17 && prefix_at(L, a, b, "request.firstline")) || prefix_at(L, a, b, "request.header.") ||
           prefix_at(L, a, b, "response.header.");
}

// Source span of URI stage u; returns false when the value is null/absent/empty
__host__ __device__ LP_INLINE bool uri_source(const Program& P, const LineOut& o, int u, int& a, int& b) {
    const UriStage& U = P.uri[u];
    uint32_t sp;
    if (U.src_q >= 0) return false;  // a derived stage (k_derived_lines)
    if (U.src_tok >= 0) {
        if (o.tok_flags & (1u << U.src_tok)) return false;  // "-" -> null
        sp = o.caps.get(U.src_tok);
    } else {
        if (o.fl_kind.get(U.src_fl) == FL_NONE) return false;
        sp = o.fl_uri.get(U.src_fl);
    }
    a = sp & 0xFFFF;
    b = sp >> 16;
    return b > a;
}

// The same from the columns phase 1 wrote (the URI kernel runs after it).
template <typename Cols>
__host__ __device__ LP_INLINE bool uri_source_cols(const Program& P, const Cols& C, int64_t li, int u, int& a, int& b) {
    const UriStage& U = P.uri[u];
    uint32_t sp;
    if (U.src_q >= 0) return false;  // a derived stage (k_derived_lines)
    if (U.src_tok >= 0) {
        if (C.tok_flags[li] & (1u << U.src_tok)) return false;  // "-" -> null
        sp = C.tok_span[U.src_tok][li];
    } else {
        if (C.fl_kind[U.src_fl][li] == FL_NONE) return false;
        sp = C.fl_uri[U.src_fl][li];
    }
    a = sp & 0xFFFF;
    b = sp >> 16;
    return b > a;
}

// Arena need of URI stage u on [a, b) (its query table): URIUtil-escaped
// bytes and '&' / '?' separators are both URI event bytes, so their count
// bounds the pieces; a URI without event bytes writes nothing to the arena.
// Rewritten / decoded parts and query values are spilled when they occur.
template <typename LN>
__host__ __device__ LP_INLINE uint32_t uri_need(const Program& P, int u, const LN& L, int a, int b, uint32_t& usep) {
    usep = count_uev(L, a, b);
    return usep != 0 && P.uri[u].query_stage >= 0 ? 16 + 16 * (usep + 1) : 0u;  // alignment, one slot per piece
}

// ---- Set-Cookie headers (ResponseSetCookieListDissector.java:79-110 with
// JDK 8 java.net.HttpCookie.parse, ResponseSetCookieDissector.java:78-151).
// The replay splits the list and names / dissects the cookies; the device
// proves the value lies in the restated subset where none of the reference's
// exceptions can occur (the oracle's sc_subset / sc_name / sc_expire):
// printable ASCII without '"', '\\' and '$', no "max-age" / "version" /
// "set-cookie" (any case: HttpCookie.parse then takes its Netscape branch, one
// cookie per string); every cookie string (the ", " parts, a part whose
// "expires=" sits within its last 15 bytes joined with the next one) has a
// first ';'-token with a '=' before which the trimmed name is a non-empty
// token that no JDK reserves; with `exp`, every "expires" attribute
// (case-sensitive key) is "EEE, dd-MMM-yyyy HH:mm:ss GMT" with in-range
// fields and the right day name (parseExpire's only reachable pattern).
template <typename LN>
__host__ __device__ LP_INLINE bool ci_lit_at(const LN& L, int q, int b, const char* lit) {  // lit lower-case
    for (int k = 0; lit[k]; ++k) {
        if (q + k >= b) return false;
        uint32_t c = L[q + k];
        if (c - 'A' < 26u) c |= 32u;
        if (c != (uint8_t)lit[k]) return false;
    }
    return true;
}
template <typename LN>
__host__ __device__ LP_INLINE bool sc_expire_ok(const LN& L, int a, int b) {
    if (b - a != 29) return false;
    const char* shape = "XXX, 00-XXX-0000 00:00:00 GMT";  // X: day / month name bytes (checked below)
    for (int i = 0; i < 29; ++i) {
        const uint32_t c = L[a + i], t = (uint8_t)shape[i];
        if (t == 'X') continue;
        if (t == '0') { if (!is_digit(c)) return false; }
        else if (c != t) return false;
    }
    const uint32_t dn = L[a] | (L[a + 1] << 8) | (L[a + 2] << 16), mn = L[a + 8] | (L[a + 9] << 8) | (L[a + 10] << 16);
    const char* days = "MonTueWedThuFriSatSun";
    const char* mons = "JanFebMarAprMayJunJulAugSepOctNovDec";
    int dow = -1, mon = -1;
    for (int k = 0; k < 7; ++k)
        if (dn == ((uint32_t)(uint8_t)days[3 * k] | ((uint32_t)(uint8_t)days[3 * k + 1] << 8) |
                   ((uint32_t)(uint8_t)days[3 * k + 2] << 16))) dow = k;
    for (int k = 0; k < 12; ++k)
        if (mn == ((uint32_t)(uint8_t)mons[3 * k] | ((uint32_t)(uint8_t)mons[3 * k + 1] << 8) |
                   ((uint32_t)(uint8_t)mons[3 * k + 2] << 16))) mon = k + 1;
    if (dow < 0 || mon < 0) return false;
    auto d2 = [&](int i) { return (int)(L[a + i] - '0') * 10 + (int)(L[a + i + 1] - '0'); };
    const int d = d2(5), y = d2(12) * 100 + d2(14), h = d2(17), mi = d2(20), se = d2(23);
    if (y < 1 || d < 1 || d > month_len(y, mon) || h > 23 || mi > 59 || se > 59) return false;
    return iso_dow(days_from_civil(y, mon, d)) == dow + 1;
}
// The cookie string [s, e): HttpCookie.parseInternal's name is valid; with
// exp, its "expires" attributes parse.
template <typename LN>
__host__ __device__ LP_INLINE bool sc_cookie_ok(const LN& L, int s, int e, bool exp) {
    int q = s;
    while (q < e && L[q] == ';') ++q;
    if (q == e) return false;  // "Empty cookie header string"
    int te = q;
    while (te < e && L[te] != ';') ++te;
    int eq = q;
    while (eq < te && L[eq] != '=') ++eq;
    if (eq == te) return false;  // "Invalid cookie name-value pair"
    int na = q, nb = eq;
    while (na < nb && L[na] <= ' ') ++na;
    while (nb > na && L[nb - 1] <= ' ') --nb;
    if (na == nb) return false;
    for (int k = na; k < nb; ++k)
        if (L[k] == ' ' || L[k] == ',') return false;  // isToken (the subset has no controls, ';' or '$')
    const int nl = nb - na;
    auto is = [&](const char* r, int n) { return nl == n && ci_lit_at(L, na, nb, r); };
    if (is("comment", 7) || is("commenturl", 10) || is("discard", 7) || is("domain", 6) || is("expires", 7) ||
        is("path", 4) || is("port", 4) || is("secure", 6))
        return false;  // names older JDKs reserve
    if (!exp) return true;
    // ResponseSetCookieDissector: split(";"), trim, split("=", 2); key "expires" (i > 0)
    for (int ps = s, i = 0; ps <= e; ++i) {
        int pe = ps;
        while (pe < e && L[pe] != ';') ++pe;
        if (i > 0) {
            int ka = ps, kb = pe;
            while (ka < kb && L[ka] <= ' ') ++ka;
            int x = ka;
            while (x < kb && L[x] != '=') ++x;
            int ke = x;
            while (ke > ka && L[ke - 1] <= ' ') --ke;
            if (ke - ka == 7 && L[ka] == 'e' && L[ka + 1] == 'x' && L[ka + 2] == 'p' && L[ka + 3] == 'i' &&
                L[ka + 4] == 'r' && L[ka + 5] == 'e' && L[ka + 6] == 's') {
                if (x == kb) return false;  // no '=': parseExpire("") throws
                int va = x + 1, vb = kb;
                while (va < vb && L[va] <= ' ') ++va;
                while (vb > va && L[vb - 1] <= ' ') --vb;
                if (!sc_expire_ok(L, va, vb)) return false;
            }
        }
        ps = pe + 1;
    }
    return true;
}
template <typename LN>
__host__ __device__ LP_INLINE bool setcookie_ok(const LN& L, int a, int b, bool exp) {
    if (b <= a) return true;  // empty: nothing is dissected
    for (int q = a; q < b; ++q) {
        const uint32_t c = L[q];
        if (c < 0x20 || c > 0x7E || c == '"' || c == '\\' || c == '$') return false;
        const uint32_t lc = c | 32u;
        if ((lc == 'm' && ci_lit_at(L, q, b, "max-age")) || (lc == 'v' && ci_lit_at(L, q, b, "version")) ||
            (lc == 's' && ci_lit_at(L, q, b, "set-cookie")))
            return false;
    }
    // split(", "): trailing empty parts are dropped
    int t = b;
    while (t - a >= 2 && L[t - 2] == ',' && L[t - 1] == ' ') t -= 2;
    if (t == a) return true;
    int prev = -1;
    for (int s = a; s <= t;) {
        int e = s;
        while (e < t && !(L[e] == ',' && e + 1 < t && L[e + 1] == ' ')) ++e;
        // a part whose "expires=" starts within its last 15 bytes waits for the next
        int ei = -1;
        for (int q = s; q + 8 <= e && ei < 0; ++q)
            if ((L[q] | 32u) == 'e' && ci_lit_at(L, q, e, "expires=")) ei = q - s;
        if (ei >= 0 && (e - s) - 15 < ei) {
            prev = s;
        } else {
            if (!sc_cookie_ok(L, prev >= 0 ? prev : s, e, exp)) return false;
            prev = -1;
        }
        if (e >= t) break;
        s = e + 2;
    }
    return true;
}

// ---- ConvertSecondsWithMillisStringDissector
// (translate/ConvertSecondsWithMillisStringDissector.java:33-40):
// value.split("\\.", 2), Long.parseLong of both, seconds * 1000 +
// milliseconds (the fraction read as an integer: "1.5" -> 1005), Java long
// arithmetic (wraps).  The element kinds deliver digits '.' digits of at
// most 18 digits each (decimal_at), so neither parse can throw.
template <typename LN>
__host__ __device__ LP_INLINE int64_t secms_value(const LN& L, int a, int b) {
    uint64_t sec = 0, frac = 0;
    int q = a;
    for (; q < b && L[q] != '.'; ++q) sec = sec * 10u + (L[q] - '0');
    for (++q; q < b; ++q) frac = frac * 10u + (L[q] - '0');
    return (int64_t)(sec * 1000u + frac);
}

// ---- UpstreamListDissector.dissect (nginxmodules/UpstreamListDissector.java:79-125):
// servers = value.split(", "); per server parts = server.split(": "); item
// k's value = parts[0].trim(), redirected = (parts.length == 1 ? parts[0] :
// parts[1]).trim().  Java String.split (limit 0): trailing empty pieces are
// dropped, a value without the separator is itself the one piece (even
// empty); String.trim drops bytes <= ' ' at both ends.  Calls f(k, va, vb,
// ra, rb) for every item in order (trimmed line positions) and returns the
// item count, -1 for a server that splits into no parts (": " pairs only: an
// ArrayIndexOutOfBoundsException in the reference; the element kinds send
// such lines to FALLBACK).
template <typename LN>
__host__ __device__ LP_INLINE int sep_at(const LN& L, int q, int e, uint32_t c0) {  // c0 then ' ' at q
    return q + 1 < e && L[q] == c0 && L[q + 1] == ' ';
}
template <typename LN, typename F>
__host__ __device__ LP_INLINE int uplist_items(const LN& L, int a, int b, F&& f) {
    auto next_sep = [&](int q, int e, uint32_t c0) {
        while (q + 1 < e && !sep_at(L, q, e, c0)) ++q;
        return q + 1 < e ? q : e;
    };
    auto strip = [&](int s, int e, uint32_t c0) {  // drop the separators of trailing empty pieces
        while (e - s >= 2 && L[e - 2] == c0 && L[e - 1] == ' ') e -= 2;
        return e;
    };
    auto trim = [&](int& s, int& e) {
        while (s < e && L[s] <= ' ') ++s;
        while (e > s && L[e - 1] <= ' ') --e;
    };
    int t = b;
    if (next_sep(a, b, ',') < b) {
        t = strip(a, b, ',');
        if (t == a) return 0;  // only empty servers
    }
    int k = 0;
    for (int s0 = a;;) {
        const int e0 = next_sep(s0, t, ',');
        const int x0 = next_sep(s0, e0, ':');
        int va = s0, vb = x0, ra = s0, rb = x0;
        if (x0 < e0) {
            // more than one part unless everything after the first ": " is empty pieces
            const int r1 = strip(x0 + 2, e0, ':');
            if (r1 > x0 + 2) {
                ra = x0 + 2;
                rb = next_sep(x0 + 2, e0, ':');
            } else if (x0 == s0) {
                return -1;  // no parts at all
            }
        }
        trim(va, vb);
        trim(ra, rb);
        f(k, va, vb, ra, rb);
        ++k;
        if (e0 >= t) break;
        s0 = e0 + 2;
    }
    return k;
}

// The same split on a token of at most 32 bytes held in registers (TokReg:
// its bytes aligned to its first byte, one word load per 4 bytes, and the
// byte-class masks the split needs), so the scans are bit operations instead
// of one dependent byte read per byte: the upstream lists of a line are split
// twice (list_need, list_fill) and their items converted, and one lane's long
// list held its whole wave.  Same steps as uplist_items, on the masks:
// next_sep = the first separator bit in [q, e - 1), strip = the separator
// bits at e - 2, trim = the first / last byte > ' '.
struct TokReg {
    RegArr<8> w;        // bytes 4j..4j+3 of the token in word j
    uint32_t comma, colon, space, le;  // bit i: byte i is ',' / ':' / ' ' / <= ' '
    __host__ __device__ LP_INLINE uint32_t byte(int i) const { return (w.get(i >> 2) >> (8 * (i & 3))) & 0xFFu; }
};
template <typename LN>
__host__ __device__ LP_INLINE bool tok_load(const LN& L, int a, int b, TokReg& T) {
    if (b - a > 32 || b < a) return false;
    const uint32_t A = L.o + (uint32_t)a, W0 = A >> 2, sh = A & 3;
    uint32_t x[9];
    LP_UNROLL for (int j = 0; j < 9; ++j) x[j] = L.word_or0(W0 + (uint32_t)j);
    T.comma = T.colon = T.space = T.le = 0;
    LP_UNROLL for (int j = 0; j < 8; ++j) {
#if defined(__HIP_DEVICE_COMPILE__)
        const uint32_t v = __builtin_amdgcn_alignbyte(x[j + 1], x[j], sh);
#else
        const uint32_t v = (uint32_t)((((uint64_t)x[j + 1] << 32) | x[j]) >> (8 * sh));
#endif
        T.w.v[j] = v;
        T.comma |= bcls::nib(swar::eq(v, ',')) << (4 * j);
        T.colon |= bcls::nib(swar::eq(v, ':')) << (4 * j);
        T.space |= bcls::nib(swar::eq(v, ' ')) << (4 * j);
        T.le |= bcls::nib(swar::lt(v, ' ' + 1)) << (4 * j);
    }
    return true;
}
__host__ __device__ LP_INLINE uint32_t bits_below(int e) { return e >= 32 ? ~0u : e <= 0 ? 0u : (1u << e) - 1u; }
template <typename F>
__host__ __device__ LP_INLINE int uplist_items_r(const TokReg& T, int a, int b, F&& f) {
    const int n = b - a;
    const uint32_t sp1 = T.space >> 1;  // bit q: byte q + 1 is ' '
    const uint32_t sepc = T.comma & sp1 & bits_below(n - 1), sepk = T.colon & sp1 & bits_below(n - 1);
    auto next_sep = [&](uint32_t sep, int q, int e) -> int {  // first separator q' >= q with q' + 1 < e, else e
        const uint32_t m = sep & ~bits_below(q) & bits_below(e - 1);
        return m ? __builtin_ctz(m) : e;
    };
    auto strip = [&](uint32_t sep, int s0, int e) {
        while (e - s0 >= 2 && ((sep >> (e - 2)) & 1u)) e -= 2;
        return e;
    };
    auto trim = [&](int& s0, int& e) {
        const uint32_t m = ~T.le & ~bits_below(s0) & bits_below(e);
        if (!m) { s0 = e; return; }
        s0 = __builtin_ctz(m);
        e = 32 - __builtin_clz(m);
    };
    int t = n;
    if (next_sep(sepc, 0, n) < n) {
        t = strip(sepc, 0, n);
        if (t == 0) return 0;  // only empty servers
    }
    int k = 0;
    for (int s0 = 0;;) {
        const int e0 = next_sep(sepc, s0, t);
        const int x0 = next_sep(sepk, s0, e0);
        int va = s0, vb = x0, ra = s0, rb = x0;
        if (x0 < e0) {
            const int r1 = strip(sepk, x0 + 2, e0);
            if (r1 > x0 + 2) {
                ra = x0 + 2;
                rb = next_sep(sepk, x0 + 2, e0);
            } else if (x0 == s0) {
                return -1;  // no parts at all
            }
        }
        trim(va, vb);
        trim(ra, rb);
        f(k, a + va, a + vb, a + ra, a + rb);
        ++k;
        if (e0 >= t) break;
        s0 = e0 + 2;
    }
    return k;
}
// secms_value on token bytes [s, e) (token-relative) in registers
__host__ __device__ LP_INLINE int64_t secms_value_r(const TokReg& T, int s, int e) {
    uint64_t sec = 0, frac = 0;
    int q = s;
    for (; q < e && T.byte(q) != '.'; ++q) sec = sec * 10u + (T.byte(q) - '0');
    for (++q; q < e; ++q) frac = frac * 10u + (T.byte(q) - '0');
    return (int64_t)(sec * 1000u + frac);
}

// ---- run histograms (lp_histograms, SURVEY.md §5 counters): one word per
// OK line, reduced on demand: bits 0..15 token k present (not "-" and not
// empty), bits 16..25 the response status code (100..599; 0: another value
// or null; 1023: the format has no status token), bits 26..30 the request
// method (0..14 the names below, 15 another, 16 none; 31: the format has no
// first-line stage).
constexpr int HIST_METHOD_OTHER = 15, HIST_METHOD_NONE = 16;
// GET POST HEAD PUT DELETE OPTIONS PATCH CONNECT TRACE PROPFIND MKCOL COPY MOVE LOCK UNLOCK
template <typename LN>
__host__ __device__ LP_INLINE int hist_method(const LN& L, int a, int b) {
    if (b <= a) return HIST_METHOD_NONE;  // no method (null or empty first line, or neither regex matched)
    const int n = b - a;
    if (n > 9) return HIST_METHOD_OTHER;
    const uint32_t w0 = load_u32_at(L, a) & (n >= 4 ? ~0u : (1u << (8 * n)) - 1u);
    const uint32_t w1 = n > 4 ? load_u32_at(L, a + 4) & (n >= 8 ? ~0u : (1u << (8 * (n - 4))) - 1u) : 0u;
    const uint32_t w2 = n > 8 ? L[a + 8] : 0u;
    auto W = [](char c0, char c1, char c2, char c3) {
        return (uint32_t)(uint8_t)c0 | ((uint32_t)(uint8_t)c1 << 8) | ((uint32_t)(uint8_t)c2 << 16) | ((uint32_t)(uint8_t)c3 << 24);
    };
    switch (n) {
    case 3:
        if (w0 == W('G', 'E', 'T', 0)) return 0;
        if (w0 == W('P', 'U', 'T', 0)) return 3;
        break;
    case 4:
        if (w0 == W('P', 'O', 'S', 'T')) return 1;
        if (w0 == W('H', 'E', 'A', 'D')) return 2;
        if (w0 == W('C', 'O', 'P', 'Y')) return 11;
        if (w0 == W('M', 'O', 'V', 'E')) return 12;
        if (w0 == W('L', 'O', 'C', 'K')) return 13;
        break;
    case 5:
        if (w0 == W('P', 'A', 'T', 'C') && w1 == 'H') return 6;
        if (w0 == W('T', 'R', 'A', 'C') && w1 == 'E') return 8;
        if (w0 == W('M', 'K', 'C', 'O') && w1 == 'L') return 10;
        break;
    case 6:
        if (w0 == W('D', 'E', 'L', 'E') && w1 == W('T', 'E', 0, 0)) return 4;
        if (w0 == W('U', 'N', 'L', 'O') && w1 == W('C', 'K', 0, 0)) return 14;
        break;
    case 7:
        if (w0 == W('O', 'P', 'T', 'I') && w1 == W('O', 'N', 'S', 0)) return 5;
        if (w0 == W('C', 'O', 'N', 'N') && w1 == W('E', 'C', 'T', 0)) return 7;
        break;
    case 8:
        if (w0 == W('P', 'R', 'O', 'P') && w1 == W('F', 'I', 'N', 'D')) return 9;
        break;
    default: break;
    }
    (void)w2;
    return HIST_METHOD_OTHER;
}
template <typename LN>
__host__ __device__ LP_INLINE uint32_t hist_word(const Program& P, const LN& L, const LineOut& o) {
    uint32_t present = 0;
    o.caps.each([&](int k, uint32_t sp) {
        if (k < P.n_tok && !((o.tok_flags >> k) & 1u) && (sp >> 16) > (sp & 0xFFFFu)) present |= 1u << k;
    });
    const int sk = P.hist_status[o.fmt];
    uint32_t code = sk >= 0 ? 0u : 1023u;  // 1023: the format has no status token (no count)
    if (sk >= 0 && !((o.tok_flags >> sk) & 1u)) {
        const uint32_t sp = o.caps.get(sk);
        const int a = (int)(sp & 0xFFFFu), b = (int)(sp >> 16);
        if (b - a == 3) {
            const uint32_t d0 = L[a] - '0', d1 = L[a + 1] - '0', d2 = L[a + 2] - '0';
            if (d0 < 10 && d1 < 10 && d2 < 10) code = d0 * 100 + d1 * 10 + d2;
            if (code < 100 || code > 599) code = 0;
        }
    }
    uint32_t m = HIST_METHOD_NONE;
    const int f = P.hist_fl[o.fmt];
    if (f >= 0) {
        const uint32_t sp = o.fl_method.get(f);
        m = (uint32_t)hist_method(L, (int)(sp & 0xFFFFu), (int)(sp >> 16));
    } else {
        m = 31;  // the format has no first-line stage: no method count
    }
    return present | (code << 16) | (m << 26);
}

// Phase 1: guard, match, tokens, time, first line (the parse kernel).
// clean: the caller already proved every byte of the line passes the
// fast-path guard (the kernel checks the whole staged window at once).
// LA: the literal-aware first candidates of [^\s]* / NGINX "$request"
// (cand_first) in the first leaf; a kernel instance without them serves the
// programs that have no such element (the code would reshape every
// program's register allocation).
// MULTI: a kernel of several-format programs (k_parse_lines): the lanes of
// a wave hold lines of different LogFormats, so the stages run by slot (the
// k-th time / first-line stage of each lane's own format together) and the
// first leaf is walked per lane.
// SIMPLE: one LogFormat of the Apache common / combined family (cand_first)
// with only Apache time stamps and no cookie / Set-Cookie guards, SECOND_MILLIS
// or BinaryIP stages: the other stages' code is left out of the instance.
// DFS = false: a line whose first leaf fails and that the prefilters do not
// rule out gets ST_REDO instead of the backtracking DFS (the one-pass chunk
// kernel queues it for k_parse_ovf_lines, which runs the whole phase 1:
// neither the DFS's code nor its registers are in the hot kernel, and a
// line that backtracks no longer holds the other lanes of its wave).
// PRE (several LogFormats, one pass): the line's format and its first-leaf
// spans are already known (fmt_match_word captured them into o.caps, the
// guard included): phase 1 starts after the match.
template <bool MULTI = false, bool LA = true, bool SIMPLE = false, bool DFS = true, bool PRE = false, typename LN,
          typename EL, typename Stk, typename Cols>
__host__ __device__ LP_INLINE void phase1(const Program& P, const EL& elems, const LN& L, LineOut& o, Stk stk, Cols& C,
                                          int64_t li, bool clean = false, int fmt = 0) {
    o.status = ST_OK;
    o.fmt = fmt;
    o.tok_flags = 0;
    o.tdone = 0;
    o.smdone = 0;
    o.bipdone = 0;
    if constexpr (!PRE) o.caps.fill(0);
    o.fl_kind.fill(FL_NONE);
    o.fl_method.fill(0);
    o.fl_uri.fill(0);
    o.fl_proto.fill(0);
    if (L.n > MAX_LINE || fmt >= P.n_fmt) { o.status = ST_FALLBACK; return; }  // too long / routing undecided
    // fast-path guard: TAB, printable ASCII and valid UTF-8 without the
    // chars java.util.regex '.' does not match (line_text_ok)
    LP_PROF(2);
    if (!PRE && !clean && !line_text_ok(L)) {
        o.status = ST_FALLBACK;
        return;
    }
    LP_PROF(3);
    // One LogFormat: every lane walks the same elements, so the DFS's first
    // leaf (each element's first candidate) is tried in lock step with the
    // elements read as wave-uniform values (scalar loads, scalar branches on
    // the element kind); lines it does not match run the backtracking DFS.
    // Lines the first leaf does not match skip the DFS when the format's
    // quote count or line tail already rules them out (exact; malformed
    // lines would otherwise backtrack while the rest of the wave waits).
    int st = ST_BAD;
    if constexpr (PRE) {
        st = ST_OK;
    } else if constexpr (MULTI) {
        const int e0 = P.fmt_elem0[fmt], ne = P.fmt_elem0[fmt + 1] - e0;
        if (match_first_leaf_lane(P, elems + e0, ne, L, o.caps)) st = ST_OK;
        else o.caps.fill(0);  // the DFS sets its own
    } else {
        if (P.n_fmt == 1 && match_first_leaf<LA, SIMPLE>(P, L, o.caps)) st = ST_OK;
    }
    if (st != ST_OK) {
        const int e0 = P.fmt_elem0[fmt], ne = P.fmt_elem0[fmt + 1] - e0;
        if (P.n_fmt == 1 && (!fmt_tail_ok(P, elems + e0, ne, L) || count_quotes(L) < P.fmt_quotes[fmt])) st = ST_BAD;
        else if constexpr (DFS) st = match_line<false, SIMPLE>(P, elems + e0, ne, L, o.caps, stk);
        else st = ST_REDO;
    }
    LP_PROF(4);
    if (st != ST_OK) { o.status = st; return; }
    // decodeExtractedValue: "-" -> null (Apache: ApacheHttpdLogFormatDissector.java:169-196,
    // NGINX: NginxHttpdLogFormatDissector.java:107-119).  Slots unrolled (the
    // spans stay in registers); only one-byte values are read.
    {
        const bool apache = P.fmt_apache[fmt] != 0;
        bool fb = false;
        uint32_t flags = 0;
        o.caps.each([&](int k, uint32_t sp) {
            if (k >= P.n_tok) return;
            const int a = sp & 0xFFFF, b = sp >> 16;
            if (b - a == 1) {
                const uint32_t c = L[a];
                flags |= (c == '-' ? 1u << k : 0u) | (c == '0' ? 1u << (16 + k) : 0u);
            }
            // the reference tests the VALUE (not the token name) against
            // "request.firstline" / "request.header." / "response.header." and
            // then unescapes \xhh sequences (ApacheHttpdLogFormatDissector.java:189-193)
            if (apache && b - a >= 15) {
                const uint32_t w = load_u32_at(L, a);
                if ((w == 0x75716572u /* "requ" */ || w == 0x70736572u /* "resp" */) && value_is_header_name(L, a, b) &&
                    find_fwd(L, a, b, [](uint32_t x) { return swar::eq(x, '\\'); }) < b)
                    fb = true;
            }
        });
        o.tok_flags = flags;
        if (fb) { o.status = ST_FALLBACK; return; }
    }
    // values the replay URL-decodes (request cookies, Utils.resilientUrlDecode):
    // ASCII, and every '%' followed by two hex digits, else FALLBACK
    if constexpr (!SIMPLE) for (uint32_t gm = (uint32_t)P.guard_pct[fmt]; gm; gm &= gm - 1) {
        const uint32_t sp = o.caps.get(__builtin_ctz(gm));
        const int a = sp & 0xFFFF, b = sp >> 16;
        if (find_fwd(L, a, b, [](uint32_t w) { return w & swar::HI; }) < b) { o.status = ST_FALLBACK; return; }
        for (int q = find_fwd(L, a, b, [](uint32_t w) { return swar::eq(w, '%'); }); q < b;
             q = find_fwd(L, q + 1, b, [](uint32_t w) { return swar::eq(w, '%'); }))
            if (q + 2 >= b || !is_hex(L[q + 1]) || !is_hex(L[q + 2])) { o.status = ST_FALLBACK; return; }
    }
    // Set-Cookie lists the replay splits (the subset where HttpCookie.parse cannot throw)
    if constexpr (!SIMPLE) for (uint32_t gm = (uint32_t)P.guard_setc[fmt]; gm; gm &= gm - 1) {
        const int k = __builtin_ctz(gm);
        if (o.tok_flags & (1u << k)) continue;  // "-": null, nothing is dissected
        const uint32_t sp = o.caps.get(k);
        if (!setcookie_ok(L, (int)(sp & 0xFFFF), (int)(sp >> 16), (P.guard_setc_exp[fmt] >> k) & 1)) {
            o.status = ST_FALLBACK;
            return;
        }
    }
    LP_PROF(5);
    // TimeStampDissector (MULTI: slot s = the s-th stage of the lane's format)
    for (int s = 0; s < P.n_time; ++s) {
        int t = s;
        if constexpr (MULTI) {
            t = -1;
            for (int u = 0, c = 0; u < P.n_time; ++u)
                if (P.time[u].fmt == fmt) { if (c == s) t = u; ++c; }
            if (t < 0) continue;
        } else {
            if (P.time[t].fmt != fmt) continue;
        }
        const TimeStage& T = P.time[t];
        const int k = T.tok;
        const uint32_t sp = o.caps.get(k);
        const int a = sp & 0xFFFF, b = sp >> 16;
        int64_t ep; uint64_t lo, ut;
        uint32_t ns = 0;
        if (T.kind == TK_APACHE) {
            if (!parse_apache_time(L, a, ep, lo, ut)) { o.status = ST_BAD; return; }
            ep *= 1000;
        } else if constexpr (SIMPLE) {
            continue;  // (not in this instance's programs)
        } else if (T.kind == TK_ISO) {
            if (!parse_iso_time(L, a, ep, lo, ut)) { o.status = ST_BAD; return; }
            ep *= 1000;
        } else {
            // an empty or "-" (null) value has no outputs (TimeStampDissector.java:412-415)
            if (b == a || (o.tok_flags & (1u << k))) continue;
            const int st = parse_strf_time(T, L, a, b, ep, lo, ut, ns);
            if (st != ST_OK) { o.status = st; return; }
        }
        o.tdone |= 1u << t;
        if constexpr (MULTI) {  // t differs between lanes: select chains
            o.ep_lo.set(t, (uint32_t)(uint64_t)ep);
            o.ep_hi.set(t, (uint32_t)((uint64_t)ep >> 32));
            o.lo_lo.set(t, (uint32_t)lo);
            o.lo_hi.set(t, (uint32_t)(lo >> 32));
            o.ut_lo.set(t, (uint32_t)ut);
            o.ut_hi.set(t, (uint32_t)(ut >> 32));
            o.nano.set(t, ns);
        } else {  // t is wave-uniform: indexed register writes
            o.ep_lo.set_u(t, (uint32_t)(uint64_t)ep);
            o.ep_hi.set_u(t, (uint32_t)((uint64_t)ep >> 32));
            o.lo_lo.set_u(t, (uint32_t)lo);
            o.lo_hi.set_u(t, (uint32_t)(lo >> 32));
            o.ut_lo.set_u(t, (uint32_t)ut);
            o.ut_hi.set_u(t, (uint32_t)(ut >> 32));
            o.nano.set_u(t, ns);
        }
    }
    LP_PROF(6);
    // HttpFirstLineDissector: ^([a-zA-Z-_]+) (.*) (HTTP/[0-9]+\.[0-9]+)$ else ^([a-zA-Z-_]+) (.*)$
    for (int s = 0; s < P.n_fl; ++s) {
        int f = s;
        if constexpr (MULTI) {
            f = -1;
            for (int u = 0, c = 0; u < P.n_fl; ++u)
                if (P.fl[u].fmt == fmt) { if (c == s) f = u; ++c; }
            if (f < 0) continue;
        } else {
            if (P.fl[f].fmt != fmt) continue;
        }
        int k = P.fl[f].tok;
        if (o.tok_flags & (1u << k)) continue;                // null
        const uint32_t sp0 = o.caps.get(k);
        int a = sp0 & 0xFFFF, b = sp0 >> 16;
        if (b <= a) continue;                                 // empty
        // method [a-zA-Z-_]+ (SWAR scan for the first other byte)
        const int q = find_fwd(L, a, b, [](uint32_t w) {
            const uint32_t l = w | 0x20202020u;
            const uint32_t alpha = swar::ge(l, 'a') & swar::lt(l, 'z' + 1) & ~(w & swar::HI);
            return ~(alpha | swar::eq(w, '-') | swar::eq(w, '_')) & swar::HI;
        });
        if (q == a || q >= b || L[q] != ' ') continue;        // neither regex matches
        o.fl_method.set(f, mkspan(a, q));
        int us = q + 1;
        // protocol: the last ' ' must be followed by HTTP/d+.d+ up to the end
        int sp = find_space_bwd(L, b - 1, us);
        if (sp < 0) sp = us - 1;
        bool full = false;
        if (sp >= us && b - sp >= 9 && load_u32_at(L, sp + 1) == 0x50545448u /* "HTTP" */ && L[sp + 5] == '/') {
            const int d1 = sp + 6, r = digits_end(L, d1);
            if (r > d1 && r < b && L[r] == '.') {
                const int d2 = r + 1, r2 = digits_end(L, d2);
                full = r2 >= b && b > d2;  // digits up to the end of the value
            }
        }
        if (full) {
            o.fl_kind.set(f, FL_FULL);
            o.fl_uri.set(f, mkspan(us, sp));
            o.fl_proto.set(f, mkspan(sp + 1, b));
        } else {
            o.fl_kind.set(f, FL_CHOPPED);
            o.fl_uri.set(f, mkspan(us, b));
            o.fl_proto.set(f, 0);
        }
    }
    // ConvertSecondsWithMillisStringDissector on this format's SECOND_MILLIS tokens
    if constexpr (!SIMPLE) for (int sm = 0; sm < P.n_secms; ++sm) {
        if (P.secms[sm].fmt != fmt) continue;
        const int k = P.secms[sm].tok;
        if ((o.tok_flags >> k) & 1u) continue;  // "-" never matches the token kinds; nothing to convert
        const uint32_t sp = o.caps.get(k);
        const int a = (int)(sp & 0xFFFFu), b = (int)(sp >> 16);
        TokReg T;  // (a short value from registers: one word load per 4 bytes)
        const int64_t ms = tok_load(L, a, b, T) ? secms_value_r(T, 0, b - a) : secms_value(L, a, b);
        o.smdone |= 1u << sm;
        o.sm_lo.set_u(sm, (uint32_t)(uint64_t)ms);
        o.sm_hi.set_u(sm, (uint32_t)((uint64_t)ms >> 32));
    }
    // BinaryIPDissector: "\xHH" x 4 (the element kind EK_BINIP proved the shape)
    if constexpr (!SIMPLE) for (int bs = 0; bs < P.n_binip; ++bs) {
        if (P.binip[bs].fmt != fmt) continue;
        const uint32_t sp = o.caps.get(P.binip[bs].tok);
        const int a = (int)(sp & 0xFFFFu);
        if ((sp >> 16) - (uint32_t)a != 16u) continue;
        uint32_t v = 0;
        for (int k = 0; k < 4; ++k) v |= (hexv(L[a + 4 * k + 2]) * 16u + hexv(L[a + 4 * k + 3])) << (8 * k);
        o.bipdone |= 1u << bs;
        o.bip.set_u(bs, v);
    }
    o.hist = hist_word(P, L, o);
    LP_PROF(7);
}

// ------------------------------------------------------------ URI stage
// A line's arena region: the reserved part (phase 1 bounds the query table
// there) written from offset 0 up, plus pieces spilled further on into the
// same shard for the rare rewritten / decoded URI parts and query values
// (sized then, exactly; refs stay region-relative: spills are allocated after
// the region, in the same shard).
struct Arena {
    LP_G uint8_t* p;  // this line's region
    uint32_t used;
    uint32_t cap;
    uint32_t slack = 0;  // reserved, never written
    uint32_t extra = 0;  // bytes written in spilled pieces
    // spill allocator: the shard's bump pointer (a device atomic; the CPU
    // emulation's counter), the region's offset in the shard, the shard size
    LP_G unsigned long long* top = nullptr;
    uint64_t base = 0, limit = 0;
    bool ovf = false;    // a spill did not fit (the batch is re-run with a larger arena)
    __host__ __device__ uint32_t put(uint32_t c) { p[used] = (uint8_t)c; return used++; }
};

// X = a fresh piece of n bytes of A's shard, written like a region (region-
// relative offsets).  false: the shard is full (A.ovf set).
__host__ __device__ LP_INLINE bool spill(Arena& A, uint32_t n, Arena& X) {
    n = (n + 3) & ~3u;  // every spilled piece starts 4-byte aligned (word stores)
    X = A;
    if (!A.top || n == 0) { A.ovf = A.top == nullptr; X.cap = X.used; return n == 0; }
#if defined(__HIP_DEVICE_COMPILE__)
    const unsigned long long x = __hip_atomic_fetch_add(A.top, (unsigned long long)n, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
#else
    const unsigned long long x = *A.top;
    *A.top += n;
#endif
    if (x < A.base || x + n > A.limit || x - A.base + n > 0x7FFFFFFFull) { A.ovf = true; return false; }
    X.used = (uint32_t)(x - A.base);
    X.cap = X.used + n;
    return true;
}

// Forward byte reader over a line: 8 bytes in registers, one aligned word
// read per 4 bytes for increasing positions (any position < n works).
template <typename LN>
struct Fwd {
    const LN& L;
    uint32_t W;
    uint64_t ww;
    __host__ __device__ LP_INLINE Fwd(const LN& l, int p) : L(l) {
        W = (L.o + (uint32_t)p) >> 2;
        ww = (uint64_t)L.word_or0(W) | ((uint64_t)L.word_or0(W + 1) << 32);
    }
    __host__ __device__ LP_INLINE uint32_t at(int p) {
        const uint32_t A = L.o + (uint32_t)p, w = A >> 2;
        if (w != W) {
            if (w == W + 1) ww = (ww >> 32) | ((uint64_t)L.word_or0(w + 1) << 32);
            else ww = (uint64_t)L.word_or0(w) | ((uint64_t)L.word_or0(w + 1) << 32);
            W = w;
        }
        return (uint32_t)(ww >> (8 * (A & 3))) & 0xFFu;
    }
};

// 128-bit character sets
__host__ __device__ LP_INLINE bool in_set(uint32_t c, uint64_t lo, uint64_t hi) {
    return c < 0x80 && (((c < 64 ? lo : hi) >> (c & 63)) & 1u);
}
// chars in both L_SERVER and L_REG_NAME of java.net.URI without '@' and
// escapes: alnum . - : _ ! ~ * ' ( ) ; = + $ ,
__host__ __device__ LP_INLINE bool authority_char(uint32_t c) { return in_set(c, 0x2FFF7F9200000000ull, 0x47FFFFFE87FFFFFEull); }
// scheme = alpha *( alpha | digit | "+" | "-" | "." )
__host__ __device__ LP_INLINE bool scheme_char(uint32_t c) { return in_set(c, 0x03FF680000000000ull, 0x07FFFFFE07FFFFFEull); }

// java.net.URI.Parser.parseIPv4Address/scanIPv4Address on [a,b) of the
// authority (JDK 8); returns end or -1.  One forward pass: up to four
// dot-separated octets of at most 9 digits (Integer.parseInt), each <= 255,
// then neither another digit/'.' nor anything but ':'.
template <typename LN>
__host__ __device__ LP_INLINE int jdk_ipv4(const LN& L, int a, int b) {
    Fwd<LN> cur(L, a);
    int p = a;
    for (int o = 0; o < 4; ++o) {
        int q = p;
        uint32_t v = 0;
        uint32_t c = 0;
        while (q < b && is_digit(c = cur.at(q))) {
            if (v < 1000) v = v * 10 + (c - '0');
            ++q;
        }
        if (q <= p || q - p > 9 || v > 255) return -1;
        p = q;
        if (o < 3) {
            if (p >= b || c != '.') return -1;
            ++p;
        } else if (p < b && c != ':') {
            return -1;  // a '.' continues the digit/dot run (scanIPv4Address fails); else not ':'
        }
    }
    return p;
}

// java.net.URI.Parser.parseHostname on [a,b) (labels alnum (alnum | '-')*
// not ending in '-', separated by '.', a trailing '.' allowed, the last
// label starting with a letter when there are several, then ':' or the end),
// one SWAR scan for the first byte outside alnum / '-' / '.' and one per
// label for its '.'.  Returns end or -1 (fail).
template <typename LN>
__host__ __device__ LP_INLINE int jdk_hostname_swar(const LN& L, int a, int b) {
    const int he = find_fwd(L, a, b, [](uint32_t w) {
        const uint32_t alnum = swar::digit(w) | (swar::ge(w, 'A') & swar::lt(w, 'Z' + 1)) |
                               (swar::ge(w, 'a') & swar::lt(w, 'z' + 1));
        return ~(alnum | swar::eq(w, '-') | swar::eq(w, '.')) & swar::HI;
    });
    int p = a, l = -1;
    while (p < he) {
        if (!is_alnum(L[p])) return -1;  // a label starts with '.' or '-'
        l = p;
        const int q = find_fwd(L, p, he, [](uint32_t w) { return swar::eq(w, '.'); });
        if (L[q - 1] == '-') return -1;
        p = q < he ? q + 1 : he;
    }
    if (he < b && L[he] != ':') return -1;
    if (l < 0) return -1;
    if (l > a && !is_alpha(L[l])) return -1;
    return he;
}

// jdk_hostname_swar for an authority of at most 32 bytes: its bytes' classes
// as 32-bit masks (one word load per 4 bytes, all issued together), then the
// label rules as bit operations: every label start (a, and after each '.')
// alnum, every label end (before each '.', and the last byte unless it is a
// '.') not '-', the last label starting with a letter when there are several.
// Longer authorities take jdk_hostname_swar.
template <typename LN>
__host__ __device__ LP_INLINE int jdk_hostname_m32(const LN& L, int a, int b) {
    const int len = b - a;
    if (len > 32) return jdk_hostname_swar(L, a, b);
    const uint32_t A = L.o + (uint32_t)a, W0 = A >> 2, sh = A & 3;
    const int nw = (int)(((A & 3) + (uint32_t)len + 3) >> 2);  // aligned words holding the bytes
    uint32_t w[9];
    LP_UNROLL for (int j = 0; j < 9; ++j) w[j] = j < nw ? L.word(W0 + (uint32_t)j) : 0u;
    uint32_t alnum = 0, alpha = 0, dot = 0, dash = 0;
    LP_UNROLL for (int j = 0; j < 8; ++j) {
#if defined(__HIP_DEVICE_COMPILE__)
        const uint32_t x = __builtin_amdgcn_alignbyte(w[j + 1], w[j], sh);
#else
        const uint32_t x = (uint32_t)((((uint64_t)w[j + 1] << 32) | w[j]) >> (8 * sh));
#endif
        const uint32_t l = x | 0x20202020u;
        const uint32_t al = swar::ge(l, 'a') & swar::lt(l, 'z' + 1) & ~(x & swar::HI);
        alpha |= bcls::nib(al) << (4 * j);
        alnum |= bcls::nib(al | swar::digit(x)) << (4 * j);
        dot |= bcls::nib(swar::eq(x, '.')) << (4 * j);
        dash |= bcls::nib(swar::eq(x, '-')) << (4 * j);
    }
    const uint32_t valid = len == 32 ? ~0u : (1u << len) - 1u;
    const uint32_t other = ~(alnum | dot | dash) & valid;
    const int he = other ? __builtin_ctz(other) : len;  // first byte outside alnum / '-' / '.'
    if (he == 0) return -1;                            // no label
    const uint32_t range = he == 32 ? ~0u : (1u << he) - 1u;
    const uint32_t d = dot & range;
    const uint32_t starts = (1u | (d << 1)) & range;
    if (starts & ~alnum) return -1;                    // a label starts with '.' or '-'
    const uint32_t ends = (d >> 1) | (((d >> (he - 1)) & 1u) ? 0u : 1u << (he - 1));
    if (ends & dash) return -1;                        // a label ends with '-'
    if (he < len && L[a + he] != ':') return -1;
    const int l = 31 - __builtin_clz(starts);          // the last label's start
    if (l > 0 && !((alpha >> l) & 1u)) return -1;
    return a + he;
}

// java.net.URI.Parser.parseHostname on [a,b); returns end or -1 (fail)
template <typename LN>
__host__ __device__ LP_INLINE int jdk_hostname(const LN& L, int a, int b) {
    Fwd<LN> cur(L, a);
    int p = a, l = -1;
    uint32_t l0 = 0;  // first char of the last label
    uint32_t c = p < b ? cur.at(p) : 0u;
    do {
        // label: alnum (alnum | '-')*, not ending in '-'
        if (!(p < b && is_alnum(c))) break;
        l = p;
        l0 = c;
        uint32_t last = c;
        ++p;
        while (p < b && (is_alnum(c = cur.at(p)) || c == '-')) {
            last = c;
            ++p;
        }
        if (last == '-') return -1;
        if (!(p < b && c == '.')) break;
        ++p;
        c = p < b ? cur.at(p) : 0u;
    } while (p < b);
    if (p < b && c != ':') return -1;
    if (l < 0) return -1;
    if (l > a && !is_alpha(l0)) return -1;
    return p;
}

// strict UTF-8 validation of a decoded byte string
template <typename BP>
__host__ __device__ LP_INLINE bool utf8_ok(BP b, uint32_t n) {
    for (uint32_t i = 0; i < n;) {
        uint32_t c = b[i];
        if (c < 0x80) { ++i; continue; }
        int need;
        uint32_t cp;
        if (c >= 0xC2 && c <= 0xDF) { need = 1; cp = c & 0x1F; }
        else if (c >= 0xE0 && c <= 0xEF) { need = 2; cp = c & 0x0F; }
        else if (c >= 0xF0 && c <= 0xF4) { need = 3; cp = c & 0x07; }
        else return false;
        if (i + (uint32_t)need >= n) return false;
        for (int r = 1; r <= need; ++r) {
            if ((b[i + r] & 0xC0) != 0x80) return false;
            cp = (cp << 6) | (b[i + r] & 0x3F);
        }
        if (need == 2 && (cp < 0x800 || (cp >= 0xD800 && cp <= 0xDFFF))) return false;
        if (need == 3 && (cp < 0x10000 || cp > 0x10FFFF)) return false;
        i += need + 1;
    }
    return true;
}

// java.net.URI.decode of [a,b) of the line (holds a '%'; escapes proven
// valid): returns an arena ref, or ~0 on FALLBACK.
template <typename LN>
__host__ __device__ LP_INLINE uint64_t decode_span(const LN& L, int a, int b, Arena& A) {
    uint32_t start = A.used;
    for (int q = a; q < b;) {
        uint32_t c = L[q];
        if (c == '%') { A.put(hexv(L[q + 1]) * 16 + hexv(L[q + 2])); q += 3; }
        else { A.put(c); ++q; }
    }
    if (!utf8_ok(A.p + start, A.used - start)) return ~0ull;
    return mkref(start, A.used - start, true);
}

__host__ __device__ LP_INLINE void put_encoded(Arena& A, uint32_t c) {
    const char* HX = "0123456789ABCDEF";
    A.put('%');
    A.put(HX[c >> 4]);
    A.put(HX[c & 15]);
}

// Utils.resilientUrlDecode of line bytes [vs, e) into the arena: every '%'
// here is followed by two hex digits (URI stage guard), so each %XX is the
// Latin-1 char U+00XX (VALID_STANDARD -> %00%XX, UTF-16 decode), '+' is a
// space, and URIUtil escapes decode back to their byte.  Output UTF-8.
// Bytes come from a two-word register window (one LDS read per 4 bytes).
// Output is gathered into 32-bit words, one aligned word store per 4 bytes
// (A.used is 4-byte aligned: spilled pieces are; the last word's padding
// bytes lie inside the spilled piece).  Each outer step produces at least 4
// bytes on every lane still decoding, so the lanes of a wave issue their word
// stores together instead of one byte store per lane and byte.
__host__ __device__ LP_INLINE void store_word(LP_G uint8_t* p, uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
    *reinterpret_cast<LP_G uint32_t*>(p) = v;
#else
    __builtin_memcpy(p, &v, 4);
#endif
}
template <typename LN>
__host__ __device__ LP_INLINE uint64_t url_decode_value(const LN& L, int vs, int e, Arena& A) {
    const uint32_t st = A.used;
    uint32_t W = (L.o + (uint32_t)vs) >> 2;
    uint64_t ww = (uint64_t)L.word(W) | ((uint64_t)L.word_or0(W + 1) << 32);
    uint64_t acc = 0;  // pending output bytes (na of them)
    uint32_t na = 0, out = st;
    for (int q = vs; q < e;) {
        while (na < 4 && q < e) {
            const uint32_t k = L.o + (uint32_t)q - 4 * W;  // 0..3
            const uint32_t c = (uint32_t)(ww >> (8 * k)) & 0xFFu;
            if (c == '%') {
                const uint32_t v =
                    hexv((uint32_t)(ww >> (8 * k + 8)) & 0xFFu) * 16 + hexv((uint32_t)(ww >> (8 * k + 16)) & 0xFFu);
                if (v < 0x80) { acc |= (uint64_t)v << (8 * na); na += 1; }
                else { acc |= (uint64_t)((0xC0 | (v >> 6)) | ((0x80 | (v & 0x3F)) << 8)) << (8 * na); na += 2; }
                q += 3;
            } else {
                acc |= (uint64_t)(c == '+' ? ' ' : c) << (8 * na);
                na += 1;
                ++q;
            }
            if (L.o + (uint32_t)q >= 4 * (W + 1)) {
                ++W;
                ww = (ww >> 32) | ((uint64_t)L.word_or0(W + 1) << 32);
            }
        }
        store_word(A.p + out, (uint32_t)acc);
        if (na >= 4) { out += 4; na -= 4; acc >>= 32; }
        else { out += na; na = 0; acc = 0; }
    }
    if (na) { store_word(A.p + out, (uint32_t)acc); out += na; }
    A.used = out;
    return mkref(st, A.used - st, true);
}

// ---- QueryStringFieldDissector (QueryStringFieldDissector.java:56-108).
// The URI stage's event pass splits the rawQuery at '&' / '?' into a table of
// one 16-byte slot per non-empty piece, noting for each piece its last '%' /
// '+' (a value that may need decoding): slot[0] = start | end << 16 |
// (lp + 1) << 48.  The kernel completes the pieces of all 64 lines of a wave
// spread evenly over its lanes: query_prep (the first '=', what the
// completion spills), one spill allocation for a batch of pieces, then
// query_finish, which overwrites the slot with the (name, value) refs.
constexpr uint64_t REF_SKIP = ~0ull;  // slot of a piece whose name was not requested

struct QueryTable {
    uint32_t tab = 0, reg = 0, count = 0, maxp = 0;
    int s = 0;
    int lp = -1;  // last '%' / '+' of the piece (a value that needs resilientUrlDecode)
    bool on = false, set = false;  // enumerating now / table laid out
    // piece [s, e) ends: its slot gets the raw piece (bounds, the last '%' /
    // '+'); one 16-byte store per slot (tables are 16-byte aligned: regions are)
    __host__ __device__ LP_INLINE void emit(LP_G uint8_t* region, int e) {
        if (e > s) {
            const uint64_t t0 = (uint64_t)(uint32_t)s | ((uint64_t)(uint32_t)e << 16) | ((uint64_t)(uint32_t)(lp + 1) << 48);
#if defined(__HIP_DEVICE_COMPILE__)
            typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
            *reinterpret_cast<LP_G u32x4_t*>(region + tab + 16 * count) = u32x4_t{(uint32_t)t0, (uint32_t)(t0 >> 32), 0u, 0u};
#else
            LP_G uint64_t* t = (LP_G uint64_t*)(region + tab) + 2 * count;
            t[0] = t0;
            t[1] = 0;
#endif
            ++count;
        }
        lp = -1;
    }
};

// First '=' of [s, e) (-1 if none) and whether the name before it (the
// whole piece without one) holds upper-case or URIUtil-escaped bytes: one
// pass over the piece's words.
template <typename LN>
__host__ __device__ LP_INLINE int piece_eq_rw(const LN& L, int s, int e, bool& rw) {
    rw = false;
    if (s >= e) return -1;
    const uint32_t A = L.o + (uint32_t)s, E = L.o + (uint32_t)e;
    uint32_t W = A >> 2;
    uint32_t valid = swar::HI << (8 * (A & 3));
    for (;;) {
        const uint32_t w = L.word(W);
        const uint32_t r = E - 4 * W;  // bytes of this word before E (>= 1)
        if (r < 4) valid &= swar::HI >> (8 * (4 - r));
        const uint32_t meq = swar::eq(w, '=') & valid;
        const uint32_t mrw = (swar::upper(w) | swar::needs_encode(w)) & valid;
        if (meq) {
            rw = rw || (mrw & ((meq & (0u - meq)) - 1u)) != 0;  // name bytes before the '='
            return (int)(4 * W + (uint32_t)swar::first(meq) - L.o);
        }
        rw = rw || mrw != 0;
        ++W;
        if (4 * W >= E) return -1;
        valid = swar::HI;
    }
}

// A query piece's split (QueryStringFieldDissector.java:75-104): bounds from
// its table slot word t0, the first '=', and the arena bytes its completion
// may write (rewritten name: 3 per name byte; decoded value: at most its
// length).
struct QPrep {
    int s = 0, e = 0, eq = -1;
    bool rw = false, pv = false;
    uint32_t need = 0;
};
template <typename LN>
__host__ __device__ LP_INLINE QPrep query_prep(const LN& L, uint64_t t0) {
    QPrep q;
    q.s = (int)(t0 & 0xFFFFu);
    q.e = (int)((t0 >> 16) & 0xFFFFu);
    const int lp = (int)((t0 >> 48) & 0xFFFFu) - 1;  // the piece's last '%' / '+'
    q.eq = piece_eq_rw(L, q.s, q.e, q.rw);
    q.pv = q.eq >= 0 && lp > q.eq;  // '%' / '+' in the value
    const int ne = q.eq >= 0 ? q.eq : q.e;
    // (whole words: the decoder's last word store pads up to 3 bytes)
    q.need = (q.rw ? (3u * (uint32_t)(ne - q.s) + 3u) & ~3u : 0u) + (q.pv ? ((uint32_t)(q.e - q.eq - 1) + 3u) & ~3u : 0u);
    return q;
}

// Completes a query piece: the name is lower-cased and keeps URIUtil's
// escapes, never decoded; a piece without '=' has value ""; else the value
// goes through Utils.resilientUrlDecode.  A: the piece's spilled bytes
// (q.need of them, A.used 4-byte aligned, offsets relative to the owning
// line's region `region`); slot: the piece's table slot.  Returns the arena
// bytes written.
template <typename LN>
__host__ __device__ LP_INLINE uint32_t query_finish(const Program& P, const QueryStage& Q, const LN& L, Arena& A,
                                                    const LP_G uint8_t* region, LP_G uint64_t* slot, const QPrep& qp) {
    const int s = qp.s, e = qp.e, eq = qp.eq;
    const int ne = eq >= 0 ? eq : e;
    const uint32_t a1 = A.used;
    // name [s, ne): URIUtil-escaped and lower-cased as in the rawQuery
    uint64_t nref;
    if (qp.rw) {
        const char* HX = "0123456789abcdef";  // URIUtil's %XX, lower-cased with the name
        const uint32_t mark = A.used;
        for (int q = s; q < ne; ++q) {
            const uint32_t c = L[q];
            if (uri_needs_encode(c)) { A.put('%'); A.put(HX[c >> 4]); A.put(HX[c & 15]); }
            else A.put((c - 'A') < 26u ? (c | 32) : c);
        }
        nref = mkref(mark, A.used - mark, true);
        A.used = (A.used + 3) & ~3u;  // the value's words start aligned
    } else {
        nref = src_ref(L, s, ne - s);
    }
    // requested?  (wantAllFields || requestedParameters.contains(name))
    bool want = Q.want_all;
    const uint32_t nlen = ref_len(nref);
    for (int k = 0; k < Q.n_names && !want; ++k) {
        if (Q.name_len[k] != nlen) continue;
        bool same = true;
        for (uint32_t q = 0; q < nlen && same; ++q) {
            const uint32_t c = qp.rw ? (uint32_t)region[ref_off(nref) + q] : L[s + (int)q];
            same = c == P.lit_byte((int)(Q.name_off[k] + q));
        }
        want = same;
    }
    if (!want) {
        slot[0] = REF_SKIP;
        slot[1] = 0;
        return A.used - a1;
    }
    uint64_t vref;
    if (eq < 0) vref = mkref(0, 0, false);  // no '=' -> ""
    else if (!qp.pv) vref = src_ref(L, eq + 1, e - eq - 1);
    else vref = url_decode_value(L, eq + 1, e, A);
    slot[0] = nref;
    slot[1] = vref;
    return A.used - a1;
}

// One query piece, its bytes spilled on its own (the test-only CPU
// emulation; the kernel allocates the spills of a whole round of pieces at
// once).  R: the owning line's arena region.  R.ovf when a spill did not fit.
template <typename LN>
__host__ __device__ LP_INLINE uint32_t query_piece(const Program& P, const QueryStage& Q, const LN& L, Arena& R,
                                                   LP_G uint64_t* slot) {
    const QPrep qp = query_prep(L, slot[0]);
    Arena A;
    if (!spill(R, qp.need, A)) {
        slot[0] = REF_SKIP;
        slot[1] = 0;
        return 0;
    }
    return query_finish(P, Q, L, A, R.p, slot, qp);
}

// State of HttpUriDissector's walk over a URI's event bytes (uri_stage): the
// guards' positions, the rawQuery rewrite bits and the query table being
// laid out.  The fast walk (uri_walk_fast, or the wave-cooperative walk of
// the URI kernel) takes the events up to the first '#', ';', non-ASCII byte
// or invalid escape; uri_stage_rest continues from there (resume).
struct UriWalk {
    int fa = -1, h = -1, nh = 0, first_pct = -1;
    // bit 0: the fragment holds '%' '?' or '&' (decoded / rewritten, not a plain span);
    // bit 1: the rawQuery is not "&" + the bytes between the first '&'/'?' and the '#'
    uint32_t rewr = 0;
    int resume = -1;
    QueryTable T;
};

// The fast walk of URI stage u over [a,b): the events before the first '#',
// ';', non-ASCII byte or invalid escape (the common bytes % & ? + and
// URIUtil-escaped ones, few branches).  A: the line's region (the query
// table starts at its next 16-byte boundary).
template <typename LN>
__host__ __device__ LP_INLINE void uri_walk_fast(const Program& P, int u, const LN& L, int a, int b, uint32_t usep,
                                                 Arena& A, UriWalk& Wk) {
    const UriStage& U = P.uri[u];
    const int qsi = U.want_query ? U.query_stage : -1;
    QueryTable& T = Wk.T;
    int& fa = Wk.fa;
    int& first_pct = Wk.first_pct;
    uint32_t& rewr = Wk.rewr;
    int& resume = Wk.resume;
    LP_PROF(50 + 4 * u);
    for_uev_w(L, a, b, [&](int q, uint32_t w) {
        const uint32_t c = w & 0xFFu;
        if (c == '#' || c == ';' || c >= 0x80) { resume = q; return false; }
        if (c == '%') {
            if (q + 2 >= b || !is_hex((w >> 8) & 0xFFu) || !is_hex((w >> 16) & 0xFFu)) { resume = q; return false; }
            first_pct = first_pct < 0 ? q : first_pct;
            T.lp = q;
            return true;
        }
        if (c == '&' || c == '?') {
            rewr |= (c == '?' && fa >= 0) ? 2u : 0u;  // a later '?' becomes '&'
            if (T.on) {
                T.emit(A.p, q);
                T.s = q + 1;
            } else if (fa < 0 && qsi >= 0) {
                T.on = T.set = true;
                T.maxp = usep + 1;
                T.tab = (A.used + 15) & ~15u;
                T.reg = T.tab + 16 * T.maxp;
                T.s = q + 1;
            }
            fa = fa < 0 ? q : fa;
            return true;
        }
        // '+' and URIUtil-escaped bytes
        rewr |= (fa >= 0 && uri_needs_encode(c)) ? 2u : 0u;
        T.lp = c == '+' ? q : T.lp;
        return true;
    });
    LP_PROF(51 + 4 * u);
}

// HttpUriDissector on the line bytes [a,b) after the fast walk: the general
// walk from Wk.resume, the query table's last piece, then the URI's parts.
// Returns status.
template <typename LN, typename Cols, typename UO>
__host__ __device__ LP_INLINE int uri_stage_rest(const Program& P, int u, const LN& L, int a, int b, uint32_t usep,
                                                 Arena& A, Cols& C, int64_t li, UO& o, UriWalk& Wk) {
    const UriStage& U = P.uri[u];
    const int qsi = U.want_query ? U.query_stage : -1;
    QueryTable& T = Wk.T;
    int& fa = Wk.fa;
    int& h = Wk.h;
    int& nh = Wk.nh;
    int& first_pct = Wk.first_pct;
    uint32_t& rewr = Wk.rewr;
    const int resume = Wk.resume;
    int st = ST_OK;
    if (resume >= 0) for_uev(L, resume, b, [&](int q, uint32_t c) {
        // non-ASCII: URIUtil.encode keeps the UTF-8 bytes raw and the
        // dissector reads them back as US-ASCII (U+FFFD each); not on the device
        if (c >= 0x80) { st = ST_FALLBACK; return false; }
        if (c == '%') {
            if (q + 2 >= b || !is_hex(L[q + 1]) || !is_hex(L[q + 2])) { st = ST_FALLBACK; return false; }  // BAD_EXCAPE_PATTERN
            if (first_pct < 0) first_pct = q;
            rewr |= h >= 0 ? 1u : 0u;
            if (T.on && h < 0) T.lp = q;
        } else if (c == '#') {
            ++nh;
            if (T.on && h < 0) {
                T.emit(A.p, q);
                T.on = false;  // the rawQuery ends at the first '#'
            }
            if (h < 0) h = q;
            if (q + 1 < b) {
                const uint32_t d = L[q + 1];
                if (d == '&' || d == '?' || d == 'x') { st = ST_FALLBACK; return false; }  // HASH_AMP, ALMOST_HTML_ENCODED
            }
            if (q > a && L[q - 1] == '=') { st = ST_FALLBACK; return false; }  // EQUALS_HASH
        } else if (c == ';') {
            // unescapeHtml4 candidate: [&?][a-zA-Z0-9#]*;
            int r = q - 1;
            while (r >= a && (is_alnum(L[r]) || L[r] == '#')) --r;
            if (r >= a && (L[r] == '&' || L[r] == '?')) { st = ST_FALLBACK; return false; }
        } else if (c == '&' || c == '?') {
            rewr |= (c == '?' && fa >= 0 && h < 0) ? 2u : 0u;  // a later '?' becomes '&'
            if (T.on) {
                T.emit(A.p, q);
                T.s = q + 1;
            } else if (fa < 0 && h < 0 && qsi >= 0) {
                // the rawQuery starts: table, pending list, piece regions
                T.on = T.set = true;
                T.maxp = usep + 1;
                T.tab = (A.used + 15) & ~15u;
                T.reg = T.tab + 16 * T.maxp;
                T.s = q + 1;
            }
            if (fa < 0) fa = q;
            rewr |= h >= 0 ? 1u : 0u;
        } else {  // '+' and URIUtil-escaped bytes
            const bool enc = uri_needs_encode(c);
            rewr |= (fa >= 0 && h < 0 && enc) ? 2u : 0u;  // URIUtil escapes it
            if (T.on && c == '+') T.lp = q;
        }
        return true;
    });
    LP_PROF(52 + 4 * u);
    if (st != ST_OK) return st;
    if (T.set) {
        if (T.on) T.emit(A.p, b);
        A.used = T.reg;
        A.slack += 16 * (T.maxp - T.count);  // unused slots
        C.q_count[qsi][li] = T.count;
        C.q_params[qsi][li] = mkref(T.tab, 16 * T.count, true);
        o.qlist.set(qsi, T.tab);
        o.qpend.set(qsi, T.count);
    }
    LP_PROF(30 + 8 * u);
    if (nh > 1) return ST_FALLBACK;                                                       // DOUBLE_HASH
    int pend = b;                              // end of path: first '?'(=fa) or '#'
    if (fa >= 0 && fa < pend) pend = fa;
    if (h >= 0 && h < pend) pend = h;
    uint32_t flags = UF_DONE | UF_PATH;
    int ps;                                    // path start
    int64_t scheme_ref = 0, host_ref = 0;
    int32_t port = -1;
    if (L[a] == '/') {
        ps = a;                                // "dummy-protocol://dummy.host.name" + uri
    } else {
        flags |= UF_IS_URL;
        // scheme: ':' before any of "/?#" (in the normalized string '?' is at fa)
        Fwd<LN> cur(L, a);
        bool sch_ok = true;
        int p = a;
        uint32_t c = 0;
        // "http://" / "https://" (no '&' / '?' among them: fa lies beyond)
        const uint32_t s0 = b - a >= 8 ? load_u32_at(L, a) : 0u, s1 = b - a >= 8 ? load_u32_at(L, a + 4) : 0u;
        if (s0 == 0x70747468u /* "http" */ && (s1 & 0xFFFFFFu) == 0x2F2F3Au /* "://" */) {
            p = a + 4;
            c = ':';
        } else if (s0 == 0x70747468u && s1 == 0x2F2F3A73u /* "s://" */) {
            p = a + 5;
            c = ':';
        } else {
            sch_ok = is_alpha(cur.at(a));
            while (p < b && p != fa) {
                c = cur.at(p);
                if (c == ':' || c == '/' || c == '#') break;
                sch_ok = sch_ok && scheme_char(c);
                ++p;
            }
        }
        LP_PROF(43);
        if (p < b && p != fa && c == ':') {
            if (p == a || !sch_ok) return ST_BAD;                                          // URISyntaxException
            flags |= UF_SCHEME;
            scheme_ref = (int64_t)src_ref(L, a, p - a);
            ++p;
            if (!(p < b && cur.at(p) == '/')) return ST_FALLBACK;                          // opaque URI
            if (p + 1 < b && cur.at(p + 1) == '/') {
                // authority [as, ae): up to '/', '#' or the first '?'; only chars
                // in both L_SERVER and L_REG_NAME of java.net.URI (no '@'
                // userinfo, no escapes), else FALLBACK
                const int as = p + 2;
                const int ae = find_fwd(L, as, b, [](uint32_t w) { return bcls::uev_hb(bcls::nonauth_bits(w)); });
                if (ae < b && ae != fa && cur.at(ae) != '/' && cur.at(ae) != '#') return ST_FALLBACK;
                if (ae == as) return ST_FALLBACK;                                          // empty authority
                LP_PROF(44);
                // parseServer; any failure -> registry-based authority (host null)
                int he = jdk_ipv4(L, as, ae);
                LP_PROF(45);
                if (he <= as) he = jdk_hostname_m32(L, as, ae);
                LP_PROF(46);
                bool ok = he > as;
                int pt = -1;
                if (ok && he < ae) {
                    // ":" port digits up to the end of the authority
                    int q = he + 1;
                    if (q < ae) {
                        Fwd<LN> pc(L, q);
                        uint64_t v = 0;
                        for (int r = q; r < ae; ++r) {
                            const uint32_t d = pc.at(r);
                            if (!is_digit(d)) { ok = false; break; }
                            v = v * 10 + (d - '0');
                            if (v > 0x7FFFFFFFull) { ok = false; break; }
                        }
                        if (ok) pt = (int)v;
                    }
                }
                LP_PROF(47);
                if (ok) {
                    flags |= UF_HOST;
                    host_ref = (int64_t)src_ref(L, as, he - as);
                    if (pt >= 0) { flags |= UF_PORT; port = pt; }
                }
                ps = ae;
            } else {
                ps = p;                                                                    // "scheme:/path"
            }
        } else {
            ps = a;                                                                        // relative, no scheme
        }
    }
    if (pend < ps) pend = ps;
    LP_PROF(31 + 8 * u);
    // ---- outputs
    C.u_scheme[u][li] = (uint64_t)scheme_ref;
    C.u_host[u][li] = (uint64_t)host_ref;
    C.u_port[u][li] = port;
    if (U.want_path) {
        uint64_t r = src_ref(L, ps, pend - ps);
        if (first_pct >= 0 && first_pct < pend) {  // decoded: at most the escaped length
            Arena X;
            if (!spill(A, (uint32_t)(pend - ps), X)) return ST_FALLBACK;
            const uint32_t x0 = X.used;
            r = decode_span(L, ps, pend, X);
            A.extra += X.used - x0;
        }
        if (r == ~0ull) return ST_FALLBACK;
        C.u_path[u][li] = r;
    }
    LP_PROF(32 + 8 * u);
    if (U.want_query) {
        if (fa >= 0 && (h < 0 || fa < h)) {
            // rawQuery = "&" + normalized text up to '#': '?'->'&', URIUtil escapes
            flags |= UF_QUERY;
            const int qs0 = fa + 1, qe = h >= 0 ? h : b;
            // the ref is formed before the scan below: with it formed after,
            // the gfx950 build (ROCm 7.2, -O3) delivered a wrong offset on
            // lanes whose scan ran an extra word (parity tests caught it)
            const uint64_t amp_ref = src_ref(L, qs0, qe - qs0) | REF_AMP;
            if (!(rewr & 2u)) {
                C.u_query[u][li] = amp_ref;
            } else {
                Arena X;  // '&' + the query, URIUtil-escaped bytes tripled
                if (!spill(A, 1u + 3u * (uint32_t)(qe - qs0), X)) return ST_FALLBACK;
                const uint32_t st = X.used;
                X.put('&');
                for (int q = fa + 1; q < qe; ++q) {
                    uint32_t c = L[q];
                    if (c == '?') X.put('&');
                    else if (uri_needs_encode(c)) put_encoded(X, c);
                    else X.put(c);
                }
                A.extra += X.used - st;
                C.u_query[u][li] = mkref(st, X.used - st, true);
            }
        } else {
            C.u_query[u][li] = mkref(0, 0, true);
            if (U.query_stage >= 0) { C.q_count[U.query_stage][li] = 0; C.q_params[U.query_stage][li] = 0; }
        }
    }
    LP_PROF(33 + 8 * u);
    if (U.want_ref && h >= 0) {
        flags |= UF_FRAG;
        // fragment = decode(normalized text after '#')
        if (!(rewr & 1u)) C.u_frag[u][li] = src_ref(L, h + 1, b - h - 1);
        else {
            Arena X;  // the decoded fragment: at most one byte more than its text
            if (!spill(A, (uint32_t)(b - h), X)) return ST_FALLBACK;
            const uint32_t st = X.used;
            for (int q = h + 1; q < b;) {
                uint32_t c = L[q];
                if (q == fa) { X.put('?'); X.put('&'); ++q; }
                else if (c == '?') { X.put('&'); ++q; }
                else if (c == '%') { X.put(hexv(L[q + 1]) * 16 + hexv(L[q + 2])); q += 3; }
                else { X.put(c); ++q; }
            }
            A.extra += X.used - st;
            if (!utf8_ok(X.p + st, X.used - st)) return ST_FALLBACK;
            C.u_frag[u][li] = mkref(st, X.used - st, true);
        }
    }
    LP_PROF(34 + 8 * u);
    C.u_flags[u][li] = flags;
    return ST_OK;
}

// HttpUriDissector fast path on the line bytes [a,b).  Returns status.
template <typename LN, typename Cols, typename UO>
__host__ __device__ LP_INLINE int uri_stage(const Program& P, int u, const LN& L, int a, int b, uint32_t usep, Arena& A,
                                            Cols& C, int64_t li, UO& o) {
    UriWalk Wk;
    uri_walk_fast(P, u, L, a, b, usep, A, Wk);
    return uri_stage_rest(P, u, L, a, b, usep, A, C, li, o, Wk);
}

// The pending query pieces of one line, one after the other (the test-only
// CPU emulation; the kernel spreads them over the wave).  LQ(us): the line
// view of URI stage us.
template <typename LQ>
__host__ __device__ LP_INLINE void query_pieces_serial(const Program& P, LQ&& lq, const UriOut& o, Arena& A) {
    for (int qs = 0; qs < P.n_query; ++qs) {
        const auto L = lq(P.query[qs].uri);
        for (uint32_t k = 0; k < o.qpend.get(qs); ++k)
            A.extra += query_piece(P, P.query[qs], L, A, (LP_G uint64_t*)(A.p + o.qlist.get(qs) + 16 * k));
    }
}

// ---- Derived URI stages: a query parameter's value that a type remapping
// turned into an HTTP.URI (Parsable.addDissection, core/Parsable.java:160-176,
// re-adds the value under the new type; Parser.findUsefulDissectorsFromField,
// core/Parser.java:446-455, gave that type its dissectors).  They run after
// the query pieces of their source are complete (k_derived_lines), one line
// per lane, on the value's bytes in place: a line span, or the decoded
// value in the line's arena region.
//
// The source: the value of the line's one occurrence of the parameter.
// Returns 0 none (no such parameter, or an empty value: HttpUriDissector
// does nothing for an empty input, HttpUriDissector.java:134-136), 1 found
// (vref), 2 FALLBACK (two or more occurrences: each is dissected in turn).
template <typename Cols>
__host__ __device__ LP_INLINE int derived_source(const Program& P, const UriStage& U, const Cols& C, int64_t li,
                                                 const LP_G uint8_t* line, const LP_G uint8_t* region, uint64_t& vref) {
    const QueryStage& Q = P.query[U.src_q];
    const uint32_t cnt = C.q_count[U.src_q][li];
    if (cnt == 0) return 0;
    const LP_G uint64_t* t = reinterpret_cast<const LP_G uint64_t*>(region + ref_off(C.q_params[U.src_q][li]));
    const uint32_t no = Q.name_off[U.src_qname], nl = Q.name_len[U.src_qname];
    int found = 0;
    for (uint32_t k = 0; k < cnt; ++k) {
        const uint64_t nref = t[2 * k];
        if (nref == REF_SKIP || ref_len(nref) != nl) continue;
        const LP_G uint8_t* np = (ref_arena(nref) ? region : line) + ref_off(nref);
        bool same = true;
        for (uint32_t q = 0; q < nl && same; ++q) same = np[q] == P.lit_byte((int)(no + q));
        if (!same) continue;
        if (++found > 1) return 2;
        vref = t[2 * k + 1];
    }
    return found && ref_len(vref) > 0 ? 1 : 0;
}

// Derived stage u on source [a, b) of L: the URI stage, then its query
// pieces one after the other.  R: the line's region with the shard's spill
// allocator (the stage's query table and every rewritten part are spilled).
template <typename LN, typename Cols>
__host__ __device__ LP_INLINE int derived_stage(const Program& P, int u, const LN& L, int a, int b, Arena& R, Cols& C,
                                                int64_t li) {
    uint32_t usep;
    const uint32_t need = uri_need(P, u, L, a, b, usep);
    Arena X = R;
    if (need && !spill(R, need, X)) return ST_FALLBACK;
    UriOut o;
    o.qlist.fill(0);
    o.qpend.fill(0);
    o.status = ST_OK;
    int st = uri_stage(P, u, L, a, b, usep, X, C, li, o);
    const int qs = P.uri[u].query_stage;
    if (st == ST_OK && qs >= 0)
        for (uint32_t k = 0; k < o.qpend.get(qs); ++k)
            query_piece(P, P.query[qs], L, X, (LP_G uint64_t*)(X.p + o.qlist.get(qs) + 16 * k));
    if (X.ovf) R.ovf = true;
    return X.ovf ? ST_FALLBACK : st;
}

// The derived stages of one OK line of LogFormat fmt.  line: the line's
// bytes (4-byte aligned base lb, line start at lb + lo, n bytes), R: its
// region (see derived_stage).  Returns the line's status.
template <typename Cols>
__host__ __device__ LP_INLINE int derived_line(const Program& P, int fmt, const LP_G uint8_t* lb, uint32_t lo, int n,
                                               Arena& R, Cols& C, int64_t li) {
    for (int u = 0; u < P.n_uri; ++u) {
        const UriStage& U = P.uri[u];
        if (U.src_q < 0 || U.fmt != fmt) continue;
        uint64_t vref = 0;
        const int f = derived_source(P, U, C, li, lb + lo, R.p, vref);
        if (f == 2) return ST_FALLBACK;
        if (f == 0) {
            C.u_flags[u][li] = 0;
            if (U.query_stage >= 0) { C.q_count[U.query_stage][li] = 0; C.q_params[U.query_stage][li] = 0; }
            continue;
        }
        const uint32_t vo = ref_off(vref), vl = ref_len(vref);
        int st;
        if (ref_arena(vref)) {
            // the decoded value in the region: positions from its first byte
            const ArenaLineT<const LP_G uint8_t*> A{{R.p + (vo & ~3u), vo & 3u, (int)vl}, vo};
            st = derived_stage(P, u, A, 0, (int)vl, R, C, li);
        } else {
            const LineT<const LP_G uint8_t*> L{lb, lo, n};
            st = derived_stage(P, u, L, (int)vo, (int)(vo + vl), R, C, li);
        }
        if (st != ST_OK) return st;
    }
    return ST_OK;
}

// Phase 2 of one line (the URI kernel): the URI stages of its LogFormat.
// lu(u): the line view of stage u's source (holding at least [a, b)), with
// sp[u] = a | b << 16 (0: no source), usep[u] its event count.
template <typename LU, typename Cols, typename SP, typename UO>
__host__ __device__ LP_INLINE void phase2(const Program& P, int fmt, LU&& lu, const SP& sp, const SP& usep, UO& o,
                                          Arena& A, Cols& C, int64_t li) {
    const int nu = P.n_uri < SP::size ? P.n_uri : SP::size;  // the caller picked SP::size >= P.n_uri
    for (int u = 0; u < nu && o.status == ST_OK; ++u) {
        if (P.uri[u].fmt != fmt) continue;  // another LogFormat's URI: nothing to write
        const uint32_t s = sp.get(u);
        const int a = (int)(s & 0xFFFF), b = (int)(s >> 16);
        if (b <= a) {
            C.u_flags[u][li] = 0;
            if (P.uri[u].query_stage >= 0) { C.q_count[P.uri[u].query_stage][li] = 0; C.q_params[P.uri[u].query_stage][li] = 0; }
            continue;
        }
        LP_PROF(10 + 2 * u);
        const int st = uri_stage(P, u, lu(u), a, b, usep.get(u), A, C, li, o);
        LP_PROF(11 + 2 * u);
        if (st != ST_OK) o.status = st;
    }
}

// Final per-line column writes (status, tokens, first line).
template <typename Cols>
__host__ __device__ LP_INLINE void write_line(const Program& P, const LineOut& o, Cols& C, int64_t li) {
    C.status[li] = (uint8_t)o.status;
    if (o.status != ST_OK) return;
    o.caps.each([&](int k, uint32_t v) { if (k < P.n_tok) C.tok_span[k][li] = v; });
    C.tok_flags[li] = o.tok_flags;
    if (C.hist) C.hist[li] = o.hist;
    o.fl_kind.each([&](int f, uint32_t v) { if (f < P.n_fl) C.fl_kind[f][li] = v; });
    o.fl_method.each([&](int f, uint32_t v) { if (f < P.n_fl) C.fl_method[f][li] = v; });
    o.fl_uri.each([&](int f, uint32_t v) { if (f < P.n_fl) C.fl_uri[f][li] = v; });
    o.fl_proto.each([&](int f, uint32_t v) { if (f < P.n_fl) C.fl_proto[f][li] = v; });
    for (int t = 0; t < P.n_time; ++t) {
        if (!((o.tdone >> t) & 1u)) continue;
        C.t_epoch[t][li] = (int64_t)(((uint64_t)o.ep_hi.get(t) << 32) | o.ep_lo.get(t));
        C.t_local[t][li] = ((uint64_t)o.lo_hi.get(t) << 32) | o.lo_lo.get(t);
        C.t_utc[t][li] = ((uint64_t)o.ut_hi.get(t) << 32) | o.ut_lo.get(t);
        if (P.time[t].kind == TK_STRF) C.t_nano[t][li] = o.nano.get(t);
    }
    for (int sm = 0; sm < P.n_secms; ++sm)
        if ((o.smdone >> sm) & 1u) C.sm_ms[sm][li] = (int64_t)(((uint64_t)o.sm_hi.get(sm) << 32) | o.sm_lo.get(sm));
    for (int bs = 0; bs < P.n_binip; ++bs)
        if ((o.bipdone >> bs) & 1u) C.bip[bs][li] = o.bip.get(bs);
}

// ---- the upstream list stages of one OK line (phase 2, after its URI
// stages: the item tables follow the URI stages' tables in the line's
// region).  L: a view of the line holding at least the list tokens.
// list_need: the region bytes the line's lists take; list_fill writes the
// tables and the l_count / l_tab columns.
template <typename LN, typename Cols>
__host__ __device__ LP_INLINE uint32_t list_need(const Program& P, int fmt, const LN& L, const Cols& C, int64_t li) {
    uint32_t need = 0;
    for (int j = 0; j < P.n_list; ++j) {
        const ListStage& S = P.list[j];
        if (S.fmt != fmt) continue;
        const uint32_t sp = C.tok_span[S.tok][li];
        const int a = (int)(sp & 0xFFFFu), b = (int)(sp >> 16);
        TokReg T;
        const int n = tok_load(L, a, b, T) ? uplist_items_r(T, a, b, [](int, int, int, int, int) {})
                                           : uplist_items(L, a, b, [](int, int, int, int, int) {});
        if (n > 0) need += 8 + (uint32_t)n * (S.secms ? LIST_ENT_MS : LIST_ENT);
    }
    return need;
}
template <typename LN, typename Cols>
__host__ __device__ LP_INLINE bool list_fill(const Program& P, int fmt, const LN& L, Arena& A, Cols& C, int64_t li) {
    for (int j = 0; j < P.n_list; ++j) {
        const ListStage& S = P.list[j];
        if (S.fmt != fmt) continue;
        const uint32_t sp = C.tok_span[S.tok][li];
        const int a = (int)(sp & 0xFFFFu), b = (int)(sp >> 16);
        const uint32_t ent = S.secms ? LIST_ENT_MS : LIST_ENT;
        TokReg T;
        const bool reg = tok_load(L, a, b, T);  // (a short token: split from registers)
        const int n = reg ? uplist_items_r(T, a, b, [](int, int, int, int, int) {})
                          : uplist_items(L, a, b, [](int, int, int, int, int) {});
        if (n < 0) return false;
        const uint32_t off = (A.used + 7u) & ~7u;
        if (n > 0 && off + (uint32_t)n * ent > A.cap) return false;
        if (n > 0) A.used = off + (uint32_t)n * ent;
        LP_G uint8_t* tab = A.p + off;
        auto put = [&](int k, int va, int vb, int ra, int rb) {
            LP_G uint32_t* e32 = reinterpret_cast<LP_G uint32_t*>(tab + (uint32_t)k * ent);
            e32[0] = mkspan((uint32_t)va, (uint32_t)vb);
            e32[1] = mkspan((uint32_t)ra, (uint32_t)rb);
            if (S.secms) {
                LP_G int64_t* e64 = reinterpret_cast<LP_G int64_t*>(tab + (uint32_t)k * ent + 8);
                e64[0] = reg ? secms_value_r(T, va - a, vb - a) : secms_value(L, va, vb);
                e64[1] = reg ? secms_value_r(T, ra - a, rb - a) : secms_value(L, ra, rb);
            }
        };
        if (reg) uplist_items_r(T, a, b, put);
        else uplist_items(L, a, b, put);
        C.l_count[j][li] = (uint32_t)n;
        C.l_tab[j][li] = n > 0 ? mkref(off, (uint32_t)n * ent, true) : 0ull;
    }
    return true;
}

// ---- name / value pieces (PairStage): f(ns, ne, vs, ve, eq) for every
// piece of [a, b) in order (eq: the piece has a '='; [vs, ve) its value).
//   PK_COOKIE (RequestCookieListDissector.dissect, :79-110): Pattern("; ").split
//     (trailing empty pieces dropped), an empty piece skipped, name = the part
//     before the first '=' trimmed, value = the trimmed rest;
//   PK_QUERY (QueryStringFieldDissector.dissect, :76-108): split("&") (trailing
//     empty pieces dropped), an empty piece skipped, name = the part before the
//     first '=' (not trimmed), value = the rest.
// (Names are lower-cased and values resilientUrlDecode'd by the caller; the
// phase-1 guard proved them ASCII with every '%' before two hex digits.)
//   PK_SETC (ResponseSetCookieListDissector.dissect, :86-110): split(", ")
//     (trailing empty parts dropped); a part whose lower-cased "expires=" starts
//     within its last 15 chars ("expires=XXXXXXX".length()) waits and is joined
//     with the next part by ", " (a later such part replaces it; one left at the
//     end is dropped); each cookie string is named by HttpCookie.parse -- on the
//     Netscape branch the phase-1 guard setcookie_ok proved: the first
//     ';'-token's part before '=', trimmed -- and its value is the cookie string
//     itself ([vs, ve) = the joined parts, contiguous in the line).
template <typename LN, typename F>
__host__ __device__ LP_INLINE int setc_pieces(const LN& L, int a, int b, F&& f) {
    int t = b;
    while (t - a >= 2 && L[t - 2] == ',' && L[t - 1] == ' ') t -= 2;
    if (t == a) return 0;
    int k = 0, prev = -1;
    for (int s0 = a;;) {
        int e0 = s0;
        while (e0 < t && !(L[e0] == ',' && e0 + 1 < t && L[e0 + 1] == ' ')) ++e0;
        int ei = -1;
        for (int q = s0; q + 8 <= e0 && ei < 0; ++q)
            if ((L[q] | 32u) == 'e' && ci_lit_at(L, q, e0, "expires=")) ei = q - s0;
        if (ei >= 0 && (e0 - s0) - 15 < ei) {
            prev = s0;
        } else {
            const int cs = prev >= 0 ? prev : s0;
            prev = -1;
            int q = cs;
            while (q < e0 && L[q] == ';') ++q;
            int eq = q;
            while (eq < e0 && L[eq] != '=' && L[eq] != ';') ++eq;
            int ns = q, ne = eq;
            while (ns < ne && L[ns] <= ' ') ++ns;
            while (ne > ns && L[ne - 1] <= ' ') --ne;
            f(ns, ne, cs, e0, true);
            ++k;
        }
        if (e0 >= t) break;
        s0 = e0 + 2;
    }
    return k;
}
template <typename LN, typename F>
__host__ __device__ LP_INLINE int pair_pieces(const LN& L, int a, int b, int kind, F&& f) {
    if (kind == PK_SETC) return setc_pieces(L, a, b, f);
    const bool ck = kind == PK_COOKIE;
    auto is_sep = [&](int q, int e) { return ck ? sep_at(L, q, e, ';') : (q < e && L[q] == '&'); };
    const int sl = ck ? 2 : 1;
    bool any = false;
    for (int q = a; q < b && !any; ++q) any = is_sep(q, b);
    int t = b;
    if (any) {
        while (t - a >= sl && is_sep(t - sl, t)) t -= sl;
        if (t == a) return 0;
    }
    int k = 0;
    for (int s0 = a;;) {
        int e0 = s0;
        while (e0 < t && !is_sep(e0, t)) ++e0;
        if (e0 > s0) {
            int eq = s0;
            while (eq < e0 && L[eq] != '=') ++eq;
            int ns = s0, ne = eq, vs = eq < e0 ? eq + 1 : e0, ve = e0;
            if (ck) {
                while (ns < ne && L[ns] <= ' ') ++ns;
                while (ne > ns && L[ne - 1] <= ' ') --ne;
                while (vs < ve && L[vs] <= ' ') ++vs;
                while (ve > vs && L[ve - 1] <= ' ') --ve;
            }
            f(ns, ne, vs, ve, eq < e0);
            ++k;
        }
        if (e0 >= t) break;
        s0 = e0 + sl;
    }
    return k;
}
template <typename LN>
__host__ __device__ LP_INLINE bool has_upper(const LN& L, int a, int b) {
    for (int q = a; q < b; ++q)
        if (L[q] - 'A' < 26u) return true;
    return false;
}
template <typename LN>
__host__ __device__ LP_INLINE bool has_escape(const LN& L, int a, int b) {
    for (int q = a; q < b; ++q)
        if (L[q] == '%' || L[q] == '+') return true;
    return false;
}
// region bytes of the line's pair stages: the piece tables and the names /
// values they rewrite (a decoded value is never longer than its source)
template <typename LN, typename Cols>
__host__ __device__ LP_INLINE uint32_t pair_need(const Program& P, int fmt, const LN& L, const Cols& C, int64_t li) {
    uint32_t need = 0;
    for (int j = 0; j < P.n_pair; ++j) {
        const PairStage& S = P.pair[j];
        if (S.fmt != fmt || ((C.tok_flags[li] >> S.tok) & 1u)) continue;
        const uint32_t sp = C.tok_span[S.tok][li];
        uint32_t bytes = 0;
        const int n = pair_pieces(L, (int)(sp & 0xFFFFu), (int)(sp >> 16), S.kind, [&](int ns, int ne, int vs, int ve, bool) {
            if (has_upper(L, ns, ne)) bytes += (uint32_t)(ne - ns) + 3;
            if (S.kind != PK_SETC && has_escape(L, vs, ve)) bytes += (uint32_t)(ve - vs) + 3;
        });
        if (n > 0) need += 8 + 16 * (uint32_t)n + bytes;
    }
    return need;
}
template <typename LN, typename Cols>
__host__ __device__ LP_INLINE bool pair_fill(const Program& P, int fmt, const LN& L, Arena& A, Cols& C, int64_t li) {
    for (int j = 0; j < P.n_pair; ++j) {
        const PairStage& S = P.pair[j];
        if (S.fmt != fmt) continue;
        if ((C.tok_flags[li] >> S.tok) & 1u) {  // "-": null, nothing is dissected
            C.p_count[j][li] = 0;
            C.p_tab[j][li] = 0;
            continue;
        }
        const uint32_t sp = C.tok_span[S.tok][li];
        const int a = (int)(sp & 0xFFFFu), b = (int)(sp >> 16);
        const int n = pair_pieces(L, a, b, S.kind, [](int, int, int, int, bool) {});
        const uint32_t off = (A.used + 7u) & ~7u;
        if (n > 0) {
            if (off + 16u * (uint32_t)n > A.cap) return false;
            A.used = off + 16u * (uint32_t)n;
        }
        LP_G uint64_t* const tab = reinterpret_cast<LP_G uint64_t*>(A.p + off);
        bool ok = true;
        uint32_t k = 0;  // the piece's entry (an index: the table pointer stays fixed)
        pair_pieces(L, a, b, S.kind, [&](int ns, int ne, int vs, int ve, bool eq) {
            const uint32_t e = 2u * k++;
            if (!ok) return;
            uint64_t nref = src_ref(L, ns, ne - ns), vref = mkref(0, 0, false);
            if (has_upper(L, ns, ne)) {
                if (A.used + (uint32_t)(ne - ns) > A.cap) { ok = false; return; }
                const uint32_t st = A.used;
                for (int q = ns; q < ne; ++q) {
                    const uint32_t c = L[q];
                    A.put(c - 'A' < 26u ? (c | 32u) : c);
                }
                nref = mkref(st, A.used - st, true);
                A.used = (A.used + 3u) & ~3u;
            }
            if (eq) {
                if (S.kind != PK_SETC && has_escape(L, vs, ve)) {  // (a cookie string is not decoded)
                    if (A.used + (uint32_t)(ve - vs) + 3 > A.cap) { ok = false; return; }
                    vref = url_decode_value(L, vs, ve, A);
                    A.used = (A.used + 3u) & ~3u;
                } else {
                    vref = src_ref(L, vs, ve - vs);
                }
            }
            tab[e] = nref;
            tab[e + 1] = vref;
        });
        if (!ok) return false;
        C.p_count[j][li] = (uint32_t)n;
        C.p_tab[j][li] = n > 0 ? mkref(off, 16u * (uint32_t)n, true) : 0ull;
    }
    return true;
}

}  // namespace lp
