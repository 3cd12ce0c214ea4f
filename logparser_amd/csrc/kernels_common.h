// Device scaffolding shared by the gfx950 kernel translation units
// (kernels.hip: line index / counters / routing scan / histograms;
// parse.hip: the parse kernels; uri.hip: the URI kernels).  The per-line
// logic is lp_device.h; this header only holds the wave-level pieces around
// it (line windows, staging, terminator masks, per-wave counts).
#pragma once
#include <hip/hip_runtime.h>

#ifndef LP_KERNEL_TU
#define LP_KERNEL_TU 1  // device column pointers are global-memory pointers (lp_program.h)
#endif

#include <algorithm>

#include "kernels.h"
#include "lp_device.h"

namespace lp {
namespace {

constexpr int CHUNK = 64 * 1024;  // bytes per workgroup in the newline passes
constexpr int NL_THREADS = 256;   // 256 threads x 16 B x 16 iterations = 64 KiB
constexpr int PW = 64;            // lanes per wave = lines per parse wave

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// exact per-byte "== c" mask of a 32-bit word (high bit of each byte)
__device__ __forceinline__ uint32_t byte_eq(uint32_t w, uint32_t c4) {
    uint32_t x = w ^ c4;
    return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
}
__device__ __forceinline__ uint32_t bits16(uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3) {
    return bcls::nib(m0) | (bcls::nib(m1) << 4) | (bcls::nib(m2) << 8) | (bcls::nib(m3) << 12);
}

// Line terminators of the 16 bytes at pos as a 16-bit mask (bit k = byte k),
// Hadoop LineReader.readDefaultLine semantics (the reader behind
// LineRecordReader, ApacheHttpdLogfileRecordReader.java:57, 115): '\n', a
// '\r' not followed by '\n', and of "\r\n" the '\n' (the '\r' is then the
// last byte of the line's bytes and the parse kernels drop it).  Bytes at or
// past nbytes are not terminators; a '\r' as the buffer's last byte is.
__device__ __forceinline__ uint32_t term_bits(uint4 v, const uint8_t* p, uint64_t pos, uint64_t nbytes) {
    uint32_t lf = bits16(byte_eq(v.x, 0x0A0A0A0Au), byte_eq(v.y, 0x0A0A0A0Au), byte_eq(v.z, 0x0A0A0A0Au),
                         byte_eq(v.w, 0x0A0A0A0Au));
    uint32_t cr = bits16(byte_eq(v.x, 0x0D0D0D0Du), byte_eq(v.y, 0x0D0D0D0Du), byte_eq(v.z, 0x0D0D0D0Du),
                         byte_eq(v.w, 0x0D0D0D0Du));
    if (pos + 16 > nbytes) {  // zero bytes past the end match neither
        const uint32_t live = nbytes > pos ? (1u << (uint32_t)(nbytes - pos)) - 1u : 0u;
        lf &= live;
        cr &= live;
    }
    if (cr) {
        uint32_t next_lf = lf >> 1;  // byte k + 1 is '\n'
        if ((cr & 0x8000u) && pos + 16 < nbytes && p[pos + 16] == '\n') next_lf |= 0x8000u;
        cr &= ~next_lf;
    }
    return lf | cr;
}
__device__ __forceinline__ uint32_t term16(const uint8_t* p, uint64_t pos, uint64_t nbytes) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (pos + 16 <= nbytes && ((uintptr_t)(p + pos) & 15) == 0) {
        v = *reinterpret_cast<const uint4*>(p + pos);
    } else {
        uint32_t w[4] = {0, 0, 0, 0};
        for (uint64_t k = pos; k < pos + 16 && k < nbytes; ++k) w[(k - pos) >> 2] |= (uint32_t)p[k] << (8 * ((k - pos) & 3));
        v = make_uint4(w[0], w[1], w[2], w[3]);
    }
    return term_bits(v, p, pos, nbytes);
}

// This lane's index in its wave (0..63; the parse / URI kernels run one wave
// per workgroup, so it equals the workitem id x), from the hardware lane
// count (v_mbcnt) instead of the workitem-ID register.  ROCm 7.2 (gfx950)
// lost that register's value on some lanes across a non-inlined call made
// under a partial EXEC mask (Program::has_phase2 inside `if (row)` in the
// chunk kernel): the next callee (chunk_excess) then got wrong lane numbers,
// scanned the wrong pieces of its window and numbered fewer lines than the
// staging pass, leaving line_off entries unwritten (the round-5 aperture
// fault in k_parse_ovf_lines).  mbcnt does not depend on it.
__device__ __forceinline__ int lane_id() {
    return (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

struct WaveStack {  // per-lane DFS stack, lane-interleaved (conflict-free)
    uint32_t* base;
    __device__ uint32_t& operator[](int k) const { return base[k * PW]; }
};

// The line of lane `own` of this wave (for work on another lane's line).
template <typename LN>
__device__ __forceinline__ LN owner_line(const LN& L, int own) {
    LN R = L;
    R.o = (uint32_t)__shfl((int)L.o, own);
    R.n = __shfl(L.n, own);
    if constexpr (!LN::has_masks)  // HBM path: every lane has its own base
        R.b = reinterpret_cast<decltype(L.b)>(__shfl((unsigned long long)(uintptr_t)L.b, own));
    return R;
}

// Lines [li0, li0 + 64) of a wave: this lane's line [s, e) and the byte
// window [w0, w1) of all of them (w0 16-byte aligned).
struct WaveLines {
    int64_t li0, li, lend;
    bool active;
    uint64_t s, e, w0, w1;
    int n;
};
__device__ __forceinline__ WaveLines wave_lines(const Columns& C, int64_t wave, int64_t n_lines, uint64_t nbytes) {
    WaveLines W;
    W.li0 = wave * PW;
    W.li = W.li0 + (int64_t)lane_id();
    W.active = W.li < n_lines;
    W.lend = W.li0 + PW < n_lines ? W.li0 + PW : n_lines;
    W.s = W.e = 0;
    if (W.active) {
        W.s = C.line_off[W.li];
        W.e = C.line_off[W.li + 1] - 1;  // exclude the terminator (or the end sentinel); see crlf_len
    }
    W.n = (int)((W.e - W.s) > (uint64_t)0x7FFFFFFF ? 0x7FFFFFFF : (W.e - W.s));
    W.w0 = C.line_off[W.li0] & ~15ull;
    W.w1 = C.line_off[W.lend];
    if (W.w1 > nbytes) W.w1 = nbytes;
    return W;
}

// Length of a line whose last byte (before its terminator) is `last`: the
// '\r' of a "\r\n" terminator is not part of the line.  (A '\r' never is
// line content: not followed by '\n' it is itself a terminator, term16.)
__device__ __forceinline__ int crlf_len(int n, uint32_t last) { return n - (n > 0 && last == '\r' ? 1 : 0); }
__device__ __forceinline__ int crlf_len_hbm(const uint8_t* buf, const WaveLines& W) {
    return W.active ? crlf_len(W.n, W.n > 0 ? buf[W.e - 1] : 0u) : W.n;
}

// Stage [w0, w1) into win (LDS) and the mask planes into msk16 (two 64-bit
// planes per 64-byte block, as 16-bit pieces).  Returns whether every byte
// but the terminators is TAB or printable ASCII (then no line needs the
// guard scan of phase 1).
__device__ __forceinline__ bool stage_window(const uint8_t* __restrict__ buf, uint64_t nbytes, uint64_t w0, uint64_t w1,
                                             uint8_t* win, uint16_t* msk16) {
    const int lane = lane_id();
    const int nv = (int)((w1 - w0 + 15) >> 4);
    const int nv4 = (nv + 3) & ~3;  // whole 64-byte mask blocks
    uint32_t bad = 0;  // guard-failing bytes other than '\n' anywhere in the window
    // SB loads in flight per lane before the first LDS store (one HBM
    // round trip per SB x 1 KiB of window instead of one per 1 KiB)
    constexpr int SB = 20;
    const uint64_t full_end = nbytes & ~15ull;  // 16-byte pieces wholly inside the buffer
    for (int k0 = lane; k0 < nv4; k0 += SB * PW) {
        u32x4 v[SB];
#pragma unroll
        for (int j = 0; j < SB; ++j) {
            const int k = k0 + j * PW;
            const uint64_t p = w0 + 16ull * k;
            v[j] = u32x4{0, 0, 0, 0};
            if (k < nv && p + 16 <= full_end) v[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(buf + p));
        }
#pragma unroll
        for (int j = 0; j < SB; ++j) {
            const int k = k0 + j * PW;
            if (k >= nv4) continue;
            const uint64_t p = w0 + 16ull * k;
            if (k < nv && p + 16 > full_end) {  // the buffer's last partial piece
                auto word = [&](uint64_t q) {
                    uint32_t w = 0;
#pragma unroll
                    for (int b = 0; b < 4; ++b) w |= q + b < nbytes ? (uint32_t)buf[q + b] << (8 * b) : 0u;
                    return w;
                };
                v[j] = u32x4{word(p), word(p + 4), word(p + 8), word(p + 12)};
            }
            *reinterpret_cast<u32x4*>(win + 16 * k) = v[j];
            uint32_t m0, m1, g = 0, lf, other, cr;
            bcls::classify16p(v[j][0], v[j][1], v[j][2], v[j][3], m0, m1, g, lf, other);
            if (other) bcls::classify16c(v[j][0], v[j][1], v[j][2], v[j][3], g, cr);  // TAB, '\r', other controls
            if (k < nv) bad |= g;
            msk16[8 * (k >> 2) + (k & 3)] = (uint16_t)m0;
            msk16[8 * (k >> 2) + 4 + (k & 3)] = (uint16_t)m1;
        }
    }
    return !__any(bad != 0);
}

// Status counts of a wave's lines (lines, ok, bad, arena bytes written).
struct WaveCounts {
    uint32_t act = 0, ok = 0, bad = 0, written = 0;
    uint32_t gathered = 0;  // URI source bytes the URI kernel read (its roofline accounting)
    __device__ __forceinline__ void store(LP_G uint32_t* wave_counts, int64_t wave) const {
        if (lane_id() == 0) {
            uint4 c, d;
            c.x = act;
            c.y = ok;
            c.z = bad;
            c.w = act - ok - bad;
            d.x = written;
            d.y = gathered;
            d.z = d.w = 0;
            uint4* wc = reinterpret_cast<uint4*>(wave_counts + WC_WORDS * (size_t)wave);
            wc[0] = c;
            wc[1] = d;
        }
    }
    __device__ __forceinline__ void store(const Columns& C, int64_t wave) const { store(C.wave_counts, wave); }
};

// Phase 1 of one wave's lines (match, tokens, time, first line) and their
// rows; adds the lines' counts to WC.  The URI stages run in k_uri_lines.
template <bool MULTI, typename LN>
__device__ __forceinline__ void parse_wave(const Program& P, const Elem* elems, const Columns& C, const LN& L,
                                           bool active, int64_t li, WaveStack stk, bool clean, WaveCounts& WC) {
    LineOut o;
    o.status = ST_OK;
    LP_PROF(1);
    if (active) phase1<MULTI>(P, elems, L, o, stk, C, li, clean, P.n_fmt > 1 ? (int)C.fmt_id[li] : 0);
    LP_PROF(9);
    if (active) write_line(P, o, C, li);
    if (active && !P.has_phase2()) C.arena_base[li] = 0;  // no URI kernel: an empty region for every line
    WC.act += (uint32_t)__popcll(__ballot(active));
    WC.ok += (uint32_t)__popcll(__ballot(active && o.status == ST_OK));
    WC.bad += (uint32_t)__popcll(__ballot(active && o.status == ST_BAD));
}

// The 16 input bytes at p (16-byte aligned): one load inside the buffer,
// bytes past nbytes read as 0.
__device__ __forceinline__ u32x4 load16(const uint8_t* __restrict__ buf, uint64_t nbytes, uint64_t p) {
    if (p + 16 <= nbytes) return *reinterpret_cast<const u32x4*>(buf + p);
    uint32_t w[4] = {0, 0, 0, 0};
    for (int c = 0; c < 16; ++c) w[c >> 2] |= p + c < nbytes ? (uint32_t)buf[p + c] << (8 * (c & 3)) : 0u;
    return u32x4{w[0], w[1], w[2], w[3]};
}

// LDS: [elements (n_elems x 16 B)][DFS stack][...]
__device__ __forceinline__ void load_elems(const Program& P, Elem* s_elems) {
    for (int k = lane_id(); k < P.n_elems; k += PW) s_elems[k] = P.elems[k];
}

// k-th set bit (0-based) of m (k < popcount(m))
__device__ __forceinline__ uint32_t select64(uint64_t m, uint32_t k) {
    uint32_t pos = 0, v = (uint32_t)m, c = (uint32_t)__popc(v);
    if (k >= c) { k -= c; v = (uint32_t)(m >> 32); pos = 32; }
    c = (uint32_t)__popc(v & 0xFFFFu);
    if (k >= c) { k -= c; v >>= 16; pos += 16; }
    c = (uint32_t)__popc(v & 0xFFu);
    if (k >= c) { k -= c; v >>= 8; pos += 8; }
    c = (uint32_t)__popc(v & 0xFu);
    if (k >= c) { k -= c; v >>= 4; pos += 4; }
    c = (uint32_t)__popc(v & 3u);
    if (k >= c) { k -= c; v >>= 2; pos += 2; }
    return pos + (k >= (v & 1u) ? 1u : 0u);
}
__device__ __forceinline__ int lsb64(uint64_t m) { return (int)__builtin_ctzll(m); }
__device__ __forceinline__ int msb64(uint64_t m) { return 63 - (int)__builtin_clzll(m); }

// inclusive scan over the wave's lanes
template <typename T>
__device__ __forceinline__ T wave_incl_scan(T x) {
    const int lane = lane_id();
    for (int d = 1; d < 64; d <<= 1) {
        const T y = __shfl_up(x, d);
        if (lane >= d) x += y;
    }
    return x;
}
template <typename T>
__device__ __forceinline__ T wave_sum(T x) {
    for (int d = 32; d > 0; d >>= 1) x += __shfl_xor(x, d);
    return x;
}

}  // namespace
}  // namespace lp
