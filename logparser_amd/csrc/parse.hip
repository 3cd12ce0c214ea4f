// gfx950 parse kernels of the logparser_amd engine (phase 1: LogFormat match,
// token flags, time stamps, first line; lp_device.h phase1).
//
//   k_parse_chunks     one-format programs: the line index and phase 1 in ONE pass
//                      over the input.  One wave per byte chunk: the chunk's window
//                      (with the tail of its last line) staged in LDS with its class
//                      masks and line terminators, the lines starting in the chunk
//                      numbered by a decoupled look-back over the chunks' line
//                      counts, one lane per line
//   k_parse_ovf_lines  the lines a chunk could not take (more than 64 lines, or a
//                      line ending past its window): read from HBM directly
//   k_parse_lines      several LogFormats: one wave per 64 lines of the line index
//                      (kernels.hip) after the routing pass; the lines' window in LDS
//   k_parse_overflow   the waves k_parse_lines queued (windows LDS cannot hold)
//   k_route_match      several LogFormats: which formats match each line (sticky
//                      routing pass 1)
#include "kernels_common.h"

namespace lp {

namespace {

// ------------------------------------------------------------ chunked parse
// Reference: the caller loop of ApacheHttpdLogfileRecordReader.nextKeyValue
// (ApacheHttpdLogfileRecordReader.java:232-280) reads lines with Hadoop's
// LineRecordReader ('\n', lone '\r' and "\r\n" end a line, the terminator is
// not part of it, a last unterminated line counts; :57, 115) and hands each
// to Parser.parse.  Here the lines of a byte chunk are found by the wave that
// parses them: a line belongs to the chunk holding its first byte.

constexpr int MAXS = PW + 1;
#ifndef LP_CHUNK_MAXW
#define LP_CHUNK_MAXW 10  // waves per CU the chunk plan may size the LDS window for
#endif
#ifndef LP_CHUNK_LMAX
#define LP_CHUNK_LMAX 54  // lines per chunk at most (one-format programs)
#endif
#ifndef LP_MF_WPE
#define LP_MF_WPE 3  // waves per SIMD the several-format chunk instance is compiled for: 3 (168 VGPRs, a few
                     // spilled) measured 10 % faster parse kernels on config 5 than 2 (216 VGPRs), profiles/r06w/mfab
#endif
#ifndef LP_CHUNK_LMAX_MF
#define LP_CHUNK_LMAX_MF 58  // the same for several-format programs (VGPR-bound at 8 waves per CU: 58 measured 6 % faster than 54 on config 5)
#endif  // line starts a chunk keeps in LDS (its 64 lines and the next start)
constexpr uint64_t CS_AGG = 1ull << 62, CS_INC = 1ull << 63, CS_CNT = CS_AGG - 1;

// the line index, written by the chunked parse kernel (read-only elsewhere)
__device__ __forceinline__ LP_G uint64_t* line_off_w(const Columns& C) { return const_cast<LP_G uint64_t*>(C.line_off); }

// Self-checks of the chunked kernels' own bookkeeping.  A failed check is
// counted in Meta::err, the first failure's kind and values kept in
// Meta::err_info, and the batch fails (LP_E_DEVICE, the values on stderr)
// instead of a kernel reading a bad entry:
//   CHK_OVF_LINE  a queued line k_parse_ovf_lines cannot take: q, li, line_off[li], line_off[li + 1]
//   CHK_EXCESS    chunk_excess numbered a different count of lines than the staging pass: c, found, counted, base
//   CHK_QUEUE     a queue append past its capacity: queue (0 lines, 1 chunks), index, entry, capacity
constexpr uint64_t CHK_OVF_LINE = 1, CHK_EXCESS = 2, CHK_QUEUE = 3;
__device__ __forceinline__ void check_fail(const Columns& C, uint64_t kind, uint64_t a, uint64_t b, uint64_t c,
                                           uint64_t d) {
    if (atomicAdd(&C.meta->err, 1ull) == 0) {
        C.meta->err_info[0] = kind;
        C.meta->err_info[1] = a;
        C.meta->err_info[2] = b;
        C.meta->err_info[3] = c;
        C.meta->err_info[4] = d;
    }
}

// Append line li to the queue of k_parse_ovf_lines (cap_lines + 1 entries).
__device__ __forceinline__ void queue_line(const Columns& C, uint64_t li) {
    const uint64_t q = atomicAdd(&C.meta->ovf_lines, 1ull);
    if (q <= (uint64_t)C.cap_lines) C.ovf_lines[q] = (uint32_t)li;
    else check_fail(C, CHK_QUEUE, 0, q, li, (uint64_t)C.cap_lines + 1);
}

// set bits of the wave mask b held by the lanes below this one
__device__ __forceinline__ uint32_t below(uint64_t b) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
}

// What the staging pass of a chunk found: the lines starting in it, the first
// terminator at or after t_hi (the end of its last line), whether the window
// passed the byte guard.
struct ChunkScan {
    uint32_t count;
    uint64_t end_term;  // absolute position, ~0: none in the window
    bool clean;
};

// Stage the window [w0, w1) (w0 64-byte aligned) into LDS with its mask
// planes, as stage_window, and find the chunk's line starts: every
// terminator t in [t_lo, t_hi) starts a line at t + 1, numbered in order
// from `first` (1 when the chunk also holds the line starting at byte 0).
// starts[r] = window offset of the r-th start (r < MAXS).
//
// The bytes reach LDS by LDS-DMA (global_load_lds_dwordx4: 1 KiB per wave
// instruction, no registers held while they are in flight) when the window
// is whole 1 KiB blocks inside the buffer, else (the batch's last chunk) by
// plain loads; then one pass over the LDS copy classifies every 16 bytes
// into the two mask planes and the line terminators.
__device__ __forceinline__ ChunkScan stage_chunk(const uint8_t* __restrict__ buf, uint64_t nbytes, uint64_t w0,
                                                 uint64_t w1, uint64_t t_lo, uint64_t t_hi, uint32_t first,
                                                 uint8_t* win, uint16_t* msk16, uint32_t* starts) {
    const int lane = lane_id();
    const int nv = (int)((w1 - w0 + 15) >> 4);
    const int nv4 = (nv + 3) & ~3;  // whole 64-byte mask blocks
    if ((nv & (PW - 1)) == 0 && w0 + 16ull * nv <= (nbytes & ~15ull)) {
        for (int k0 = 0; k0 < nv; k0 += PW)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(buf + w0 + 16ull * (k0 + lane)),
                                             (__attribute__((address_space(3))) void*)(win + 16 * k0), 16, 0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        for (int k = lane; k < nv4; k += PW) {
            u32x4 v = u32x4{0, 0, 0, 0};
            if (k < nv) v = load16(buf, nbytes, w0 + 16ull * k);
            *reinterpret_cast<u32x4*>(win + 16 * k) = v;
        }
    }
    // window-relative 32-bit positions (a window is at most 48 KiB); the
    // rounds inside [t_lo, t_hi) and the input (all but the first and the
    // last) skip the boundary masks
    const uint32_t nrel = nbytes - w0 < 16ull * (uint64_t)(nv4 + 1) ? (uint32_t)(nbytes - w0) : 16u * (uint32_t)(nv4 + 1);
    const uint32_t tl = (uint32_t)(t_lo - w0), th = (uint32_t)(t_hi - w0);
    uint32_t bad = 0;
    uint32_t run = first;        // starts numbered so far (wave-uniform)
    uint32_t end_rel = ~0u;      // this lane's first terminator >= t_hi (relative)
    u32x4 vn = lane < nv4 ? *reinterpret_cast<const u32x4*>(win + 16 * lane) : u32x4{0, 0, 0, 0};
    for (int k0 = 0; k0 < nv4; k0 += PW) {  // wave-uniform rounds: every lane joins the ballots
        const int k = k0 + lane;
        const uint32_t q = 16u * (uint32_t)k;
        const uint32_t r0 = 16u * (uint32_t)k0, r1 = r0 + 16u * PW;
        const bool inner = r0 >= tl && r1 <= th && r1 <= nrel && k0 + PW <= nv;  // wave-uniform
        uint32_t tm = 0;
        const u32x4 v = vn;
        if (k + PW < nv4) vn = *reinterpret_cast<const u32x4*>(win + 16 * (k + PW));  // the next round's piece
        if (k < nv4) {
            uint32_t m0, m1, g = 0, lf, other;
            bcls::classify16p(v[0], v[1], v[2], v[3], m0, m1, g, lf, other);
            msk16[8 * (k >> 2) + (k & 3)] = (uint16_t)m0;
            msk16[8 * (k >> 2) + 4 + (k & 3)] = (uint16_t)m1;
            tm = lf;
            if (other) {  // TAB, '\r' or another control byte (rare): the exact guard and CR terminators
                uint32_t cr;
                bcls::classify16c(v[0], v[1], v[2], v[3], g, cr);
                if (cr) {
                    // "\r\n": the '\n' ends the line; a lone '\r' does (term_bits)
                    const uint64_t p = w0 + q;
                    uint32_t next_lf = lf >> 1;
                    if ((cr & 0x8000u) && p + 16 < nbytes && buf[p + 16] == '\n') next_lf |= 0x8000u;
                    tm |= cr & ~next_lf;
                }
            }
            if (inner) {
                bad |= g;
            } else {
                if (k < nv) bad |= g;
                if (q + 16 > nrel) tm &= nrel > q ? (1u << (nrel - q)) - 1u : 0u;
            }
        }
        // terminators in [t_lo, t_hi): line starts; the first at or after t_hi: the end
        uint32_t ms = tm;
        if (!inner) {
            uint32_t me = 0;
            if (q < tl) ms &= tl - q >= 16 ? 0u : ~0u << (tl - q);
            if (q + 16 > th) {
                const uint32_t lo = th > q ? (1u << (th - q)) - 1u : 0u;
                me = tm & ~lo;
                ms &= lo;
            }
            if (me) end_rel = min(end_rel, q + (uint32_t)__builtin_ctz(me));
        }
        // rank of this lane's first start in the round: the counts (0..16) of
        // the lanes below it, bit plane by bit plane (ballot + mbcnt; no
        // cross-lane permutes in the loop)
        const uint32_t c = (uint32_t)__popc(ms);
        const uint64_t b0 = __ballot(c & 1u), b1 = __ballot(c & 2u);
        uint32_t excl = below(b0) + 2 * below(b1);
        uint32_t tot = (uint32_t)(__popcll(b0) + 2 * __popcll(b1));
        const uint64_t bh = __ballot(c >= 4u);
        if (bh) {  // wave-uniform: a lane with 4 or more terminators in 16 bytes (short lines)
            const uint64_t b2 = __ballot(c & 4u), b3 = __ballot(c & 8u), b4 = __ballot(c & 16u);
            excl += 4 * below(b2) + 8 * below(b3) + 16 * below(b4);
            tot += (uint32_t)(4 * __popcll(b2) + 8 * __popcll(b3) + 16 * __popcll(b4));
        }
        uint32_t r = run + excl;
        run += tot;
        for (uint32_t m = ms; m; m &= m - 1, ++r)
            if (r < (uint32_t)MAXS) starts[r] = q + (uint32_t)__builtin_ctz(m) + 1u;
    }
    ChunkScan S;
    S.count = run;
    // wave minimum of the end terminator
    for (int d = 32; d > 0; d >>= 1) end_rel = min(end_rel, (uint32_t)__shfl_xor((int)end_rel, d));
    S.end_term = end_rel == ~0u ? ~0ull : w0 + end_rel;
    S.clean = !__any(bad != 0);
    return S;
}

// The chunks' line numbers.  Chunk c's wave publishes its line count (an
// aggregate) right after staging, without waiting for anything; one scanner
// wave (block 0 of the launch) walks the chunks in order, 512 state words
// per round, and turns every published aggregate into the inclusive prefix;
// chunk c's wave reads its prefix back after phase 1, by when the scanner has
// long passed it.  The scanner only waits for chunks dispatched before the
// ones it has reached, and those publish without waiting, so every wait
// ends.  Each state word is one 8-byte value (status bits and count), stored
// and polled with agent-scope (sc1) accesses: no payload travels beside it.
__device__ __forceinline__ void chunk_publish(LP_G uint64_t* st, int64_t c, uint64_t count) {
    if (lane_id() == 0) __hip_atomic_store(&st[c], CS_AGG | count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __noinline__ void chunk_scanner(LP_G uint64_t* st, int64_t n_chunks) {
    constexpr int PER = 8;  // state words per lane per round
    const int lane = lane_id();
    uint64_t run = 0;
    int64_t c = 0;
    while (c < n_chunks) {
        uint64_t v[PER];
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int64_t idx = c + PER * lane + i;
            v[i] = idx < n_chunks ? __hip_atomic_load(&st[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
        }
        // this lane's leading published words and their line count
        int pub = 0;
        uint64_t sum = 0;
        bool stop = false;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            stop = stop || !(v[i] & CS_AGG);
            if (!stop) { sum += v[i] & CS_CNT; ++pub; }
        }
        const uint64_t full = __ballot(pub == PER);
        const int L = full == ~0ull ? PW : (int)__builtin_ctzll(~full);  // the first lane with a gap
        const uint64_t mine = lane <= L ? sum : 0ull;
        const uint64_t incl = wave_incl_scan(mine);
        const uint64_t total = __shfl(incl, PW - 1);
        const int pub_L = L < PW ? __shfl(pub, L) : 0;
        if (lane <= L) {
            uint64_t r = run + incl - mine;
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                if (i >= pub) break;
                r += v[i] & CS_CNT;
                __hip_atomic_store(&st[c + PER * lane + i], CS_INC | r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        const int64_t adv = (int64_t)L * PER + pub_L;
        run += total;
        c += adv;
        if (adv == 0) __builtin_amdgcn_s_sleep(8);
    }
}

// chunk c's first line number (the scanner's prefix minus the chunk's own
// count), or ~0 when the scanner has not reached the chunk after
// CHUNK_WAIT_MAX polls (~10 ms; in a normal launch it has long passed it):
// the wave then leaves the chunk to the deferred pass instead of waiting on,
// so that no wait depends on the order in which the dispatcher starts the
// workgroups (a chunk whose wave was never started cannot hold the others).
// (wait_max: LP_OPT_CHUNK_WAIT, tests; 0 = CHUNK_WAIT_MAX, -1 = defer
// without polling, -2 = defer the odd chunks without polling, the even ones
// as normal: finished and deferred chunks side by side, deterministically)
constexpr uint32_t CHUNK_WAIT_MAX = 1u << 14;
__device__ __forceinline__ uint64_t chunk_base(LP_G uint64_t* st, int64_t c, uint64_t count, int wait_max) {
    if (wait_max < 0 && (wait_max != -2 || (c & 1))) return ~0ull;
    uint64_t v = 0;
    const uint32_t lim = wait_max <= 0 ? CHUNK_WAIT_MAX : (uint32_t)wait_max;
    if (lane_id() == 0) {
        for (uint32_t it = 0;; ++it) {
            v = __hip_atomic_load(&st[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (v & CS_INC) break;
            if (it >= lim) { v = ~0ull; break; }
            __builtin_amdgcn_s_sleep(4);
        }
    }
    v = __shfl(v, 0);
    return v == ~0ull ? ~0ull : (v & CS_CNT) - count;
}

// Lines with rank >= 64 in a chunk (more than a wave's lanes): found again
// from the staged window, their line_off entries written and the lines
// queued for k_parse_ovf_lines.  Rare (very short lines).
__device__ __noinline__ void chunk_excess(const uint8_t* __restrict__ buf, uint64_t nbytes, const Columns& C,
                                         const uint8_t* win, uint64_t w0, uint64_t w1, uint64_t t_lo, uint64_t t_hi,
                                         uint32_t first, uint64_t base, int64_t chunk, uint32_t count) {
    const int lane = lane_id();
    const int nv = (int)((w1 - w0 + 15) >> 4);
    uint32_t run = first;
    for (int k0 = 0; k0 < nv; k0 += PW) {
        const int k = k0 + lane;
        const uint64_t p = w0 + 16ull * k;
        uint32_t ms = 0;
        if (k < nv) {
            const u32x4 v = *reinterpret_cast<const u32x4*>(win + 16 * k);
            ms = term_bits(make_uint4(v[0], v[1], v[2], v[3]), buf, p, nbytes);
            if (p < t_lo) ms &= t_lo - p >= 16 ? 0u : ~0u << (uint32_t)(t_lo - p);
            if (p + 16 > t_hi) ms &= t_hi > p ? (1u << (uint32_t)(t_hi - p)) - 1u : 0u;
        }
        const uint32_t c = (uint32_t)__popc(ms);
        const uint32_t incl = wave_incl_scan(c);
        uint32_t r = run + incl - c;
        run += (uint32_t)__shfl((int)incl, 63);
        for (uint32_t m = ms; m; m &= m - 1, ++r) {
            if (r < (uint32_t)PW) continue;
            const uint64_t li = base + r;
            if ((int64_t)li >= C.cap_lines) continue;
            line_off_w(C)[li] = p + (uint64_t)__builtin_ctz(m) + 1;
            queue_line(C, li);
        }
    }
    // the staging pass counted (and published) `count` lines for this chunk
    if (lane == 0 && run != count) {
        check_fail(C, CHK_EXCESS, (uint64_t)chunk, run, count, base);
        if (C.meta->err_info[1] == (uint64_t)chunk) {  // (this chunk's record: the arguments it received)
            C.meta->err_info[5] = w0;
            C.meta->err_info[6] = w1;
            C.meta->err_info[7] = t_lo;
            C.meta->err_info[8] = t_hi;
            C.meta->err_info[9] = first;
            C.meta->err_info[10] = (uint64_t)(uintptr_t)win;
            C.meta->err_info[11] = nbytes;
            C.meta->err_info[12] = (uint64_t)(uintptr_t)buf;
        }
    }
}

// Chunk c of cb bytes on one wave: stage its window, publish its line count,
// phase 1 of its lines, then (its first line number known) the line index
// entries and rows.  LDS: [elements][DFS stack][starts][window (win_cap)]
// [mask planes (win_cap / 4)].  direct: every line goes to the direct kernel
// (LP_OPT_FORCE_DIRECT, tests).
// second: the deferred pass (the chunk's count is published and the scanner
// has finished: the line number is read, not waited for).
// MF: a program of several LogFormats (HttpdLogFormatDissector.java:173-204):
// each lane first computes its line's match word without the DFS; a line
// that exactly one format matches is routed to it whatever the sticky state
// is (the active format, if it is not that one, fails, and the first that
// matches becomes active), and one that no format matches is BAD whatever
// the state is; so phase 1 runs here for those.  A line several formats
// match, or whose word needs the DFS, is queued: k_route_ovf computes its
// word, the routing scan (k_fmt_*) then gives every line its format, and
// k_parse_ovf_lines parses it.  Every line's word is written to fmt_match.
template <bool LA, bool SIMPLE, bool MF = false>
__device__ __forceinline__ void parse_chunk(const uint8_t* __restrict__ buf, uint64_t nbytes, const Program& P,
                                            const Columns& C, const Elem* s_elems, uint8_t* smem, int64_t c,
                                            int64_t n_chunks, uint32_t cb, uint32_t win_cap, uint32_t stk_words,
                                            int direct, int wait_max, bool second) {
    const uint64_t c0 = (uint64_t)c * cb;
    const uint64_t c1 = c0 + cb < nbytes ? c0 + cb : nbytes;
    const int lane = lane_id();
    WaveStack stk{reinterpret_cast<uint32_t*>(smem + 16 * P.n_elems) + lane};
    uint32_t* starts = reinterpret_cast<uint32_t*>(smem + 16 * P.n_elems + 4 * stk_words);
    uint8_t* win = smem + 16 * P.n_elems + 4 * stk_words + 16 * ((4 * MAXS + 15) / 16);
    uint16_t* msk16 = reinterpret_cast<uint16_t*>(win + win_cap);
    // window: 64 bytes before the chunk (its first start needs the byte
    // before it), the chunk, then the tail of its last line
    const uint64_t w0 = c0 >= 64 ? c0 - 64 : 0;
    const uint64_t w1 = w0 + win_cap < nbytes ? w0 + win_cap : nbytes;
    const uint64_t t_lo = c0 ? c0 - 1 : 0, t_hi = c1 - 1;
    const uint32_t first = c0 == 0 ? 1u : 0u;
    if (first && lane == 0) starts[0] = 0;
    LP_PROF(0);
    const ChunkScan S = stage_chunk(buf, nbytes, w0, w1, t_lo, t_hi, first, win, msk16, starts);
    if (!second) chunk_publish(C.chunk_state, c, S.count);
    LP_PROF(60);
    __syncthreads();  // starts[] written by every lane
    const uint32_t nl = S.count < (uint32_t)PW ? S.count : (uint32_t)PW;  // lines on this wave's lanes
    const bool has = (uint32_t)lane < nl;
    // this lane's line [s, e) in window offsets; e = its terminator (or end)
    uint32_t s = 0, e = 0;
    bool known = false;
    if (has) {
        s = starts[lane];
        if ((uint32_t)lane + 1 < S.count) {
            e = starts[lane + 1] - 1;
            known = true;
        } else if (S.end_term != ~0ull) {
            e = (uint32_t)(S.end_term - w0);
            known = true;
        } else if (w1 == nbytes) {  // a last line without terminator
            e = (uint32_t)(nbytes - w0);
            known = true;
        }
    }
    const bool lds_line = has && known && !direct;
    const int n = lds_line ? crlf_len((int)(e - s), e > s ? win[e - 1] : 0u) : 0;
    const LineT<lds_bytes, lds_u64> L{(lds_bytes)win, lds_line ? s : 0u, n, (lds_u64)reinterpret_cast<uint64_t*>(msk16)};
    // phase 1 before the line numbers are known (its row is written after)
    LineOut o;
    o.status = ST_OK;
    o.tdone = o.smdone = o.bipdone = 0;
    LP_PROF(1);
    uint32_t mword = 0;  // MF: the line's match word (bit f: format f matches)
    if constexpr (MF) {
        if (lds_line) {
            bool redo = false;
            // (the spans of the first matching format's first leaf in o.caps)
            mword = fmt_match_word<false>(P, s_elems, L, stk, S.clean, &redo, &o.caps);
            const uint32_t mm = mword & 0xFFu;
            if (redo || (mword >> 8) || (mm & (mm - 1))) o.status = ST_REDO;  // the DFS or the sticky state decides
            else if (mm == 0) o.status = ST_BAD;  // no format matches: BAD in every state
            else phase1<true, LA, false, false, true>(P, s_elems, L, o, stk, C, 0, S.clean, __builtin_ctz(mm));
        }
    } else {
#if defined(LP_DFS_IN_CHUNKS)  // (experiment builds: the backtracking DFS inside the chunk kernel, as before round 6)
        if (lds_line) phase1<false, LA, SIMPLE, true>(P, s_elems, L, o, stk, C, 0, S.clean, 0);
#else
        if (lds_line) phase1<false, LA, SIMPLE, false>(P, s_elems, L, o, stk, C, 0, S.clean, 0);  // (no DFS: ST_REDO)
#endif
    }
    LP_PROF(9);
    const uint64_t base = chunk_base(C.chunk_state, c, S.count, second ? (int)CHUNK_WAIT_MAX : wait_max);
    if (base == ~0ull) {  // (never in a normal launch) the deferred pass redoes the chunk
        if (lane == 0) {
            const uint64_t q = atomicAdd(&C.meta->deferred, 1ull);
            if (q < (uint64_t)n_chunks) C.deferred_chunks[q] = (uint32_t)c;
            else check_fail(C, CHK_QUEUE, 1, q, (uint64_t)c, (uint64_t)n_chunks);
        }
        return;
    }
    LP_PROF(61);
    const int64_t cap = C.cap_lines;
    const int64_t li = (int64_t)base + lane;
    const bool mine = has && li < cap;
    if (mine) line_off_w(C)[li] = w0 + s;
    if constexpr (MF) {
        if (mine) C.fmt_match[li] = (uint16_t)mword;  // (a queued line's word: k_route_ovf)
    }
    // a line the window does not hold, or that needs the backtracking DFS,
    // is queued for k_parse_ovf_lines (the whole phase 1, from HBM)
    const bool redo = lds_line && o.status == ST_REDO;
    const bool row = mine && lds_line && !redo;
    if (mine && (!lds_line || redo)) queue_line(C, (uint64_t)li);
    if (row) {
        write_line(P, o, C, li);
        if (!P.has_phase2()) C.arena_base[li] = 0;  // no URI kernel: an empty region for every line
    }
    if (S.count > (uint32_t)PW)
        chunk_excess(buf, nbytes, C, win, w0, w1, t_lo, t_hi, first, base, c, S.count);
    if (c == n_chunks - 1 && lane == 0) {
        // the batch's line count (Hadoop: a last line without terminator counts)
        const uint64_t total = base + S.count;
        C.meta->n_lines = total;
        C.meta->cap_ovf = (int64_t)total > cap ? 1ull : 0ull;
        if ((int64_t)total <= cap) {
            const uint8_t last = buf[nbytes - 1];
            line_off_w(C)[total] = last == '\n' || last == '\r' ? nbytes : nbytes + 1;  // sentinel
        }
    }
    WaveCounts WC;
    WC.act = (uint32_t)__popcll(__ballot(row));
    WC.ok = (uint32_t)__popcll(__ballot(row && o.status == ST_OK));
    WC.bad = (uint32_t)__popcll(__ballot(row && o.status == ST_BAD));
    WC.store(C.chunk_counts, c);
    LP_PROF(62);
}

// Block 0: the scanner; block c + 1: chunk c.  Chunks whose wave stopped
// waiting for the scanner (chunk_base) are redone by k_parse_deferred.
// SIMPLE: the instance for Apache common / combined family programs
// (phase1; the host's simple_program picks it).
template <bool LA, bool SIMPLE, bool MF>
__global__ __launch_bounds__(PW, MF ? LP_MF_WPE : 2) void k_parse_chunks(const uint8_t* __restrict__ buf, uint64_t nbytes,
                                                     const DeviceArgs* __restrict__ args, uint32_t cb, uint32_t win_cap,
                                                     uint32_t stk_words, int direct, int wait_max) {
    const Program& P = args->prog;
    const Columns& C = args->cols;
    const int64_t n_chunks = (int64_t)((nbytes + cb - 1) / cb);
    if (blockIdx.x == 0) {
        chunk_scanner(C.chunk_state, n_chunks);
        return;
    }
    const int64_t c = (int64_t)blockIdx.x - 1;
    if ((uint64_t)c * cb >= nbytes) return;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    Elem* s_elems = reinterpret_cast<Elem*>(smem);
    load_elems(P, s_elems);
    parse_chunk<LA, SIMPLE, MF>(buf, nbytes, P, C, s_elems, smem, c, n_chunks, cb, win_cap, stk_words, direct, wait_max,
                                false);
}

// The deferred pass: the chunks in C.deferred_chunks (none in a normal
// launch: its blocks return at once), after k_parse_chunks, whose scanner has
// then finished, so their line numbers are read, not waited for.
template <bool LA, bool SIMPLE, bool MF>
__global__ __launch_bounds__(PW, 2) void k_parse_deferred(const uint8_t* __restrict__ buf, uint64_t nbytes,
                                                       const DeviceArgs* __restrict__ args, uint32_t cb,
                                                       uint32_t win_cap, uint32_t stk_words, int direct) {
    const Program& P = args->prog;
    const Columns& C = args->cols;
    const uint64_t nd = C.meta->deferred;
    if (blockIdx.x >= nd) return;
    const int64_t n_chunks = (int64_t)((nbytes + cb - 1) / cb);
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    Elem* s_elems = reinterpret_cast<Elem*>(smem);
    load_elems(P, s_elems);
    for (uint64_t q = blockIdx.x; q < nd; q += gridDim.x) {
        parse_chunk<LA, SIMPLE, MF>(buf, nbytes, P, C, s_elems, smem, (int64_t)C.deferred_chunks[q], n_chunks, cb,
                                    win_cap, stk_words, direct, 0, true);
        __syncthreads();  // this chunk's LDS reads are done before the next one is staged
    }
}

// The lines k_parse_chunks queued, 64 per wave on a persistent grid, read
// from HBM.  Without URI stages (whose kernel re-counts every line) their
// status counts go to the batch counters here.
__global__ __launch_bounds__(PW) void k_parse_ovf_lines(const uint8_t* __restrict__ buf, uint64_t nbytes,
                                                        const DeviceArgs* __restrict__ args, uint32_t stk_words) {
    const Program& P = args->prog;
    const Columns& C = args->cols;
    if (C.meta->cap_ovf) return;
    const uint64_t nq = min((uint64_t)C.meta->ovf_lines, (uint64_t)C.cap_lines + 1);  // (queue_line checked the rest)
    const uint64_t n_lines = C.meta->n_lines;
    if ((uint64_t)blockIdx.x * PW >= nq) return;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    Elem* s_elems = reinterpret_cast<Elem*>(smem);
    WaveStack stk{reinterpret_cast<uint32_t*>(smem + 16 * P.n_elems) + lane_id()};
    load_elems(P, s_elems);
    __syncthreads();
    WaveCounts WC;
    for (uint64_t q0 = (uint64_t)blockIdx.x * PW; q0 < nq; q0 += (uint64_t)gridDim.x * PW) {
        const uint64_t q = q0 + lane_id();
        bool active = q < nq;
        const int64_t li = active ? (int64_t)C.ovf_lines[q] : 0;
        uint64_t s = 0, e = 0;
        if (active) {
            // a queued line is one of the batch's lines, and its index entries
            // bound a line of the buffer (the sentinel is nbytes or nbytes + 1)
            uint64_t e1 = 0;
            const bool in = (uint64_t)li < n_lines;
            if (in) {
                s = C.line_off[li];
                e1 = C.line_off[li + 1];
            }
            if (!in || s >= e1 || e1 > nbytes + 1) {
                check_fail(C, CHK_OVF_LINE, q, (uint64_t)li, s, e1);
                active = false;
                s = 0;
            } else {
                e = e1 - 1;
            }
        }
        const uint64_t len = e - s;
        const int n0 = (int)(len > (uint64_t)0x7FFFFFFF ? 0x7FFFFFFF : len);
        const int n = active ? crlf_len(n0, n0 > 0 ? buf[e - 1] : 0u) : 0;
        const LP_G uint8_t* ls = (const LP_G uint8_t*)(buf) + s;
        const uint32_t mis = (uint32_t)((uintptr_t)ls & 3);
        const LineT<const LP_G uint8_t*> L{ls - mis, mis, n};
        parse_wave<false>(P, s_elems, C, L, active, li, stk, false, WC);
    }
    if (!P.has_phase2() && lane_id() == 0 && WC.act) {
        atomicAdd(&C.meta->counters[0], (unsigned long long)WC.act);
        atomicAdd(&C.meta->counters[1], (unsigned long long)WC.ok);
        atomicAdd(&C.meta->counters[2], (unsigned long long)WC.bad);
        atomicAdd(&C.meta->counters[3], (unsigned long long)(WC.act - WC.ok - WC.bad));
    }
}

// Several LogFormats, one pass: the match words (with the DFS) of the lines
// the chunk kernel queued, 64 per wave on a persistent grid, from HBM; the
// routing scan (k_fmt_*) runs after it.
__global__ __launch_bounds__(PW) void k_route_ovf(const uint8_t* __restrict__ buf, uint64_t nbytes,
                                                  const DeviceArgs* __restrict__ args, uint32_t stk_words) {
    const Program& P = args->prog;
    const Columns& C = args->cols;
    if (C.meta->cap_ovf) return;
    const uint64_t nq = min((uint64_t)C.meta->ovf_lines, (uint64_t)C.cap_lines + 1);
    const uint64_t n_lines = C.meta->n_lines;
    if ((uint64_t)blockIdx.x * PW >= nq) return;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    Elem* s_elems = reinterpret_cast<Elem*>(smem);
    WaveStack stk{reinterpret_cast<uint32_t*>(smem + 16 * P.n_elems) + lane_id()};
    load_elems(P, s_elems);
    __syncthreads();
    for (uint64_t q0 = (uint64_t)blockIdx.x * PW; q0 < nq; q0 += (uint64_t)gridDim.x * PW) {
        const uint64_t q = q0 + lane_id();
        if (q >= nq) continue;
        const int64_t li = (int64_t)C.ovf_lines[q];
        if ((uint64_t)li >= n_lines) continue;  // (k_parse_ovf_lines reports it)
        const uint64_t s = C.line_off[li], e1 = C.line_off[li + 1];
        if (s >= e1 || e1 > nbytes + 1) continue;  // (idem)
        const uint64_t e = e1 - 1, len = e - s;
        const int n0 = (int)(len > (uint64_t)0x7FFFFFFF ? 0x7FFFFFFF : len);
        const int n = crlf_len(n0, n0 > 0 ? buf[e - 1] : 0u);
        const LP_G uint8_t* ls = (const LP_G uint8_t*)(buf) + s;
        const uint32_t mis = (uint32_t)((uintptr_t)ls & 3);
        const LineT<const LP_G uint8_t*> L{ls - mis, mis, n};
        C.fmt_match[li] = (uint16_t)fmt_match_word(P, s_elems, L, stk, false);
    }
}

// ------------------------------------------------ line-index parse (several LogFormats)

// One wave's 64 lines on the staged path (k_parse_lines), or queued for
// k_parse_overflow when even half its window exceeds LDS.
__device__ __forceinline__ void parse_group(const uint8_t* __restrict__ buf, uint64_t nbytes, const Program& P,
                                            const Columns& C, const Elem* s_elems, WaveStack stk, uint8_t* win,
                                            uint16_t* msk16, uint32_t win_cap, int64_t wave, int64_t n_lines) {
    const WaveLines W = wave_lines(C, wave, n_lines, nbytes);
    // the lines' window in one staged round; a window larger than LDS in two
    // rounds of 32 lines (lanes 0-31, then 32-63) when each half fits, else
    // the wave is queued for k_parse_overflow (lines read from HBM)
    uint64_t a0 = W.w0, b0 = W.w1, a1 = 0, b1 = 0;
    int rounds = 1;
    if (W.w1 - W.w0 > win_cap) {
        const int64_t mid = W.li0 + PW / 2 < W.lend ? W.li0 + PW / 2 : W.lend;
        const uint64_t lm = C.line_off[mid];
        b0 = lm < nbytes ? lm : nbytes;
        a1 = lm & ~15ull;
        b1 = W.w1;
        rounds = mid < W.lend ? 2 : 1;
        if (b0 - a0 > win_cap || (rounds == 2 && b1 - a1 > win_cap)) {
            if (lane_id() == 0) C.ovf_list[atomicAdd(&C.meta->ovf_waves, 1ull)] = (uint32_t)wave;
            return;
        }
    }
    LP_PROF(0);
    WaveCounts WC;
#pragma nounroll
    for (int r = 0; r < rounds; ++r) {
        const uint64_t a = r ? a1 : a0, b = r ? b1 : b0;
        const bool clean = stage_window(buf, nbytes, a, b, win, msk16);
        __syncthreads();
        const bool mine = W.active && (rounds == 1 || (lane_id() >= PW / 2) == (r != 0));
        const int n = mine ? crlf_len(W.n, W.n > 0 ? win[W.e - 1 - a] : 0u) : 0;
        const LineT<lds_bytes, lds_u64> L{(lds_bytes)win, mine ? (uint32_t)(W.s - a) : 0u, n,
                                          (lds_u64)reinterpret_cast<uint64_t*>(msk16)};
        parse_wave<true>(P, s_elems, C, L, mine, W.li, stk, clean, WC);
        if (r + 1 < rounds) __syncthreads();  // this round's LDS reads are done before the next staging
    }
    WC.store(C, wave);
}

__global__ __launch_bounds__(PW, 2) void k_parse_lines(const uint8_t* __restrict__ buf, uint64_t nbytes,
                                                    const DeviceArgs* __restrict__ args, uint32_t win_cap,
                                                    uint32_t stk_words) {
    const Program& P = args->prog;
    const Columns& C = args->cols;
    const int64_t n_lines = (int64_t)C.meta->n_lines;
    const int64_t wave = blockIdx.x;
    if (wave * PW >= n_lines || C.meta->cap_ovf) return;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    Elem* s_elems = reinterpret_cast<Elem*>(smem);
    WaveStack stk{reinterpret_cast<uint32_t*>(smem + 16 * P.n_elems) + lane_id()};
    uint8_t* win = smem + 16 * P.n_elems + stk_words * 4;
    uint16_t* msk16 = reinterpret_cast<uint16_t*>(win + win_cap);
    load_elems(P, s_elems);
    parse_group(buf, nbytes, P, C, s_elems, stk, win, msk16, win_cap, wave, n_lines);
}

// The waves k_parse_lines queued (even half their window exceeds LDS: very
// long lines), on a persistent grid: the lines are read from HBM directly.
__global__ __launch_bounds__(PW) void k_parse_overflow(const uint8_t* __restrict__ buf, uint64_t nbytes,
                                                       const DeviceArgs* __restrict__ args, uint32_t stk_words) {
    const Program& P = args->prog;
    const Columns& C = args->cols;
    const int64_t n_lines = (int64_t)C.meta->n_lines;
    const uint64_t nq = C.meta->ovf_waves;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    Elem* s_elems = reinterpret_cast<Elem*>(smem);
    WaveStack stk{reinterpret_cast<uint32_t*>(smem + 16 * P.n_elems) + lane_id()};
    load_elems(P, s_elems);
    __syncthreads();
    for (uint64_t q = blockIdx.x; q < nq; q += gridDim.x) {
        const int64_t wave = C.ovf_list[q];
        const WaveLines W = wave_lines(C, wave, n_lines, nbytes);
        WaveCounts WC;
        // base = the line start aligned down to 4 bytes: word reads never
        // leave the 4-byte words holding the line's bytes
        const LP_G uint8_t* ls = (const LP_G uint8_t*)(buf) + W.s;
        const uint32_t mis = (uint32_t)((uintptr_t)ls & 3);
        const LineT<const LP_G uint8_t*> L{ls - mis, mis, crlf_len_hbm(buf, W)};
        parse_wave<true>(P, s_elems, C, L, W.active, W.li, stk, false, WC);
        __syncthreads();
        WC.store(C, wave);
    }
}

// Sticky routing pass 1: the match word of every line (bit f = format f matches).
__global__ __launch_bounds__(PW) void k_route_match(const uint8_t* __restrict__ buf, uint64_t nbytes,
                                                    const DeviceArgs* __restrict__ args, uint32_t win_cap,
                                                    uint32_t stk_words) {
    const Program& P = args->prog;
    const Columns& C = args->cols;
    const int64_t n_lines = (int64_t)C.meta->n_lines;
    const int64_t wave = blockIdx.x;
    if (wave * PW >= n_lines || C.meta->cap_ovf) return;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    Elem* s_elems = reinterpret_cast<Elem*>(smem);
    WaveStack stk{reinterpret_cast<uint32_t*>(smem + 16 * P.n_elems) + lane_id()};
    uint8_t* win = smem + 16 * P.n_elems + stk_words * 4;
    uint16_t* msk16 = reinterpret_cast<uint16_t*>(win + win_cap);
    load_elems(P, s_elems);
    const WaveLines W = wave_lines(C, wave, n_lines, nbytes);
    if (W.w1 - W.w0 <= win_cap) {
        const bool clean = stage_window(buf, nbytes, W.w0, W.w1, win, msk16);
        __syncthreads();
        const int n = W.active ? crlf_len(W.n, W.n > 0 ? win[W.e - 1 - W.w0] : 0u) : W.n;
        const LineT<lds_bytes, lds_u64> L{(lds_bytes)win, (uint32_t)(W.s - W.w0), n, (lds_u64)reinterpret_cast<uint64_t*>(msk16)};
        if (W.active) C.fmt_match[W.li] = (uint16_t)fmt_match_word(P, s_elems, L, stk, clean);
    } else {
        __syncthreads();
        const LP_G uint8_t* ls = (const LP_G uint8_t*)(buf) + W.s;
        const uint32_t mis = (uint32_t)((uintptr_t)ls & 3);
        const LineT<const LP_G uint8_t*> L{ls - mis, mis, crlf_len_hbm(buf, W)};
        if (W.active) C.fmt_match[W.li] = (uint16_t)fmt_match_word(P, s_elems, L, stk, false);
    }
}

// LDS window of a wave: sized to the most waves per CU that still leave >= 4 %
// over the mean 64 lines (the few windows that do not fit go to the direct
// kernel).  Measured on gfx950: W waves of one 64-thread workgroup each fit
// when a wave's LDS is at most 160 KiB / W - 640 B.
struct WindowPlan {
    uint32_t cap, stk_words;
    size_t lds;
};
WindowPlan window_plan(const ParseLaunch& a) {
    WindowPlan w;
    w.stk_words = (uint32_t)(a.stack_depth > 0 ? a.stack_depth : 1) * PW;
    const uint64_t fixed = 16 * (uint64_t)a.n_elems + 4 * (uint64_t)w.stk_words;
    const uint64_t per8 = 8 + MC_N;  // LDS bytes per 8 window bytes (window + mask planes)
    const uint64_t mean = a.mean_line ? a.mean_line : 256;
    const uint64_t need = PW * mean + PW * mean / 25 + 64;
    uint64_t cap = 0;
    for (int k = 8; k >= 2 && !cap; --k) {
        const uint64_t budget = 160 * 1024 / k - 640;
        if (budget <= fixed) continue;
        const uint64_t c = ((budget - fixed) * 8 / per8) & ~63ull;
        if (c >= need) cap = c;
    }
    if (!cap) cap = ((PW * mean * 110) / 100 + 512 + 63) & ~63ull;
    if (cap > 48 * 1024) cap = 48 * 1024;
    if (a.force_direct) cap = 0;
    w.cap = (uint32_t)cap;
    w.lds = fixed + cap + MC_N * (cap / 8);
    return w;
}

}  // namespace

// The chunked kernel's LDS: a window of the most waves per CU that still
// holds the chunk (target_lines x the mean line) plus 64 bytes before it and
// an overhang of at least 2 mean lines for the tail of its last line.
ChunkPlan chunk_plan(const ParseLaunch& a) {
    ChunkPlan c{};
    c.stk_words = (uint32_t)(a.stack_depth > 0 ? a.stack_depth : 1) * PW;
    // the chunk kernels run no DFS (ST_REDO lines are queued): no stack in
    // their LDS (the queued lines' kernels have theirs)
#if defined(LP_DFS_IN_CHUNKS)
    c.chunk_stk = c.stk_words;
#else
    c.chunk_stk = 0;
#endif
    const uint64_t fixed = 16 * (uint64_t)a.n_elems + 4 * (uint64_t)c.chunk_stk + 16 * ((4 * MAXS + 15) / 16);
    const uint64_t per8 = 8 + MC_N;  // LDS bytes per 8 window bytes (window + mask planes)
    const uint64_t mean = a.mean_line ? a.mean_line : 256;
    const uint64_t oh = std::max<uint64_t>(512, ((2 * mean + 63) & ~63ull));
    // lines per chunk: at most 54 (measured best at 8 waves per CU, config 2:
    // tools/chunk_sweep.py), and the count that puts the most lines in
    // flight per CU (waves x lines) over the wave counts the registers allow
    // (the several-format instance: LP_MF_WPE waves per SIMD); LP_OPT_CHUNK_LINES
    // fixes the count
    uint64_t lines = a.chunk_lines ? a.chunk_lines : 54;
    if (!a.chunk_lines) {
        const int maxw = a.multi ? 4 * LP_MF_WPE : LP_CHUNK_MAXW;
        const uint64_t lmax = a.multi ? LP_CHUNK_LMAX_MF : LP_CHUNK_LMAX;
        uint64_t best = 0;
        for (int k = 8; k <= maxw; ++k) {
            const uint64_t budget = 160 * 1024 / k - 640;
            if (budget <= fixed) break;
            const uint64_t capk = std::min<uint64_t>(((budget - fixed) * 8 / per8) & ~63ull, 48 * 1024) & ~1023ull;
            const uint64_t lk = capk > 64 + oh + 63 ? std::min<uint64_t>(lmax, (capk - 64 - oh - 63) / mean) : 0;
            if (lk >= 16 && (uint64_t)k * lk > best) {
                best = (uint64_t)k * lk;
                lines = lk;
            }
        }
    }
    uint64_t cb = ((lines * mean) + 63) & ~63ull;
    if (cb < 1024) cb = 1024;
    const uint64_t need = cb + 64 + oh;
    uint64_t cap = 0;
    int waves = 0;
    for (int k = LP_CHUNK_MAXW; k >= 2 && !cap; --k) {
        const uint64_t budget = 160 * 1024 / k - 640;
        if (budget <= fixed) continue;
        const uint64_t w = ((budget - fixed) * 8 / per8) & ~63ull;
        if (w >= need || k == 2) {
            // whole 1 KiB LDS-DMA blocks, no more than the chunk needs (a
            // wave stages its whole window: a larger one only re-reads the
            // next chunk's bytes)
            cap = std::min<uint64_t>(std::min<uint64_t>(w, 48 * 1024), (need + 1023) & ~1023ull) & ~1023ull;
            waves = k;
        }
    }
    if (cap < need) cb = cap > 64 + oh + 1024 ? ((cap - 64 - oh) & ~63ull) : 1024;  // long lines: fewer per chunk
    if (cap < cb + 64 + 64) cap = (cb + 128 + 1023) & ~1023ull;
    c.cb = (uint32_t)cb;
    c.win_cap = (uint32_t)cap;
    c.waves_per_cu = waves;
    c.lds = fixed + cap + MC_N * (cap / 8);
    c.n_chunks = a.nbytes ? (int64_t)((a.nbytes + cb - 1) / cb) : 0;
    return c;
}

#if defined(LP_PROFILE)
int prof_read_parse(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof), sizeof(unsigned long long) * PROF_WAVES * PROF_POINTS) == hipSuccess ? 0 : -1;
}
int prof_clear_parse() {
    static unsigned long long z[PROF_WAVES * PROF_POINTS];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof z) == hipSuccess ? 0 : -1;
}
#endif

int launch_route_match(const ParseLaunch& a, const DeviceArgs* d_args, hipStream_t s) {
    const int64_t waves = parse_waves(a.cap_lines);
    if (waves == 0) return 0;
    const WindowPlan w = window_plan(a);
    hipLaunchKernelGGL(k_route_match, dim3((unsigned)waves), dim3(PW), w.lds, s, a.buf, a.nbytes, d_args, w.cap,
                       w.stk_words);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_parse(const ParseLaunch& a, const DeviceArgs* d_args, const Columns& C, hipStream_t s) {
    const int64_t waves = parse_waves(a.cap_lines);
    if (waves == 0 && !a.chunked) {
        if (a.mid_event) hipEventRecord((hipEvent_t)a.mid_event, s);
        return 0;
    }
    const int64_t grid = std::max<int64_t>(1, waves < 1024 ? waves : 1024);
    if (a.chunked) {
        // one pass: line index + phase 1, then the queued lines from HBM
        const ChunkPlan cp = chunk_plan(a);
        if (cp.n_chunks > 0) {
            // the instance per program shape: literal-aware first candidates
            // only for programs that have such an element, SIMPLE for the
            // Apache common / combined family; the chunks, then the deferred pass (its blocks return at once
            // when no wave gave up waiting, the normal case)
            const unsigned g0 = (unsigned)cp.n_chunks + 1, g1 = (unsigned)std::min<int64_t>(cp.n_chunks, 1024);
            const int fd = a.force_direct ? 1 : 0;
            // (the instance per program shape: LA, SIMPLE)
            auto run = [&](auto chunks, auto deferred) {
                hipLaunchKernelGGL(chunks, dim3(g0), dim3(PW), cp.lds, s, a.buf, a.nbytes, d_args, cp.cb, cp.win_cap,
                                   cp.chunk_stk, fd, a.chunk_wait);
                hipLaunchKernelGGL(deferred, dim3(g1), dim3(PW), cp.lds, s, a.buf, a.nbytes, d_args, cp.cb,
                                   cp.win_cap, cp.chunk_stk, fd);
            };
#if defined(LP_NO_SIMPLE)  // (experiment builds: every program on the general instances)
            const bool simple = false;
#else
            const bool simple = a.simple;
#endif
            // (several LogFormats: one instance; their first leaves are walked per lane)
            if (a.multi) run(k_parse_chunks<true, false, true>, k_parse_deferred<true, false, true>);
            else if (a.lit_aware && simple) run(k_parse_chunks<true, true, false>, k_parse_deferred<true, true, false>);
            else if (a.lit_aware) run(k_parse_chunks<true, false, false>, k_parse_deferred<true, false, false>);
            else if (simple) run(k_parse_chunks<false, true, false>, k_parse_deferred<false, true, false>);
            else run(k_parse_chunks<false, false, false>, k_parse_deferred<false, false, false>);
            const size_t lds_ovf = 16 * (size_t)a.n_elems + 4 * (size_t)cp.stk_words;
            if (a.multi) {
                // the queued lines' match words, then the sticky routing scan
                // over every line's word (fmt_id of every line, the state after
                // the batch)
                hipLaunchKernelGGL(k_route_ovf, dim3((unsigned)grid), dim3(PW), lds_ovf, s, a.buf, a.nbytes, d_args,
                                   cp.stk_words);
                if (launch_route(d_args, a.cap_lines, s) != 0) return -1;
            }
            hipLaunchKernelGGL(k_parse_ovf_lines, dim3((unsigned)grid), dim3(PW), lds_ovf, s, a.buf, a.nbytes, d_args,
                               cp.stk_words);
        }
        if (a.mid_event) hipEventRecord((hipEvent_t)a.mid_event, s);
        if (launch_uri(a, d_args, s) != 0) return -1;
        // without URI stages the chunks' counts (plus the queued lines' own
        // atomics); with them the URI kernel re-counted every 64-line group
        if (a.uri) return launch_reduce_counts(C.wave_counts, waves, true, C.meta, s);
        return launch_reduce_counts(C.chunk_counts, cp.n_chunks, false, C.meta, s);
    }
    const WindowPlan w = window_plan(a);
    hipLaunchKernelGGL(k_parse_lines, dim3((unsigned)waves), dim3(PW), w.lds, s, a.buf, a.nbytes, d_args, w.cap,
                       w.stk_words);
    // the queued waves (even half the window exceeds LDS): persistent grid,
    // lines read from HBM (LDS: the elements and the DFS stack only)
    const size_t lds_ovf = 16 * (size_t)a.n_elems + 4 * (size_t)w.stk_words;
    hipLaunchKernelGGL(k_parse_overflow, dim3((unsigned)grid), dim3(PW), lds_ovf, s, a.buf, a.nbytes, d_args,
                       w.stk_words);
    if (a.mid_event) hipEventRecord((hipEvent_t)a.mid_event, s);
    if (launch_uri(a, d_args, s) != 0) return -1;
    return launch_reduce_counts(C.wave_counts, waves, true, C.meta, s);
}

}  // namespace lp
