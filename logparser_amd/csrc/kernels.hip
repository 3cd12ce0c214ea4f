// gfx950 kernels of the logparser_amd engine.
//
//   k_count_newlines  per-chunk line terminator count and terminator bit masks ('\n', lone '\r',
//                     the '\n' of "\r\n"; 16-byte loads, SWAR byte compare)
//   k_scan_counts     exclusive scan of the chunk counts (single workgroup); the batch's line
//                     count, line_off[0] and the end sentinel, written on the device
//   k_line_offsets    line start offsets from the bit masks (Hadoop LineRecordReader '\n' semantics)
//   k_parse_lines     one wave per 64 lines, one lane per line: the lines' byte window and
//                     its byte-class masks staged in LDS, LogFormat match + token / time /
//                     first-line stages (phase 1), wave-aggregated arena allocation from a
//                     sharded bump pointer, URI + query-string stages (phase 2); a wave whose
//                     window does not fit LDS is queued for k_parse_overflow
//   k_parse_overflow  the queued waves: two staged rounds of 32 lines, or the lines read
//                     from HBM (very long lines), on a persistent grid
//   k_route_match     several LogFormats: which formats match each line (sticky routing pass 1)
//   k_fmt_*           the sticky active-format scan (routing pass 2)
//   k_reduce_counts   per-wave status counts -> the batch counters
//
// The per-line logic is lp_device.h; this file only adds the data-parallel
// scaffolding around it.  The staged kernel carries exactly one line type
// (the LDS window with masks): its code is what the hot loop keeps in the
// instruction cache.
#include <hip/hip_runtime.h>

#define LP_KERNEL_TU 1  // device column pointers are global-memory pointers (lp_program.h)

#include <algorithm>

#include "kernels.h"
#include "lp_device.h"

namespace lp {

namespace {

constexpr int CHUNK = 64 * 1024;  // bytes per workgroup in the newline passes
constexpr int NL_THREADS = 256;   // 256 threads x 16 B x 16 iterations = 64 KiB

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

// Pass 1 of the line index: line terminators per 64 KiB chunk, and the
// terminator bit mask of every 16-byte piece (1 bit per input byte) so that
// pass 2 reads nbytes / 8 bytes instead of the input again.
__global__ __launch_bounds__(NL_THREADS) void k_count_newlines(const uint8_t* __restrict__ buf, uint64_t nbytes,
                                                                uint64_t* __restrict__ counts,
                                                                uint16_t* __restrict__ nlmask) {
    const uint64_t base = (uint64_t)blockIdx.x * CHUNK;
    constexpr int IT = CHUNK / (NL_THREADS * 16);
    uint32_t c = 0;
    if (base + CHUNK <= nbytes && ((uintptr_t)(buf + base) & 15) == 0) {
        // a whole chunk: every load in flight before the first use
        typedef uint32_t w4 __attribute__((ext_vector_type(4)));
        w4 v[IT];
#pragma unroll
        for (int it = 0; it < IT; ++it)
            v[it] = __builtin_nontemporal_load(
                reinterpret_cast<const w4*>(buf + base + ((uint64_t)it * NL_THREADS + threadIdx.x) * 16));
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const uint64_t pos = base + ((uint64_t)it * NL_THREADS + threadIdx.x) * 16;
            const uint32_t m = term_bits(make_uint4(v[it][0], v[it][1], v[it][2], v[it][3]), buf, pos, nbytes);
            c += (uint32_t)__popc(m);
            nlmask[pos >> 4] = (uint16_t)m;
        }
    } else {
        for (int it = 0; it < IT; ++it) {
            uint64_t pos = base + ((uint64_t)it * NL_THREADS + threadIdx.x) * 16;
            uint32_t m = 0;
            if (pos < nbytes) {
                m = term16(buf, pos, nbytes);
                c += (uint32_t)__popc(m);
            }
            nlmask[pos >> 4] = (uint16_t)m;
        }
    }
    // block reduction
    __shared__ uint32_t red[NL_THREADS / 64];
    for (int d = 32; d > 0; d >>= 1) c += __shfl_down(c, d);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (int w = 0; w < NL_THREADS / 64; ++w) t += red[w];
        counts[blockIdx.x] = t;
    }
}

// exclusive scan of n counts in place; total written to counts[n]; then the
// batch's line count (a final line without '\n' counts), line_off[0] = 0 and
// the end sentinel of an unterminated last line (line_off[n_lines] = nbytes + 1)
__global__ __launch_bounds__(1024) void k_scan_counts(uint64_t* __restrict__ counts, int64_t n,
                                                      const uint8_t* __restrict__ buf, uint64_t nbytes,
                                                      uint64_t* __restrict__ line_off, int64_t cap_lines,
                                                      Meta* __restrict__ meta) {
    // one contiguous segment per thread; loads issued 8 at a time so their
    // latencies overlap (a dependent load per element took ~1 ms at 386 K
    // chunks)
    __shared__ uint64_t part[1024];
    const int64_t per = (n + 1023) / 1024;
    const int64_t a = (int64_t)threadIdx.x * per, b = a + per < n ? a + per : n;
    uint64_t s = 0;
    int64_t i = a;
    for (; i + 8 <= b; i += 8) {
        uint64_t v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = counts[i + k];
#pragma unroll
        for (int k = 0; k < 8; ++k) s += v[k];
    }
    for (; i < b; ++i) s += counts[i];
    part[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x < 64) {  // exclusive scan of the 1024 partial sums by one wave
        uint64_t v[16], t = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) { v[k] = part[threadIdx.x * 16 + k]; t += v[k]; }
        uint64_t x = t;
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t y = __shfl_up(x, d);
            if ((int)threadIdx.x >= d) x += y;
        }
        uint64_t run = x - t;
#pragma unroll
        for (int k = 0; k < 16; ++k) { part[threadIdx.x * 16 + k] = run; run += v[k]; }
        if (threadIdx.x == 63) {
            counts[n] = run;
            // Hadoop LineRecordReader: lines = terminator count, plus a last line without one
            const bool open_end = nbytes > 0 && buf[nbytes - 1] != '\n' && buf[nbytes - 1] != '\r';
            const int64_t lines = (int64_t)run + (open_end ? 1 : 0);
            meta->n_lines = (unsigned long long)lines;
            // cap_lines < 0: only count (the host sizes the buffers from the count)
            meta->cap_ovf = cap_lines >= 0 && lines > cap_lines ? 1ull : 0ull;
            line_off[0] = 0;
            if (open_end && cap_lines >= 0 && lines <= cap_lines) line_off[lines] = nbytes + 1;
        }
    }
    __syncthreads();
    uint64_t run = part[threadIdx.x];
    i = a;
    for (; i + 8 <= b; i += 8) {
        uint64_t v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = counts[i + k];
#pragma unroll
        for (int k = 0; k < 8; ++k) { counts[i + k] = run; run += v[k]; }
    }
    for (; i < b; ++i) { uint64_t v = counts[i]; counts[i] = run; run += v; }
}

// line_off[j] = start of line j.  line_off[0] = 0 and the entry after every
// terminator that is not the last byte; line_off[n_lines] = end sentinel.
// Entries past cap_lines are not written (the batch is then re-run with
// larger columns).  Thread t of a chunk takes 16 consecutive mask words (256
// input bytes): one block scan of the per-thread counts, then each thread
// writes its lines' starts.
__global__ __launch_bounds__(NL_THREADS) void k_line_offsets(const uint16_t* __restrict__ nlmask, uint64_t nbytes,
                                                              const uint64_t* __restrict__ chunk_base,
                                                              uint64_t* __restrict__ line_off, int64_t cap_lines) {
    constexpr int WPT = CHUNK / 16 / NL_THREADS;  // mask words per thread (16)
    const uint64_t base = (uint64_t)blockIdx.x * CHUNK;
    const uint64_t pos0 = base + (uint64_t)threadIdx.x * WPT * 16;  // first input byte of this thread
    __shared__ uint32_t wsum[NL_THREADS / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t m[WPT];
    const uint64_t nwords = (nbytes + 15) >> 4;
    const uint64_t w0 = pos0 >> 4;
    if (w0 + WPT <= nwords) {
        const uint4* q = reinterpret_cast<const uint4*>(nlmask + w0);  // 32-byte aligned
        const uint4 a = q[0], b = q[1];
        const uint32_t x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int k = 0; k < 8; ++k) { m[2 * k] = x[k] & 0xFFFFu; m[2 * k + 1] = x[k] >> 16; }
    } else {
#pragma unroll
        for (int k = 0; k < WPT; ++k) m[k] = w0 + k < nwords ? (uint32_t)nlmask[w0 + k] : 0u;
    }
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < WPT; ++k) c += (uint32_t)__popc(m[k]);
    // block exclusive scan of c
    uint32_t x = c;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if (lane >= d) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint32_t wpre = 0;
    for (int w = 0; w < NL_THREADS / 64; ++w)
        if (w < wave) wpre += wsum[w];
    uint64_t k = chunk_base[blockIdx.x] + wpre + x - c;  // index of this thread's first terminator
#pragma unroll
    for (int j = 0; j < WPT; ++j) {
        uint32_t mm = m[j];
        while (mm) {
            const uint32_t b = (uint32_t)__builtin_ctz(mm);
            mm &= mm - 1;
            if ((int64_t)(k + 1) <= cap_lines) line_off[k + 1] = pos0 + 16ull * j + b + 1;
            ++k;
        }
    }
}

// ---------------------------------------------------------------- parse
// One workgroup = one wave = 64 consecutive lines.  The wave copies the byte
// window holding its lines into LDS with coalesced 16-byte loads (classifying
// every byte into the two mask planes on the way), then every lane runs the
// per-line stages of lp_device.h on its own line out of LDS.
constexpr int PW = 64;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#ifndef LP_STAGE_PRIO
#define LP_STAGE_PRIO 0
#endif

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
    W.li = W.li0 + (int64_t)threadIdx.x;
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
    const int lane = threadIdx.x;
    const int nv = (int)((w1 - w0 + 15) >> 4);
    const int nv4 = (nv + 3) & ~3;  // whole 64-byte mask blocks
    uint32_t bad = 0;  // guard-failing bytes other than '\n' anywhere in the window
    // SB loads in flight per lane before the first LDS store (one HBM
    // round trip per SB x 1 KiB of window instead of one per 1 KiB)
    constexpr int SB = 20;
    const uint64_t full_end = nbytes & ~15ull;  // 16-byte pieces wholly inside the buffer
    for (int k0 = lane; k0 < nv4; k0 += SB * PW) {
        u32x4 v[SB];
#if LP_STAGE_PRIO
        // the window's loads leave before the other waves' ALU work (they
        // are this wave's critical path; the CU has other waves to issue)
        __builtin_amdgcn_s_setprio(3);
#endif
#pragma unroll
        for (int j = 0; j < SB; ++j) {
            const int k = k0 + j * PW;
            const uint64_t p = w0 + 16ull * k;
            v[j] = u32x4{0, 0, 0, 0};
            if (k < nv && p + 16 <= full_end) v[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(buf + p));
        }
#if LP_STAGE_PRIO
        __builtin_amdgcn_s_setprio(0);
#endif
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
            uint32_t m0, m1, g = 0;
            bcls::classify16g(v[j][0], v[j][1], v[j][2], v[j][3], m0, m1, g);
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
    __device__ __forceinline__ void store(const Columns& C, int64_t wave) const {
        if (threadIdx.x == 0) {
            uint4 c, d;
            c.x = act;
            c.y = ok;
            c.z = bad;
            c.w = act - ok - bad;
            d.x = written;
            d.y = gathered;
            d.z = d.w = 0;
            uint4* wc = reinterpret_cast<uint4*>(C.wave_counts + WC_WORDS * (size_t)wave);
            wc[0] = c;
            wc[1] = d;
        }
    }
};

// Phase 1 of one wave's lines (match, tokens, time, first line) and their
// rows; adds the lines' counts to WC.  The URI stages run in k_uri_lines.
template <typename LN>
__device__ __forceinline__ void parse_wave(const Program& P, const Elem* elems, const Columns& C, const LN& L,
                                           bool active, int64_t li, WaveStack stk, bool clean, WaveCounts& WC) {
    LineOut o;
    o.status = ST_OK;
    LP_PROF(1);
    if (active) phase1(P, elems, L, o, stk, C, li, clean, P.n_fmt > 1 ? (int)C.fmt_id[li] : 0);
    LP_PROF(9);
    if (active) write_line(P, o, C, li);
    if (active && P.n_uri == 0) C.arena_base[li] = 0;  // no URI kernel: an empty region for every line
    WC.act += (uint32_t)__popcll(__ballot(active));
    WC.ok += (uint32_t)__popcll(__ballot(active && o.status == ST_OK));
    WC.bad += (uint32_t)__popcll(__ballot(active && o.status == ST_BAD));
}

// ------------------------------------------------------------------ URIs
// The URI and query-string stages of a wave's 64 lines (HttpUriDissector,
// QueryStringFieldDissector), after k_parse_lines wrote the lines' status and
// spans.  Each lane's URI sources (request URI, referer, ...) are gathered
// from the input into a compact LDS buffer (only the URI bytes: a few KiB per
// wave, so many waves share a CU and hide the arena atomics and the query
// passes' latencies), with their one-plane UEV mask; then phase 2 per lane,
// a wave-aggregated arena allocation, and the query pieces spread over the
// lanes.  A wave whose URI bytes do not fit runs on the direct (HBM) path.
// compact URI bytes per wave: with its mask plane within the LDS share of a
// CU running 16 waves (config 2: 7.3 KiB per wave on average, 8.3 KiB at the
// 99th percentile; a wave needing more runs on the direct path)
constexpr uint32_t URI_CAP = 8512;

// Per lane: the line's URI sources.  sp[u] = a | b << 16 (line-relative, 0 =
// none), cs[u] = the compact buffer offset of line byte a.  NU: the URI
// stages this kernel instance handles (>= P.n_uri; most programs have at
// most two, whose per-lane arrays then take two registers each)
template <int NU>
struct UriLane {
    bool ok;
    int fmt;
    uint64_t ls;  // line start in the input
    RegArr<NU> sp, cs, usep;
};

template <int NU>
__device__ __forceinline__ UriLane<NU> uri_lane(const Program& P, const Columns& C, int64_t li, bool active) {
    UriLane<NU> U;
    U.sp.fill(0);
    U.cs.fill(0);
    U.usep.fill(0);
    U.ok = false;
    U.fmt = 0;
    U.ls = 0;
    if (!active) return U;
    // every column read issued before the status is known (one round trip;
    // the values of a line that is not OK are not used)
    const uint8_t st = C.status[li];
    const int fmt = P.n_fmt > 1 ? (int)C.fmt_id[li] : 0;
    U.ls = C.line_off[li];
    const uint32_t tf = C.tok_flags[li];
    uint32_t raw[NU], kind[NU];
    for (int u = 0; u < NU; ++u) {
        raw[u] = 0;
        kind[u] = FL_FULL;
        if (u >= P.n_uri || P.uri[u].src_q >= 0) continue;
        if (P.uri[u].src_tok >= 0) {
            raw[u] = C.tok_span[P.uri[u].src_tok][li];
            kind[u] = (tf >> P.uri[u].src_tok) & 1u ? FL_NONE : FL_FULL;  // "-" -> null
        } else {
            raw[u] = C.fl_uri[P.uri[u].src_fl][li];
            kind[u] = C.fl_kind[P.uri[u].src_fl][li];
        }
    }
    U.ok = st == ST_OK;
    U.fmt = U.ok ? fmt : 0;
    if (U.ok)
        for (int u = 0; u < P.n_uri && u < NU; ++u) {
            // uri_source_cols (lp_device.h) on the values read above
            const int a = (int)(raw[u] & 0xFFFF), b = (int)(raw[u] >> 16);
            if (P.uri[u].fmt == U.fmt && P.uri[u].src_q < 0 && kind[u] != FL_NONE && b > a) U.sp.set(u, mkspan(a, b));
        }
    return U;
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

// The fast walk of URI stage u (lp_device.h uri_walk_fast) for all lines of
// the wave at once.  A line's event bytes (its UEV bits in [a, b), usep of
// them) are numbered line after line; each round, every lane takes one event
// of the wave: its byte, its class, and from ballots over its line's earlier
// events in the round plus the line's carried state (the owner lane's
// registers) what the sequential walk would know there -- whether an
// earlier event stopped the walk, the first '&' / '?' (fa), the previous
// query-piece boundary, the last '%' / '+'.  A boundary event that ends a
// non-empty piece writes its table slot; at the end of each round every
// owner lane folds its events of the round into its state.  The result per
// lane (part: the lane's line takes part) is exactly the sequential walk's
// state: resume, fa, first_pct, rewr bit 1, the query table (slots, count,
// s, lp).  L: the lane's line view (compact buffer with its UEV plane);
// A.p / A.used: the line's region and where its table starts.
template <typename CL>
__device__ __forceinline__ void uri_walk_coop(const Program& P, int u, const CL& L, bool part, int a, int b,
                                              uint32_t usep, const Arena& A, UriWalk& Wk) {
    const int lane = threadIdx.x;
    const bool table = P.uri[u].want_query && P.uri[u].query_stage >= 0;  // uniform
    const uint32_t cnt = part ? usep : 0u;
    uint32_t x = cnt;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if (lane >= d) x += y;
    }
    const uint32_t eb = x - cnt, E = __shfl(x, 63);
    const uint32_t tab = (A.used + 15) & ~15u;
    const unsigned long long reg = (unsigned long long)(uintptr_t)A.p;
    // the owner's state (this lane's line)
    int resume = -1, fa = -1, fpct = -1, lastB = -1, lastPP = -1;
    uint32_t count = 0;
    bool rw = false;
    for (uint32_t g0 = 0; g0 < E; g0 += PW) {
        const uint32_t g = g0 + (uint32_t)lane;
        const bool valid = g < E;
        int ow = 0;  // last lane whose first event is <= g
        for (int st = 32; st; st >>= 1)
            if (__shfl((int)eb, ow + st) <= (int)g) ow += st;
        const uint32_t ebo = (uint32_t)__shfl((int)eb, ow);
        const uint32_t oo = (uint32_t)__shfl((int)L.o, ow);
        const int oa = __shfl(a, ow), ob = __shfl(b, ow);
        // the event: the (g - ebo)-th UEV bit of the owner's [oa, ob)
        uint32_t Aq = 0;
        if (valid) {
            const uint32_t A0 = oo + (uint32_t)oa, A1 = oo + (uint32_t)ob, WL = (A1 - 1) >> 6;
            uint32_t W = A0 >> 6, k = g - ebo;
            uint64_t m = L.mask(MC_UEV, W) & (~0ull << (A0 & 63));
            for (;;) {
                if (W == WL) m &= ~0ull >> (63 - ((A1 - 1) & 63));
                const uint32_t c = (uint32_t)__popcll(m);
                if (k < c || W >= WL) break;  // (the count came from the same plane: k < c by WL)
                k -= c;
                ++W;
                m = L.mask(MC_UEV, W);
            }
            Aq = (W << 6) + select64(m, k);
        }
        const int q = (int)(Aq - oo);
        CL Lo = L;
        Lo.o = oo;
        Lo.n = ob;
        const uint32_t w = valid ? load_u32_at(Lo, q) : 0u;
        const uint32_t c = w & 0xFFu;
        const bool pct = c == '%';
        const bool bad_pct = pct && (q + 2 >= ob || !is_hex((w >> 8) & 0xFFu) || !is_hex((w >> 16) & 0xFFu));
        const bool stop = valid && (c == '#' || c == ';' || c >= 0x80 || bad_pct);
        const bool aq = c == '&' || c == '?';
        // the owner's state before this round
        const int cres = __shfl(resume, ow), cfa = __shfl(fa, ow), clB = __shfl(lastB, ow), clPP = __shfl(lastPP, ow);
        const uint32_t ccount = (uint32_t)__shfl((int)count, ow);
        // my line's earlier events in this round: lanes [seg0, lane)
        const int s0 = (int)ebo - (int)g0;
        const uint64_t below = (1ull << lane) - 1ull;
        const uint64_t seg_lt = valid ? below & (~0ull << (s0 > 0 ? s0 : 0)) : 0ull;
        const uint64_t Bstop = __ballot(stop);
        const bool live = valid && !stop && cres < 0 && !(Bstop & seg_lt);  // the fast walk takes this event
        const uint64_t Baq = __ballot(live && aq);
        const uint64_t mfa = Baq & seg_lt;
        const int qfa = __shfl(q, mfa ? lsb64(mfa) : lane);
        const int fa_j = cfa >= 0 ? cfa : (mfa ? qfa : -1);  // the first '&' / '?' before me
        const bool pp = live && ((pct && !bad_pct) || c == '+');
        const bool isB = table && live && aq && fa_j >= 0;   // a piece boundary after fa
        const uint64_t BB = __ballot(isB), BPP = __ballot(pp);
        const uint64_t mB = BB & seg_lt, mP = BPP & seg_lt;
        const int qpb = __shfl(q, mB ? msb64(mB) : lane), qpp = __shfl(q, mP ? msb64(mP) : lane);
        const bool first_piece = !mB && clB < 0;  // the previous boundary is fa
        const int pb = mB ? qpb : (clB >= 0 ? clB : fa_j);
        const int lpp = mP ? qpp : clPP;  // the last '%' / '+' before me
        const int lp = first_piece ? lpp : (lpp > pb ? lpp : -1);
        const bool emit = isB && q > pb + 1;
        const uint64_t BE = __ballot(emit);
        const bool rwj = live && fa_j >= 0 && ((aq && c == '?') || (!aq && !pct && uri_needs_encode(c)));
        const uint64_t BR = __ballot(rwj);
        const unsigned long long oreg = __shfl(reg, ow);
        const uint32_t otab = (uint32_t)__shfl((int)tab, ow);
        if (emit) {
            const uint32_t idx = ccount + (uint32_t)__popcll(BE & seg_lt);
            const uint64_t t0 = (uint64_t)(uint32_t)(pb + 1) | ((uint64_t)(uint32_t)q << 16) | ((uint64_t)(uint32_t)(lp + 1) << 48);
            *reinterpret_cast<LP_G u32x4*>(reinterpret_cast<LP_G uint8_t*>(oreg) + otab + 16 * idx) =
                u32x4{(uint32_t)t0, (uint32_t)(t0 >> 32), 0u, 0u};
        }
        // owners fold their events of this round into their state
        const int so = (int)eb - (int)g0, eo = (int)(eb + cnt) - (int)g0;
        const int so_c = so < 0 ? 0 : so > PW ? PW : so, eo_c = eo < 0 ? 0 : eo > PW ? PW : eo;
        const uint64_t segm = so_c < eo_c ? ((eo_c == PW ? ~0ull : (1ull << eo_c) - 1ull) & (~0ull << so_c)) : 0ull;
        const uint64_t ms = Bstop & segm, mf = Baq & segm, mpct = __ballot(live && pct) & segm, mb = BB & segm,
                       mpp = BPP & segm;
        const int q_s = __shfl(q, ms ? lsb64(ms) : lane), q_f = __shfl(q, mf ? lsb64(mf) : lane);
        const int q_p = __shfl(q, mpct ? lsb64(mpct) : lane), q_b = __shfl(q, mb ? msb64(mb) : lane);
        const int q_pp = __shfl(q, mpp ? msb64(mpp) : lane);
        if (resume < 0 && ms) resume = q_s;
        if (fa < 0 && mf) fa = q_f;
        if (fpct < 0 && mpct) fpct = q_p;
        if (mb) lastB = q_b;
        if (mpp) lastPP = q_pp;
        count += (uint32_t)__popcll(BE & segm);
        rw = rw || (BR & segm) != 0;
    }
    if (!part) return;
    Wk.resume = resume;
    Wk.fa = fa;
    Wk.first_pct = fpct;
    Wk.rewr = rw ? 2u : 0u;
    QueryTable& T = Wk.T;
    if (table && fa >= 0) {
        T.on = T.set = true;
        T.maxp = usep + 1;
        T.tab = tab;
        T.reg = tab + 16 * T.maxp;
        T.s = (lastB >= 0 ? lastB : fa) + 1;
        T.count = count;
        T.lp = lastB >= 0 ? (lastPP > lastB ? lastPP : -1) : lastPP;
    } else {
        T.lp = lastPP;
    }
}

// Phase 2, the arena allocation and the query pieces of one wave; lu(u) is
// the lane's line view of URI stage u (valid for every lane, empty stages
// included: the query pass reads other lanes' views).
template <int NU, int NQ, bool COOP, typename LU>
__device__ __forceinline__ void uri_wave(const Program& P, const Columns& C, UriLane<NU>& U, LU&& lu, bool active,
                                         int64_t li, int64_t wave, WaveCounts& WC) {
    const int lane = threadIdx.x;
    const int nq = P.n_query < NQ ? P.n_query : NQ;
    uint32_t need = 0;
    if (U.ok)
        for (int u = 0; u < P.n_uri && u < NU; ++u) {
            const uint32_t s = U.sp.get(u);
            if (!s) continue;
            uint32_t ev;
            need += uri_need(P, u, lu(u), (int)(s & 0xFFFF), (int)(s >> 16), ev);
            U.usep.set(u, ev);
        }
    need = (need + 15) & ~15u;
    // wave-aggregated arena allocation from the wave's shard
    uint32_t x = need;
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(x, d);
        if (lane >= d) x += y;
    }
    const uint32_t total = __shfl(x, 63);
    const int shard = (int)(wave % ARENA_SHARDS);
    unsigned long long wbase = 0;
    // regions start 16-byte aligned (their query tables take 16-byte slot
    // stores; spills keep the bump pointer only 4-byte aligned)
    if (lane == 63 && total) wbase = atomicAdd(&C.meta->shard_top[16 * shard], (unsigned long long)total + 12ull);
    wbase = (__shfl(wbase, 63) + 15) & ~15ull;
    const bool fits = wbase + total <= C.shard_cap;
    LP_PROF(26);
    uint32_t written = 0;
    unsigned long long my_region = 0;
    UriOutT<NQ> o;
    o.qlist.fill(0);
    o.qpend.fill(0);
    o.status = U.ok ? ST_OK : ST_BAD;
    Arena A{C.arena, 0, 0};
    bool live = false;  // the line's region is allocated: phase 2 runs
    if (U.ok) {
        if (!fits && need) {
            // the shard is full: the batch is re-run with a larger arena
            o.status = ST_FALLBACK;
            atomicAdd(&C.meta->arena_ovf, 1ull);
        } else {
            const unsigned long long mine = (unsigned long long)shard * C.shard_cap + wbase + x - need;
            my_region = mine;
            C.arena_base[li] = mine;  // also for an empty region: spills are region-relative
            A = Arena{C.arena + mine, 0, need};
            A.top = &C.meta->shard_top[16 * shard];  // spills come from the same shard
            A.base = wbase + x - need;
            A.limit = C.shard_cap;
            live = true;
        }
    }
    // phase 2 (lp_device.h phase2), stage by stage for the whole wave: the
    // compact path walks the stages' event bytes cooperatively
    const int nu = P.n_uri < NU ? P.n_uri : NU;
    for (int u = 0; u < nu; ++u) {
        const bool fmt_ok = live && o.status == ST_OK && P.uri[u].fmt == U.fmt;
        const uint32_t sp = U.sp.get(u);
        const int a = (int)(sp & 0xFFFF), b = (int)(sp >> 16);
        const bool part = fmt_ok && b > a;
        if (fmt_ok && !part) {
            C.u_flags[u][li] = 0;
            if (P.uri[u].query_stage >= 0) { C.q_count[P.uri[u].query_stage][li] = 0; C.q_params[P.uri[u].query_stage][li] = 0; }
        }
        LP_PROF(10 + 2 * u);
        UriWalk Wk;
        if constexpr (COOP) {
            LP_PROF(50 + 4 * u);
            uri_walk_coop(P, u, lu(u), part, a, b, U.usep.get(u), A, Wk);
            LP_PROF(51 + 4 * u);
        } else if (part) {
            uri_walk_fast(P, u, lu(u), a, b, U.usep.get(u), A, Wk);
        }
        if (part) {
            const int st = uri_stage_rest(P, u, lu(u), a, b, U.usep.get(u), A, C, li, o, Wk);
            if (st != ST_OK) o.status = st;
        }
        LP_PROF(11 + 2 * u);
    }
    if (live) {
        if (A.ovf) {
            o.status = ST_FALLBACK;
            atomicAdd(&C.meta->arena_ovf, 1ull);
        }
        written = A.used - A.slack + A.extra;
    }
    LP_PROF(21);
    // QueryStringFieldDissector pieces of all lines of the wave, spread evenly
    // over the lanes (a line's pieces vary from 0 to dozens; one lane per line
    // would leave most lanes idle while the longest query finishes): the
    // pieces of every query stage in one numbering (a lane's stage-0 pieces,
    // then its stage-1 pieces, ...), QR blocks of 64 pieces per round: their
    // table slots loaded together, then query_prep, ONE spill allocation for
    // the round, query_finish.  Most waves need one round for all stages.
    if (nq > 0) {
        constexpr int QR = 4;
        __syncthreads();  // the table slots written in phase 2 are visible to every lane
        const bool has = U.ok && o.status == ST_OK && need != 0;
        const unsigned long long my_ab = has ? my_region : 0ull;
        uint64_t piece_ovf = 0;  // lanes whose line lost a piece for want of arena
        uint32_t np = 0;
        for (int qs = 0; qs < nq; ++qs) np += has ? o.qpend.get(qs) : 0u;
        uint32_t incl = np;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(incl, d);
            if (lane >= d) incl += y;
        }
        const uint32_t base = incl - np, tot = __shfl(incl, 63);
        // piece j of lane ow: its query stage and its slot in ow's region;
        // OL = ow's line view of that stage (every lane takes part in the shuffles)
        auto piece = [&](int ow, uint32_t j, int& pq, uint32_t& soff) {
            uint32_t cum = 0;
            pq = 0;
            soff = 0;
            for (int qs = 0; qs < nq; ++qs) {
                const uint32_t c = (uint32_t)__shfl((int)(has ? o.qpend.get(qs) : 0u), ow);
                const uint32_t l = (uint32_t)__shfl((int)o.qlist.get(qs), ow);
                if (j >= cum && j < cum + c) {
                    pq = qs;
                    soff = l + 16 * (j - cum);
                }
                cum += c;
            }
        };
        auto owner_view = [&](int ow, int pq) {
            auto OL = owner_line(lu(P.query[0].uri), ow);
            for (int qs = 1; qs < nq; ++qs) {
                const auto V = owner_line(lu(P.query[qs].uri), ow);
                if (pq == qs) OL = V;
            }
            return OL;
        };
        for (uint32_t g0 = 0; g0 < tot; g0 += QR * PW) {
            int own[QR], pqs[QR];
            uint32_t soffs[QR];
            uint64_t t0[QR];
#pragma unroll
            for (int k = 0; k < QR; ++k) {
                own[k] = 0;
                pqs[k] = 0;
                soffs[k] = 0;
                t0[k] = 0;
                if (g0 + (uint32_t)(k * PW) >= tot) continue;  // no piece in this block (uniform)
                const uint32_t g = g0 + (uint32_t)(k * PW + lane);
                int ow = 0;  // last lane whose first pending piece index is <= g
                for (int st = 32; st; st >>= 1)
                    if (__shfl(base, ow + st) <= g) ow += st;
                own[k] = ow;
                const uint32_t ob = __shfl(base, ow);
                const unsigned long long oab = __shfl(my_ab, ow);
                piece(ow, g - ob, pqs[k], soffs[k]);
                if (g < tot) t0[k] = *reinterpret_cast<const LP_G uint64_t*>(C.arena + oab + soffs[k]);
            }
            QPrep qp[QR];
            uint32_t mine = 0;
#pragma unroll
            for (int k = 0; k < QR; ++k) {
                if (g0 + (uint32_t)(k * PW) >= tot) continue;
                const uint32_t g = g0 + (uint32_t)(k * PW + lane);
                const auto OL = owner_view(own[k], pqs[k]);
                if (g < tot) qp[k] = query_prep(OL, t0[k]);
                mine += qp[k].need;
            }
            // the round's spilled bytes in one allocation from the wave's
            // shard (every owner is a line of this wave)
            uint32_t x = mine;
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(x, d);
                if (lane >= d) x += y;
            }
            const uint32_t rtot = __shfl(x, 63);
            unsigned long long rbase = 0;
            if (lane == 63 && rtot) rbase = atomicAdd(&C.meta->shard_top[16 * shard], (unsigned long long)rtot);
            unsigned long long at = __shfl(rbase, 63) + x - mine;  // this lane's first piece in the shard
#pragma unroll
            for (int k = 0; k < QR; ++k) {
                if (g0 + (uint32_t)(k * PW) >= tot) continue;
                const uint32_t g = g0 + (uint32_t)(k * PW + lane);
                const int ow = own[k];
                const unsigned long long oab = __shfl(my_ab, ow);
                const auto OL = owner_view(ow, pqs[k]);
                bool povf = false;
                if (g < tot) {
                    LP_G uint64_t* slot = reinterpret_cast<LP_G uint64_t*>(C.arena + oab + soffs[k]);
                    const unsigned long long rel = oab - (unsigned long long)shard * C.shard_cap;  // region in the shard
                    if (qp[k].need && (at + qp[k].need > C.shard_cap || at - rel + qp[k].need > 0x7FFFFFFFull)) {
                        slot[0] = REF_SKIP;
                        slot[1] = 0;
                        povf = true;
                        atomicAdd(&C.meta->arena_ovf, 1ull);  // the batch is re-run with a larger arena
                    } else {
                        Arena A{C.arena + oab, (uint32_t)(at - rel), (uint32_t)(at - rel + qp[k].need)};
                        written += query_finish(P, P.query[pqs[k]], OL, A, C.arena + oab, slot, qp[k]);
                    }
                    at += qp[k].need;
                }
                // a piece that did not fit: its line goes to FALLBACK (the
                // batch is re-run with a larger arena, or, when the re-runs
                // are spent, delivered with those lines FALLBACK)
                for (uint64_t m = __ballot(povf); m; m &= m - 1) piece_ovf |= 1ull << __shfl(ow, (int)__builtin_ctzll(m));
            }
        }
        if (((piece_ovf >> lane) & 1) && o.status == ST_OK) o.status = ST_FALLBACK;
    }
    LP_PROF(22);
    if (U.ok && o.status != ST_OK) C.status[li] = (uint8_t)o.status;
    for (int d = 32; d > 0; d >>= 1) written += __shfl_xor(written, d);
    const int st = !active ? -1 : U.ok ? o.status : (int)C.status[li];
    WC.act += (uint32_t)__popcll(__ballot(active));
    WC.ok += (uint32_t)__popcll(__ballot(st == ST_OK));
    WC.bad += (uint32_t)__popcll(__ballot(st == ST_BAD));
    WC.written += written;
}

// The 16 input bytes at p (16-byte aligned): one load inside the buffer,
// bytes past nbytes read as 0.
__device__ __forceinline__ u32x4 load16(const uint8_t* __restrict__ buf, uint64_t nbytes, uint64_t p) {
    if (p + 16 <= nbytes) return *reinterpret_cast<const u32x4*>(buf + p);
    uint32_t w[4] = {0, 0, 0, 0};
    for (int c = 0; c < 16; ++c) w[c >> 2] |= p + c < nbytes ? (uint32_t)buf[p + c] << (8 * (c & 3)) : 0u;
    return u32x4{w[0], w[1], w[2], w[3]};
}

// The URI stages of one wave on the compact path: its lines' URI bytes
// gathered into cbuf (CAP bytes) with their UEV plane, then uri_wave.
// Returns false, having done nothing, when the wave's bytes exceed CAP.
template <int NU, int NQ, uint32_t CAP>
__device__ __forceinline__ bool uri_compact(const uint8_t* __restrict__ buf, uint64_t nbytes, const Program& P,
                                            const Columns& C, int64_t wave, int64_t n_lines, uint32_t* cbuf,
                                            uint64_t* plane, WaveCounts& WC) {
    const int lane = threadIdx.x;
    const int64_t li = wave * PW + lane;
    const bool active = li < n_lines;
    LP_PROF(23);
    UriLane<NU> U = uri_lane<NU>(P, C, li, active);
    // one region per line: the 16-byte input blocks holding all its URI
    // sources (request URI, referer, ...: close together in a line), in
    // line order; a block keeps its alignment, so the wave gathers whole
    // aligned 16-byte blocks, consecutive lanes taking consecutive blocks
    uint64_t lo = ~0ull, hi = 0;
    for (int u = 0; u < P.n_uri && u < NU; ++u) {
        const uint32_t s = U.sp.get(u);
        if (!s) continue;
        lo = min(lo, U.ls + (s & 0xFFFF));
        hi = max(hi, U.ls + (s >> 16));
    }
    const uint64_t r0 = hi ? lo & ~15ull : 0;
    const uint32_t nblk = hi ? (uint32_t)((((hi + 15) & ~15ull) - r0) >> 4) : 0u;
    uint32_t x = nblk;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if (lane >= d) x += y;
    }
    const uint32_t tot = __shfl(x, 63), cb = x - nblk;  // blocks of the wave, this line's first block
    if (16 * tot + 16 > CAP) return false;
    WC.gathered = 16 * tot;
    for (int u = 0; u < P.n_uri && u < NU; ++u) {
        const uint32_t s = U.sp.get(u);
        if (s) U.cs.set(u, 16 * cb + (uint32_t)(U.ls + (s & 0xFFFF) - r0));
    }
    // gather: block g of the wave is block g - cb[own] of line own's region,
    // own = the last lane whose first block is <= g; every round's load in
    // flight before the first store
    constexpr int GR = 9;  // rounds per batch (the main kernel's CAP / 1024, rounded up)
    uint16_t* pl16 = reinterpret_cast<uint16_t*>(plane);
    for (uint32_t g0 = 0; g0 < tot; g0 += GR * PW) {
        u32x4 v[GR];
#pragma unroll
        for (int k = 0; k < GR; ++k) {
            const uint32_t g = g0 + (uint32_t)(k * PW + lane);
            int own = 0;
            for (int st = 32; st; st >>= 1)
                if (__shfl(cb, own + st) <= g) own += st;
            const uint64_t src = (uint64_t)__shfl((unsigned long long)r0, own) + 16ull * (g - __shfl(cb, own));
            v[k] = u32x4{0, 0, 0, 0};
            if (g < tot) v[k] = load16(buf, nbytes, src);
        }
#pragma unroll
        for (int k = 0; k < GR; ++k) {
            const uint32_t g = g0 + (uint32_t)(k * PW + lane);
            if (g >= tot) continue;
            *reinterpret_cast<u32x4*>(cbuf + 4 * g) = v[k];
            uint32_t m0, m1;
            bcls::classify16(v[k][0], v[k][1], v[k][2], v[k][3], m0, m1);
            pl16[g] = (uint16_t)(m0 | m1);
        }
    }
    LP_PROF(24);
    // one zero block after the last (the scanners' look-ahead word) and the
    // rest of the last 64-byte mask block
    for (uint32_t g = tot + lane; g < ((tot + 1 + 3) & ~3u); g += PW) {
        *reinterpret_cast<u32x4*>(cbuf + 4 * g) = u32x4{0, 0, 0, 0};
        pl16[g] = 0;
    }
    __syncthreads();
    LP_PROF(25);
    typedef LineT<lds_bytes, lds_u64, 1> CL;
    auto lu = [&](int u) {
        const uint32_t s = U.sp.get(u);
        // line byte q lives at cbuf + cs + (q - a): origin cs - a (mod 2^32)
        return CL{(lds_bytes)cbuf, U.cs.get(u) - (s & 0xFFFFu), (int)(s >> 16), (lds_u64)plane};
    };
    uri_wave<NU, NQ, true>(P, C, U, lu, active, li, wave, WC);
    return true;
}

// 16 waves per CU: the LDS share allows them, and __launch_bounds__(64, 4)
// (4 waves per SIMD) keeps the registers within 128
template <int NU, int NQ>
__global__ __launch_bounds__(PW, 4) void k_uri_lines(const uint8_t* __restrict__ buf, uint64_t nbytes,
                                                     const DeviceArgs* __restrict__ args) {
    const Program& P = args->prog;
    const Columns& C = args->cols;
    const int64_t n_lines = (int64_t)C.meta->n_lines;
    const int64_t wave = blockIdx.x;
    if (wave * PW >= n_lines || C.meta->cap_ovf) return;
    __shared__ __attribute__((aligned(16))) uint32_t cbuf[URI_CAP / 4 + 16];
    __shared__ uint64_t plane[URI_CAP / 64 + 1];
    WaveCounts WC;
    if (uri_compact<NU, NQ, URI_CAP>(buf, nbytes, P, C, wave, n_lines, cbuf, plane, WC)) WC.store(C, wave);
    else if (threadIdx.x == 0) C.uri_ovf_list[atomicAdd(&C.meta->uri_ovf_waves, 1ull)] = (uint32_t)wave;
}

// The waves k_uri_lines queued (their URI bytes exceed its compact buffer),
// on a persistent grid: the same path with a buffer four times as large (few
// waves: their occupancy does not matter), and for a wave exceeding even
// that, the lines' bytes read from HBM directly.
constexpr uint32_t URI_CAP_OVF = 4 * URI_CAP;
template <int NU, int NQ>
__global__ __launch_bounds__(PW) void k_uri_overflow(const uint8_t* __restrict__ buf, uint64_t nbytes,
                                                     const DeviceArgs* __restrict__ args) {
    const Program& P = args->prog;
    const Columns& C = args->cols;
    const int64_t n_lines = (int64_t)C.meta->n_lines;
    const uint64_t nq = C.meta->uri_ovf_waves;
    __shared__ __attribute__((aligned(16))) uint32_t cbuf[URI_CAP_OVF / 4 + 16];
    __shared__ uint64_t plane[URI_CAP_OVF / 64 + 1];
    for (uint64_t q = blockIdx.x; q < nq; q += gridDim.x) {
        const int64_t wave = C.uri_ovf_list[q];
        WaveCounts WC;
        if (!uri_compact<NU, NQ, URI_CAP_OVF>(buf, nbytes, P, C, wave, n_lines, cbuf, plane, WC)) {
            const WaveLines W = wave_lines(C, wave, n_lines, nbytes);
            UriLane<NU> U = uri_lane<NU>(P, C, W.li, W.active);
            const LP_G uint8_t* ls = (const LP_G uint8_t*)(buf) + W.s;
            const uint32_t mis = (uint32_t)((uintptr_t)ls & 3);
            const LineT<const LP_G uint8_t*> L{ls - mis, mis, crlf_len_hbm(buf, W)};
            auto lu = [&](int) { return L; };
            uri_wave<NU, NQ, false>(P, C, U, lu, W.active, W.li, wave, WC);
        }
        __syncthreads();
        WC.store(C, wave);
    }
}

// Derived URI stages (type-remapped query parameters, lp_device.h
// derived_line), after both URI kernels: one line per lane, the sources read
// in place (the input, or the decoded value in the line's region), every
// table and rewritten part spilled from the region's shard.  Only launched
// for programs that have such stages.  Re-counts the wave's statuses.
__global__ __launch_bounds__(PW) void k_derived_lines(const uint8_t* __restrict__ buf, uint64_t nbytes,
                                                      const DeviceArgs* __restrict__ args) {
    const Program& P = args->prog;
    const Columns& C = args->cols;
    const int64_t n_lines = (int64_t)C.meta->n_lines;
    const int64_t wave = blockIdx.x;
    if (wave * PW >= n_lines || C.meta->cap_ovf) return;
    const WaveLines W = wave_lines(C, wave, n_lines, nbytes);
    int st = W.active ? (int)C.status[W.li] : -1;
    if (st == ST_OK) {
        const int fmt = P.n_fmt > 1 ? (int)C.fmt_id[W.li] : 0;
        const LP_G uint8_t* ls = (const LP_G uint8_t*)(buf) + W.s;
        const uint32_t mis = (uint32_t)((uintptr_t)ls & 3);
        const unsigned long long ab = C.arena_base[W.li];
        const int shard = (int)(ab / C.shard_cap);
        Arena R{C.arena + ab, 0, 0};
        R.top = &C.meta->shard_top[16 * shard];
        R.base = ab - (unsigned long long)shard * C.shard_cap;
        R.limit = C.shard_cap;
        st = derived_line(P, fmt, ls - mis, mis, crlf_len_hbm(buf, W), R, C, W.li);
        if (R.ovf) atomicAdd(&C.meta->arena_ovf, 1ull);  // the batch is re-run with a larger arena
        if (st != ST_OK) C.status[W.li] = (uint8_t)st;
    }
    const uint32_t ok = (uint32_t)__popcll(__ballot(st == ST_OK)), bad = (uint32_t)__popcll(__ballot(st == ST_BAD));
    if (threadIdx.x == 0) {
        LP_G uint32_t* wc = C.wave_counts + WC_WORDS * (size_t)wave;
        const uint32_t act = wc[0];
        wc[1] = ok;
        wc[2] = bad;
        wc[3] = act - ok - bad;
    }
}

// LDS: [elements (n_elems x 16 B)][DFS stack][byte window (win_cap, a multiple of 64)][mask planes (win_cap / 4)]
__device__ __forceinline__ void load_elems(const Program& P, Elem* s_elems) {
    for (int k = threadIdx.x; k < P.n_elems; k += PW) s_elems[k] = P.elems[k];
}

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
            if (threadIdx.x == 0) C.ovf_list[atomicAdd(&C.meta->ovf_waves, 1ull)] = (uint32_t)wave;
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
        const bool mine = W.active && (rounds == 1 || ((int)threadIdx.x >= PW / 2) == (r != 0));
        const int n = mine ? crlf_len(W.n, W.n > 0 ? win[W.e - 1 - a] : 0u) : 0;
        const LineT<lds_bytes, lds_u64> L{(lds_bytes)win, mine ? (uint32_t)(W.s - a) : 0u, n,
                                          (lds_u64)reinterpret_cast<uint64_t*>(msk16)};
        parse_wave(P, s_elems, C, L, mine, W.li, stk, clean, WC);
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
    WaveStack stk{reinterpret_cast<uint32_t*>(smem + 16 * P.n_elems) + threadIdx.x};
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
    WaveStack stk{reinterpret_cast<uint32_t*>(smem + 16 * P.n_elems) + threadIdx.x};
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
        parse_wave(P, s_elems, C, L, W.active, W.li, stk, false, WC);
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
    WaveStack stk{reinterpret_cast<uint32_t*>(smem + 16 * P.n_elems) + threadIdx.x};
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

// meta->counters[0..5] += sum of the per-wave counts (lines ok bad fallback arena-bytes URI-source-bytes)
__global__ __launch_bounds__(256) void k_reduce_counts(const uint32_t* __restrict__ wc, Meta* __restrict__ meta) {
    const int64_t n_lines = meta->cap_ovf ? 0 : (int64_t)meta->n_lines;
    const int64_t n_waves = (n_lines + PW - 1) / PW;
    unsigned long long a[6] = {0, 0, 0, 0, 0, 0};
    for (int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x; w < n_waves; w += (int64_t)gridDim.x * 256) {
        const uint4 c = reinterpret_cast<const uint4*>(wc + WC_WORDS * w)[0];
        const uint4 d = reinterpret_cast<const uint4*>(wc + WC_WORDS * w)[1];
        a[0] += c.x; a[1] += c.y; a[2] += c.z; a[3] += c.w; a[4] += d.x; a[5] += d.y;
    }
    __shared__ unsigned long long red[6][4];
    for (int k = 0; k < 6; ++k) {
        unsigned long long v = a[k];
        for (int d = 32; d > 0; d >>= 1) v += __shfl_down(v, d);
        if ((threadIdx.x & 63) == 0) red[k][threadIdx.x >> 6] = v;
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        unsigned long long v = red[threadIdx.x][0] + red[threadIdx.x][1] + red[threadIdx.x][2] + red[threadIdx.x][3];
        if (v) atomicAdd(&meta->counters[threadIdx.x], v);
    }
}

// ------------------------------------------------------ sticky routing scan
// The routed format of line i = the fold of the per-line transition tables
// (lp_device.h fmt_table) from the handle's state.  Chunks of FMT_CHUNK
// lines: one wave per chunk, FMT_LPL lines per lane.
constexpr int FMT_LPL = FMT_CHUNK / PW;

__device__ __forceinline__ uint64_t lane_table(const Columns& C, const Program& P, int64_t l0, int64_t n_lines) {
    uint64_t t = 0xFEDCBA9876543210ull;  // identity
    for (int k = 0; k < FMT_LPL; ++k) {
        const int64_t li = l0 + k;
        if (li >= n_lines) break;
        t = fmt_compose(t, fmt_table(C.fmt_match[li], P.n_fmt));
    }
    return t;
}

// inclusive scan of the lanes' tables in lane order (table of lanes 0..lane)
__device__ __forceinline__ uint64_t wave_scan_tables(uint64_t t) {
    const int lane = threadIdx.x;
    for (int d = 1; d < PW; d <<= 1) {
        const uint64_t o = __shfl_up(t, d);
        if (lane >= d) t = fmt_compose(o, t);
    }
    return t;
}

__device__ __forceinline__ int64_t routed_lines(const Columns& C) {
    return C.meta->cap_ovf ? 0 : (int64_t)C.meta->n_lines;
}

__global__ __launch_bounds__(PW) void k_fmt_reduce(const DeviceArgs* __restrict__ args) {
    const Program& P = args->prog;
    const Columns& C = args->cols;
    const int64_t n_lines = routed_lines(C);
    if ((int64_t)blockIdx.x * FMT_CHUNK >= n_lines) return;
    const int64_t l0 = (int64_t)blockIdx.x * FMT_CHUNK + (int64_t)threadIdx.x * FMT_LPL;
    const uint64_t t = wave_scan_tables(lane_table(C, P, l0, n_lines));
    if (threadIdx.x == PW - 1) C.fmt_chunk[blockIdx.x] = t;
}

// one thread: chunk tables -> entry state of every chunk (in place), final
// state after the last chunk at [n_chunks] and in meta->fmt_state
__global__ void k_fmt_chunks(const DeviceArgs* __restrict__ args) {
    const Columns& C = args->cols;
    const int64_t n_chunks = fmt_chunks(routed_lines(C));
    uint32_t s = C.fmt_init;
    for (int64_t c = 0; c < n_chunks; ++c) {
        const uint64_t t = C.fmt_chunk[c];
        C.fmt_chunk[c] = s;
        s = fmt_apply(t, s);
    }
    C.fmt_chunk[n_chunks] = s;
    C.meta->fmt_state = s;
}

__global__ __launch_bounds__(PW) void k_fmt_apply(const DeviceArgs* __restrict__ args) {
    const Program& P = args->prog;
    const Columns& C = args->cols;
    const int64_t n_lines = routed_lines(C);
    if ((int64_t)blockIdx.x * FMT_CHUNK >= n_lines) return;
    const int64_t l0 = (int64_t)blockIdx.x * FMT_CHUNK + (int64_t)threadIdx.x * FMT_LPL;
    const uint64_t incl = wave_scan_tables(lane_table(C, P, l0, n_lines));
    uint64_t excl = __shfl_up(incl, 1);
    if (threadIdx.x == 0) excl = 0xFEDCBA9876543210ull;
    uint32_t s = fmt_apply(excl, (uint32_t)C.fmt_chunk[blockIdx.x]);
    for (int k = 0; k < FMT_LPL; ++k) {
        const int64_t li = l0 + k;
        if (li >= n_lines) break;
        s = fmt_apply(fmt_table(C.fmt_match[li], P.n_fmt), s);
        C.fmt_id[li] = (uint8_t)s;
    }
}

// ------------------------------------------------------------- histograms
// Run counters of a parsed batch (device counters all-reduced
// over RCCL by multi-GPU callers): per-status line counts, per-token null /
// present counts, response status codes and request methods of the OK lines.
// Grid-stride over lines, one LDS histogram per block, flushed with global
// atomics (a few thousand per launch).
__device__ __constant__ const char HIST_METHODS[15][10] = {
    "GET", "POST", "HEAD", "PUT", "DELETE", "OPTIONS", "PATCH", "CONNECT", "TRACE",
    "PROPFIND", "MKCOL", "COPY", "MOVE", "LOCK", "UNLOCK"};

__global__ __launch_bounds__(256) void k_histograms(const DeviceArgs* __restrict__ args, const uint8_t* __restrict__ buf,
                                                    unsigned long long* __restrict__ hist) {
    const Program& P = args->prog;
    const Columns& C = args->cols;
    __shared__ unsigned long long h[HIST_WORDS];
    for (int k = threadIdx.x; k < HIST_WORDS; k += blockDim.x) h[k] = 0;
    __syncthreads();
    const int64_t n = C.meta->cap_ovf ? 0 : (int64_t)C.meta->n_lines;
    for (int64_t li = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; li < n; li += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t st = C.status[li] < 3 ? C.status[li] : 2u;
        atomicAdd(&h[0], 1ull);
        atomicAdd(&h[1 + st], 1ull);
        if (st != ST_OK) continue;
        const int fmt = P.n_fmt > 1 ? (int)C.fmt_id[li] : 0;
        if (fmt >= P.n_fmt) continue;
        const uint8_t* line = buf + C.line_off[li];
        const uint32_t flags = C.tok_flags[li];
        for (int k = 0; k < P.n_tok; ++k) {
            const uint32_t sp = C.tok_span[k][li];
            if ((flags >> k) & 1u) atomicAdd(&h[16 + k], 1ull);
            else if ((sp >> 16) > (sp & 0xFFFFu)) atomicAdd(&h[32 + k], 1ull);
        }
        const int sk = P.hist_status[fmt];
        if (sk >= 0) {
            const uint32_t sp = C.tok_span[sk][li];
            const uint32_t a = sp & 0xFFFFu, b = sp >> 16;
            int code = -1;
            if (b - a == 3 && !((flags >> sk) & 1u)) {
                const uint32_t d0 = line[a] - '0', d1 = line[a + 1] - '0', d2 = line[a + 2] - '0';
                if (d0 < 10 && d1 < 10 && d2 < 10) code = (int)(d0 * 100 + d1 * 10 + d2);
            }
            if (code >= 100 && code <= 599) atomicAdd(&h[100 + code], 1ull);
            else atomicAdd(&h[48], 1ull);
        }
        const int f = P.hist_fl[fmt];
        if (f >= 0) {
            const uint32_t sp = C.fl_method[f][li];
            const uint32_t a = sp & 0xFFFFu, b = sp >> 16;
            int m = 15;
            if (b <= a) m = 16;  // no method (null or empty first line, or neither regex matched)
            else if (b - a <= 9) {
                for (int t = 0; t < 15 && m == 15; ++t) {
                    uint32_t q = 0;
                    while (q < b - a && HIST_METHODS[t][q] == (char)line[a + q]) ++q;
                    if (q == b - a && HIST_METHODS[t][q] == 0) m = t;
                }
            }
            atomicAdd(&h[64 + m], 1ull);
        }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < HIST_WORDS; k += blockDim.x)
        if (h[k]) atomicAdd(&hist[k], h[k]);
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


int64_t count_chunks(uint64_t nbytes) { return (int64_t)((nbytes + CHUNK - 1) / CHUNK); }

int launch_count(const uint8_t* d_buf, uint64_t nbytes, uint64_t* d_chunk, uint16_t* d_nlmask, uint64_t* d_line_off,
                 int64_t cap_lines, Meta* d_meta, hipStream_t s) {
    const int64_t nc = count_chunks(nbytes);
    if (nc > 0)
        hipLaunchKernelGGL(k_count_newlines, dim3((unsigned)nc), dim3(NL_THREADS), 0, s, d_buf, nbytes, d_chunk, d_nlmask);
    hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, s, d_chunk, nc, d_buf, nbytes, d_line_off, cap_lines, d_meta);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_offsets(const uint16_t* d_nlmask, uint64_t nbytes, const uint64_t* d_chunk, uint64_t* d_line_off,
                   int64_t cap_lines, hipStream_t s) {
    int64_t nc = count_chunks(nbytes);
    if (nc == 0) return 0;
    hipLaunchKernelGGL(k_line_offsets, dim3((unsigned)nc), dim3(NL_THREADS), 0, s, d_nlmask, nbytes, d_chunk, d_line_off,
                       cap_lines);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int64_t parse_waves(int64_t n_lines) { return (n_lines + PW - 1) / PW; }

#if defined(LP_PROFILE)
// profiling build: copy out (and clear) the per-wave timestamps
// (PROF_WAVES x PROF_POINTS u64)
extern "C" int lp_profile_read(unsigned long long* out, int n) {
    if (n < PROF_WAVES * PROF_POINTS) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof), sizeof(unsigned long long) * PROF_WAVES * PROF_POINTS) != hipSuccess)
        return -1;
    static unsigned long long z[PROF_WAVES * PROF_POINTS];
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof z);
    return 0;
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

int launch_route(const DeviceArgs* d_args, int64_t cap_lines, hipStream_t s) {
    const int64_t nc = fmt_chunks(cap_lines);
    if (nc == 0) return 0;
    hipLaunchKernelGGL(k_fmt_reduce, dim3((unsigned)nc), dim3(PW), 0, s, d_args);
    hipLaunchKernelGGL(k_fmt_chunks, dim3(1), dim3(1), 0, s, d_args);
    hipLaunchKernelGGL(k_fmt_apply, dim3((unsigned)nc), dim3(PW), 0, s, d_args);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_histograms(const DeviceArgs* d_args, const uint8_t* buf, int64_t cap_lines, uint64_t* hist, hipStream_t s) {
    if (hipMemsetAsync(hist, 0, sizeof(uint64_t) * HIST_WORDS, s) != hipSuccess) return -1;
    if (cap_lines <= 0) return 0;
    const int64_t blocks = std::min<int64_t>(2048, (cap_lines + 255) / 256);
    hipLaunchKernelGGL(k_histograms, dim3((unsigned)blocks), dim3(256), 0, s, d_args, buf,
                       reinterpret_cast<unsigned long long*>(hist));
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_parse(const ParseLaunch& a, const DeviceArgs* d_args, const uint32_t* d_wave_counts, Meta* d_meta,
                 hipStream_t s) {
    const int64_t waves = parse_waves(a.cap_lines);
    if (waves == 0) {
        if (a.mid_event) hipEventRecord((hipEvent_t)a.mid_event, s);
        return 0;
    }
    const WindowPlan w = window_plan(a);
    hipLaunchKernelGGL(k_parse_lines, dim3((unsigned)waves), dim3(PW), w.lds, s, a.buf, a.nbytes, d_args, w.cap,
                       w.stk_words);
    // the queued waves (even half the window exceeds LDS): persistent grid,
    // lines read from HBM (LDS: the elements and the DFS stack only)
    const int64_t grid = waves < 1024 ? waves : 1024;
    const size_t lds_ovf = 16 * (size_t)a.n_elems + 4 * (size_t)w.stk_words;
    hipLaunchKernelGGL(k_parse_overflow, dim3((unsigned)grid), dim3(PW), lds_ovf, s, a.buf, a.nbytes, d_args,
                       w.stk_words);
    if (a.mid_event) hipEventRecord((hipEvent_t)a.mid_event, s);
    if (a.uri) {
        // most programs have at most two URI and two query stages (the
        // request URI and the referer): an instance keeping two of each
        if (a.n_uri <= 2 && a.n_query <= 2) {
            hipLaunchKernelGGL((k_uri_lines<2, 2>), dim3((unsigned)waves), dim3(PW), 0, s, a.buf, a.nbytes, d_args);
            hipLaunchKernelGGL((k_uri_overflow<2, 2>), dim3((unsigned)grid), dim3(PW), 0, s, a.buf, a.nbytes, d_args);
        } else {
            hipLaunchKernelGGL((k_uri_lines<MAX_URI, MAX_QUERY>), dim3((unsigned)waves), dim3(PW), 0, s, a.buf,
                               a.nbytes, d_args);
            hipLaunchKernelGGL((k_uri_overflow<MAX_URI, MAX_QUERY>), dim3((unsigned)grid), dim3(PW), 0, s, a.buf,
                               a.nbytes, d_args);
        }
        if (a.derived) hipLaunchKernelGGL(k_derived_lines, dim3((unsigned)waves), dim3(PW), 0, s, a.buf, a.nbytes, d_args);
    }
    int64_t rb = (waves + 255) / 256;
    if (rb > 1024) rb = 1024;
    hipLaunchKernelGGL(k_reduce_counts, dim3((unsigned)rb), dim3(256), 0, s, d_wave_counts, d_meta);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace lp
