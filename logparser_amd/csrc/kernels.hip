// gfx950 kernels of the logparser_amd engine.
//
//   k_count_newlines  per-chunk '\n' count and '\n' bit masks (16-byte loads, SWAR byte compare)
//   k_scan_counts     exclusive scan of the chunk counts (single workgroup)
//   k_line_offsets    line start offsets from the bit masks (Hadoop LineRecordReader '\n' semantics)
//   k_parse_lines     one wave per 64 lines, one lane per line: the lines'
//                     byte window staged in LDS, LogFormat match + token /
//                     time / first-line stages (phase 1), wave-aggregated
//                     arena allocation, URI + query-string stages (phase 2)
//   k_reduce_counts   per-wave status counts -> the batch counters
//
// The per-line logic is lp_device.h; this file only adds the data-parallel
// scaffolding around it.
#include <hip/hip_runtime.h>

#define LP_KERNEL_TU 1  // device column pointers are global-memory pointers (lp_program.h)

#include <cstdlib>

#include "kernels.h"
#include "lp_device.h"

namespace lp {

namespace {

constexpr int CHUNK = 64 * 1024;  // bytes per workgroup in the newline passes
constexpr int NL_THREADS = 256;   // 256 threads x 16 B x 16 iterations = 64 KiB

// exact per-byte "== '\n'" mask of a 32-bit word (high bit of each byte)
__device__ __forceinline__ uint32_t nl_mask(uint32_t w) {
    uint32_t x = w ^ 0x0A0A0A0Au;
    return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
}

// the 16 bytes at pos (zero past nbytes) and their '\n' masks (bit 7 of
// each byte, one 32-bit mask per word)
struct Piece16 {
    uint32_t m[4];
    __device__ __forceinline__ uint32_t count() const {
        return __popc(m[0]) + __popc(m[1]) + __popc(m[2]) + __popc(m[3]);
    }
};
__device__ __forceinline__ Piece16 nl16(const uint8_t* p, uint64_t pos, uint64_t nbytes) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (pos + 16 <= nbytes && ((uintptr_t)(p + pos) & 15) == 0) {
        v = *reinterpret_cast<const uint4*>(p + pos);
    } else {
        uint32_t w[4] = {0, 0, 0, 0};
        for (uint64_t k = pos; k < pos + 16 && k < nbytes; ++k) w[(k - pos) >> 2] |= (uint32_t)p[k] << (8 * ((k - pos) & 3));
        v = make_uint4(w[0], w[1], w[2], w[3]);
    }
    Piece16 r;
    r.m[0] = nl_mask(v.x);
    r.m[1] = nl_mask(v.y);
    r.m[2] = nl_mask(v.z);
    r.m[3] = nl_mask(v.w);
    if (pos + 16 > nbytes) {  // zero bytes past the end are not newlines anyway
        for (int j = 0; j < 4; ++j)
            for (int b = 0; b < 4; ++b)
                if (pos + 4 * j + b >= nbytes) r.m[j] &= ~(0x80u << (8 * b));
    }
    return r;
}

// '\n' bits of a 16-byte piece as a 16-bit mask (bit k = byte k)
__device__ __forceinline__ uint32_t piece_bits(const Piece16& pc) {
    return bcls::nib(pc.m[0]) | (bcls::nib(pc.m[1]) << 4) | (bcls::nib(pc.m[2]) << 8) | (bcls::nib(pc.m[3]) << 12);
}

// Pass 1 of the line index: '\n' count per 64 KiB chunk, and the '\n' bit
// mask of every 16-byte piece (1 bit per input byte) so that pass 2 reads
// nbytes / 8 bytes instead of the input again.
__global__ __launch_bounds__(NL_THREADS) void k_count_newlines(const uint8_t* __restrict__ buf, uint64_t nbytes,
                                                                uint64_t* __restrict__ counts,
                                                                uint16_t* __restrict__ nlmask) {
    const uint64_t base = (uint64_t)blockIdx.x * CHUNK;
    uint32_t c = 0;
    for (int it = 0; it < CHUNK / (NL_THREADS * 16); ++it) {
        uint64_t pos = base + ((uint64_t)it * NL_THREADS + threadIdx.x) * 16;
        uint32_t m = 0;
        if (pos < nbytes) {
            const Piece16 pc = nl16(buf, pos, nbytes);
            c += pc.count();
            m = piece_bits(pc);
        }
        nlmask[pos >> 4] = (uint16_t)m;
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

// exclusive scan of n counts in place; total written to counts[n]
__global__ __launch_bounds__(1024) void k_scan_counts(uint64_t* __restrict__ counts, int64_t n) {
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
        if (threadIdx.x == 63) counts[n] = run;
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
// '\n' that is not the last byte; line_off[n_lines] = end sentinel.
__global__ __launch_bounds__(NL_THREADS) void k_line_offsets(const uint16_t* __restrict__ nlmask, uint64_t nbytes,
                                                              const uint64_t* __restrict__ chunk_base,
                                                              uint64_t* __restrict__ line_off) {
    const uint64_t base = (uint64_t)blockIdx.x * CHUNK;
    __shared__ uint32_t wsum[NL_THREADS / 64];
    uint64_t run = chunk_base[blockIdx.x];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int it = 0; it < CHUNK / (NL_THREADS * 16); ++it) {
        uint64_t pos = base + ((uint64_t)it * NL_THREADS + threadIdx.x) * 16;
        uint32_t m = pos < nbytes ? (uint32_t)nlmask[pos >> 4] : 0u;
        const uint32_t c = (uint32_t)__popc(m);
        // block exclusive scan of c
        uint32_t x = c;
        for (int d = 1; d < 64; d <<= 1) {
            uint32_t y = __shfl_up(x, d);
            if (lane >= d) x += y;
        }
        if (lane == 63) wsum[wave] = x;
        __syncthreads();
        uint32_t wpre = 0, tot = 0;
        for (int w = 0; w < NL_THREADS / 64; ++w) {
            if (w < wave) wpre += wsum[w];
            tot += wsum[w];
        }
        uint64_t k = run + wpre + x - c;  // index of this thread's first '\n'
        while (m) {
            const uint32_t b = (uint32_t)__builtin_ctz(m);
            m &= m - 1;
            line_off[++k] = pos + b + 1;
        }
        run += tot;
        __syncthreads();
    }
}

// ---------------------------------------------------------------- parse
// One workgroup = one wave = 64 consecutive lines.  The wave copies the byte
// window holding its lines into LDS with coalesced 16-byte loads, then every
// lane runs the per-line stages of lp_device.h on its own line out of LDS.
// Windows larger than the LDS budget (very long lines) read HBM directly.
constexpr int PW = 64;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

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

template <typename LN>
__device__ __forceinline__ void parse_wave(const Program& P, const Elem* elems, const Columns& C, const LN& L,
                                           bool active, int64_t li, WaveStack stk, bool clean, int mode) {
    if (mode == PM_MATCH) {  // sticky routing, pass 1: which formats match each line
        if (active) C.fmt_match[li] = (uint16_t)fmt_match_word(P, elems, L, stk, clean);
        return;
    }
    LineOut o;
    o.status = ST_OK;
    o.arena_need = 0;
    LP_PROF(1);
    if (active) phase1(P, elems, L, o, stk, C, li, clean, P.n_fmt > 1 ? (int)C.fmt_id[li] : 0);
    LP_PROF(9);
    // wave-aggregated arena allocation (every lane reaches this point)
    const uint32_t need = (active && o.status == ST_OK) ? o.arena_need : 0u;
    const int lane = threadIdx.x;
    uint32_t x = need;
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(x, d);
        if (lane >= d) x += y;
    }
    const uint32_t total = __shfl(x, 63);
    unsigned long long wbase = 0;
    if (lane == 63 && total) wbase = atomicAdd(C.arena_top, (unsigned long long)total);
    wbase = __shfl(wbase, 63);
    uint32_t written = 0;
    if (active) {
        if (o.status == ST_OK && need) {
            const unsigned long long mine = wbase + x - need;
            if (mine + need > C.arena_cap) o.status = ST_FALLBACK;
            else {
                C.arena_base[li] = mine;
                Arena A{C.arena + mine, 0, need};
                phase2(P, L, o, A, C, li);
                written = A.used - A.slack;
            }
        } else if (o.status == ST_OK) {
            C.arena_base[li] = 0;
        }
        LP_PROF(20);
        write_line(P, o, C, li);
    }
    LP_PROF(21);
    // QueryStringFieldDissector pieces of all lines of the wave, spread evenly
    // over the lanes (a line's pieces vary from 0 to dozens; one lane per line
    // would leave most lanes idle while the longest query finishes)
    if (P.n_query > 0) {
        __syncthreads();  // the table slots written in phase 2 are visible to every lane
        const bool has = active && o.status == ST_OK && need != 0;
        const unsigned long long my_ab = has ? C.arena_base[li] : 0ull;
        for (int qs = 0; qs < P.n_query; ++qs) {
            const uint32_t np = has ? o.qpend.get(qs) : 0u;
            const uint32_t my_list = o.qlist.get(qs);
            uint32_t incl = np;
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(incl, d);
                if (lane >= d) incl += y;
            }
            const uint32_t base = incl - np, total = __shfl(incl, 63);
            for (uint32_t g0 = 0; g0 < total; g0 += PW) {
                const uint32_t g = g0 + (uint32_t)lane;
                int own = 0;  // last lane whose first pending piece index is <= g
                for (int st = 32; st; st >>= 1)
                    if (__shfl(base, own + st) <= g) own += st;
                const uint32_t ob = __shfl(base, own), olist = __shfl(my_list, own);
                const unsigned long long oab = __shfl(my_ab, own);
                const auto OL = owner_line(L, own);
                if (g < total) {
                    LP_G uint8_t* region = C.arena + oab;
                    LP_G uint64_t* slot = reinterpret_cast<LP_G uint64_t*>(region + olist + 16 * (g - ob));
                    const uint64_t a0 = slot[0];
                    const uint32_t reserved = 3u * (uint32_t)(((a0 >> 16) & 0xFFFFu) - (a0 & 0xFFFFu));
                    const uint32_t used = query_piece(P, P.query[qs], OL, region, slot);
                    written += used - reserved;  // modulo 2^32: the wave sum is exact
                }
            }
        }
    }
    LP_PROF(22);
    for (int d = 32; d > 0; d >>= 1) written += __shfl_xor(written, d);
    const uint64_t m_act = __ballot(active);
    const uint64_t m_ok = __ballot(active && o.status == ST_OK);
    const uint64_t m_bad = __ballot(active && o.status == ST_BAD);
    if (lane == 0) {
        uint4 c, d;
        c.x = (uint32_t)__popcll(m_act);
        c.y = (uint32_t)__popcll(m_ok);
        c.z = (uint32_t)__popcll(m_bad);
        c.w = c.x - c.y - c.z;
        d.x = written;
        d.y = d.z = d.w = 0;
        uint4* wc = reinterpret_cast<uint4*>(C.wave_counts + WC_WORDS * (size_t)blockIdx.x);
        wc[0] = c;
        wc[1] = d;
    }
}

// MASKS: the staging pass also builds the byte-class masks (MC_N bits per
// window byte) for the 64-bytes-per-step scanners; without them the
// scanners classify 4 bytes per step and a wave needs less LDS.
template <bool MASKS>
__global__ __launch_bounds__(PW) void k_parse_lines(const uint8_t* __restrict__ buf, uint64_t nbytes, int64_t n_lines,
                                                    const DeviceArgs* __restrict__ args, uint32_t win_cap, int stage,
                                                    uint32_t stk_words, int mode) {
    const Program& P = args->prog;
    const Columns& C = args->cols;
    // LDS: [elements (n_elems x 16 B)][DFS stack][byte window (win_cap, a multiple of 64)][MC_N class masks]
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    Elem* s_elems = reinterpret_cast<Elem*>(smem);
    for (int k = threadIdx.x; k < P.n_elems; k += PW) s_elems[k] = P.elems[k];
    WaveStack stk{reinterpret_cast<uint32_t*>(smem + 16 * P.n_elems) + threadIdx.x};
    uint8_t* win = smem + 16 * P.n_elems + stk_words * 4;
    const uint32_t mwords = win_cap >> 6;
    uint16_t* msk16 = reinterpret_cast<uint16_t*>(win + win_cap);
    const int lane = threadIdx.x;
    const int64_t li0 = (int64_t)blockIdx.x * PW;
    const int64_t li = li0 + lane;
    const bool active = li < n_lines;
    const int64_t lend = li0 + PW < n_lines ? li0 + PW : n_lines;
    uint64_t s = 0, e = 0;
    if (active) {
        s = C.line_off[li];
        e = C.line_off[li + 1] - 1;  // exclude '\n' (or the end sentinel)
    }
    const int n = (int)((e - s) > (uint64_t)0x7FFFFFFF ? 0x7FFFFFFF : (e - s));
    const uint64_t w0 = C.line_off[li0] & ~15ull;
    uint64_t w1 = C.line_off[lend];
    if (w1 > nbytes) w1 = nbytes;
    LP_PROF(0);
    if (stage && w1 - w0 <= win_cap) {
        // stage the window with coalesced 16-byte loads and classify every
        // byte once (nibble-LUT classes -> 16 bits per class per 16 bytes)
        const int nv = (int)((w1 - w0 + 15) >> 4);
        const int nv4 = (nv + 3) & ~3;  // whole 64-bit mask words
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
                if (k < nv)
                    for (int w = 0; w < 4; ++w) bad |= swar::guard_bad(v[j][w]) & ~swar::eq(v[j][w], '\n');
                *reinterpret_cast<u32x4*>(win + 16 * k) = v[j];
                if constexpr (MASKS) {
                    uint32_t m0, m1;
                    bcls::classify16(v[j][0], v[j][1], v[j][2], v[j][3], m0, m1);
                    if (MC_QUOTE >= 0) msk16[4 * mwords * MC_QUOTE + k] = (uint16_t)m0;
                    msk16[4 * mwords * MC_UEV + k] = (uint16_t)m1;
                }
            }
        }
        const bool clean = !__any(bad != 0);
        __syncthreads();
        if constexpr (MASKS) {
            const LineT<lds_bytes, lds_u64> L{(lds_bytes)win, (uint32_t)(s - w0), n,
                                              (lds_u64)reinterpret_cast<uint64_t*>(msk16), mwords};
            parse_wave(P, s_elems, C, L, active, li, stk, clean, mode);
        } else {
            const LineT<lds_bytes> L{(lds_bytes)win, (uint32_t)(s - w0), n};
            parse_wave(P, s_elems, C, L, active, li, stk, clean, mode);
        }
    } else {
        __syncthreads();
        // base = the line start aligned down to 4 bytes: word reads never
        // leave the 4-byte words holding the line's bytes
        const LP_G uint8_t* ls = (const LP_G uint8_t*)(buf) + s;
        const uint32_t mis = (uint32_t)((uintptr_t)ls & 3);
        const LineT<const LP_G uint8_t*> L{ls - mis, mis, n};
        parse_wave(P, s_elems, C, L, active, li, stk, false, mode);
    }
}

// counters[0..4] += sum of the per-wave counts (lines ok bad fallback arena-bytes)
__global__ __launch_bounds__(256) void k_reduce_counts(const uint32_t* __restrict__ wc, int64_t n_waves,
                                                       unsigned long long* __restrict__ counters) {
    unsigned long long a[5] = {0, 0, 0, 0, 0};
    for (int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x; w < n_waves; w += (int64_t)gridDim.x * 256) {
        const uint4 c = reinterpret_cast<const uint4*>(wc + WC_WORDS * w)[0];
        const uint4 d = reinterpret_cast<const uint4*>(wc + WC_WORDS * w)[1];
        a[0] += c.x; a[1] += c.y; a[2] += c.z; a[3] += c.w; a[4] += d.x;
    }
    __shared__ unsigned long long red[5][4];
    for (int k = 0; k < 5; ++k) {
        unsigned long long v = a[k];
        for (int d = 32; d > 0; d >>= 1) v += __shfl_down(v, d);
        if ((threadIdx.x & 63) == 0) red[k][threadIdx.x >> 6] = v;
    }
    __syncthreads();
    if (threadIdx.x < 5) {
        unsigned long long v = red[threadIdx.x][0] + red[threadIdx.x][1] + red[threadIdx.x][2] + red[threadIdx.x][3];
        if (v) atomicAdd(&counters[threadIdx.x], v);
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

__global__ __launch_bounds__(PW) void k_fmt_reduce(const DeviceArgs* __restrict__ args, int64_t n_lines) {
    const Program& P = args->prog;
    const Columns& C = args->cols;
    const int64_t l0 = (int64_t)blockIdx.x * FMT_CHUNK + (int64_t)threadIdx.x * FMT_LPL;
    const uint64_t t = wave_scan_tables(lane_table(C, P, l0, n_lines));
    if (threadIdx.x == PW - 1) C.fmt_chunk[blockIdx.x] = t;
}

// one thread: chunk tables -> entry state of every chunk (in place), final
// state after the last chunk at [n_chunks]
__global__ void k_fmt_chunks(const DeviceArgs* __restrict__ args, int64_t n_chunks) {
    const Columns& C = args->cols;
    uint32_t s = C.fmt_init;
    for (int64_t c = 0; c < n_chunks; ++c) {
        const uint64_t t = C.fmt_chunk[c];
        C.fmt_chunk[c] = s;
        s = fmt_apply(t, s);
    }
    C.fmt_chunk[n_chunks] = s;
}

__global__ __launch_bounds__(PW) void k_fmt_apply(const DeviceArgs* __restrict__ args, int64_t n_lines) {
    const Program& P = args->prog;
    const Columns& C = args->cols;
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

}  // namespace


int64_t count_chunks(uint64_t nbytes) { return (int64_t)((nbytes + CHUNK - 1) / CHUNK); }

int launch_count(const uint8_t* d_buf, uint64_t nbytes, uint64_t* d_chunk, uint16_t* d_nlmask, hipStream_t s) {
    int64_t nc = count_chunks(nbytes);
    if (nc == 0) return 0;
    hipLaunchKernelGGL(k_count_newlines, dim3((unsigned)nc), dim3(NL_THREADS), 0, s, d_buf, nbytes, d_chunk, d_nlmask);
    hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, s, d_chunk, nc);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_offsets(const uint16_t* d_nlmask, uint64_t nbytes, const uint64_t* d_chunk, uint64_t* d_line_off,
                   hipStream_t s) {
    int64_t nc = count_chunks(nbytes);
    if (nc == 0) return 0;
    hipLaunchKernelGGL(k_line_offsets, dim3((unsigned)nc), dim3(NL_THREADS), 0, s, d_nlmask, nbytes, d_chunk, d_line_off);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int64_t parse_waves(int64_t n_lines) { return (n_lines + PW - 1) / PW; }

#if defined(LP_PROFILE)
// profiling build: copy out (and clear) the per-point timestamp sums
extern "C" int lp_profile_read(unsigned long long* out, int n) {
    unsigned long long h[64 * 16];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_prof), sizeof h) != hipSuccess) return -1;
    for (int k = 0; k < n && k < 64; ++k) { out[2 * k] = h[k * 16]; out[2 * k + 1] = h[k * 16 + 1]; }
    hipMemset(nullptr, 0, 0);
    unsigned long long z[64 * 16] = {};
    hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof z);
    return 0;
}
#endif

int launch_route(const DeviceArgs* d_args, int64_t n_lines, hipStream_t s) {
    if (n_lines == 0) return 0;
    const int64_t nc = fmt_chunks(n_lines);
    hipLaunchKernelGGL(k_fmt_reduce, dim3((unsigned)nc), dim3(PW), 0, s, d_args, n_lines);
    hipLaunchKernelGGL(k_fmt_chunks, dim3(1), dim3(1), 0, s, d_args, nc);
    hipLaunchKernelGGL(k_fmt_apply, dim3((unsigned)nc), dim3(PW), 0, s, d_args, n_lines);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_parse(const uint8_t* d_buf, uint64_t nbytes, int64_t n_lines, const DeviceArgs* d_args, int n_elems,
                 int stack_depth, const uint32_t* d_wave_counts, unsigned long long* counters, hipStream_t s, int mode) {
    if (n_lines == 0) return 0;
    const int64_t waves = parse_waves(n_lines);
    // LDS window per wave: ~1.1x the mean bytes of 64 lines (+512 B), so
    // nearly every wave stages; at most 48 KiB (+ 18 KiB of class masks).  A window that does not fit
    // reads HBM directly.
    const uint64_t mean = (nbytes + n_lines - 1) / n_lines;
    // tuning knobs for profiling experiments (defaults are the product setting)
    const char* e1 = getenv("LP_WIN_PCT");
    const char* e2 = getenv("LP_NO_STAGE");
    const char* e4 = getenv("LP_MASKS");
    const bool masks = e4 ? atoi(e4) != 0 : true;
    const int force_global = e2 ? atoi(e2) : 0;
    const uint32_t stk_words = (uint32_t)(stack_depth > 0 ? stack_depth : 1) * PW;
    const uint64_t fixed = 16 * (uint64_t)n_elems + 4 * (uint64_t)stk_words;
    const uint64_t per8 = masks ? 8 + MC_N : 8;  // LDS bytes per 8 window bytes
    // The parse kernel is latency bound: its speed follows the waves a CU
    // holds, and LDS sets that number.  The window of a wave is sized to the
    // most waves per CU that still leave >= 4 % over the mean 64 lines (the
    // few windows that do not fit read HBM directly).  Measured on gfx950:
    // W waves of one 64-thread workgroup each fit when a wave's LDS is at
    // most 160 KiB / W - 640 B.
    const uint64_t need = PW * mean + PW * mean / 25 + 64;
    uint64_t cap = 0;
    for (int w = 8; w >= 2 && !cap; --w) {
        const uint64_t budget = 160 * 1024 / w - 640;
        if (budget <= fixed) continue;
        const uint64_t c = ((budget - fixed) * 8 / per8) & ~63ull;
        if (c >= need) cap = c;
    }
    if (!cap || e1) cap = ((PW * mean * (uint64_t)(e1 ? atoi(e1) : 110)) / 100 + 512 + 63) & ~63ull;
    if (cap > 48 * 1024) cap = 48 * 1024;
    const int stage = ((uintptr_t)d_buf & 15) == 0 && !force_global;
    const char* e3 = getenv("LP_LDS_PAD");  // profiling experiments: extra LDS per wave (lower occupancy)
    const size_t lds = 16 * (size_t)n_elems + stk_words * 4 + cap + (masks ? MC_N * (cap / 8) : 0) +
                       (e3 ? (size_t)atoi(e3) : 0);
    if (masks)
        hipLaunchKernelGGL(k_parse_lines<true>, dim3((unsigned)waves), dim3(PW), lds, s, d_buf, nbytes, n_lines, d_args,
                           (uint32_t)cap, stage, stk_words, mode);
    else
        hipLaunchKernelGGL(k_parse_lines<false>, dim3((unsigned)waves), dim3(PW), lds, s, d_buf, nbytes, n_lines,
                           d_args, (uint32_t)cap, stage, stk_words, mode);
    if (mode == PM_MATCH) return hipGetLastError() == hipSuccess ? 0 : -1;
    int64_t rb = (waves + 255) / 256;
    if (rb > 1024) rb = 1024;
    hipLaunchKernelGGL(k_reduce_counts, dim3((unsigned)rb), dim3(256), 0, s, d_wave_counts, waves, counters);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace lp
