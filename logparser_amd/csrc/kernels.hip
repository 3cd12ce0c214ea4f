// gfx950 kernels of the logparser_amd engine: the separate line index (the
// first batch of a handle, and multi-format programs, whose routing pass
// needs the index first), the counter reduction, the sticky active-format
// scan and the run histograms.  The parse kernels are parse.hip, the URI
// kernels uri.hip; the shared wave scaffolding is kernels_common.h and the
// per-line logic lp_device.h.
//
//   k_count_newlines  per-chunk line terminator count and terminator bit masks ('\n', lone '\r',
//                     the '\n' of "\r\n"; 16-byte loads, SWAR byte compare)
//   k_scan_counts     exclusive scan of the chunk counts (single workgroup); the batch's line
//                     count, line_off[0] and the end sentinel, written on the device
//   k_line_offsets    line start offsets from the bit masks (Hadoop LineRecordReader '\n' semantics)
//   k_reduce_counts   per-wave status counts -> the batch counters
//   k_fmt_*           the sticky active-format scan (routing pass 2)
//   k_histograms      run histograms of a parsed batch (on demand)
#include "kernels_common.h"

namespace lp {

namespace {

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

// meta->counters[0..5] += sum of the per-wave counts (lines ok bad fallback arena-bytes URI-source-bytes)
// n_entries: the per-chunk count records of the launch that wrote them, or
// (per_group) at most that many records of 64-line groups, of which only the
// batch's lines' groups were written; nothing is counted when the batch
// overflowed its columns
__global__ __launch_bounds__(256) void k_reduce_counts(const uint32_t* __restrict__ wc, int64_t n_entries, int per_group,
                                                       Meta* __restrict__ meta) {
    int64_t n_waves = meta->cap_ovf ? 0 : n_entries;
    if (per_group) n_waves = min(n_waves, (int64_t)((meta->n_lines + PW - 1) / PW));
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
// The parse kernels left one histogram word per OK line (lp_device.h
// hist_word: present tokens, status code, method), so this pass reads 9
// bytes per line (status, token flags, that word), not the input.
// Grid-stride over lines, one LDS histogram per block, flushed with global
// atomics (a few thousand per launch).
__global__ __launch_bounds__(256) void k_histograms(const DeviceArgs* __restrict__ args,
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
        if (P.n_fmt > 1 && C.fmt_id[li] >= P.n_fmt) continue;
        const uint32_t flags = C.tok_flags[li], w = C.hist[li];
        for (uint32_t m = flags & 0xFFFFu & ((1u << P.n_tok) - 1u); m; m &= m - 1) atomicAdd(&h[16 + __builtin_ctz(m)], 1ull);
        for (uint32_t m = w & 0xFFFFu; m; m &= m - 1) atomicAdd(&h[32 + __builtin_ctz(m)], 1ull);
        const uint32_t code = (w >> 16) & 1023u, meth = w >> 26;
        if (code != 1023u) atomicAdd(&h[code ? 100 + code : 48], 1ull);
        if (meth != 31u) atomicAdd(&h[64 + meth], 1ull);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < HIST_WORDS; k += blockDim.x)
        if (h[k]) atomicAdd(&hist[k], h[k]);
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
    (void)buf;
    hipLaunchKernelGGL(k_histograms, dim3((unsigned)blocks), dim3(256), 0, s, d_args,
                       reinterpret_cast<unsigned long long*>(hist));
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_reduce_counts(const uint32_t* d_wave_counts, int64_t n_entries, bool per_group, Meta* d_meta, hipStream_t s) {
    int64_t rb = (n_entries + 255) / 256;
    if (rb > 1024) rb = 1024;
    if (rb < 1) rb = 1;
    hipLaunchKernelGGL(k_reduce_counts, dim3((unsigned)rb), dim3(256), 0, s, d_wave_counts, n_entries, per_group ? 1 : 0,
                       d_meta);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace lp
