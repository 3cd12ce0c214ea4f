// gfx950 kernels of the logparser_amd engine.
//
//   k_count_newlines  per-chunk '\n' count (16-byte loads, SWAR byte compare)
//   k_scan_counts     exclusive scan of the chunk counts (single workgroup)
//   k_line_offsets    line start offsets (Hadoop LineRecordReader '\n' semantics)
//   k_parse_lines     one thread per line: LogFormat match + token / time /
//                     first-line stages (phase 1), wave-aggregated arena
//                     allocation, URI + query-string stages (phase 2)
//
// The per-line logic is lp_device.h; this file only adds the data-parallel
// scaffolding around it.
#include <hip/hip_runtime.h>

#include "kernels.h"
#include "lp_device.h"

namespace lp {

__constant__ Program c_prog;

namespace {

constexpr int CHUNK = 64 * 1024;  // bytes per workgroup in the newline passes
constexpr int NL_THREADS = 256;   // 256 threads x 16 B x 16 iterations = 64 KiB

// exact per-byte "== '\n'" mask of a 32-bit word (high bit of each byte)
__device__ __forceinline__ uint32_t nl_mask(uint32_t w) {
    uint32_t x = w ^ 0x0A0A0A0Au;
    return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
}

__device__ __forceinline__ uint32_t count_nl16(const uint8_t* p, uint64_t pos, uint64_t nbytes) {
    if (pos + 16 <= nbytes && ((uintptr_t)(p + pos) & 15) == 0) {
        uint4 v = *reinterpret_cast<const uint4*>(p + pos);
        return __popc(nl_mask(v.x)) + __popc(nl_mask(v.y)) + __popc(nl_mask(v.z)) + __popc(nl_mask(v.w));
    }
    uint32_t c = 0;
    for (uint64_t k = pos; k < pos + 16 && k < nbytes; ++k) c += p[k] == '\n';
    return c;
}

__global__ __launch_bounds__(NL_THREADS) void k_count_newlines(const uint8_t* __restrict__ buf, uint64_t nbytes,
                                                                uint64_t* __restrict__ counts) {
    const uint64_t base = (uint64_t)blockIdx.x * CHUNK;
    uint32_t c = 0;
    for (int it = 0; it < CHUNK / (NL_THREADS * 16); ++it) {
        uint64_t pos = base + ((uint64_t)it * NL_THREADS + threadIdx.x) * 16;
        if (pos < nbytes) c += count_nl16(buf, pos, nbytes);
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
    __shared__ uint64_t part[1024];
    const int64_t per = (n + 1023) / 1024;
    const int64_t a = (int64_t)threadIdx.x * per, b = a + per < n ? a + per : n;
    uint64_t s = 0;
    for (int64_t i = a; i < b; ++i) s += counts[i];
    part[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t run = 0;
        for (int t = 0; t < 1024; ++t) { uint64_t v = part[t]; part[t] = run; run += v; }
        counts[n] = run;
    }
    __syncthreads();
    uint64_t run = part[threadIdx.x];
    for (int64_t i = a; i < b; ++i) { uint64_t v = counts[i]; counts[i] = run; run += v; }
}

// line_off[j] = start of line j.  line_off[0] = 0 and the entry after every
// '\n' that is not the last byte; line_off[n_lines] = end sentinel.
__global__ __launch_bounds__(NL_THREADS) void k_line_offsets(const uint8_t* __restrict__ buf, uint64_t nbytes,
                                                              const uint64_t* __restrict__ chunk_base,
                                                              uint64_t* __restrict__ line_off) {
    const uint64_t base = (uint64_t)blockIdx.x * CHUNK;
    __shared__ uint32_t wsum[NL_THREADS / 64];
    uint64_t run = chunk_base[blockIdx.x];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int it = 0; it < CHUNK / (NL_THREADS * 16); ++it) {
        uint64_t pos = base + ((uint64_t)it * NL_THREADS + threadIdx.x) * 16;
        uint32_t c = pos < nbytes ? count_nl16(buf, pos, nbytes) : 0;
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
        if (c) {
            for (uint64_t q = pos; q < pos + 16 && q < nbytes; ++q)
                if (buf[q] == '\n') line_off[++k] = q + 1;
        }
        run += tot;
        __syncthreads();
    }
}

// per-thread DFS stack interleaved in LDS (conflict-free: lane-contiguous)
struct LdsStack {
    uint32_t* base;
    __device__ uint32_t& operator[](int k) const { return base[k * 256]; }
};

__global__ __launch_bounds__(256) void k_parse_lines(const uint8_t* __restrict__ buf, int64_t n_lines, Columns C) {
    __shared__ uint32_t stk[MAX_STACK * 256];
    __shared__ unsigned long long cnt[4];
    if (threadIdx.x < 4) cnt[threadIdx.x] = 0;
    __syncthreads();
    const int64_t li = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool active = li < n_lines;
    const Program& P = c_prog;
    LineOut o;
    o.status = ST_OK;
    o.arena_need = 0;
    Line L{buf, 0};
    if (active) {
        const uint64_t s = C.line_off[li], e = C.line_off[li + 1] - 1;  // exclude '\n'
        L.s = buf + s;
        L.n = (int)((e - s) > (uint64_t)0x7FFFFFFF ? 0x7FFFFFFF : (e - s));
        phase1(P, L, o, LdsStack{stk + threadIdx.x}, C, li);
    }
    // wave-aggregated arena allocation (every lane reaches this point)
    uint32_t need = (active && o.status == ST_OK) ? o.arena_need : 0u;
    const int lane = threadIdx.x & 63;
    uint32_t x = need;
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(x, d);
        if (lane >= d) x += y;
    }
    uint32_t total = __shfl(x, 63);
    unsigned long long wbase = 0;
    if (lane == 63 && total) wbase = atomicAdd(C.arena_top, (unsigned long long)total);
    wbase = __shfl(wbase, 63);
    if (active) {
        if (o.status == ST_OK && need) {
            unsigned long long mine = wbase + x - need;
            if (mine + need > C.arena_cap) o.status = ST_FALLBACK;
            else {
                C.arena_base[li] = mine;
                Arena A{C.arena + mine, 0, need};
                phase2(P, L, o, A, C, li);
            }
        } else if (o.status == ST_OK) {
            C.arena_base[li] = 0;
        }
        write_line(P, o, C, li);
        atomicAdd(&cnt[0], 1ull);
        atomicAdd(&cnt[1 + o.status], 1ull);
    }
    __syncthreads();
    if (threadIdx.x < 4 && cnt[threadIdx.x]) atomicAdd(&C.counters[threadIdx.x], cnt[threadIdx.x]);
}

}  // namespace

int set_program(const Program& p, hipStream_t s) {
    return hipMemcpyToSymbolAsync(HIP_SYMBOL(c_prog), &p, sizeof(Program), 0, hipMemcpyHostToDevice, s) == hipSuccess ? 0 : -1;
}

int64_t count_chunks(uint64_t nbytes) { return (int64_t)((nbytes + CHUNK - 1) / CHUNK); }

int launch_count(const uint8_t* d_buf, uint64_t nbytes, uint64_t* d_chunk, hipStream_t s) {
    int64_t nc = count_chunks(nbytes);
    if (nc == 0) return 0;
    hipLaunchKernelGGL(k_count_newlines, dim3((unsigned)nc), dim3(NL_THREADS), 0, s, d_buf, nbytes, d_chunk);
    hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, s, d_chunk, nc);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_offsets(const uint8_t* d_buf, uint64_t nbytes, const uint64_t* d_chunk, uint64_t* d_line_off, hipStream_t s) {
    int64_t nc = count_chunks(nbytes);
    if (nc == 0) return 0;
    hipLaunchKernelGGL(k_line_offsets, dim3((unsigned)nc), dim3(NL_THREADS), 0, s, d_buf, nbytes, d_chunk, d_line_off);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_parse(const uint8_t* d_buf, int64_t n_lines, const Columns& C, hipStream_t s) {
    if (n_lines == 0) return 0;
    unsigned blocks = (unsigned)((n_lines + 255) / 256);
    hipLaunchKernelGGL(k_parse_lines, dim3(blocks), dim3(256), 0, s, d_buf, n_lines, C);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace lp
