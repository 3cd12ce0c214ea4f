// Host-callable launchers of the gfx950 kernels (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "lp_program.h"

namespace lp {

// Everything the parse kernel reads besides the input: copied to the device
// per batch (stream-ordered), so concurrent handles never share state.
struct DeviceArgs {
    Program prog;
    Columns cols;
};

int64_t count_chunks(uint64_t nbytes);
// index pass 1: per-chunk '\n' counts, exclusively scanned in place;
// d_chunk needs count_chunks()+1 entries, d_chunk[nc] = total '\n' count
// and d_nlmask[i] = '\n' bits of bytes [16 i, 16 i + 16) (nlmask_words() entries)
int launch_count(const uint8_t* d_buf, uint64_t nbytes, uint64_t* d_chunk, uint16_t* d_nlmask, hipStream_t s);
inline int64_t nlmask_words(uint64_t nbytes) { return count_chunks(nbytes) * (64 * 1024 / 16); }
// index pass 2 (from the masks): d_line_off[k] = start of line k for k >= 1 (caller sets [0])
int launch_offsets(const uint16_t* d_nlmask, uint64_t nbytes, const uint64_t* d_chunk, uint64_t* d_line_off,
                   hipStream_t s);
// parse kernels: number of waves (C.wave_counts needs WC_WORDS u32 per wave)
constexpr int WC_WORDS = 8;
int64_t parse_waves(int64_t n_lines);
// parse every line, then counters[0..4] += lines, ok, bad, fallback, arena bytes written
// (mode PM_PARSE); mode PM_MATCH only writes C.fmt_match (sticky routing pass 1)
enum { PM_PARSE = 0, PM_MATCH = 1 };
int launch_parse(const uint8_t* d_buf, uint64_t nbytes, int64_t n_lines, const DeviceArgs* d_args, int n_elems,
                 int stack_depth, const uint32_t* d_wave_counts, unsigned long long* counters, hipStream_t s,
                 int mode = PM_PARSE);
// sticky routing pass 2: C.fmt_match -> C.fmt_id (C.fmt_chunk: fmt_chunks()+1 words, the
// state after the last line at [fmt_chunks()])
constexpr int FMT_CHUNK = 4096;
inline int64_t fmt_chunks(int64_t n_lines) { return (n_lines + FMT_CHUNK - 1) / FMT_CHUNK; }
int launch_route(const DeviceArgs* d_args, int64_t n_lines, hipStream_t s);

}  // namespace lp
