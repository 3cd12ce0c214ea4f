// Host-callable launchers of the gfx950 kernels (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "lp_program.h"

namespace lp {

int set_program(const Program& p, hipStream_t s);
int64_t count_chunks(uint64_t nbytes);
// index pass 1: per-chunk '\n' counts, exclusively scanned in place;
// d_chunk needs count_chunks()+1 entries, d_chunk[nc] = total '\n' count
int launch_count(const uint8_t* d_buf, uint64_t nbytes, uint64_t* d_chunk, hipStream_t s);
// index pass 2: d_line_off[k] = start of line k for k >= 1 (caller sets [0])
int launch_offsets(const uint8_t* d_buf, uint64_t nbytes, const uint64_t* d_chunk, uint64_t* d_line_off, hipStream_t s);
int launch_parse(const uint8_t* d_buf, int64_t n_lines, const Columns& C, hipStream_t s);

}  // namespace lp
