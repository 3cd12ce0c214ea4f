// Host-callable launchers of the gfx950 kernels (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "lp_program.h"
#include "lp_table.h"

namespace lp {

// Everything the parse kernels read besides the input: copied to the device
// per batch (stream-ordered), so concurrent handles never share state.
struct DeviceArgs {
    Program prog;
    Columns cols;
};

int64_t count_chunks(uint64_t nbytes);
inline int64_t nlmask_words(uint64_t nbytes) { return count_chunks(nbytes) * (64 * 1024 / 16); }
// line index, pass 1: per-chunk '\n' counts (exclusively scanned in place,
// d_chunk needs count_chunks()+1 entries) and the '\n' bit mask of every 16
// input bytes (d_nlmask, nlmask_words() entries); the scan also sets
// meta->n_lines (Hadoop LineRecordReader count: a final unterminated line
// counts), line_off[0] and the end sentinel, and meta->cap_ovf when the
// batch has more lines than the columns hold (cap_lines).
int launch_count(const uint8_t* d_buf, uint64_t nbytes, uint64_t* d_chunk, uint16_t* d_nlmask, uint64_t* d_line_off,
                 int64_t cap_lines, Meta* d_meta, hipStream_t s);
// line index, pass 2 (from the masks): line_off[k] = start of line k (k <= cap_lines)
int launch_offsets(const uint16_t* d_nlmask, uint64_t nbytes, const uint64_t* d_chunk, uint64_t* d_line_off,
                   int64_t cap_lines, hipStream_t s);

// parse kernels: one wave per 64 lines (C.wave_counts needs WC_WORDS u32 per wave)
constexpr int WC_WORDS = 8;
int64_t parse_waves(int64_t n_lines);
struct ParseLaunch {
    const uint8_t* buf;
    uint64_t nbytes;
    int64_t cap_lines;      // grid: parse_waves(cap_lines) waves; lines >= meta->n_lines exit
    uint64_t mean_line;     // expected mean line length (sizes the LDS window)
    int n_elems, stack_depth;
    bool force_direct;      // every wave on the direct (HBM) path: tests / diagnostics only
    bool uri;               // the program has URI stages (k_uri_lines after the parse kernel)
    bool derived;           // ... some of them derived (type remapping: k_derived_lines after those)
    int n_uri, n_query;     // URI / query stages (the URI kernel instance)
    void* mid_event = nullptr;  // hipEvent_t recorded between the parse kernels and the URI kernels
    bool chunked = false;       // one-format program: k_parse_chunks builds the line index itself
    uint32_t chunk_lines = 0;   // lines per byte chunk the chunked kernel aims for (0: default)
    int32_t chunk_wait = 0;     // polls for a chunk's line number before deferring it (0: default, < 0: none)
    bool lit_aware = true;      // the program has a [^\s]* / "$request" element a shorter end of which can meet
                                // its literal (the chunked kernel's instance with literal-aware first candidates)
    bool simple = false;        // one format of the Apache common / combined family (capi simple_program)
    bool multi = false;         // several LogFormats on the one-pass path (routing inside the chunk kernel)
};
// The chunked parse kernel's geometry: cb input bytes per chunk (one wave
// each), an LDS window of win_cap bytes (the chunk, 64 bytes before it, the
// tail of its last line), n_chunks chunks.
struct ChunkPlan {
    uint32_t cb, win_cap, stk_words, chunk_stk;  // stk_words: the queued lines' kernels; chunk_stk: the chunk kernels'
    int waves_per_cu;
    size_t lds;
    int64_t n_chunks;
};
ChunkPlan chunk_plan(const ParseLaunch& a);
// parse every line, then the URI stages (k_uri_lines, and its direct path),
// then meta->counters[0..4] += lines, ok, bad, fallback, arena bytes written.
// Chunked (a.chunked): k_parse_chunks writes the line index, meta->n_lines /
// cap_ovf and the lines' rows, k_parse_ovf_lines the lines it queued
// (C.chunk_state zeroed, C.chunk_counts and C.deferred_chunks: chunk_plan().n_chunks records,
// C.ovf_lines: cap_lines entries).  Otherwise the line index exists and the
// staged waves, then the waves whose window did not fit LDS, run
// (C.ovf_list and C.uri_ovf_list: parse_waves(cap_lines) + 1 entries each).
// C: the host copy of the columns the device holds.
int launch_parse(const ParseLaunch& a, const DeviceArgs* d_args, const Columns& C, hipStream_t s);
// the URI kernels of a launch (uri.hip)
int launch_uri(const ParseLaunch& a, const DeviceArgs* d_args, hipStream_t s);
// meta->counters[0..5] += the sum of n_entries count records (per_group: of
// 64-line groups, only those holding the batch's meta->n_lines lines)
int launch_reduce_counts(const uint32_t* d_wave_counts, int64_t n_entries, bool per_group, Meta* d_meta, hipStream_t s);
#if defined(LP_PROFILE)
int prof_read_parse(unsigned long long* out);
int prof_clear_parse();
int prof_read_uri(unsigned long long* out);
int prof_clear_uri();
#endif
// sticky routing pass 1: C.fmt_match of every line
int launch_route_match(const ParseLaunch& a, const DeviceArgs* d_args, hipStream_t s);
// sticky routing pass 2: C.fmt_match -> C.fmt_id (C.fmt_chunk: fmt_chunks()+1 words, the
// state after the last line at [fmt_chunks(n_lines)])
constexpr int FMT_CHUNK = 4096;
__host__ __device__ inline int64_t fmt_chunks(int64_t n_lines) { return (n_lines + FMT_CHUNK - 1) / FMT_CHUNK; }
int launch_route(const DeviceArgs* d_args, int64_t cap_lines, hipStream_t s);

// run histograms of the parsed batch (buf: its input) into hist
// (HIST_WORDS u64, zeroed here): layout in include/logparser_amd.h
constexpr int HIST_WORDS = 1024;
int launch_histograms(const DeviceArgs* d_args, const uint8_t* buf, int64_t cap_lines, uint64_t* hist, hipStream_t s);

// device table (table.hip, lp_table.h): scratch bytes for count rows; the
// values / validity / STRING offsets of rows [ta.first, ta.first + ta.count)
// (d_targs: ta on the device; buf: the batch's input); then, once the caller
// checked the offsets' totals against its capacities, the STRING bytes
size_t table_scratch_bytes(int64_t count, int n_str);
// where TableArgs::srcw starts in that scratch
size_t table_srcw_offset(int64_t count);
// mid (optional): recorded after k_table_values, before the offset scans
int launch_table_values(const DeviceArgs* d_args, const TableArgs* d_targs, const TableArgs& ta, const uint8_t* buf,
                        void* scratch, size_t scratch_bytes, hipStream_t s, hipEvent_t mid = nullptr);
int launch_table_chars(const DeviceArgs* d_args, const TableArgs* d_targs, const TableArgs& ta, const uint8_t* buf,
                       hipStream_t s);

}  // namespace lp
