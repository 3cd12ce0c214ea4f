/*
 * logparser_amd -- MI355X (gfx950) batch engine for logparser's per-line hot
 * path: match Apache HTTPD access-log lines against a LogFormat and extract
 * typed fields (tokens, epoch-millisecond timestamps, request first line,
 * URI parts, percent-decoded query parameters).
 *
 * Drop-in boundary.  Every entry point below replaces a piece of the
 * reference's per-line Java path (paths relative to the reference repo,
 * hp/ = httpdlog/httpdlog-parser/src/main/java/nl/basjes/parse/httpdlog/,
 * core/ = parser-core/src/main/java/nl/basjes/parse/core/):
 *
 *   lp_compile        new HttpdLoglineParser<>(cls, logformat) + addParseTarget(...)
 *                     + the lazy Parser.assembleDissectors on first parse
 *                     (hp/HttpdLoglineParser.java:44-50,104-126;
 *                      core/Parser.java:237-356, 581-635;
 *                      hp/dissectors/tokenformat/TokenFormatDissector.java:127-213)
 *   lp_possible_paths Parser.getPossiblePaths() (core/Parser.java:904-1012)
 *   lp_parse_batch    a loop of Parser.parse(record, line) over a batch of
 *                     '\n'-separated lines (core/Parser.java:716-756), i.e.
 *                     HttpdLogFormatDissector.dissect + TokenFormatDissector.dissect
 *                     (hp/HttpdLogFormatDissector.java:173-204,
 *                      hp/dissectors/tokenformat/TokenFormatDissector.java:243-275)
 *                     and the downstream TimeStamp / HttpFirstLine / HttpUri /
 *                     QueryStringField / CLF converter dissectors -- run on the GPU.
 *   lp_line_status    the per-line outcome the caller's loop sees
 *                     (ApacheHttpdLogfileRecordReader.java:256-269): OK, BAD
 *                     (= DissectionFailure), FALLBACK (= not proven on device:
 *                     hand the line to the reference Java dissector).
 *   lp_line_record_json  the values the reference would have delivered to the
 *                     record's setters for that line (Parser.store,
 *                     core/Parser.java:760-876), as a canonical JSON object.
 *   lp_counters       the RecordReader counters "Lines read / Good lines /
 *                     Bad lines" (ApacheHttpdLogfileRecordReader.java:118-120)
 *                     plus the FALLBACK count.
 *   lp_result_*       the whole batch's SoA results in bulk: what a Java
 *                     GpuHttpdLogFormatDissector replays into
 *                     Parsable.addDissection (core/Dissector.java:62-186,
 *                     core/Parsable.java:77-140), see INTEGRATION.md.
 *
 * Threading: like the reference Parser (not thread-safe), one handle per
 * host thread / GPU.  Ownership: the caller owns the input buffer; the
 * handle owns device scratch and results until the next lp_parse_batch or
 * lp_free.  No torch types cross this boundary.
 */
#ifndef LOGPARSER_AMD_H
#define LOGPARSER_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* return codes */
#define LP_OK 0
#define LP_E_INVALID (-1)      /* bad arguments / logformat (InvalidDissectorException) */
#define LP_E_MISSING (-2)      /* MissingDissectorsException */
#define LP_E_UNSUPPORTED (-3)  /* compiled, but some requested path needs a dissector
                                  not implemented on the device: every line -> FALLBACK */
#define LP_E_DEVICE (-4)       /* HIP error / no device / extension not usable */
#define LP_E_NOMEM (-5)
#define LP_E_STATE (-6)        /* called in the wrong order */

/* per-line status */
#define LP_LINE_OK 0
#define LP_LINE_BAD 1          /* the reference throws DissectionFailure */
#define LP_LINE_FALLBACK 2     /* outside the device's proven subset */

/* lp_parse_batch buffer flags */
#define LP_BUF_HOST 0          /* host memory: copied H2D on the stream */
#define LP_BUF_DEVICE 1        /* device pointer, already resident in HBM */

typedef struct lp_handle lp_handle;

/* Compile a LogFormat (one or more, '\n' separated; aliases common /
 * combined / combinedio / referer / agent) and the requested "TYPE:path"
 * targets.  device: HIP device ordinal.  Returns NULL on failure; *status
 * receives LP_OK / LP_E_UNSUPPORTED (handle still usable) / error code. */
lp_handle *lp_compile(const char *logformats, const char *const *paths, int n_paths,
                      int device, int *status, char *err, size_t errlen);

/* Parser.addTypeRemapping(input, newType, casts) (core/Parser.java:636-677):
 * a value delivered at path `input` is delivered again as type `type`
 * (Parsable.addDissection, core/Parsable.java:160-176), where that type's
 * dissectors take it further (Parser.java:446-455): e.g. a query parameter
 * holding a URL, remapped to HTTP.URI, is dissected by HttpUriDissector on
 * the device (the "derived" URI stages).  casts: LP_CAST_* bits of the
 * remapped target (the reference's STRING_ONLY default is LP_CAST_STRING). */
typedef struct lp_remap {
    const char *input;
    const char *type;
    int32_t casts;
} lp_remap;
/* lp_compile with the parser's type remappings (n_remaps may be 0). */
lp_handle *lp_compile_remapped(const char *logformats, const char *const *paths, int n_paths,
                               const lp_remap *remaps, int n_remaps, int device, int *status, char *err,
                               size_t errlen);
void lp_free(lp_handle *h);

/* Parser.getPossiblePaths(max_depth) for a logformat: '\n'-separated, sorted.
 * Returns the number of bytes written (excluding NUL) or a negative error. */
int64_t lp_possible_paths(const char *logformats, int max_depth, char *out, size_t cap);
/* The same with type remappings: each remapped path and what the new type's
 * dissectors produce below it (core/Parser.java:954-962). */
int64_t lp_possible_paths_remapped(const char *logformats, int max_depth, const lp_remap *remaps, int n_remaps,
                                   char *out, size_t cap);

/* Options (lp_set_option). */
#define LP_OPT_FORCE_DIRECT 1  /* 1: every wave reads its lines from HBM (no LDS window);
                                  diagnostics and tests of the direct path only */
#define LP_OPT_MAX_RETRIES 2   /* re-runs of a batch whose ARENA estimate was short (default 3,
                                  0..16); an arena still short after them degrades: the lines
                                  that did not fit are FALLBACK, lp_counters out[6].  A short
                                  line capacity is always re-run with the exact count (at most
                                  twice, not bounded by this option): nothing is parsed without
                                  columns for every line */
#define LP_OPT_ARENA_BYTES 3   /* tests: exact arena capacity of each batch's first run (0 = estimate) */
#define LP_OPT_CHUNK_LINES 4   /* one-format programs: lines per byte chunk the one-pass parse kernel
                                  aims for (1..64, 0 = default 54; a chunk's 65th line onwards is
                                  parsed from HBM by a second kernel) */
#define LP_OPT_CHUNK_WAIT 5    /* tests: polls a chunk's wave makes for its first line number before it
                                  leaves the chunk to the deferred pass (0 = default 16384; -1: none,
                                  every chunk goes to the deferred pass; -2: the odd chunks go to it
                                  without polling, the even ones wait as by default) */
#define LP_OPT_ONE_PASS 6      /* several LogFormats: 1 (default) one pass over the input (the chunk kernel
                                  routes every line exactly one format matches; the rest after the
                                  routing scan), 0 the line index, routing and parse passes */
int lp_set_option(lp_handle *h, int option, int64_t value);

/* Capacity for the coming batches: columns for max_lines lines and at least
 * arena_bytes of side arena (0 = estimated; the estimate wins when larger).
 * With it (or after a first batch, whose line count sizes the buffers)
 * lp_parse_batch enqueues the whole batch without waiting for the device; a
 * batch that outgrows the buffers is re-run with exact sizes inside lp_sync
 * (a short arena at most LP_OPT_MAX_RETRIES times, after which the lines that
 * did not fit go to FALLBACK instead of failing the batch; a short line
 * capacity at most twice, with the exact count). */
int lp_reserve(lp_handle *h, int64_t max_lines, uint64_t arena_bytes);

/* Parse every line of buf[0, nbytes), Hadoop LineRecordReader semantics
 * (ApacheHttpdLogfileRecordReader.java:57, 115): a line ends at '\n', at a
 * lone '\r' or at "\r\n", the terminator is not part of it, and a final
 * line without one counts.  stream: a hipStream_t (NULL = default stream).
 * Enqueues all work on the stream and returns without synchronizing (except a
 * handle's first batch without a reservation, which waits for its line
 * count); call lp_sync before reading results.  A batch still pending on the
 * handle is finished first: to overlap batches, use one handle per stream.
 * On error the handle holds no batch (the accessors return LP_E_STATE) until
 * a batch succeeds.
 * first_line_no (lp_parse_batch_at): the global number of the batch's first
 * line (a split reader's position in the stream); it comes
 * back in lp_result.first_line.  lp_parse_batch continues the handle's
 * numbering (0 for its first batch, then the previous batch's first line +
 * its line count). */
int lp_parse_batch(lp_handle *h, const uint8_t *buf, uint64_t nbytes, int buf_flags, void *stream);
int lp_parse_batch_at(lp_handle *h, const uint8_t *buf, uint64_t nbytes, int64_t first_line_no, int buf_flags,
                      void *stream);
int lp_sync(lp_handle *h);

/* Results of the last batch (after lp_sync). */
int64_t lp_num_lines(lp_handle *h);
/* copies statuses of lines [first, first+count) to host memory */
int lp_line_status(lp_handle *h, int64_t first, int64_t count, uint8_t *out);
/* byte offset of line i in the batch (i <= num_lines) */
int64_t lp_line_offset(lp_handle *h, int64_t i);
/* canonical record of line i (status must be OK):
 *   {"TYPE:path": [v, ...], ...}  keys sorted; v = "str" | null | {"l": n}
 * returns bytes written (excluding NUL) or negative (LP_E_STATE if the line
 * is not OK, -100 - needed if cap is too small). */
int64_t lp_line_record_json(lp_handle *h, int64_t i, char *out, size_t cap);
/* out[0..3] = lines, ok, bad, fallback of the last batch (device counters);
 * diagnostics: out[4] = one LogFormat: lines parsed by the direct kernel (a
 * byte chunk's 65th line onwards, or a line ending past the chunk's LDS
 * window); several LogFormats: waves parsed by the overflow kernel (their
 * lines' window exceeded the main kernel's LDS window), out[5] = re-runs of the
 * batch (capacity / arena estimates exceeded), out[6] = arena overflows the
 * final run left (lines sent to FALLBACK for want of arena; 0 normally),
 * out[7] = waves whose URI bytes exceeded the URI kernel's compact buffer
 * (their URI stages read the input from HBM directly), out[8] = one-format
 * programs: byte chunks redone by the deferred pass (their wave stopped
 * waiting for its first line number; 0 normally, see LP_OPT_CHUNK_WAIT).
 * Returns the words written (at most 9). */
int lp_counters(lp_handle *h, uint64_t *out, int n);

/* Device-side timing of the last batch, in milliseconds, measured with HIP
 * events on the batch's stream: [0] whole batch, [1] separate line index
 * kernels (0 for one-LogFormat programs after a handle's first batch: their
 * parse kernel finds the lines itself), [2] parse pass (every kernel after
 * the index), [3] of it the parse kernels (one LogFormat: k_parse_chunks +
 * k_parse_ovf_lines; several: routing match + k_parse_lines + its direct
 * path), [4] of it the URI kernels (+ the counter reduction); then the last
 * complete lp_result_table on a device view: [5] k_table_values, [6] the
 * STRING columns' offset scans, [7] k_table_chars.  Returns the number of
 * values written. */
int lp_last_timing(lp_handle *h, float *out_ms, int n);

/* Run histograms of the last batch, computed on the device (SURVEY.md §5
 * counters; multi-GPU callers all-reduce them, e.g. over RCCL).  out: 1024
 * u64 words, host memory, or device memory on the handle's device when
 * out_on_device (then usable directly as an all-reduce buffer).  The batch's
 * input must still be valid.  Layout (word: count):
 *   0 lines, 1 OK, 2 BAD, 3 FALLBACK lines
 *   16 + k: OK lines whose captured token slot k is "-" (null)
 *   32 + k: OK lines whose token slot k is present and non-empty
 *   48: OK lines whose status value (token request.status.last, else
 *       request.status, if requested) is not a code 100..599
 *   64 + m: OK lines by request method (first-line dissector, if requested):
 *       m = 0 GET 1 POST 2 HEAD 3 PUT 4 DELETE 5 OPTIONS 6 PATCH 7 CONNECT
 *       8 TRACE 9 PROPFIND 10 MKCOL 11 COPY 12 MOVE 13 LOCK 14 UNLOCK
 *       15 other, 16 no method
 *   100 + c: OK lines with status code c (100 <= c <= 599)
 * Replaces the reference's Hadoop counters (ApacheHttpdLogfileRecordReader.java:118-120)
 * for a batch; returns LP_OK or an error. */
#define LP_HIST_WORDS 1024
#define LP_HIST_LINES 0
#define LP_HIST_OK 1
#define LP_HIST_BAD 2
#define LP_HIST_FALLBACK 3
#define LP_HIST_TOK_NULL 16
#define LP_HIST_TOK_PRESENT 32
#define LP_HIST_STATUS_OTHER 48
#define LP_HIST_METHOD 64
#define LP_HIST_STATUS 100
int lp_histograms(lp_handle *h, uint64_t *out, int out_on_device);

/* Algorithmic bytes of the last batch: [0] input bytes read, [1] bytes of
 * SoA results + arena written, [2] the parse kernels' bytes (input once,
 * line index, their columns), [3] the URI kernels' bytes (URI source bytes
 * gathered, the per-line columns they read, their columns and arena
 * writes) -- roofline accounting per kernel (timings [3] and [4]). */
int lp_last_bytes(lp_handle *h, uint64_t *out, int n);

/* ---- Bulk results: the SoA the kernels wrote (SURVEY.md §8(b) lp_result). ----
 * Per line i: status[i] (LP_LINE_*), and for the compiled program's stages
 * the columns listed in lp_result.column (name, stage index, element size,
 * byte offset from lp_result.columns), each n_lines elements:
 *   status (u8), tok_span[k] (u32 start | end << 16, line-relative) and
 *   tok_flags (u32: bit k value "-" = null, bit 16+k value "0") per captured
 *   token k; t_epoch[t] (i64 epoch ms), t_local[t] / t_utc[t] (u64 packed
 *   calendar, lp_program.h pack_cal), t_nano[t] (u32) per timestamp stage;
 *   fl_kind / fl_method / fl_uri / fl_proto (u32 kind, spans) per first-line
 *   stage; u_flags (u32 UF_* bits), u_scheme / u_host / u_path / u_query /
 *   u_frag (u64 refs) and u_port (i32) per URI stage; q_count (u32) and
 *   q_params (u64 ref of a table of q_count (name ref, value ref) pairs) per
 *   query stage; arena_base (u64, the line's arena region); fmt_id (u8, the
 *   routed LogFormat) with several LogFormats.
 * A ref is off | len << 32 (len 30 bits); bit 63 set: the bytes are in the
 * line's arena region, else line-relative; bit 62: '&' followed by those
 * bytes.  A q_params table slot whose parameter name was not requested holds
 * ~0 (REF_SKIP) as its name ref: skip it.  Arena offsets b live in shard
 * s = b / shard_cap, at arena + shard_off[s] + (b - s * shard_cap). */
#define LP_ARENA_SHARDS 64
typedef struct lp_column {
    char name[16];
    int32_t index;
    int32_t elem_size;
    uint64_t offset;
} lp_column;
typedef struct lp_result {
    int64_t n_lines;
    int64_t first_line;        /* global number of line 0 of the batch (lp_parse_batch_at) */
    uint64_t input_bytes;
    const uint8_t *input;      /* line i = input[line_off[i], line_off[i+1] - 1), less the '\r' of a
                                  "\r\n" terminator; NULL if not copied */
    const uint64_t *line_off;  /* n_lines + 1 entries */
    const uint8_t *columns;
    uint64_t columns_bytes;
    const uint8_t *arena;
    uint64_t arena_bytes;
    uint64_t shard_cap;
    uint64_t shard_off[LP_ARENA_SHARDS];
    int32_t n_columns;
    int32_t on_host;           /* 0: device pointers (lp_result_view), 1: host copy (lp_result_copy) */
    const lp_column *column;   /* view: owned by the handle, valid until its next batch;
                                  host copy: inside the copy's buffer */
} lp_result;
/* Device pointers of the last batch's results (valid until the next batch). */
int lp_result_view(lp_handle *h, lp_result *out);
/* Copy the last batch's results (line index, columns, used arena, and the
 * input when with_input) into host memory (pinned memory copies fastest) in
 * one call.  Returns the bytes used, or -(bytes needed) when host is NULL or
 * cap is too small. */
int64_t lp_result_copy(lp_handle *h, void *host, uint64_t cap, int with_input, lp_result *out);
/* The canonical record of line i (as lp_line_record_json) from a host copy
 * made with the input: no device access. */
int64_t lp_result_record_json(lp_handle *h, const lp_result *r, int64_t i, char *out, size_t cap);

/* The reference's Parsable.addDissection(base, type, name, value) calls
 * that deliver line i's requested values (core/Parsable.java:77-193), from a
 * host copy made with the input, in the reference's emission order: what a
 * Java GpuHttpdLogFormatDissector.dissect replays.  kind:
 * LP_VALUE_STRING (bytes p[0, len), UTF-8), LP_VALUE_NULL, LP_VALUE_LONG (l).
 * Returns the number of calls, or LP_E_STATE when line i is not OK. */
#define LP_VALUE_STRING 0
#define LP_VALUE_NULL 1
#define LP_VALUE_LONG 2
typedef void (*lp_emit_fn)(void *ctx, const char *base, const char *type, const char *name, int kind,
                           const uint8_t *p, uint32_t len, int64_t l);
int lp_result_emit(lp_handle *h, const lp_result *r, int64_t i, lp_emit_fn fn, void *ctx);

/* Parser.getCasts(name) (parser-core/.../core/Parser.java:127-129, filled
 * at :438-439 from each dissector's prepareForDissect): the casts of a
 * "TYPE:path" the handle delivers, as LP_CAST_* bits (0 = NO_CASTS), or
 * LP_E_MISSING when no dissector delivers it.  The caller's setter side
 * (Parser.store, :760-876) needs them to pick String / Long / Double setters. */
#define LP_CAST_STRING 1
#define LP_CAST_LONG 2
#define LP_CAST_DOUBLE 4
int lp_casts(lp_handle *h, const char *target);

/* Typed columns of a batch, the output side of a parse: what a caller with
 * one setter per column type builds per line -- the Hadoop ParsedRecord
 * (httpdlog-inputformat/.../ParsedRecord.java:154-214: set(name, String /
 * Long / Double), nulls ignored, the last value wins) read back column by
 * column as the Hive SerDe does (httpdlog-serde/.../ApacheHttpdlogDeserializer.java:
 * 224-240 STRING / BIGINT / DOUBLE columns, :295-323 one row per line).
 * From a host copy (lp_result_copy with the input), rows [first, first+count):
 *   kind LP_CAST_STRING: i64 = byte offsets [count + 1] into chars (Arrow
 *        layout: row k = chars[i64[k], i64[k + 1])), chars_cap bytes at chars;
 *   kind LP_CAST_LONG:   i64 = values [count];  LP_CAST_DOUBLE: f64 = values;
 *   valid[k] = 1 when row k has a value (lines not OK have none).
 * path: a requested "TYPE:path" (a wildcard request's member by its full
 * path).  Returns LP_OK; LP_E_NOMEM when a STRING column's chars_cap is too
 * small (chars_len = bytes needed: call again); LP_E_MISSING for a path the
 * handle does not deliver; LP_E_INVALID when the path's casts (lp_casts) do
 * not include the column's type (the reference's store would call no setter).
 * threads: host threads to replay with.
 * On a device view (r from lp_result_view, on_host 0) the table is built on
 * the GPU from the batch still in HBM (its input must still be valid):
 * valid / i64 / f64 / chars are then device buffers of the handle's device,
 * the call returns once they are filled.  Request cookies, raw-token query
 * strings, Set-Cookie cookies and their value / expires / domain / comment /
 * path attributes, upstream list items (N.value / N.redirected, SECOND_MILLIS
 * in ms and us), BinaryIP and the first line / URI / query values are device
 * columns.  LP_E_UNSUPPORTED names a path whose value only the host replay
 * derives (a converter applied to an already converted value) or a DOUBLE
 * column of a string-valued path (Double.parseDouble): build those from a
 * host copy. */
typedef struct lp_table_col {
    const char *path;
    int32_t kind;
    uint8_t *valid;
    int64_t *i64;
    double *f64;
    char *chars;
    uint64_t chars_cap;
    uint64_t chars_len;
} lp_table_col;
int lp_result_table(lp_handle *h, const lp_result *r, int64_t first, int64_t count, lp_table_col *cols, int n_cols,
                    int threads);

/* Description of the compiled device program (for logs/tests), NUL-terminated. */
int64_t lp_describe(lp_handle *h, char *out, size_t cap);

/* Synthetic 'combined' access-log generator (deterministic per seed), used
 * by bench.py and tests to build BASELINE.json config-2 inputs.  Writes
 * complete lines into out (cap bytes) starting at line index first_line;
 * returns bytes written and sets *n_lines. */
int64_t lp_synth_combined(uint64_t seed, int64_t first_line, int64_t max_lines,
                          char *out, size_t cap, int64_t *n_lines);

/* The same for each BASELINE.json workload:
 *   LP_SYNTH_COMBINED  config 2, 'combined'
 *   LP_SYNTH_STRFTIME  config 3, '%h %l %u [%{%d/%b/%Y %T}t.%{msec_frac}t] "%r" %>s %b
 *                      "%{Referer}i" "%{User-Agent}i" %I %O', 5 % malformed lines
 *   LP_SYNTH_NGINX     config 4, the NGINX log_format of
 *                      hpt/nginxmodules/NginxUpstreamTest.java:94
 *   LP_SYNTH_MIXED     config 5, 40 % config-2, 30 % config-4 and 30 % 'common'
 *                      lines (mutually exclusive formats), chosen per line
 * Returns LP_E_INVALID for an unknown workload. */
#define LP_SYNTH_COMBINED 2
#define LP_SYNTH_STRFTIME 3
#define LP_SYNTH_NGINX 4
#define LP_SYNTH_MIXED 5
int64_t lp_synth(int workload, uint64_t seed, int64_t first_line, int64_t max_lines,
                 char *out, size_t cap, int64_t *n_lines);

#ifdef __cplusplus
}
#endif
#endif
