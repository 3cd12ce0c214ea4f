// C-ABI of the logparser_amd engine (include/logparser_amd.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <cmath>
#include <regex>
#include <thread>
#include <unordered_map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/logparser_amd.h"
#include "kernels.h"
#include "plan.h"

#if defined(LP_PROFILE)
// profiling build: copy out (and clear) the per-wave timestamps of the parse
// and URI kernels (PROF_WAVES x PROF_POINTS u64; the two kernel translation
// units mark disjoint points)
extern "C" int lp_profile_read(unsigned long long* out, int n) {
    if (n < lp::PROF_WAVES * lp::PROF_POINTS) return -1;
    std::vector<unsigned long long> u((size_t)lp::PROF_WAVES * lp::PROF_POINTS);
    if (lp::prof_read_parse(out) != 0 || lp::prof_read_uri(u.data()) != 0) return -1;
    for (size_t k = 0; k < u.size(); ++k) out[k] += u[k];
    lp::prof_clear_parse();
    lp::prof_clear_uri();
    return 0;
}
#endif

static_assert(LP_ARENA_SHARDS == lp::ARENA_SHARDS, "arena shard count of the ABI and the kernels");

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    bool ensure(size_t n) {
        if (n <= cap && p) return true;
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
        if (n == 0) n = 256;
        if (hipMalloc(&p, n) != hipSuccess) return false;
        cap = n;
        return true;
    }
    void release() {
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <typename T>
    T* as(size_t off = 0) const { return reinterpret_cast<T*>((char*)p + off); }
};

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// One SoA column of the program: its ABI name, stage index, element size and
// the Columns field that points at it.
struct ColSpec {
    const char* name;
    int index;
    int esz;
    void** field;
    int uri;  // written by the URI kernels (1) or the parse kernels (0): lp_last_bytes' per-kernel split
};

}  // namespace

struct lp_handle {
    lp::Plan plan;
    int compile_status = LP_OK;
    int device = 0;
    hipStream_t stream = nullptr;
    DevBuf input, chunk, line_off, cols, arena, meta, waves, args, route, ovf, hist;
    DevBuf cstate;  // chunked parse: look-back words, per-chunk counts, queued lines
    DevBuf targs, tscratch;  // device table (lp_result_table on a device view)
    lp::DeviceArgs host_args{};
    lp::Columns C{};
    std::vector<ColSpec> specs;
    std::vector<lp_column> dev_cols;
    // the batch (valid once lp_parse_batch succeeded)
    bool valid = false, pending = false;
    int64_t n_lines = 0;
    uint64_t nbytes = 0;
    const uint8_t* d_buf = nullptr;
    // capacities of the column and arena buffers, and what sizes the next batch
    int64_t cap_lines = 0;
    uint64_t shard_cap = 0;
    int64_t reserve_lines = 0;
    uint64_t reserve_arena = 0;
    double mean_line = 0;          // input bytes per line of the last batch
    double arena_per_line = 0;     // arena bytes (largest shard x shards) per line of the last batch
    bool force_direct = false;
    int max_retries = 3;           // re-runs of a batch whose estimates were short (LP_OPT_MAX_RETRIES)
    uint64_t arena_first = 0;      // LP_OPT_ARENA_BYTES: exact arena of a batch's first run (tests)
    uint64_t arena_ovf = 0;        // arena overflow events of the last batch's final run (its lines FALLBACK)
    int64_t first_line = 0;        // global number of the last batch's first line
    int64_t next_line = 0;         // ... of the next batch's (lp_parse_batch continues the numbering)
    hipEvent_t ev[5]{};  // batch start, index done, parse start, batch end, parse kernels done
    hipEvent_t tev[4]{}; // device table: start, values kernel done, scans done, bytes done
    float tms[3] = {0, 0, 0};  // the last device table's values / scans / bytes phases
    bool have_events = false;
    uint64_t counters[4]{};
    uint32_t chunk_lines = 0;      // LP_OPT_CHUNK_LINES (0: the kernel's default)
    int32_t chunk_wait = 0;        // LP_OPT_CHUNK_WAIT (tests: 0 default, < 0 defer every chunk not yet reached)
    bool one_pass = true;          // LP_OPT_ONE_PASS: several LogFormats on the chunked one-pass path
    bool chunked = false;          // the last batch ran the chunked parse (line index inside the parse kernel)
    uint64_t ovf_waves = 0;        // waves of the last batch parsed by k_parse_overflow (chunked: lines by k_parse_ovf_lines)
    uint64_t uri_ovf_waves = 0;    // ... whose URI stages ran in k_uri_overflow
    uint64_t deferred = 0;         // chunks of the last batch parsed by the deferred pass (normally 0)
    uint64_t shard_top[LP_ARENA_SHARDS]{};
    lp::ParseLaunch last_launch{};  // the last enqueue's launch parameters (diagnostics)
    uint64_t arena_written = 0;
    uint64_t uri_src_bytes = 0;  // URI source bytes the URI kernels read (meta counters[5])
    int retries = 0;
    float ms[5]{};
    // host copy for lp_line_record_json / lp_line_status
    bool host_valid = false;
    std::vector<uint8_t> hostbuf;
    lp_result host_res{};
    lp::ResultView view;
    // HttpdLogFormatDissector's active format, carried from batch to batch
    // like the reference parser's (format 0 before the first line)
    uint32_t fmt_state = 0;
};

namespace {

// column capacity for n (expected) lines: 25 % more for the next batches of
// a stream, at most 4 M lines more (a huge batch keeps its footprint close to
// its size; a larger next batch re-runs once with exact capacity)
int64_t headroom(int64_t n) { return n + std::min<int64_t>(n / 4, 1 << 22) + 1024; }

void set_err(char* err, size_t errlen, const std::string& s) {
    if (err && errlen) snprintf(err, errlen, "%s", s.c_str());
}

// The program's SoA columns, in layout order.
void build_specs(lp_handle* h) {
    const lp::Program& P = h->plan.program();
    lp::Columns& C = h->C;
    auto& v = h->specs;
    v.clear();
    int uri = 0;
    auto add = [&](const char* nm, int idx, int esz, void* field) { v.push_back({nm, idx, esz, (void**)field, uri}); };
    add("status", 0, 1, &C.status);
    for (int k = 0; k < P.n_tok; ++k) add("tok_span", k, 4, &C.tok_span[k]);
    add("tok_flags", 0, 4, &C.tok_flags);
    add("hist", 0, 4, &C.hist);
    for (int t = 0; t < P.n_time; ++t) {
        add("t_epoch", t, 8, &C.t_epoch[t]);
        add("t_local", t, 8, &C.t_local[t]);
        add("t_utc", t, 8, &C.t_utc[t]);
        if (P.time[t].kind == lp::TK_STRF) add("t_nano", t, 4, &C.t_nano[t]);  // only strftime has fractions
    }
    for (int k = 0; k < P.n_secms; ++k) add("sm_ms", k, 8, &C.sm_ms[k]);
    for (int k = 0; k < P.n_binip; ++k) add("bip", k, 4, &C.bip[k]);
    for (int f = 0; f < P.n_fl; ++f) {
        add("fl_kind", f, 4, &C.fl_kind[f]);
        add("fl_method", f, 4, &C.fl_method[f]);
        add("fl_uri", f, 4, &C.fl_uri[f]);
        add("fl_proto", f, 4, &C.fl_proto[f]);
    }
    uri = 1;  // the URI kernels' columns
    for (int u = 0; u < P.n_uri; ++u) {
        add("u_flags", u, 4, &C.u_flags[u]);
        add("u_scheme", u, 8, &C.u_scheme[u]);
        add("u_host", u, 8, &C.u_host[u]);
        add("u_port", u, 4, &C.u_port[u]);
        add("u_path", u, 8, &C.u_path[u]);
        add("u_query", u, 8, &C.u_query[u]);
        add("u_frag", u, 8, &C.u_frag[u]);
    }
    for (int q = 0; q < P.n_query; ++q) {
        add("q_count", q, 4, &C.q_count[q]);
        add("q_params", q, 8, &C.q_params[q]);
    }
    for (int j = 0; j < P.n_list; ++j) {
        add("l_count", j, 4, &C.l_count[j]);
        add("l_tab", j, 8, &C.l_tab[j]);
    }
    for (int j = 0; j < P.n_pair; ++j) {
        add("p_count", j, 4, &C.p_count[j]);
        add("p_tab", j, 8, &C.p_tab[j]);
    }
    add("arena_base", 0, 8, &C.arena_base);
    uri = 0;
    if (P.n_fmt > 1) {
        add("fmt_match", 0, 2, &C.fmt_match);
        add("fmt_id", 0, 1, &C.fmt_id);
    }
}

// column descriptors for columns of `rows` rows
std::vector<lp_column> layout(const std::vector<ColSpec>& specs, int64_t rows, uint64_t* total) {
    std::vector<lp_column> out;
    uint64_t off = 0;
    for (const auto& c : specs) {
        lp_column d{};
        snprintf(d.name, sizeof d.name, "%s", c.name);
        d.index = c.index;
        d.elem_size = c.esz;
        d.offset = off;
        out.push_back(d);
        off += align256((size_t)c.esz * (size_t)(rows > 0 ? rows : 1));
    }
    *total = off;
    return out;
}

// Columns for cap lines in one allocation.
bool alloc_columns(lp_handle* h, int64_t cap) {
    uint64_t total = 0;
    h->dev_cols = layout(h->specs, cap, &total);
    if (!h->cols.ensure(total)) return false;
    for (size_t k = 0; k < h->specs.size(); ++k) *h->specs[k].field = h->cols.as<char>(h->dev_cols[k].offset);
    return true;
}

// A view of a result (device or host copy) for the replay.
void make_view(lp_handle* h, const lp_result& r, lp::ResultView& V) {
    V = lp::ResultView{};
    V.n = r.n_lines;
    V.line_off = r.line_off;
    V.input = r.input;
    V.arena = r.arena;
    V.shard_cap = r.shard_cap;
    for (int s = 0; s < LP_ARENA_SHARDS; ++s) V.shard_off[s] = r.shard_off[s];
    for (int k = 0; k < r.n_columns; ++k) {
        const lp_column& c = r.column[k];
        const void* p = r.columns + c.offset;
        const std::string nm = c.name;
        const int i = c.index;
        if (nm == "status") V.status = (const uint8_t*)p;
        else if (nm == "tok_span") V.tok_span[i] = (const uint32_t*)p;
        else if (nm == "tok_flags") V.tok_flags = (const uint32_t*)p;
        else if (nm == "t_epoch") V.t_epoch[i] = (const int64_t*)p;
        else if (nm == "t_local") V.t_local[i] = (const uint64_t*)p;
        else if (nm == "t_utc") V.t_utc[i] = (const uint64_t*)p;
        else if (nm == "t_nano") V.t_nano[i] = (const uint32_t*)p;
        else if (nm == "fl_kind") V.fl_kind[i] = (const uint32_t*)p;
        else if (nm == "fl_method") V.fl_method[i] = (const uint32_t*)p;
        else if (nm == "fl_uri") V.fl_uri[i] = (const uint32_t*)p;
        else if (nm == "fl_proto") V.fl_proto[i] = (const uint32_t*)p;
        else if (nm == "u_flags") V.u_flags[i] = (const uint32_t*)p;
        else if (nm == "u_scheme") V.u_scheme[i] = (const uint64_t*)p;
        else if (nm == "u_host") V.u_host[i] = (const uint64_t*)p;
        else if (nm == "u_port") V.u_port[i] = (const int32_t*)p;
        else if (nm == "u_path") V.u_path[i] = (const uint64_t*)p;
        else if (nm == "u_query") V.u_query[i] = (const uint64_t*)p;
        else if (nm == "u_frag") V.u_frag[i] = (const uint64_t*)p;
        else if (nm == "q_count") V.q_count[i] = (const uint32_t*)p;
        else if (nm == "q_params") V.q_params[i] = (const uint64_t*)p;
        else if (nm == "arena_base") V.arena_base = (const uint64_t*)p;
        else if (nm == "sm_ms") V.sm_ms[i] = (const int64_t*)p;
        else if (nm == "l_count") V.l_count[i] = (const uint32_t*)p;
        else if (nm == "l_tab") V.l_tab[i] = (const uint64_t*)p;
        else if (nm == "bip") V.bip[i] = (const uint32_t*)p;
        else if (nm == "p_count") V.p_count[i] = (const uint32_t*)p;
        else if (nm == "p_tab") V.p_tab[i] = (const uint64_t*)p;
        else if (nm == "fmt_id") V.fmt_id = (const uint8_t*)p;
    }
    if (!V.arena) V.arena_base = nullptr;
}

// Enqueue the whole batch (index, routing, parse) with the current
// capacities.  sync_count: count the lines first and size the buffers from
// the exact count (the handle has no estimate yet).
// One LogFormat of the Apache common / combined family: literals, [^\s]*,
// the number kinds, .* / .*? and the %t time stamp, Apache time stages only,
// no cookie / Set-Cookie guards, SECOND_MILLIS or BinaryIP stages (the parse
// kernel's SIMPLE instance leaves the other kinds and stages out).
bool simple_program(const lp::Program& P) {
    if (P.n_fmt != 1 || P.n_secms || P.n_binip || P.guard_pct[0] || P.guard_setc[0]) return false;
    for (int t = 0; t < P.n_time; ++t)
        if (P.time[t].kind != lp::TK_APACHE) return false;
    for (int i = 0; i < P.n_elems; ++i) {
        switch (lp::load_elem(P.elems + i).kind) {
        case lp::EK_LIT: case lp::EK_NOSPACE: case lp::EK_NUMBER: case lp::EK_CLFNUMBER: case lp::EK_HEXNUMBER:
        case lp::EK_CLFHEXNUMBER: case lp::EK_NONZERO: case lp::EK_ANY_GREEDY: case lp::EK_ANY_LAZY:
        case lp::EK_TIME_US: break;
        default: return false;
        }
    }
    return true;
}

int enqueue(lp_handle* h, bool sync_count) {
    hipStream_t s = h->stream;
    const uint64_t nbytes = h->nbytes;
    const lp::Program& P = h->plan.program();
    const int64_t nc = lp::count_chunks(nbytes);
    const size_t cbytes = align256(sizeof(uint64_t) * (size_t)(nc + 2));
    if (!h->chunk.ensure(cbytes + 2 * (size_t)lp::nlmask_words(nbytes))) return LP_E_NOMEM;
    if (!h->meta.ensure(sizeof(lp::Meta))) return LP_E_NOMEM;
    uint64_t* d_chunk = h->chunk.as<uint64_t>();
    uint16_t* d_nlmask = h->chunk.as<uint16_t>(cbytes);
    lp::Meta* d_meta = h->meta.as<lp::Meta>();
    if (hipMemsetAsync(d_meta, 0, sizeof(lp::Meta), s) != hipSuccess) return LP_E_DEVICE;
    hipEventRecord(h->ev[0], s);
    int64_t cap = h->cap_lines;
    // one LogFormat: the parse kernel finds the lines itself (k_parse_chunks);
    // several: the routing pass needs the line index first
    // one pass: the parse kernel finds the lines itself (k_parse_chunks);
    // several LogFormats route inside it too (LP_OPT_ONE_PASS 0: the line
    // index, the routing passes, then the parse)
    const bool chunked = h->plan.device_ok() && (P.n_fmt == 1 || h->one_pass);
    h->chunked = chunked;
    if (sync_count && chunked) {
        // first batch of a one-format handle: the line length of an 8 MiB
        // prefix sizes the columns (no pass over the whole input; a short
        // estimate sets cap_ovf and finish() re-runs with the exact count)
        const uint64_t pre = std::min<uint64_t>(nbytes, 8ull << 20);
        if (!h->line_off.ensure(16)) return LP_E_NOMEM;
        if (lp::launch_count(h->d_buf, pre, d_chunk, d_nlmask, h->line_off.as<uint64_t>(), -1, d_meta, s) != 0)
            return LP_E_DEVICE;
        unsigned long long n = 0;
        if (hipMemcpyAsync(&n, &d_meta->n_lines, sizeof n, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess || hipMemsetAsync(d_meta, 0, sizeof(lp::Meta), s) != hipSuccess)
            return LP_E_DEVICE;
        const double mean = n ? (double)pre / (double)n : (double)std::max<uint64_t>(pre, 1);
        cap = std::max<int64_t>(headroom((int64_t)((double)nbytes / mean * 1.02)), h->reserve_lines);
        h->mean_line = mean;  // sizes this batch's LDS windows
    } else if (sync_count) {
        // first batch of a handle: the exact line count sizes the columns
        if (!h->line_off.ensure(16)) return LP_E_NOMEM;
        if (lp::launch_count(h->d_buf, nbytes, d_chunk, d_nlmask, h->line_off.as<uint64_t>(), -1, d_meta, s) != 0)
            return LP_E_DEVICE;
        unsigned long long n = 0;
        if (hipMemcpyAsync(&n, &d_meta->n_lines, sizeof n, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return LP_E_DEVICE;
        // headroom for the next batches of the stream (sized like the estimate below)
        cap = std::max<int64_t>(headroom((int64_t)n), h->reserve_lines);
        if (n) h->mean_line = (double)nbytes / (double)n;  // sizes this batch's LDS windows
    } else if (!chunked) {
        if (!h->line_off.ensure(sizeof(uint64_t) * (size_t)(cap + 2))) return LP_E_NOMEM;
        if (lp::launch_count(h->d_buf, nbytes, d_chunk, d_nlmask, h->line_off.as<uint64_t>(), cap, d_meta, s) != 0)
            return LP_E_DEVICE;
    }
    if (!h->line_off.ensure(sizeof(uint64_t) * (size_t)(cap + 2))) return LP_E_NOMEM;
    if (sync_count && !chunked) {  // the scan ran without the line index buffer: its ends now
        unsigned long long n = 0;
        hipMemcpy(&n, &d_meta->n_lines, sizeof n, hipMemcpyDeviceToHost);
        uint64_t ends[2] = {0, nbytes + 1};
        hipMemcpy(h->line_off.as<uint64_t>(), &ends[0], 8, hipMemcpyHostToDevice);
        uint8_t last = '\n';
        if (nbytes) hipMemcpy(&last, h->d_buf + nbytes - 1, 1, hipMemcpyDeviceToHost);
        if (nbytes && last != '\n' && last != '\r') hipMemcpy(h->line_off.as<uint64_t>() + n, &ends[1], 8, hipMemcpyHostToDevice);
    }
    h->cap_lines = cap;
    if (!chunked && lp::launch_offsets(d_nlmask, nbytes, d_chunk, h->line_off.as<uint64_t>(), cap, s) != 0)
        return LP_E_DEVICE;
    hipEventRecord(h->ev[1], s);
    if (!alloc_columns(h, cap)) return LP_E_NOMEM;
    // arena: ARENA_SHARDS shards of shard_cap bytes; the reservation is a
    // minimum (a re-run after an overflow needs the grown estimate)
    const double per = h->arena_per_line > 0 ? h->arena_per_line * 1.25 : 64.0;
    uint64_t acap = std::max<uint64_t>(h->reserve_arena, (uint64_t)(per * (double)cap) + (1u << 20));
    if (h->arena_first && h->retries == 0) acap = h->arena_first;
    if (!h->plan.device_ok() || !P.has_phase2()) acap = 4096 * LP_ARENA_SHARDS;
    h->shard_cap = (acap / LP_ARENA_SHARDS + 255) & ~255ull;
    if (!h->arena.ensure(h->shard_cap * LP_ARENA_SHARDS)) return LP_E_NOMEM;
    lp::Columns& C = h->C;
    C.line_off = h->line_off.as<uint64_t>();
    C.arena = h->arena.as<uint8_t>();
    C.shard_cap = h->shard_cap;
    C.meta = d_meta;
    C.cap_lines = cap;
    const int64_t waves = lp::parse_waves(cap);
    if (!h->waves.ensure(4 * lp::WC_WORDS * (size_t)(waves + 1))) return LP_E_NOMEM;
    if (!h->ovf.ensure(8 * (size_t)(waves + 1))) return LP_E_NOMEM;
    C.wave_counts = h->waves.as<uint32_t>();
    C.ovf_list = h->ovf.as<uint32_t>();
    C.uri_ovf_list = h->ovf.as<uint32_t>() + (waves + 1);
    if (h->plan.device_ok()) {
        if (P.n_fmt > 1) {  // sticky multi-format routing scratch
            if (!h->route.ensure(8 * (size_t)(lp::fmt_chunks(cap) + 1))) return LP_E_NOMEM;
            C.fmt_chunk = h->route.as<uint64_t>();
            C.fmt_init = h->fmt_state;
        }
        if (!h->args.ensure(sizeof(lp::DeviceArgs))) return LP_E_NOMEM;
        lp::ParseLaunch pl{h->d_buf, nbytes, cap, (uint64_t)(h->mean_line > 0 ? h->mean_line + 0.5 : 0),
                           P.n_elems, P.max_stack, h->force_direct, P.has_phase2(), false, P.n_uri, P.n_query,
                           h->ev[4]};
        for (int u = 0; u < P.n_uri; ++u) pl.derived = pl.derived || P.uri[u].src_q >= 0;
        if (!pl.mean_line && cap > 0) pl.mean_line = (nbytes + cap - 1) / (uint64_t)cap;
        pl.chunked = chunked;
        pl.chunk_lines = h->chunk_lines;
        pl.chunk_wait = h->chunk_wait;
        pl.multi = chunked && P.n_fmt > 1;
        pl.lit_aware = false;
        for (int i = 0; i < P.n_elems; ++i) {
            const lp::ElemV e = lp::load_elem(P.elems + i);
            if (e.nlit && !e.last && ((e.kind == lp::EK_NOSPACE && !e.det) || e.kind == lp::EK_NOSPACE3))
                pl.lit_aware = true;
        }
        pl.simple = simple_program(P);
        h->last_launch = pl;
        if (chunked) {
            // look-back words (zeroed), per-chunk counts, the queued line list
            const lp::ChunkPlan cp = lp::chunk_plan(pl);
            const size_t sb = align256(8 * (size_t)(cp.n_chunks + 1)), cb = align256(4 * lp::WC_WORDS * (size_t)(cp.n_chunks + 1));
            const size_t ob = align256(4 * (size_t)(cap + 1));
            if (!h->cstate.ensure(sb + cb + ob + 4 * (size_t)(cp.n_chunks + 1))) return LP_E_NOMEM;
            C.chunk_state = h->cstate.as<uint64_t>();
            C.chunk_counts = h->cstate.as<uint32_t>(sb);
            C.ovf_lines = h->cstate.as<uint32_t>(sb + cb);
            C.deferred_chunks = h->cstate.as<uint32_t>(sb + cb + ob);
            if (hipMemsetAsync(C.chunk_state, 0, sb, s) != hipSuccess) return LP_E_DEVICE;
        }
        h->host_args.prog = P;
        h->host_args.cols = C;
        if (hipMemcpyAsync(h->args.p, &h->host_args, sizeof(lp::DeviceArgs), hipMemcpyHostToDevice, s) != hipSuccess)
            return LP_E_DEVICE;
        hipEventRecord(h->ev[2], s);
        const lp::DeviceArgs* d_args = h->args.as<lp::DeviceArgs>();
        if (P.n_fmt > 1 && !chunked) {
            // HttpdLogFormatDissector routing: every format's match per line,
            // then the scan of the sticky active format (one pass: inside
            // launch_parse, after the chunk kernel)
            if (lp::launch_route_match(pl, d_args, s) != 0 || lp::launch_route(d_args, cap, s) != 0) return LP_E_DEVICE;
        }
        if (lp::launch_parse(pl, d_args, C, s) != 0) return LP_E_DEVICE;
    } else {
        // the requested paths need a dissector that is not on the device:
        // every line goes back to the reference (FALLBACK)
        hipEventRecord(h->ev[2], s);
        if (cap) hipMemsetAsync(C.status, LP_LINE_FALLBACK, (size_t)cap, s);
        hipEventRecord(h->ev[4], s);
    }
    hipEventRecord(h->ev[3], s);
    return LP_OK;
}

// Wait for the batch, read its bookkeeping; when its line count or arena
// need outgrew the buffers, re-run it with exact sizes.
int finish(lp_handle* h) {
    int cap_reruns = 0;    // re-runs for a short line capacity: always (the re-run has the exact count)
    int arena_reruns = 0;  // ... for a short arena: at most LP_OPT_MAX_RETRIES
    for (;;) {
        if (hipStreamSynchronize(h->stream) != hipSuccess) return LP_E_DEVICE;
        lp::Meta m;
        if (hipMemcpy(&m, h->meta.p, sizeof m, hipMemcpyDeviceToHost) != hipSuccess) return LP_E_DEVICE;
        if (m.err) {
            // a kernel's self-check of its own bookkeeping failed (parse.hip check_fail)
            fprintf(stderr,
                    "logparser_amd: internal check failed %llu time(s); first: kind %llu values %llu %llu %llu %llu "
                    "(batch %llu bytes, %llu lines)\n",
                    m.err, m.err_info[0], m.err_info[1], m.err_info[2], m.err_info[3], m.err_info[4],
                    (unsigned long long)h->nbytes, m.n_lines);
            if (m.err_info[0] == 2) {
                const lp::ChunkPlan cp = lp::chunk_plan(h->last_launch);
                fprintf(stderr,
                        "  chunk_excess received w0 %llu w1 %llu t_lo %llu t_hi %llu first %llu win %llx nbytes %llu "
                        "buf %llx (host: buf %llx cb %u win_cap %u)\n",
                        m.err_info[5], m.err_info[6], m.err_info[7], m.err_info[8], m.err_info[9], m.err_info[10],
                        m.err_info[11], m.err_info[12], (unsigned long long)(uintptr_t)h->d_buf, cp.cb, cp.win_cap);
            }
            return LP_E_DEVICE;
        }
        uint64_t top_max = 0;
        for (int s = 0; s < LP_ARENA_SHARDS; ++s) {
            h->shard_top[s] = m.shard_top[16 * s];
            top_max = std::max<uint64_t>(top_max, h->shard_top[s]);
        }
        const int64_t n = (int64_t)m.n_lines;
        // LP_OPT_MAX_RETRIES bounds the arena re-runs only: a short arena has
        // a fallback (its lines go FALLBACK), a short line capacity has none
        const bool cap_rerun = m.cap_ovf && cap_reruns < 2;
        const bool arena_rerun = !m.cap_ovf && m.arena_ovf && arena_reruns < h->max_retries;
        if (h->plan.device_ok() && (cap_rerun || arena_rerun)) {
            // exact sizes: the line count, every shard as large as the largest
            // request (shard tops count what was asked for, also past the end)
            if (cap_rerun) ++cap_reruns;
            else ++arena_reruns;
            ++h->retries;
            h->cap_lines = std::max<int64_t>(n, h->cap_lines);
            if (n > 0) h->mean_line = (double)h->nbytes / (double)n;
            // the next estimate (arena_per_line x 1.25 x capacity) covers the largest shard
            if (m.arena_ovf && n > 0)
                h->arena_per_line = std::max(h->arena_per_line, (double)(top_max + 4096) * LP_ARENA_SHARDS / (double)n);
            const int st = enqueue(h, false);
            if (st != LP_OK) return st;
            continue;
        }
        // more lines than columns: nothing was parsed.  An arena that is still
        // short after the re-runs degrades instead: the lines whose region or
        // pieces did not fit are FALLBACK (the kernels marked them), the rest
        // of the batch is delivered
        if (m.cap_ovf) return LP_E_NOMEM;
        h->arena_ovf = m.arena_ovf;
        h->n_lines = n;
        if (h->plan.device_ok()) {
            for (int k = 0; k < 4; ++k) h->counters[k] = m.counters[k];
            h->arena_written = m.counters[4];
            h->uri_src_bytes = m.counters[5];
            h->ovf_waves = h->chunked ? m.ovf_lines : m.ovf_waves;
            h->uri_ovf_waves = m.uri_ovf_waves;
            h->deferred = h->chunked ? m.deferred : 0;
        } else {
            h->counters[0] = (uint64_t)n;
            h->counters[1] = h->counters[2] = 0;
            h->counters[3] = (uint64_t)n;
            h->arena_written = 0;
            h->uri_src_bytes = 0;
        }
        for (int s = 0; s < LP_ARENA_SHARDS; ++s) h->shard_top[s] = std::min<uint64_t>(h->shard_top[s], h->shard_cap);
        const lp::Program& P = h->plan.program();
        if (h->plan.device_ok() && P.n_fmt > 1 && n > 0) h->fmt_state = (uint32_t)m.fmt_state;
        if (n > 0) {
            h->mean_line = (double)h->nbytes / (double)n;
            h->arena_per_line = (double)top_max * LP_ARENA_SHARDS / (double)n;
        }
        float a = 0, b = 0, c = 0, d = 0, e = 0;
        hipEventElapsedTime(&a, h->ev[0], h->ev[3]);
        hipEventElapsedTime(&b, h->ev[0], h->ev[1]);
        hipEventElapsedTime(&c, h->ev[2], h->ev[3]);
        hipEventElapsedTime(&d, h->ev[2], h->ev[4]);
        hipEventElapsedTime(&e, h->ev[4], h->ev[3]);
        h->ms[0] = a; h->ms[1] = b; h->ms[2] = c; h->ms[3] = d; h->ms[4] = e;
        return LP_OK;
    }
}

int ensure_synced(lp_handle* h) {
    if (h->pending) {
        const int st = lp_sync(h);
        if (st != LP_OK) return st;
    }
    return h->valid ? LP_OK : LP_E_STATE;
}

// Bytes of a host copy (line index, columns, arena shards, input) and its
// layout; fills r when dst is non-null.
int64_t copy_result(lp_handle* h, uint8_t* dst, uint64_t cap, bool with_input, lp_result* r) {
    const int64_t n = h->n_lines;
    uint64_t cols_bytes = 0;
    // the column table travels in the copy: the result never points into the
    // handle (a later copy or batch must not invalidate an earlier copy)
    const std::vector<lp_column> cols = layout(h->specs, n, &cols_bytes);
    const uint64_t tab_bytes = sizeof(lp_column) * cols.size();
    uint64_t arena_bytes = 0;
    uint64_t shard_off[LP_ARENA_SHARDS];
    for (int s = 0; s < LP_ARENA_SHARDS; ++s) {
        shard_off[s] = arena_bytes;
        arena_bytes += (h->shard_top[s] + 15) & ~15ull;
    }
    const uint64_t o_tab = 0, o_lines = align256(tab_bytes), o_cols = o_lines + align256(8 * (uint64_t)(n + 1));
    const uint64_t o_arena = o_cols + cols_bytes;
    const uint64_t o_input = align256(o_arena + arena_bytes);
    const uint64_t total = with_input ? o_input + h->nbytes + 64 : o_input;
    if (!dst) return -(int64_t)total;
    if (cap < total) return -(int64_t)total;
    auto cp = [&](uint64_t off, const void* src, uint64_t bytes) {
        return bytes == 0 || hipMemcpy(dst + off, src, bytes, hipMemcpyDeviceToHost) == hipSuccess;
    };
    if (tab_bytes) memcpy(dst + o_tab, cols.data(), tab_bytes);
    bool ok = cp(o_lines, h->line_off.p, 8 * (uint64_t)(n + 1));
    for (size_t k = 0; k < h->specs.size() && ok; ++k)
        ok = cp(o_cols + cols[k].offset, *h->specs[k].field, (uint64_t)h->specs[k].esz * (uint64_t)n);
    for (int s = 0; s < LP_ARENA_SHARDS && ok; ++s)
        ok = cp(o_arena + shard_off[s], h->arena.as<uint8_t>((size_t)s * h->shard_cap), h->shard_top[s]);
    if (with_input && ok) {
        ok = cp(o_input, h->d_buf, h->nbytes);
        memset(dst + o_input + h->nbytes, '\n', 64);
    }
    if (!ok) return LP_E_DEVICE;
    lp_result& R = *r;
    R = lp_result{};
    R.n_lines = n;
    R.first_line = h->first_line;
    R.input_bytes = h->nbytes;
    R.input = with_input ? dst + o_input : nullptr;
    R.line_off = reinterpret_cast<const uint64_t*>(dst + o_lines);
    R.columns = dst + o_cols;
    R.columns_bytes = cols_bytes;
    R.arena = dst + o_arena;
    R.arena_bytes = arena_bytes;
    R.shard_cap = h->shard_cap;
    for (int s = 0; s < LP_ARENA_SHARDS; ++s) R.shard_off[s] = shard_off[s];
    R.n_columns = (int32_t)cols.size();
    R.column = reinterpret_cast<const lp_column*>(dst + o_tab);
    R.on_host = 1;
    return (int64_t)total;
}

bool fetch_host(lp_handle* h) {
    if (h->host_valid) return true;
    if (ensure_synced(h) != LP_OK) return false;
    const int64_t need = -copy_result(h, nullptr, 0, true, nullptr);
    h->hostbuf.resize((size_t)need);
    if (copy_result(h, h->hostbuf.data(), (uint64_t)need, true, &h->host_res) < 0) return false;
    make_view(h, h->host_res, h->view);
    h->host_valid = true;
    return true;
}

}  // namespace

extern "C" {

lp_handle* lp_compile(const char* logformats, const char* const* paths, int n_paths, int device, int* status,
                      char* err, size_t errlen) {
    return lp_compile_remapped(logformats, paths, n_paths, nullptr, 0, device, status, err, errlen);
}

lp_handle* lp_compile_remapped(const char* logformats, const char* const* paths, int n_paths, const lp_remap* remaps,
                               int n_remaps, int device, int* status, char* err, size_t errlen) {
    if (status) *status = LP_E_INVALID;
    if (!logformats || (n_paths > 0 && !paths) || (n_remaps > 0 && !remaps)) { set_err(err, errlen, "null argument"); return nullptr; }
    std::vector<lp::Remap> rm;
    for (int i = 0; i < n_remaps; ++i) {
        if (!remaps[i].input || !remaps[i].type) { set_err(err, errlen, "null remapping"); return nullptr; }
        rm.push_back(lp::Remap{remaps[i].input, remaps[i].type, (int)remaps[i].casts});
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        if (status) *status = LP_E_DEVICE;
        set_err(err, errlen, "logparser_amd: no HIP device available (the engine runs only on the GPU)");
        return nullptr;
    }
    if (device < 0 || device >= ndev) { if (status) *status = LP_E_DEVICE; set_err(err, errlen, "bad device ordinal"); return nullptr; }
    auto h = std::make_unique<lp_handle>();
    h->device = device;
    std::vector<std::string> f;
    for (int i = 0; i < n_paths; ++i) f.emplace_back(paths[i]);
    std::string e;
    int st = h->plan.build(logformats, f, e, rm);
    if (st != LP_OK && st != LP_E_UNSUPPORTED) {
        if (status) *status = st;
        set_err(err, errlen, e);
        return nullptr;
    }
    if (st == LP_E_UNSUPPORTED) set_err(err, errlen, h->plan.unsupported_reason());
    h->compile_status = st;
    build_specs(h.get());
    if (hipSetDevice(device) != hipSuccess) { if (status) *status = LP_E_DEVICE; return nullptr; }
    for (auto& ev : h->ev) hipEventCreate(&ev);
    for (auto& ev : h->tev) hipEventCreate(&ev);
    h->have_events = true;
    if (!h->meta.ensure(sizeof(lp::Meta))) { if (status) *status = LP_E_NOMEM; return nullptr; }
    if (status) *status = st;
    return h.release();
}

void lp_free(lp_handle* h) {
    if (!h) return;
    hipSetDevice(h->device);
    if (h->pending) hipStreamSynchronize(h->stream);
    for (auto* b : {&h->input, &h->chunk, &h->line_off, &h->cols, &h->arena, &h->meta, &h->waves, &h->args, &h->route,
                    &h->ovf, &h->hist, &h->cstate, &h->targs, &h->tscratch})
        b->release();
    if (h->have_events) {
        for (auto& ev : h->ev) hipEventDestroy(ev);
        for (auto& ev : h->tev) hipEventDestroy(ev);
    }
    delete h;
}

int64_t lp_possible_paths(const char* logformats, int max_depth, char* out, size_t cap) {
    return lp_possible_paths_remapped(logformats, max_depth, nullptr, 0, out, cap);
}

int64_t lp_possible_paths_remapped(const char* logformats, int max_depth, const lp_remap* remaps, int n_remaps,
                                   char* out, size_t cap) {
    if (n_remaps > 0 && !remaps) return LP_E_INVALID;
    std::vector<lp::Remap> rm;
    for (int i = 0; i < n_remaps; ++i) {
        if (!remaps[i].input || !remaps[i].type) return LP_E_INVALID;
        rm.push_back(lp::Remap{remaps[i].input, remaps[i].type, (int)remaps[i].casts});
    }
    std::vector<std::string> paths;
    std::string err;
    lp::Plan::possible_paths(logformats ? logformats : "", max_depth, paths, err, rm);
    std::string s;
    for (auto& p : paths) s += p + "\n";
    if (!out || s.size() + 1 > cap) return -(int64_t)(s.size() + 1);
    memcpy(out, s.c_str(), s.size() + 1);
    return (int64_t)s.size();
}

int lp_set_option(lp_handle* h, int option, int64_t value) {
    if (!h) return LP_E_INVALID;
    switch (option) {
    case LP_OPT_FORCE_DIRECT: h->force_direct = value != 0; return LP_OK;
    case LP_OPT_CHUNK_LINES:
        if (value < 0 || value > 64) return LP_E_INVALID;
        h->chunk_lines = (uint32_t)value;
        return LP_OK;
    case LP_OPT_ONE_PASS:
        h->one_pass = value != 0;
        return LP_OK;
    case LP_OPT_CHUNK_WAIT:
        h->chunk_wait = value == -2 ? -2 : value < 0 ? -1 : (int32_t)std::min<int64_t>(value, 1 << 30);
        return LP_OK;
    case LP_OPT_MAX_RETRIES:
        if (value < 0 || value > 16) return LP_E_INVALID;
        h->max_retries = (int)value;
        return LP_OK;
    case LP_OPT_ARENA_BYTES:
        if (value < 0) return LP_E_INVALID;
        h->arena_first = (uint64_t)value;
        return LP_OK;
    default: return LP_E_INVALID;
    }
}

int lp_reserve(lp_handle* h, int64_t max_lines, uint64_t arena_bytes) {
    if (!h || max_lines < 0) return LP_E_INVALID;
    h->reserve_lines = max_lines;
    h->reserve_arena = arena_bytes;
    if (max_lines > h->cap_lines) h->cap_lines = max_lines;
    return LP_OK;
}

int lp_parse_batch(lp_handle* h, const uint8_t* buf, uint64_t nbytes, int buf_flags, void* stream) {
    if (!h) return LP_E_INVALID;
    if (h->pending) lp_sync(h);  // the previous batch's line count continues the numbering
    return lp_parse_batch_at(h, buf, nbytes, h->next_line, buf_flags, stream);
}

int lp_parse_batch_at(lp_handle* h, const uint8_t* buf, uint64_t nbytes, int64_t first_line_no, int buf_flags,
                      void* stream) {
    if (!h || (!buf && nbytes) || first_line_no < 0) return LP_E_INVALID;
    if (hipSetDevice(h->device) != hipSuccess) return LP_E_DEVICE;
    if (h->pending) lp_sync(h);
    // the handle holds no valid batch until this one has been enqueued
    h->valid = false;
    h->host_valid = false;
    h->n_lines = 0;
    h->retries = 0;
    h->arena_ovf = 0;
    h->first_line = h->next_line = first_line_no;
    hipStream_t s = (hipStream_t)stream;
    h->stream = s;
    h->nbytes = nbytes;
    if (buf_flags == LP_BUF_HOST) {
        if (!h->input.ensure(nbytes + 16)) return LP_E_NOMEM;
        if (nbytes && hipMemcpyAsync(h->input.p, buf, nbytes, hipMemcpyHostToDevice, s) != hipSuccess) return LP_E_DEVICE;
        h->d_buf = h->input.as<uint8_t>();
    } else if (((uintptr_t)buf & 15u) != 0) {
        // the index and staging passes stream 16-byte aligned loads; a batch
        // that starts mid-word (a line-aligned slice of a larger buffer) is
        // first copied to the handle's aligned buffer (measured: misaligned
        // streaming ran the index 4.5x and the parse kernel 2.2x slower)
        if (!h->input.ensure(nbytes + 16)) return LP_E_NOMEM;
        if (nbytes && hipMemcpyAsync(h->input.p, buf, nbytes, hipMemcpyDeviceToDevice, s) != hipSuccess) return LP_E_DEVICE;
        h->d_buf = h->input.as<uint8_t>();
    } else {
        h->d_buf = buf;
    }
    // capacity from the reservation or the previous batch's line length; a
    // handle without either counts its lines first (one synchronisation)
    bool sync_count = false;
    if (h->reserve_lines > 0) {
        h->cap_lines = std::max<int64_t>(h->cap_lines, h->reserve_lines);
    } else if (h->mean_line > 0) {
        const int64_t est = headroom((int64_t)((double)nbytes / h->mean_line));
        h->cap_lines = std::max<int64_t>(h->cap_lines, est);
    } else {
        sync_count = true;
    }
    const int st = enqueue(h, sync_count);
    if (st != LP_OK) return st;
    h->pending = true;
    h->valid = true;
    return LP_OK;
}

int lp_sync(lp_handle* h) {
    if (!h) return LP_E_INVALID;
    if (!h->pending) return h->valid ? LP_OK : LP_E_STATE;
    hipSetDevice(h->device);
    h->pending = false;
    const int st = finish(h);
    if (st != LP_OK) {
        h->valid = false;
        h->n_lines = 0;
    } else {
        h->next_line = h->first_line + h->n_lines;
    }
    return st;
}

int64_t lp_num_lines(lp_handle* h) {
    if (!h) return LP_E_INVALID;
    const int st = ensure_synced(h);
    return st == LP_OK ? h->n_lines : st;
}

int lp_line_status(lp_handle* h, int64_t first, int64_t count, uint8_t* out) {
    if (!h) return LP_E_INVALID;
    const int st = ensure_synced(h);
    if (st != LP_OK) return st;
    if (first < 0 || count < 0 || first + count > h->n_lines || (count && !out)) return LP_E_INVALID;
    if (!count) return LP_OK;
    if (h->host_valid) {  // served from the host copy
        memcpy(out, h->view.status + first, (size_t)count);
        return LP_OK;
    }
    if (hipMemcpy(out, h->C.status + first, (size_t)count, hipMemcpyDeviceToHost) != hipSuccess) return LP_E_DEVICE;
    return LP_OK;
}

int64_t lp_line_offset(lp_handle* h, int64_t i) {
    if (!h) return LP_E_INVALID;
    const int st = ensure_synced(h);
    if (st != LP_OK) return st;
    if (i < 0 || i > h->n_lines) return LP_E_INVALID;
    if (h->host_valid) return (int64_t)h->view.line_off[i];
    uint64_t v = 0;
    if (hipMemcpy(&v, h->line_off.as<uint64_t>() + i, sizeof v, hipMemcpyDeviceToHost) != hipSuccess) return LP_E_DEVICE;
    return (int64_t)v;
}

int64_t lp_line_record_json(lp_handle* h, int64_t i, char* out, size_t cap) {
    if (!h) return LP_E_INVALID;
    const int st = ensure_synced(h);
    if (st != LP_OK) return st;
    if (i < 0 || i >= h->n_lines) return LP_E_INVALID;
    if (!fetch_host(h)) return LP_E_DEVICE;
    if (h->view.status[i] != LP_LINE_OK) return LP_E_STATE;
    std::string js = h->plan.record_json(h->view, i);
    if (!out || js.size() + 1 > cap) return -100 - (int64_t)(js.size() + 1);
    memcpy(out, js.c_str(), js.size() + 1);
    return (int64_t)js.size();
}

int lp_counters(lp_handle* h, uint64_t* out, int n) {
    if (!h || !out) return LP_E_INVALID;
    const int st = ensure_synced(h);
    if (st != LP_OK) return st;
    const uint64_t v[9] = {h->counters[0], h->counters[1], h->counters[2], h->counters[3], h->ovf_waves,
                           (uint64_t)h->retries, h->arena_ovf, h->uri_ovf_waves, h->deferred};
    for (int k = 0; k < n && k < 9; ++k) out[k] = v[k];
    return n < 9 ? n : 9;
}

int lp_histograms(lp_handle* h, uint64_t* out, int out_on_device) {
    if (!h || !out) return LP_E_INVALID;
    const int st = ensure_synced(h);
    if (st != LP_OK) return st;
    if (!h->valid) return LP_E_INVALID;
    static_assert(lp::HIST_WORDS == LP_HIST_WORDS, "histogram layout");
    if (!h->plan.device_ok()) {  // every line FALLBACK
        std::vector<uint64_t> v(LP_HIST_WORDS, 0);
        v[LP_HIST_LINES] = h->counters[0];
        v[LP_HIST_FALLBACK] = h->counters[3];
        if (!out_on_device) memcpy(out, v.data(), 8 * v.size());
        else if (hipMemcpy(out, v.data(), 8 * v.size(), hipMemcpyHostToDevice) != hipSuccess) return LP_E_DEVICE;
        return LP_OK;
    }
    uint64_t* d = out;
    if (!out_on_device) {
        if (!h->hist.ensure(8 * (size_t)LP_HIST_WORDS)) return LP_E_NOMEM;
        d = h->hist.as<uint64_t>();
    }
    if (lp::launch_histograms(h->args.as<lp::DeviceArgs>(), h->d_buf, h->n_lines, d, h->stream) != 0) return LP_E_DEVICE;
    if (!out_on_device && hipMemcpyAsync(out, d, 8 * (size_t)LP_HIST_WORDS, hipMemcpyDeviceToHost, h->stream) != hipSuccess)
        return LP_E_DEVICE;
    return hipStreamSynchronize(h->stream) == hipSuccess ? LP_OK : LP_E_DEVICE;
}

int lp_last_timing(lp_handle* h, float* out, int n) {
    if (!h || !out) return LP_E_INVALID;
    const int st = ensure_synced(h);
    if (st != LP_OK) return st;
    for (int k = 0; k < n && k < 5; ++k) out[k] = h->ms[k];
    for (int k = 5; k < n && k < 8; ++k) out[k] = h->tms[k - 5];
    return n < 8 ? n : 8;
}

int lp_last_bytes(lp_handle* h, uint64_t* out, int n) {
    if (!h || !out) return LP_E_INVALID;
    const int st = ensure_synced(h);
    if (st != LP_OK) return st;
    uint64_t row = 8;  // line index entry
    uint64_t row_uri = 0;  // the columns the URI kernels write
    for (const auto& c : h->specs) {
        row += (uint64_t)c.esz;
        if (c.uri) row_uri += (uint64_t)c.esz;
    }
    const uint64_t n1 = (uint64_t)h->n_lines;
    const lp::Program& P = h->plan.program();
    // parse kernels: the input once, the line index, their columns;
    // URI kernels: the gathered URI bytes, per line the status, line start,
    // token flags and one source span per URI stage, their columns and arena
    const uint64_t parse_b = h->nbytes + 8 * (n1 + 1) + n1 * (row - 8 - row_uri);
    const uint64_t uri_b = P.has_phase2() ? h->uri_src_bytes + n1 * (1 + 8 + 4 + 4 * (uint64_t)P.n_uri) + n1 * row_uri +
                                         h->arena_written : 0;
    uint64_t v[4] = {h->nbytes, n1 * row + h->arena_written, parse_b, uri_b};
    for (int k = 0; k < n && k < 4; ++k) out[k] = v[k];
    return n < 4 ? n : 4;
}

int lp_casts(lp_handle* h, const char* target) {
    if (!h || !target) return LP_E_INVALID;
    const int c = h->plan.casts(target);
    return c < 0 ? LP_E_MISSING : c;
}

int64_t lp_describe(lp_handle* h, char* out, size_t cap) {
    if (!h) return LP_E_INVALID;
    std::string d = h->plan.describe();
    if (!out || d.size() + 1 > cap) return -(int64_t)(d.size() + 1);
    memcpy(out, d.c_str(), d.size() + 1);
    return (int64_t)d.size();
}

int lp_result_view(lp_handle* h, lp_result* out) {
    if (!h || !out) return LP_E_INVALID;
    const int st = ensure_synced(h);
    if (st != LP_OK) return st;
    lp_result& R = *out;
    R = lp_result{};
    R.n_lines = h->n_lines;
    R.first_line = h->first_line;
    R.input_bytes = h->nbytes;
    R.input = h->d_buf;
    R.line_off = h->line_off.as<uint64_t>();
    R.columns = h->cols.as<uint8_t>();
    R.columns_bytes = h->cols.cap;
    R.arena = h->arena.as<uint8_t>();
    R.arena_bytes = h->shard_cap * LP_ARENA_SHARDS;
    R.shard_cap = h->shard_cap;
    for (int s = 0; s < LP_ARENA_SHARDS; ++s) R.shard_off[s] = (uint64_t)s * h->shard_cap;
    R.n_columns = (int32_t)h->dev_cols.size();
    R.column = h->dev_cols.data();
    R.on_host = 0;
    return LP_OK;
}

int64_t lp_result_copy(lp_handle* h, void* host, uint64_t cap, int with_input, lp_result* out) {
    if (!h || (host && !out)) return LP_E_INVALID;
    const int st = ensure_synced(h);
    if (st != LP_OK) return st;
    return copy_result(h, (uint8_t*)host, host ? cap : 0, with_input != 0, out);
}

int64_t lp_result_record_json(lp_handle* h, const lp_result* r, int64_t i, char* out, size_t cap) {
    if (!h || !r || !r->on_host || !r->input) return LP_E_INVALID;
    if (i < 0 || i >= r->n_lines) return LP_E_INVALID;
    lp::ResultView V;
    make_view(h, *r, V);
    if (!V.status || V.status[i] != LP_LINE_OK) return LP_E_STATE;
    std::string js = h->plan.record_json(V, i);
    if (!out || js.size() + 1 > cap) return -100 - (int64_t)(js.size() + 1);
    memcpy(out, js.c_str(), js.size() + 1);
    return (int64_t)js.size();
}

// ---- typed columns of a batch (the output side: ParsedRecord / the Hive SerDe)
namespace {
// Long.parseLong: optional sign, decimal digits only, in range
bool java_parse_long(const uint8_t* p, uint32_t n, int64_t& out) {
    uint32_t k = 0;
    bool neg = false;
    if (n && (p[0] == '-' || p[0] == '+')) { neg = p[0] == '-'; k = 1; }
    if (k == n) return false;
    unsigned __int128 v = 0;
    for (; k < n; ++k) {
        if (p[k] < '0' || p[k] > '9') return false;
        v = v * 10 + (p[k] - '0');
        if (v > ((unsigned __int128)1 << 63)) return false;
    }
    if (!neg && v == ((unsigned __int128)1 << 63)) return false;
    out = neg ? (int64_t)(0 - (uint64_t)v) : (int64_t)v;
    return true;
}
// Double.parseDouble (FloatingDecimal.readJavaFormatString): chars <= ' '
// trimmed; [+-] then NaN | Infinity | decimal digits with an optional '.',
// exponent and f/F/d/D suffix | a hex float with a binary exponent
bool java_parse_double(const uint8_t* p, uint32_t n, double& out) {
    uint32_t a = 0, b = n;
    while (a < b && p[a] <= ' ') ++a;
    while (b > a && p[b - 1] <= ' ') --b;
    std::string t((const char*)p + a, b - a);
    static const std::regex dec("[+-]?(NaN|Infinity|(([0-9]+\\.?[0-9]*|\\.[0-9]+)([eE][+-]?[0-9]+)?)[fFdD]?)");
    static const std::regex hex("[+-]?0[xX]([0-9a-fA-F]+\\.?[0-9a-fA-F]*|\\.[0-9a-fA-F]+)[pP][+-]?[0-9]+[fFdD]?");
    const bool d = std::regex_match(t, dec), x = !d && std::regex_match(t, hex);
    if (!d && !x) return false;
    const bool neg = !t.empty() && t[0] == '-';
    if (t.find("NaN") != std::string::npos) { out = std::nan(""); return true; }
    if (t.find("Infinity") != std::string::npos) { out = neg ? -HUGE_VAL : HUGE_VAL; return true; }
    if (!t.empty() && strchr("fFdD", t.back())) t.pop_back();
    out = strtod(t.c_str(), nullptr);
    return true;
}
struct TableCtx {
    const std::unordered_map<std::string, std::vector<int>>* by_path;
    lp_table_col* cols;
    int64_t row;           // row in the output
    std::vector<std::string>* sbuf;  // per column: this chunk's STRING bytes
    std::vector<std::vector<std::pair<uint64_t, uint32_t>>>* sref;  // per column: (offset, len) per chunk row
    int64_t row0;          // first output row of the chunk
};
void table_value(void* vctx, const std::string& target, const lp::MVal& v) {
    TableCtx& t = *(TableCtx*)vctx;
    auto it = t.by_path->find(target);
    if (it == t.by_path->end()) return;
    for (int c : it->second) {
        lp_table_col& C = t.cols[c];
        // ParsedRecord.set(name, value) (ParsedRecord.java:154-170): a null is
        // ignored, the last value wins (Value.getString / getLong / getDouble)
        if (v.null) continue;
        if (C.kind == LP_CAST_STRING) {
            std::string& buf = (*t.sbuf)[c];
            const uint64_t off = buf.size();  // a chunk's bytes of one column may pass 4 GiB
            if (v.is_long) buf += std::to_string(v.l);
            else buf.append((const char*)v.p, v.len);
            (*t.sref)[c][t.row - t.row0] = {off, (uint32_t)(buf.size() - off)};
            C.valid[t.row] = 1;
        } else if (C.kind == LP_CAST_LONG) {
            int64_t x;
            if (v.is_long) x = v.l;
            else if (!java_parse_long(v.p, v.len, x)) continue;
            C.i64[t.row] = x;
            C.valid[t.row] = 1;
        } else {
            double x;
            if (v.is_long) x = (double)v.l;
            else if (!java_parse_double(v.p, v.len, x)) continue;
            C.f64[t.row] = x;
            C.valid[t.row] = 1;
        }
    }
}
}  // namespace

// lp_result_table on a device view: the columns built in HBM (table.hip)
static int table_device(lp_handle* h, int64_t first, int64_t count, lp_table_col* cols, int n_cols) {
    if (ensure_synced(h) != LP_OK) return LP_E_STATE;
    if (first < 0 || count < 0 || first + count > h->n_lines || n_cols > lp::MAX_TABLE_COLS) return LP_E_INVALID;
    auto ta = std::make_unique<lp::TableArgs>();
    memset(ta.get(), 0, sizeof(lp::TableArgs));
    ta->first = first;
    ta->count = count;
    ta->n_cols = n_cols;
    std::string names;
    for (int c = 0; c < n_cols; ++c) {
        lp_table_col& C = cols[c];
        lp::TableCol& T = ta->cols[c];
        T.kind = C.kind;
        if (!h->plan.table_src(C.path, T.src, names, T.alt)) return LP_E_UNSUPPORTED;
        if (C.kind == LP_CAST_DOUBLE)  // Double.parseDouble of a string stays on the host table
            for (int f = 0; f < 2 * lp::MAX_FMT; ++f) {
                const lp::TableSrc& x = f < lp::MAX_FMT ? T.src[f] : T.alt[f - lp::MAX_FMT];
                const bool long_valued = x.kind == lp::TC_NONE || x.kind == lp::TC_NULL ||
                                         (x.kind == lp::TC_URI && x.b == lp::UP_PORT) ||
                                         (x.kind == lp::TC_TIME && x.b != lp::TF_MONTHNAME && x.b != lp::TF_DATE &&
                                          x.b != lp::TF_TIME) ||
                                         x.kind == lp::TC_SECMS || x.kind == lp::TC_LIST_MS;
                // a SECOND_MILLIS list item: digits '.' digits, parsed on the device (decimal_to_double)
                const bool decimal = x.kind == lp::TC_LIST && h->plan.program().list[x.a].secms;
                if (!long_valued && !decimal) return LP_E_UNSUPPORTED;
            }
        T.valid = C.valid;
        T.i64 = C.i64;
        T.f64 = C.f64;
        T.chars = (uint8_t*)C.chars;
    }
    memcpy(ta->names, names.data(), names.size());
    hipSetDevice(h->device);
    hipStream_t s = h->stream;
    if (!h->targs.ensure(sizeof(lp::TableArgs))) return LP_E_NOMEM;
    int n_str = 0;
    for (int c = 0; c < n_cols; ++c) n_str += cols[c].kind == LP_CAST_STRING ? 1 : 0;
    const size_t scratch = lp::table_scratch_bytes(count, n_str);
    if (!h->tscratch.ensure(scratch)) return LP_E_NOMEM;
    ta->srcw = reinterpret_cast<uint64_t*>((char*)h->tscratch.p + lp::table_srcw_offset(count));
    if (hipMemcpyAsync(h->targs.p, ta.get(), sizeof(lp::TableArgs), hipMemcpyHostToDevice, s) != hipSuccess) return LP_E_DEVICE;
    const lp::DeviceArgs* d_args = h->args.as<lp::DeviceArgs>();
    const lp::TableArgs* d_targs = h->targs.as<lp::TableArgs>();
    hipEventRecord(h->tev[0], s);
    if (lp::launch_table_values(d_args, d_targs, *ta, h->d_buf, h->tscratch.p, h->tscratch.cap, s, h->tev[1]) != 0)
        return LP_E_DEVICE;
    hipEventRecord(h->tev[2], s);
    // the STRING columns' byte counts decide whether their bytes fit
    std::vector<int64_t> tot(n_cols, 0);
    for (int c = 0; c < n_cols; ++c)
        if (cols[c].kind == LP_CAST_STRING &&
            hipMemcpyAsync(&tot[c], cols[c].i64 + count, 8, hipMemcpyDeviceToHost, s) != hipSuccess)
            return LP_E_DEVICE;
    if (hipStreamSynchronize(s) != hipSuccess) return LP_E_DEVICE;
    bool fits = true;
    for (int c = 0; c < n_cols; ++c) {
        if (cols[c].kind != LP_CAST_STRING) continue;
        cols[c].chars_len = (uint64_t)tot[c];
        if (cols[c].chars_len > cols[c].chars_cap || (tot[c] && !cols[c].chars)) fits = false;
    }
    if (!fits) return LP_E_NOMEM;
    if (lp::launch_table_chars(d_args, d_targs, *ta, h->d_buf, s) != 0) return LP_E_DEVICE;
    hipEventRecord(h->tev[3], s);
    if (hipStreamSynchronize(s) != hipSuccess) return LP_E_DEVICE;
    float a = 0, b = 0, c = 0;
    hipEventElapsedTime(&a, h->tev[0], h->tev[1]);
    hipEventElapsedTime(&b, h->tev[1], h->tev[2]);
    hipEventElapsedTime(&c, h->tev[2], h->tev[3]);
    h->tms[0] = a;
    h->tms[1] = b;
    h->tms[2] = c;
    return LP_OK;
}

int lp_result_table(lp_handle* h, const lp_result* r, int64_t first, int64_t count, lp_table_col* cols, int n_cols,
                    int threads) {
    if (!h || !r || !cols || n_cols <= 0) return LP_E_INVALID;
    for (int c = 0; c < n_cols; ++c) {  // the same validation in both modes
        const lp_table_col& C = cols[c];
        if (!C.path || !C.valid || (C.kind == LP_CAST_STRING ? !C.i64 : C.kind == LP_CAST_LONG ? !C.i64 : !C.f64))
            return LP_E_INVALID;
        if (C.kind != LP_CAST_STRING && C.kind != LP_CAST_LONG && C.kind != LP_CAST_DOUBLE) return LP_E_INVALID;
        std::string p = C.path;
        int casts = h->plan.casts(p);
        if (casts < 0) {
            const size_t dot = p.rfind('.');
            if (dot != std::string::npos) casts = h->plan.casts(p.substr(0, dot) + ".*");
        }
        if (casts < 0) return LP_E_MISSING;
        if (!(casts & C.kind)) return LP_E_INVALID;
    }
    if (!r->on_host) {
        // a device view is only good for the batch the handle holds now
        if (!h->valid || r->n_lines != h->n_lines || r->first_line != h->first_line || r->input != h->d_buf ||
            r->line_off != h->line_off.as<uint64_t>())
            return LP_E_STATE;
        return table_device(h, first, count, cols, n_cols);
    }
    if (!r->input) return LP_E_INVALID;
    if (first < 0 || count < 0 || first + count > r->n_lines) return LP_E_INVALID;
    std::unordered_map<std::string, std::vector<int>> by_path;
    for (int c = 0; c < n_cols; ++c) {
        const lp_table_col& C = cols[c];
        if (!C.path || !C.valid || (C.kind == LP_CAST_STRING ? !C.i64 : C.kind == LP_CAST_LONG ? !C.i64 : !C.f64))
            return LP_E_INVALID;
        if (C.kind != LP_CAST_STRING && C.kind != LP_CAST_LONG && C.kind != LP_CAST_DOUBLE) return LP_E_INVALID;
        // the casts of the requested path (or of its wildcard request) must
        // allow the column type: else the reference's store finds no setter
        std::string p = C.path;
        int casts = h->plan.casts(p);
        if (casts < 0) {
            const size_t dot = p.rfind('.');
            if (dot != std::string::npos) casts = h->plan.casts(p.substr(0, dot) + ".*");
        }
        if (casts < 0) return LP_E_MISSING;
        if (!(casts & C.kind)) return LP_E_INVALID;
        by_path[p].push_back(c);
    }
    lp::ResultView V;
    make_view(h, *r, V);
    const int T = std::max(1, std::min(threads > 0 ? threads : 1, 64));
    const int64_t per = (count + T - 1) / T;
    std::vector<std::vector<std::string>> sbuf(T, std::vector<std::string>(n_cols));
    std::vector<std::vector<std::vector<std::pair<uint64_t, uint32_t>>>> sref(T);
    auto work = [&](int t) {
        const int64_t a = std::min(count, t * per), b = std::min(count, a + per);
        sref[t].assign(n_cols, std::vector<std::pair<uint64_t, uint32_t>>((size_t)(b - a), {0ull, 0u}));
        TableCtx ctx{&by_path, cols, 0, &sbuf[t], &sref[t], a};
        for (int64_t k = a; k < b; ++k) {
            for (int c = 0; c < n_cols; ++c) cols[c].valid[k] = 0;
            const int64_t i = first + k;
            if (!V.status || V.status[i] != LP_LINE_OK) continue;
            ctx.row = k;
            h->plan.rec_row(V, i, table_value, &ctx);
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < T; ++t) pool.emplace_back(work, t);
    work(0);
    for (auto& th : pool) th.join();
    // STRING columns (Arrow layout): row k = chars[offsets[k], offsets[k + 1]),
    // the row's last value; a row without one is empty (valid 0)
    int rc = LP_OK;
    for (int c = 0; c < n_cols; ++c) {
        lp_table_col& C = cols[c];
        if (C.kind != LP_CAST_STRING) continue;
        uint64_t need = 0;
        for (int64_t k = 0; k < count; ++k)
            if (C.valid[k]) need += sref[(size_t)(k / per)][c][(size_t)(k % per)].second;
        C.chars_len = need;
        if (need > C.chars_cap || (need && !C.chars)) { rc = LP_E_NOMEM; continue; }
        uint64_t pos = 0;
        for (int64_t k = 0; k < count; ++k) {
            C.i64[k] = (int64_t)pos;
            if (!C.valid[k]) continue;
            const int t = (int)(k / per);
            const auto& pr = sref[(size_t)t][c][(size_t)(k % per)];
            memcpy(C.chars + pos, sbuf[(size_t)t][c].data() + pr.first, pr.second);
            pos += pr.second;
        }
        C.i64[count] = (int64_t)pos;
    }
    return rc;
}

int lp_result_emit(lp_handle* h, const lp_result* r, int64_t i, lp_emit_fn fn, void* ctx) {
    if (!h || !r || !fn || !r->on_host || !r->input) return LP_E_INVALID;
    if (i < 0 || i >= r->n_lines) return LP_E_INVALID;
    lp::ResultView V;
    make_view(h, *r, V);
    if (!V.status || V.status[i] != LP_LINE_OK) return LP_E_STATE;
    return h->plan.emit_row(V, i, fn, ctx);
}

}  // extern "C"
