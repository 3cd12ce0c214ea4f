// C-ABI of the logparser_amd engine (include/logparser_amd.h).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/logparser_amd.h"
#include "kernels.h"
#include "plan.h"

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

}  // namespace

struct lp_handle {
    lp::Plan plan;
    int compile_status = LP_OK;
    int device = 0;
    hipStream_t stream = nullptr;
    DevBuf input, chunk, line_off, cols, arena, misc, waves, args, route;
    lp::DeviceArgs host_args{};
    lp::Columns C{};
    int64_t n_lines = 0;
    uint64_t nbytes = 0;
    const uint8_t* d_buf = nullptr;
    hipEvent_t ev[4]{};
    bool have_events = false;
    bool pending = false;
    uint64_t row_bytes = 0;
    uint64_t counters[4]{};
    uint64_t arena_used = 0;     // arena bytes allocated (bump pointer)
    uint64_t arena_written = 0;  // arena bytes actually written
    float ms[3]{};
    bool host_valid = false;
    lp::HostResults host;
    // HttpdLogFormatDissector's active format, carried from batch to batch
    // like the reference parser's (format 0 before the first line)
    uint32_t fmt_state = 0;
};

namespace {

void set_err(char* err, size_t errlen, const std::string& s) {
    if (err && errlen) snprintf(err, errlen, "%s", s.c_str());
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Lay out the result columns for n lines in one allocation.
bool alloc_columns(lp_handle* h, int64_t n) {
    const lp::Program& P = h->plan.program();
    struct Col { void** dst; size_t esz; };
    std::vector<Col> cols;
    lp::Columns& C = h->C;
    cols.push_back({(void**)&C.status, 1});
    for (int k = 0; k < P.n_tok; ++k) cols.push_back({(void**)&C.tok_span[k], 4});
    cols.push_back({(void**)&C.tok_flags, 4});
    for (int t = 0; t < P.n_time; ++t) {
        cols.push_back({(void**)&C.t_epoch[t], 8});
        cols.push_back({(void**)&C.t_local[t], 8});
        cols.push_back({(void**)&C.t_utc[t], 8});
        if (P.time[t].kind == lp::TK_STRF) cols.push_back({(void**)&C.t_nano[t], 4});  // only strftime has fractions
    }
    for (int f = 0; f < P.n_fl; ++f) {
        cols.push_back({(void**)&C.fl_kind[f], 4});
        cols.push_back({(void**)&C.fl_method[f], 4});
        cols.push_back({(void**)&C.fl_uri[f], 4});
        cols.push_back({(void**)&C.fl_proto[f], 4});
    }
    for (int u = 0; u < P.n_uri; ++u) {
        cols.push_back({(void**)&C.u_flags[u], 4});
        cols.push_back({(void**)&C.u_scheme[u], 8});
        cols.push_back({(void**)&C.u_host[u], 8});
        cols.push_back({(void**)&C.u_port[u], 4});
        cols.push_back({(void**)&C.u_path[u], 8});
        cols.push_back({(void**)&C.u_query[u], 8});
        cols.push_back({(void**)&C.u_frag[u], 8});
    }
    for (int q = 0; q < P.n_query; ++q) {
        cols.push_back({(void**)&C.q_count[q], 4});
        cols.push_back({(void**)&C.q_params[q], 8});
    }
    cols.push_back({(void**)&C.arena_base, 8});
    if (P.n_fmt > 1) {
        cols.push_back({(void**)&C.fmt_match, 2});
        cols.push_back({(void**)&C.fmt_id, 1});
    }
    size_t total = 0;
    uint64_t row = 0;
    for (auto& c : cols) {
        total += align256(c.esz * (size_t)(n > 0 ? n : 1));
        row += c.esz;
    }
    if (!h->cols.ensure(total)) return false;
    size_t off = 0;
    for (auto& c : cols) {
        *c.dst = h->cols.as<char>(off);
        off += align256(c.esz * (size_t)(n > 0 ? n : 1));
    }
    h->row_bytes = row;
    return true;
}

template <typename T>
void fetch(std::vector<T>& dst, const T* src, int64_t n) {
    dst.resize((size_t)(n > 0 ? n : 0));
    if (n > 0 && src) hipMemcpy(dst.data(), src, sizeof(T) * (size_t)n, hipMemcpyDeviceToHost);
}

bool fetch_host(lp_handle* h) {
    if (h->host_valid) return true;
    if (h->pending) lp_sync(h);
    const lp::Program& P = h->plan.program();
    lp::HostResults& R = h->host;
    const int64_t n = h->n_lines;
    R.n = n;
    fetch(R.line_off, h->line_off.as<uint64_t>(), n + 1);
    fetch(R.status, h->C.status, n);
    R.input.resize(h->nbytes);
    if (h->nbytes) hipMemcpy(R.input.data(), h->d_buf, h->nbytes, hipMemcpyDeviceToHost);
    R.input.push_back('\n');
    if (!h->plan.device_ok()) { h->host_valid = true; return true; }
    if (P.n_fmt > 1) fetch(R.fmt_id, h->C.fmt_id, n);
    R.tok_span.resize(lp::MAX_TOK);
    for (int k = 0; k < P.n_tok; ++k) fetch(R.tok_span[k], h->C.tok_span[k], n);
    fetch(R.tok_flags, h->C.tok_flags, n);
    R.t_epoch.resize(lp::MAX_TIME); R.t_local.resize(lp::MAX_TIME); R.t_utc.resize(lp::MAX_TIME);
    R.t_nano.resize(lp::MAX_TIME);
    for (int t = 0; t < P.n_time; ++t) {
        fetch(R.t_epoch[t], h->C.t_epoch[t], n);
        fetch(R.t_local[t], h->C.t_local[t], n);
        fetch(R.t_utc[t], h->C.t_utc[t], n);
        if (P.time[t].kind == lp::TK_STRF) fetch(R.t_nano[t], h->C.t_nano[t], n);
    }
    R.fl_kind.resize(lp::MAX_FL); R.fl_method.resize(lp::MAX_FL); R.fl_uri.resize(lp::MAX_FL); R.fl_proto.resize(lp::MAX_FL);
    for (int f = 0; f < P.n_fl; ++f) {
        fetch(R.fl_kind[f], h->C.fl_kind[f], n);
        fetch(R.fl_method[f], h->C.fl_method[f], n);
        fetch(R.fl_uri[f], h->C.fl_uri[f], n);
        fetch(R.fl_proto[f], h->C.fl_proto[f], n);
    }
    for (auto* v : {&R.u_scheme, &R.u_host, &R.u_path, &R.u_query, &R.u_frag}) v->resize(lp::MAX_URI);
    R.u_flags.resize(lp::MAX_URI); R.u_port.resize(lp::MAX_URI);
    for (int u = 0; u < P.n_uri; ++u) {
        fetch(R.u_flags[u], h->C.u_flags[u], n);
        fetch(R.u_scheme[u], h->C.u_scheme[u], n);
        fetch(R.u_host[u], h->C.u_host[u], n);
        fetch(R.u_port[u], h->C.u_port[u], n);
        fetch(R.u_path[u], h->C.u_path[u], n);
        fetch(R.u_query[u], h->C.u_query[u], n);
        fetch(R.u_frag[u], h->C.u_frag[u], n);
    }
    R.q_count.resize(lp::MAX_QUERY); R.q_params.resize(lp::MAX_QUERY);
    for (int q = 0; q < P.n_query; ++q) {
        fetch(R.q_count[q], h->C.q_count[q], n);
        fetch(R.q_params[q], h->C.q_params[q], n);
    }
    fetch(R.arena_base, h->C.arena_base, n);
    R.arena.resize(h->arena_used + 64);
    if (h->arena_used) hipMemcpy(R.arena.data(), h->C.arena, h->arena_used, hipMemcpyDeviceToHost);
    h->host_valid = true;
    return true;
}

}  // namespace

extern "C" {

lp_handle* lp_compile(const char* logformats, const char* const* paths, int n_paths, int device, int* status,
                      char* err, size_t errlen) {
    if (status) *status = LP_E_INVALID;
    if (!logformats || (n_paths > 0 && !paths)) { set_err(err, errlen, "null argument"); return nullptr; }
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
    int st = h->plan.build(logformats, f, e);
    if (st != LP_OK && st != LP_E_UNSUPPORTED) {
        if (status) *status = st;
        set_err(err, errlen, e);
        return nullptr;
    }
    if (st == LP_E_UNSUPPORTED) set_err(err, errlen, h->plan.unsupported_reason());
    h->compile_status = st;
    if (hipSetDevice(device) != hipSuccess) { if (status) *status = LP_E_DEVICE; return nullptr; }
    for (auto& ev : h->ev) hipEventCreate(&ev);
    h->have_events = true;
    if (!h->misc.ensure(256)) { if (status) *status = LP_E_NOMEM; return nullptr; }
    if (status) *status = st;
    return h.release();
}

void lp_free(lp_handle* h) {
    if (!h) return;
    hipSetDevice(h->device);
    if (h->pending) hipStreamSynchronize(h->stream);
    for (auto* b : {&h->input, &h->chunk, &h->line_off, &h->cols, &h->arena, &h->misc, &h->waves, &h->args, &h->route})
        b->release();
    if (h->have_events)
        for (auto& ev : h->ev) hipEventDestroy(ev);
    delete h;
}

int64_t lp_possible_paths(const char* logformats, int max_depth, char* out, size_t cap) {
    std::vector<std::string> paths;
    std::string err;
    lp::Plan::possible_paths(logformats ? logformats : "", max_depth, paths, err);
    std::string s;
    for (auto& p : paths) s += p + "\n";
    if (!out || s.size() + 1 > cap) return -(int64_t)(s.size() + 1);
    memcpy(out, s.c_str(), s.size() + 1);
    return (int64_t)s.size();
}

int lp_parse_batch(lp_handle* h, const uint8_t* buf, uint64_t nbytes, int buf_flags, void* stream) {
    if (!h || (!buf && nbytes)) return LP_E_INVALID;
    if (hipSetDevice(h->device) != hipSuccess) return LP_E_DEVICE;
    if (h->pending) lp_sync(h);
    hipStream_t s = (hipStream_t)stream;
    h->stream = s;
    h->host_valid = false;
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
    const int64_t nc = lp::count_chunks(nbytes);
    const size_t cbytes = align256(sizeof(uint64_t) * (size_t)(nc + 2));
    if (!h->chunk.ensure(cbytes + 2 * (size_t)lp::nlmask_words(nbytes))) return LP_E_NOMEM;
    uint64_t* d_chunk = h->chunk.as<uint64_t>();
    uint16_t* d_nlmask = h->chunk.as<uint16_t>(cbytes);
    hipEventRecord(h->ev[0], s);
    // index pass 1 (count + scan), then the line count on the host
    if (lp::launch_count(h->d_buf, nbytes, d_chunk, d_nlmask, s) != 0) return LP_E_DEVICE;
    uint64_t total = 0;
    uint8_t last = '\n';
    if (nc > 0) {
        hipMemcpyAsync(&total, d_chunk + nc, sizeof total, hipMemcpyDeviceToHost, s);
        hipMemcpyAsync(&last, h->d_buf + nbytes - 1, 1, hipMemcpyDeviceToHost, s);
    }
    if (hipStreamSynchronize(s) != hipSuccess) return LP_E_DEVICE;
    const int64_t n = (int64_t)total + (nbytes > 0 && last != '\n' ? 1 : 0);
    h->n_lines = n;
    if (!h->line_off.ensure(sizeof(uint64_t) * (size_t)(n + 2))) return LP_E_NOMEM;
    uint64_t* d_off = h->line_off.as<uint64_t>();
    uint64_t head = 0, tail = nbytes + 1;
    hipMemcpyAsync(d_off, &head, sizeof head, hipMemcpyHostToDevice, s);
    if (lp::launch_offsets(d_nlmask, nbytes, d_chunk, d_off, s) != 0) return LP_E_DEVICE;
    if (nbytes > 0 && last != '\n') hipMemcpyAsync(d_off + n, &tail, sizeof tail, hipMemcpyHostToDevice, s);
    hipEventRecord(h->ev[1], s);
    // results
    if (!alloc_columns(h, n)) return LP_E_NOMEM;
    const lp::Program& P = h->plan.program();
    // arena: generous bound (only written bytes cost bandwidth)
    uint64_t acap = h->plan.device_ok() && P.n_uri > 0 ? 3 * nbytes + 64 * (uint64_t)n + 4096 : 4096;
    if (!h->arena.ensure(acap)) return LP_E_NOMEM;
    lp::Columns& C = h->C;
    C.line_off = d_off;
    C.arena = h->arena.as<uint8_t>();
    C.arena_cap = h->arena.cap;
    if (!h->waves.ensure(4 * lp::WC_WORDS * (size_t)(lp::parse_waves(n) + 1))) return LP_E_NOMEM;
    C.wave_counts = h->waves.as<uint32_t>();
    C.arena_top = h->misc.as<unsigned long long>(64);
    hipMemsetAsync(h->misc.p, 0, 128, s);
    if (h->plan.device_ok()) {
        if (P.n_fmt > 1) {  // sticky multi-format routing scratch
            if (!h->route.ensure(8 * (size_t)(lp::fmt_chunks(n) + 1))) return LP_E_NOMEM;
            C.fmt_chunk = h->route.as<uint64_t>();
            C.fmt_init = h->fmt_state;
        }
        if (!h->args.ensure(sizeof(lp::DeviceArgs))) return LP_E_NOMEM;
        h->host_args.prog = P;
        h->host_args.cols = C;
        if (hipMemcpyAsync(h->args.p, &h->host_args, sizeof(lp::DeviceArgs), hipMemcpyHostToDevice, s) != hipSuccess)
            return LP_E_DEVICE;
        hipEventRecord(h->ev[2], s);
        if (P.n_fmt > 1) {
            // HttpdLogFormatDissector routing: every format's match per line,
            // then the scan of the sticky active format
            if (lp::launch_parse(h->d_buf, nbytes, n, h->args.as<lp::DeviceArgs>(), P.n_elems, P.max_stack, C.wave_counts,
                                 h->misc.as<unsigned long long>(), s, lp::PM_MATCH) != 0 ||
                lp::launch_route(h->args.as<lp::DeviceArgs>(), n, s) != 0)
                return LP_E_DEVICE;
        }
        if (lp::launch_parse(h->d_buf, nbytes, n, h->args.as<lp::DeviceArgs>(), P.n_elems, P.max_stack, C.wave_counts,
                             h->misc.as<unsigned long long>(), s) != 0)
            return LP_E_DEVICE;
    } else {
        // the requested paths need a dissector that is not on the device:
        // every line goes back to the reference (FALLBACK)
        hipEventRecord(h->ev[2], s);
        if (n) hipMemsetAsync(C.status, LP_LINE_FALLBACK, (size_t)n, s);
    }
    hipEventRecord(h->ev[3], s);
    h->pending = true;
    return LP_OK;
}

int lp_sync(lp_handle* h) {
    if (!h) return LP_E_INVALID;
    if (!h->pending) return LP_OK;
    hipSetDevice(h->device);
    if (hipStreamSynchronize(h->stream) != hipSuccess) return LP_E_DEVICE;
    h->pending = false;
    unsigned long long m[16];
    hipMemcpy(m, h->misc.p, sizeof m, hipMemcpyDeviceToHost);
    if (h->plan.device_ok()) {
        for (int k = 0; k < 4; ++k) h->counters[k] = m[k];
    } else {
        h->counters[0] = (uint64_t)h->n_lines;
        h->counters[1] = h->counters[2] = 0;
        h->counters[3] = (uint64_t)h->n_lines;
    }
    h->arena_used = m[8];
    const lp::Program& P = h->plan.program();
    if (h->plan.device_ok() && P.n_fmt > 1 && h->n_lines > 0) {  // the active format after the batch's last line
        uint64_t st = 0;
        hipMemcpy(&st, h->C.fmt_chunk + lp::fmt_chunks(h->n_lines), sizeof st, hipMemcpyDeviceToHost);
        h->fmt_state = (uint32_t)st;
    }
    h->arena_written = h->plan.device_ok() ? m[4] : 0;
    float a = 0, b = 0, c = 0;
    hipEventElapsedTime(&a, h->ev[0], h->ev[3]);
    hipEventElapsedTime(&b, h->ev[0], h->ev[1]);
    hipEventElapsedTime(&c, h->ev[2], h->ev[3]);
    h->ms[0] = a; h->ms[1] = b; h->ms[2] = c;
    return LP_OK;
}

int64_t lp_num_lines(lp_handle* h) { return h ? h->n_lines : LP_E_INVALID; }

int lp_line_status(lp_handle* h, int64_t first, int64_t count, uint8_t* out) {
    if (!h || first < 0 || count < 0 || first + count > h->n_lines) return LP_E_INVALID;
    if (h->pending) lp_sync(h);
    if (count && hipMemcpy(out, h->C.status + first, (size_t)count, hipMemcpyDeviceToHost) != hipSuccess) return LP_E_DEVICE;
    return LP_OK;
}

int64_t lp_line_offset(lp_handle* h, int64_t i) {
    if (!h || i < 0 || i > h->n_lines) return LP_E_INVALID;
    if (h->pending) lp_sync(h);
    uint64_t v = 0;
    hipMemcpy(&v, h->line_off.as<uint64_t>() + i, sizeof v, hipMemcpyDeviceToHost);
    return (int64_t)v;
}

int64_t lp_line_record_json(lp_handle* h, int64_t i, char* out, size_t cap) {
    if (!h || i < 0 || i >= h->n_lines) return LP_E_INVALID;
    if (!fetch_host(h)) return LP_E_DEVICE;
    if (h->host.status[(size_t)i] != LP_LINE_OK) return LP_E_STATE;
#ifdef LP_DEBUG_HOST
    for (int u = 0; u < h->plan.program().n_uri; ++u)
        fprintf(stderr, "host i=%lld u=%d flags=%x query=%llx path=%llx line_off=%llu\n", (long long)i, u,
                h->host.u_flags[u][i], (unsigned long long)h->host.u_query[u][i], (unsigned long long)h->host.u_path[u][i],
                (unsigned long long)h->host.line_off[i]);
#endif
    std::string js = h->plan.record_json(h->host, i);
    if (!out || js.size() + 1 > cap) return -100 - (int64_t)(js.size() + 1);
    memcpy(out, js.c_str(), js.size() + 1);
    return (int64_t)js.size();
}

int lp_counters(lp_handle* h, uint64_t* out, int n) {
    if (!h || !out) return LP_E_INVALID;
    if (h->pending) lp_sync(h);
    for (int k = 0; k < n && k < 4; ++k) out[k] = h->counters[k];
    return n < 4 ? n : 4;
}

int lp_last_timing(lp_handle* h, float* out, int n) {
    if (!h || !out) return LP_E_INVALID;
    if (h->pending) lp_sync(h);
    for (int k = 0; k < n && k < 3; ++k) out[k] = h->ms[k];
    return n < 3 ? n : 3;
}

int lp_last_bytes(lp_handle* h, uint64_t* out, int n) {
    if (!h || !out) return LP_E_INVALID;
    if (h->pending) lp_sync(h);
    uint64_t v[2] = {h->nbytes, (uint64_t)h->n_lines * (h->row_bytes + 8) + h->arena_written};
    for (int k = 0; k < n && k < 2; ++k) out[k] = v[k];
    return n < 2 ? n : 2;
}

int64_t lp_describe(lp_handle* h, char* out, size_t cap) {
    if (!h) return LP_E_INVALID;
    std::string d = h->plan.describe();
    if (!out || d.size() + 1 > cap) return -(int64_t)(d.size() + 1);
    memcpy(out, d.c_str(), d.size() + 1);
    return (int64_t)d.size();
}

}  // extern "C"
