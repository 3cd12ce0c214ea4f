// TEST-ONLY CPU emulation of the device per-line logic.
//
// Compiles logparser_amd/csrc/lp_device.h (the exact source of the gfx950
// kernel's per-line code) and plan.cpp with g++ so the planner, matcher and
// stages can be diffed against the oracle in the CPU test suite.  It is never
// part of the product: the product library (liblogparser_amd.so) only runs
// this logic inside the HIP kernel and fails when no GPU is present.
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../logparser_amd/csrc/lp_device.h"
#include "../../logparser_amd/csrc/plan.h"

using namespace lp;

struct Emu {
    Plan plan;
    int status;
    std::string err;
    uint32_t fmt_state = 0;  // sticky active LogFormat (HttpdLogFormatDissector), carried line to line
};

// the kernel instance a one-format program runs in (capi.cpp enqueue: the
// literal-aware first candidates only for programs that have such elements)
static bool lit_aware(const Program& P) {
    for (int i = 0; i < P.n_elems; ++i) {
        const ElemV e = load_elem(P.elems + i);
        if (e.nlit && !e.last && ((e.kind == EK_NOSPACE && !e.det) || e.kind == EK_NOSPACE3)) return true;
    }
    return false;
}

extern "C" {

// with type remappings: rm_in[k] -> rm_type[k] (STRING_ONLY casts)
void* emu_new_remapped(const char* fmt, const char* const* fields, int n, const char* const* rm_in,
                       const char* const* rm_type, int n_rm, int* status, char* err, int errlen) {
    Emu* e = new Emu();
    std::vector<std::string> f(fields, fields + n);
    std::vector<Remap> rm;
    for (int k = 0; k < n_rm; ++k) rm.push_back(Remap{rm_in[k], rm_type[k], CAST_S});
    e->status = e->plan.build(fmt, f, e->err, rm);
    *status = e->status;
    if (err && errlen) snprintf(err, errlen, "%s%s", e->err.c_str(), e->plan.device_ok() ? "" : e->plan.unsupported_reason().c_str());
    if (e->status != 0 && e->status != -3) { delete e; return nullptr; }
    return e;
}

void* emu_new(const char* fmt, const char* const* fields, int n, int* status, char* err, int errlen) {
    return emu_new_remapped(fmt, fields, n, nullptr, nullptr, 0, status, err, errlen);
}

void emu_free(void* h) { delete (Emu*)h; }

// Parser.getCasts of a "TYPE:path" (the planner's castsOfTargets), -1 unknown
int emu_casts(void* h, const char* target) { return ((Emu*)h)->plan.casts(target); }

int emu_describe(void* h, char* out, int cap) {
    std::string d = ((Emu*)h)->plan.describe();
    snprintf(out, cap, "%s", d.c_str());
    return (int)d.size();
}

static int parse_impl(Emu* e, const char* line, int len, const uint8_t* base, uint32_t base_off, char* out, int cap);
static int g_masks_fwd(int on);

// returns line status (0 OK, 1 BAD, 2 FALLBACK), fills out with the record JSON when OK
int emu_parse(void* h, const char* line, int len, char* out, int cap) {
    // the line at a varying offset of a 4-byte aligned base, as inside the
    // kernel's LDS window (exercises the word-at-a-time scanners' edges)
    const uint32_t off = (uint32_t)(len * 7 + (len > 0 ? (uint8_t)line[0] : 0)) & 3u;
    std::vector<uint8_t> padded(off, 0xFF);
    padded.insert(padded.end(), line, line + len);
    padded.push_back('\n');
    padded.resize(padded.size() + 8, 0xFF);  // word reads of the last bytes
    return parse_impl((Emu*)h, line, len, padded.data(), off, out, cap);
}

// the line is buf[start, start+len) of a whole batch buffer (as the kernel
// sees it: neighbouring lines around it); buf must be 4-byte aligned and
// readable up to the next multiple of 4 after the line
int emu_parse_in(void* h, const char* buf, int64_t start, int len, char* out, int cap) {
    return parse_impl((Emu*)h, buf + start, len, (const uint8_t*)buf, (uint32_t)start, out, cap);
}

void emu_set_masks(int on) { g_masks_fwd(on); }

// uplist_at (byte reads) and uplist_at_r (register masks) on the line
// buf[0, len) at offset p, the line at byte offset `off` of an aligned
// buffer: out = {uplist_at, uplist_at_r}
void emu_uplist(const char* v, int len, int p, int off, int dec, int* out) {
    std::vector<uint8_t> buf((size_t)off, 0xA5);
    buf.insert(buf.end(), v, v + len);
    buf.resize(((buf.size() + 8 + 3) & ~(size_t)3) + 40, 0xA5);
    const Line L{buf.data(), (uint32_t)off, len};
    out[0] = uplist_at(L, p, dec != 0);
    out[1] = uplist_at_r(L, p, dec != 0);
}

// UpstreamListDissector's split of the token v[0, len) (at byte offset `off`
// of an aligned buffer): uplist_items (byte reads) and, when tok_load takes
// the token (at most 32 bytes), uplist_items_r (registers); per item its
// four trimmed positions and secms_value / secms_value_r of the value and
// redirected spans (digits '.' digits items only: dec).  out: [0] the byte
// count, [1] the register count (-2: not loaded), then 16 items x 8 int64
// for each version.  Returns 0.
int emu_uplist_items(const char* v, int len, int off, int dec, int64_t* out) {
    std::vector<uint8_t> buf((size_t)off, 0xA5);
    buf.insert(buf.end(), v, v + len);
    buf.resize(((buf.size() + 8 + 3) & ~(size_t)3) + 40, 0xA5);
    const Line L{buf.data(), (uint32_t)off, len};
    for (int k = 0; k < 2 + 2 * 16 * 8; ++k) out[k] = 0;
    auto rec = [&](int64_t* o, auto&& sm) {
        return [o, &sm](int k, int va, int vb, int ra, int rb) {
            if (k >= 16) return;
            int64_t* e = o + 8 * k;
            e[0] = va; e[1] = vb; e[2] = ra; e[3] = rb;
            e[4] = sm(va, vb);
            e[5] = sm(ra, rb);
        };
    };
    auto sm_b = [&](int a, int b) -> int64_t { return dec ? secms_value(L, a, b) : 0; };
    out[0] = uplist_items(L, 0, len, rec(out + 2, sm_b));
    TokReg T;
    if (tok_load(L, 0, len, T)) {
        auto sm_r = [&](int a, int b) -> int64_t { return dec ? secms_value_r(T, a, b) : 0; };
        out[1] = uplist_items_r(T, 0, len, rec(out + 2 + 16 * 8, sm_r));
    } else {
        out[1] = -2;
    }
    return 0;
}

// parse_strf_time of the program's first time stage on the value v[0, len)
// placed at byte offset `off` (0..3) of an aligned buffer, with the stage's
// fixed-layout plan (use_fixed 1) or the general element loop only (0):
// out = {status, epoch_ms, local, utc, nanos}; returns -1 without a strftime stage
int emu_strf(void* h, const char* v, int len, int off, int use_fixed, int64_t* out) {
    const Program& P = ((Emu*)h)->plan.program();
    if (P.n_time < 1 || P.time[0].kind != TK_STRF) return -1;
    TimeStage T = P.time[0];
    if (!use_fixed) { T.fx_n = 0; T.fixed_w = 0; }
    std::vector<uint8_t> buf((size_t)off, 0xA5);
    buf.insert(buf.end(), v, v + len);
    buf.resize(((buf.size() + 8 + 3) & ~(size_t)3) + 40, 0xA5);  // word reads past the value
    const Line L{buf.data(), (uint32_t)off, len};
    int64_t ep = 0;
    uint64_t lo = 0, ut = 0;
    uint32_t ns = 0;
    const int st = parse_strf_time(T, L, 0, len, ep, lo, ut, ns);
    out[0] = st;
    out[1] = ep;
    out[2] = (int64_t)lo;
    out[3] = (int64_t)ut;
    out[4] = ns;
    return T.fx_n;
}

// the planner's token table (plan.cpp) as canonical JSON; returns its length
int emu_token_table(int nginx, char* out, int cap) {
    const std::string j = lp::token_table_json(nginx != 0);
    if (out && cap > 0) snprintf(out, cap, "%s", j.c_str());
    return (int)j.size();
}

}  // extern "C"

// One line's results, stored in vectors (the emulation's columns, one row).
struct Store {
    std::vector<uint64_t> line_off;
    std::vector<uint8_t> status, input, arena, fmt_id;
    std::vector<uint64_t> arena_base;
    std::vector<std::vector<uint32_t>> tok_span, t_nano, fl_kind, fl_method, fl_uri, fl_proto, u_flags, q_count;
    std::vector<uint32_t> tok_flags;
    std::vector<std::vector<int64_t>> t_epoch;
    std::vector<std::vector<uint64_t>> t_local, t_utc, u_scheme, u_host, u_path, u_query, u_frag, q_params;
    std::vector<std::vector<int32_t>> u_port;
    std::vector<std::vector<int64_t>> sm_ms;
    std::vector<std::vector<uint32_t>> l_count;
    std::vector<std::vector<uint64_t>> l_tab;
    std::vector<std::vector<uint32_t>> bip, p_count;
    std::vector<std::vector<uint64_t>> p_tab;
};

// The URI kernel's view of one URI source [a, b) of the line at base + off:
// the source's whole 4-byte words copied into a compact buffer (the span
// starts at the same offset mod 4), a zero word after them, zero-filled to
// 64 bytes, and the buffer's one-plane UEV mask (g_masks), or the whole line
// (the URI kernel's direct path, SWAR scanners).
struct UriView {
    std::vector<uint64_t> buf, plane;
    uint32_t o = 0;
    int n = 0;
};
static UriView uri_view(const uint8_t* base, uint32_t off, int a, int b) {
    UriView V;
    const uint32_t s0 = (off + (uint32_t)a) & ~3u, s1 = (off + (uint32_t)b + 3) & ~3u;
    const uint32_t lead = 8;  // the span's words do not start the buffer (as in the kernel)
    const uint32_t used = lead + (s1 - s0) + 4, tot = (used + 63) & ~63u;
    V.buf.assign(tot / 8 + 1, 0);
    memset(V.buf.data(), 0x5A, lead);
    memcpy((uint8_t*)V.buf.data() + lead, base + s0, s1 - s0);
    V.plane.assign(tot / 64 + 1, 0);
    build_uev_plane((const uint8_t*)V.buf.data(), tot, V.plane.data());
    V.o = lead + ((off + (uint32_t)a) & 3u) - (uint32_t)a;
    V.n = b;
    return V;
}

static int g_masks = 1;  // 1: lines carry byte-class masks (the kernels' LDS paths), 0: SWAR scanners (HBM paths)

template <typename LN>
static int run_line(const Program& P, const LN& L, const uint8_t* base, uint32_t off, LineOut& o, uint32_t* stk,
                    Columns& C, Store& R, char* out, int cap, uint32_t& fmt_state) {
    if (P.n_fmt > 1) {  // sticky routing, one line at a time (the kernels do it as a scan)
        const uint32_t m = fmt_match_word(P, P.elems, L, stk, false);
        fmt_state = fmt_apply(fmt_table(m, P.n_fmt), fmt_state);
        R.fmt_id.assign(1, (uint8_t)fmt_state);
    }
    bool pre = false;
    if (P.n_fmt > 1) {
        // as the one-pass chunk kernel (parse.hip parse_chunk<..., MF>): a line
        // exactly one format matches without the DFS is parsed from the spans
        // the routing word captured (phase1 PRE); the rest as k_parse_ovf_lines
        // does after the routing scan (the whole phase 1 on the routed format)
        bool redo = false;
        const uint32_t w = fmt_match_word<false>(P, P.elems, L, stk, false, &redo, &o.caps);
        const uint32_t mm = w & 0xFFu;
        pre = !redo && !(w >> 8) && mm && !(mm & (mm - 1));
        if (pre && (uint32_t)__builtin_ctz(mm) != fmt_state) return -2;  // (the state must agree: exactness check)
    }
    if (pre) phase1<true, true, false, false, true>(P, P.elems, L, o, stk, C, 0, false, (int)fmt_state);
    else if (P.n_fmt > 1) phase1<false>(P, P.elems, L, o, stk, C, 0, false, (int)fmt_state);  // as k_parse_ovf_lines
    else if (lit_aware(P)) phase1<false, true>(P, P.elems, L, o, stk, C, 0, false, 0);  // as k_parse_chunks<true>
    else phase1<false, false>(P, P.elems, L, o, stk, C, 0, false, 0);            // as k_parse_chunks<false>
    write_line(P, o, C, 0);
    if (o.status != ST_OK || !P.has_phase2()) return 0;
    // the URI kernel: its sources from the columns phase 1 wrote
    RegArr<MAX_URI> sp, usep;
    sp.fill(0);
    usep.fill(0);
    std::vector<UriView> views(MAX_URI);
    uint32_t need = 0;
    for (int u = 0; u < P.n_uri; ++u) {
        int a, b;
        if (P.uri[u].fmt != o.fmt || !uri_source_cols(P, C, 0, u, a, b)) continue;
        sp.set(u, mkspan(a, b));
        views[u] = uri_view(base, off, a, b);
        uint32_t ev;
        if (g_masks) need += uri_need(P, u, ULine{(const uint8_t*)views[u].buf.data(), views[u].o, views[u].n,
                                                   views[u].plane.data()}, a, b, ev);
        else need += uri_need(P, u, L, a, b, ev);
        usep.set(u, ev);
    }
    // the upstream list stages read the line itself (the URI kernel: from HBM)
    const Line LH{base, off, L.n};
    need += list_need(P, o.fmt, LH, C, 0) + pair_need(P, o.fmt, LH, C, 0);
    need = (need + 15) & ~15u;
    // the region, then room for spills (a shard of its own: bump counter
    // after the region, as the kernel's shard_top)
    const uint64_t room = need + 64ull * (uint64_t)L.n + 8192;
    R.arena.assign(room + 64, 0);
    unsigned long long top = need;
    Arena A{R.arena.data(), 0, need};
    A.top = &top;
    A.base = 0;
    A.limit = room;
    UriOut uo;
    uo.qlist.fill(0);
    uo.qpend.fill(0);
    if (g_masks) {
        auto lu = [&](int u) {
            return ULine{(const uint8_t*)views[u].buf.data(), views[u].o, views[u].n, views[u].plane.data()};
        };
        phase2(P, o.fmt, lu, sp, usep, uo, A, C, 0);
        if (uo.status == ST_OK) query_pieces_serial(P, lu, uo, A);
    } else {
        auto lu = [&](int) { return L; };
        phase2(P, o.fmt, lu, sp, usep, uo, A, C, 0);
        if (uo.status == ST_OK) query_pieces_serial(P, lu, uo, A);
    }
    if (uo.status == ST_OK && (!list_fill(P, o.fmt, LH, A, C, 0) || !pair_fill(P, o.fmt, LH, A, C, 0))) uo.status = ST_FALLBACK;
    if (A.used > need) { snprintf(out, cap, "ARENA OVERFLOW %u > %u", A.used, need); return 3; }
    if (A.ovf) { snprintf(out, cap, "ARENA SPILL OVERFLOW"); return 3; }
    // k_derived_lines: the remapped query parameters' URI stages, on the
    // line in the input and the values in the region
    if (uo.status == ST_OK) {
        Arena D{R.arena.data(), 0, 0};
        D.top = &top;
        D.base = 0;
        D.limit = room;
        uo.status = derived_line(P, o.fmt, base + (off & ~3u), off & 3u, L.n, D, C, 0);
        if (D.ovf) { snprintf(out, cap, "ARENA SPILL OVERFLOW (derived)"); return 3; }
    }
    o.status = uo.status;
    C.status[0] = (uint8_t)o.status;
    return 0;
}

extern "C" {

static int parse_impl(Emu* e, const char* line, int len, const uint8_t* base, uint32_t base_off, char* out, int cap) {
    if (!e->plan.device_ok()) return 2;
    const Program& P = e->plan.program();
    Store R;
    R.input.assign(line, line + len);
    R.input.push_back('\n');
    R.line_off = {0, (uint64_t)len + 1};
    R.status.assign(1, 0);
    R.tok_span.assign(MAX_TOK, std::vector<uint32_t>(1));
    R.tok_flags.assign(1, 0);
    R.t_epoch.assign(MAX_TIME, std::vector<int64_t>(1));
    R.t_local.assign(MAX_TIME, std::vector<uint64_t>(1));
    R.t_utc.assign(MAX_TIME, std::vector<uint64_t>(1));
    R.t_nano.assign(MAX_TIME, std::vector<uint32_t>(1));
    for (auto* v : {&R.fl_kind, &R.fl_method, &R.fl_uri, &R.fl_proto}) v->assign(MAX_FL, std::vector<uint32_t>(1));
    R.u_flags.assign(MAX_URI, std::vector<uint32_t>(1));
    for (auto* v : {&R.u_scheme, &R.u_host, &R.u_path, &R.u_query, &R.u_frag})
        v->assign(MAX_URI, std::vector<uint64_t>(1));
    R.u_port.assign(MAX_URI, std::vector<int32_t>(1));
    R.q_count.assign(MAX_QUERY, std::vector<uint32_t>(1));
    R.q_params.assign(MAX_QUERY, std::vector<uint64_t>(1));
    R.arena_base.assign(1, 0);
    R.sm_ms.assign(MAX_SECMS, std::vector<int64_t>(1));
    R.l_count.assign(MAX_LIST, std::vector<uint32_t>(1));
    R.l_tab.assign(MAX_LIST, std::vector<uint64_t>(1));
    R.bip.assign(MAX_BINIP, std::vector<uint32_t>(1));
    R.p_count.assign(MAX_PAIR, std::vector<uint32_t>(1));
    R.p_tab.assign(MAX_PAIR, std::vector<uint64_t>(1));
    Columns C;
    memset(&C, 0, sizeof C);
    C.status = R.status.data();
    C.line_off = R.line_off.data();
    for (int k = 0; k < MAX_TOK; ++k) C.tok_span[k] = R.tok_span[k].data();
    C.tok_flags = R.tok_flags.data();
    for (int t = 0; t < MAX_TIME; ++t) { C.t_epoch[t] = R.t_epoch[t].data(); C.t_local[t] = R.t_local[t].data(); C.t_utc[t] = R.t_utc[t].data(); C.t_nano[t] = R.t_nano[t].data(); }
    for (int f = 0; f < MAX_FL; ++f) { C.fl_kind[f] = R.fl_kind[f].data(); C.fl_method[f] = R.fl_method[f].data(); C.fl_uri[f] = R.fl_uri[f].data(); C.fl_proto[f] = R.fl_proto[f].data(); }
    for (int u = 0; u < MAX_URI; ++u) {
        C.u_flags[u] = R.u_flags[u].data(); C.u_scheme[u] = R.u_scheme[u].data(); C.u_host[u] = R.u_host[u].data();
        C.u_port[u] = R.u_port[u].data(); C.u_path[u] = R.u_path[u].data(); C.u_query[u] = R.u_query[u].data();
        C.u_frag[u] = R.u_frag[u].data();
    }
    for (int q = 0; q < MAX_QUERY; ++q) { C.q_count[q] = R.q_count[q].data(); C.q_params[q] = R.q_params[q].data(); }
    for (int k = 0; k < MAX_SECMS; ++k) C.sm_ms[k] = R.sm_ms[k].data();
    for (int j = 0; j < MAX_LIST; ++j) { C.l_count[j] = R.l_count[j].data(); C.l_tab[j] = R.l_tab[j].data(); }
    for (int k = 0; k < MAX_BINIP; ++k) C.bip[k] = R.bip[k].data();
    for (int j = 0; j < MAX_PAIR; ++j) { C.p_count[j] = R.p_count[j].data(); C.p_tab[j] = R.p_tab[j].data(); }
    C.arena_base = R.arena_base.data();
    LineOut o;
    uint32_t stk[MAX_STACK];
    int st = 0;
    if (g_masks) {
        // as the kernel's LDS window: a 64-byte aligned copy of the bytes
        // around the line plus the byte-class masks of that copy
        const uint32_t lo = base_off & ~63u, hi = (base_off + (uint32_t)len + 4) & ~3u;
        const uint32_t wn = ((hi - lo) + 63) & ~63u;
        std::vector<uint64_t> wbuf(wn / 8 + 8, ~0ull);
        memcpy(wbuf.data(), base + lo, hi - lo);
        std::vector<uint64_t> masks(MC_N * (wn / 64));
        build_masks((const uint8_t*)wbuf.data(), wn, masks.data());
        MLine L{(const uint8_t*)wbuf.data(), base_off - lo, len, masks.data()};
        st = run_line(P, L, base, base_off, o, stk, C, R, out, cap, e->fmt_state);
    } else {
        Line L{base, base_off, len};
        st = run_line(P, L, base, base_off, o, stk, C, R, out, cap, e->fmt_state);
    }
    if (st) return st;
    if (o.status != ST_OK) return o.status;
    ResultView V;
    V.n = 1;
    V.line_off = R.line_off.data();
    V.status = R.status.data();
    V.input = R.input.data();
    V.arena = R.arena.empty() ? nullptr : R.arena.data();
    V.arena_base = R.arena_base.data();
    for (int k = 0; k < MAX_TOK; ++k) V.tok_span[k] = R.tok_span[k].data();
    V.tok_flags = R.tok_flags.data();
    for (int t = 0; t < MAX_TIME; ++t) { V.t_epoch[t] = R.t_epoch[t].data(); V.t_local[t] = R.t_local[t].data(); V.t_utc[t] = R.t_utc[t].data(); V.t_nano[t] = R.t_nano[t].data(); }
    for (int f = 0; f < MAX_FL; ++f) { V.fl_kind[f] = R.fl_kind[f].data(); V.fl_method[f] = R.fl_method[f].data(); V.fl_uri[f] = R.fl_uri[f].data(); V.fl_proto[f] = R.fl_proto[f].data(); }
    for (int u = 0; u < MAX_URI; ++u) {
        V.u_flags[u] = R.u_flags[u].data(); V.u_scheme[u] = R.u_scheme[u].data(); V.u_host[u] = R.u_host[u].data();
        V.u_port[u] = R.u_port[u].data(); V.u_path[u] = R.u_path[u].data(); V.u_query[u] = R.u_query[u].data();
        V.u_frag[u] = R.u_frag[u].data();
    }
    for (int q = 0; q < MAX_QUERY; ++q) { V.q_count[q] = R.q_count[q].data(); V.q_params[q] = R.q_params[q].data(); }
    for (int k = 0; k < MAX_SECMS; ++k) V.sm_ms[k] = R.sm_ms[k].data();
    for (int j = 0; j < MAX_LIST; ++j) { V.l_count[j] = R.l_count[j].data(); V.l_tab[j] = R.l_tab[j].data(); }
    for (int k = 0; k < MAX_BINIP; ++k) V.bip[k] = R.bip[k].data();
    for (int j = 0; j < MAX_PAIR; ++j) { V.p_count[j] = R.p_count[j].data(); V.p_tab[j] = R.p_tab[j].data(); }
    V.fmt_id = R.fmt_id.empty() ? nullptr : R.fmt_id.data();
    std::string js = e->plan.record_json(V, 0);
    if ((int)js.size() + 1 > cap) return -1;
    memcpy(out, js.c_str(), js.size() + 1);
    return 0;
}

static int g_masks_fwd(int on) { return g_masks = on; }

// How the lines of a one-format program reach their match result in the
// parse kernel's phase 1 (k_parse_chunks): out[0] lines, [1] the first DFS
// leaf matches, [2] ruled out by the quote-count / line-tail prefilters,
// [3] the backtracking DFS decides.  (Diagnostics for the kernel design:
// which lines a lean first-leaf kernel would hand to the queued-line kernel.)
int emu_leaf_stats(void* h, const char* data, int64_t n, int64_t* out) {
    Emu* e = (Emu*)h;
    if (!e->plan.device_ok()) return 2;
    const Program& P = e->plan.program();
    if (P.n_fmt != 1) return 3;
    const bool la = lit_aware(P);
    for (int k = 0; k < 4; ++k) out[k] = 0;
    const uint8_t* base = (const uint8_t*)data;
    for (int64_t s = 0; s < n;) {
        int64_t t = s;
        while (t < n && data[t] != '\n') ++t;
        const uint32_t off = (uint32_t)s, len = (uint32_t)(t - s);
        const uint32_t lo = off & ~63u, hi = (off + len + 4) & ~3u;
        const uint32_t wn = ((hi - lo) + 63) & ~63u;
        std::vector<uint64_t> wbuf(wn / 8 + 8, ~0ull);
        memcpy(wbuf.data(), base + lo, std::min<uint64_t>(hi - lo, (uint64_t)n - lo));
        std::vector<uint64_t> masks(MC_N * (wn / 64));
        build_masks((const uint8_t*)wbuf.data(), wn, masks.data());
        MLine L{(const uint8_t*)wbuf.data(), off - lo, (int)len, masks.data()};
        RegArr<MAX_TOK> caps;
        caps.fill(0);
        ++out[0];
        const bool leaf = la ? match_first_leaf<true>(P, L, caps) : match_first_leaf<false>(P, L, caps);
        if (leaf) ++out[1];
        else if (!fmt_tail_ok(P, P.elems, P.n_elems, L) || count_quotes(L) < P.fmt_quotes[0]) ++out[2];
        else ++out[3];
        s = t + 1;
    }
    return 0;
}

int emu_possible_paths(const char* fmt, int depth, char* out, int cap) {
    std::vector<std::string> paths;
    std::string err;
    Plan::possible_paths(fmt, depth, paths, err);
    std::string s;
    for (auto& p : paths) s += p + "\n";
    if ((int)s.size() + 1 > cap) return -1;
    memcpy(out, s.c_str(), s.size() + 1);
    return (int)s.size();
}
}
