// Per-line hot path of the logparser reference, written once for the GPU
// (gfx950 kernel in kernels.hip; every function is __host__ __device__ so the
// test-only CPU emulation in tests/ can run the identical source).
//
// One thread owns one line.  Phase 1 matches the LogFormat and runs the
// token / timestamp / first-line stages; phase 2 (after a wave-aggregated
// arena allocation) runs the URI and query-string stages that produce bytes
// that are not substrings of the line.
//
// Any input the device cannot prove it handles exactly returns FALLBACK
// (status 2): the caller hands that line to the reference Java dissector.
#pragma once
#include "lp_program.h"

namespace lp {

enum : int { ST_OK = 0, ST_BAD = 1, ST_FALLBACK = 2 };

// ----------------------------------------------------------- byte classes
__host__ __device__ inline bool is_ws(uint32_t c) { return c == ' ' || (c >= 9 && c <= 13); }      // \s
__host__ __device__ inline bool is_digit(uint32_t c) { return c - '0' < 10u; }
__host__ __device__ inline bool is_hex(uint32_t c) { return is_digit(c) || ((c | 32u) - 'a') < 6u; }
__host__ __device__ inline bool is_alpha(uint32_t c) { return ((c | 32u) - 'a') < 26u; }
__host__ __device__ inline bool is_alnum(uint32_t c) { return is_alpha(c) || is_digit(c); }
__host__ __device__ inline uint32_t hexv(uint32_t c) { return c <= '9' ? c - '0' : (c | 32u) - 'a' + 10; }
// chars commons-httpclient URIUtil.encode escapes with the HttpUriDissector
// "badUriChars" set (HttpUriDissector.java:111-120): control, space, unwise
// {}|\^[]` and <>"  (ASCII only; non-ASCII lines never reach this point)
__host__ __device__ inline bool uri_needs_encode(uint32_t c) {
    if (c <= 0x20 || c == 0x7F) return true;
    switch (c) {
    case '{': case '}': case '|': case '\\': case '^': case '[': case ']': case '`': case '<': case '>': case '"':
        return true;
    }
    return false;
}

// -------------------------------------------------------------- matcher
struct Line {
    const uint8_t* s;
    int n;
    __host__ __device__ uint32_t operator[](int i) const { return s[i]; }
};

__host__ __device__ inline bool lit_at(const Program& P, const Line& L, int pos, int off, int len) {
    if (pos + len > L.n) return false;
    for (int k = 0; k < len; ++k)
        if (L[pos + k] != P.lit[off + k]) return false;
    return true;
}

// Java Pattern.Dot: everything except line terminators.  The fast-path guard
// already rejected \n \r and non-ASCII, so '.' runs to end of line.
__host__ __device__ inline int dot_end(const Line& L, int p) { return L.n; }

__host__ __device__ inline bool time_us_ok(const Line& L, int p) {
    if (p + 26 > L.n) return false;
    const uint8_t* c = L.s + p;
    if (!(c[0] >= '0' && c[0] <= '3') || !is_digit(c[1]) || c[2] != '/') return false;
    if (!is_alpha(c[3]) || !is_alpha(c[4]) || !is_alpha(c[5]) || c[6] != '/') return false;
    if (!(c[7] >= '1' && c[7] <= '9') || !is_digit(c[8]) || !is_digit(c[9]) || !is_digit(c[10]) || c[11] != ':') return false;
    if (!is_digit(c[12]) || !is_digit(c[13]) || c[14] != ':' || !is_digit(c[15]) || !is_digit(c[16]) || c[17] != ':') return false;
    if (!is_digit(c[18]) || !is_digit(c[19]) || c[20] != ' ') return false;
    if (!(c[21] == '+' || c[21] == '|' || c[21] == '-')) return false;   // [\+|\-]
    return is_digit(c[22]) && is_digit(c[23]) && is_digit(c[24]) && is_digit(c[25]);
}

// The highest-priority IPv4 alternative of FORMAT_IPV4
// (TokenParser.java:43-46) when every octet is taken whole: returns end or -1.
__host__ __device__ inline int ipv4_first(const Line& L, int p) {
    int q = p;
    for (int o = 0; o < 4; ++o) {
        int a = q;
        while (q < L.n && q - a < 4 && is_digit(L[q])) ++q;
        int nd = q - a;
        if (nd < 1 || nd > 3) return -1;
        if (nd == 3) {
            uint32_t d1 = L[a], v = (L[a] - '0') * 100 + (L[a + 1] - '0') * 10 + (L[a + 2] - '0');
            // 25[0-5] | 2[0-4][0-9] | [01][0-9][0-9] take three digits
            if (!(d1 == '0' || d1 == '1' || (v >= 200 && v <= 255))) return -1;
        }
        if (q < L.n && is_digit(L[q])) return -1;
        if (o < 3) {
            if (q >= L.n || L[q] != '.') return -1;
            ++q;
        }
    }
    return q;
}

// First candidate end of element e at position p (exact leftmost-first
// order), -1 = none, -2 = FALLBACK.
__host__ __device__ inline int cand_first(const Program& P, const Elem& e, const Line& L, int p) {
    switch (e.kind) {
    case EK_NOSPACE: { int q = p; while (q < L.n && !is_ws(L[q])) ++q; return q; }
    case EK_NUMBER: { int q = p; while (q < L.n && is_digit(L[q])) ++q; return q > p ? q : -1; }
    case EK_CLFNUMBER: {
        int q = p; while (q < L.n && is_digit(L[q])) ++q;
        if (q > p) return q;
        return (p < L.n && L[p] == '-') ? p + 1 : -1;
    }
    case EK_HEXNUMBER: { int q = p; while (q < L.n && is_hex(L[q])) ++q; return q > p ? q : -1; }
    case EK_CLFHEXNUMBER: {
        int q = p; while (q < L.n && is_hex(L[q])) ++q;
        if (q > p) return q;
        return (p < L.n && L[p] == '-') ? p + 1 : -1;
    }
    case EK_NONZERO: {
        if (p >= L.n || !(L[p] >= '1' && L[p] <= '9')) return -1;
        int q = p + 1; while (q < L.n && is_digit(L[q])) ++q; return q;
    }
    case EK_ANY_GREEDY: {
        int m = dot_end(L, p);
        if (e.last) return m == L.n ? m : -1;
        if (!e.nlit) return m;
        for (int q = m; q >= p; --q) if (lit_at(P, L, q, e.lit_off, e.lit_len)) return q;
        return -1;
    }
    case EK_ANY_LAZY: {
        int m = dot_end(L, p);
        if (e.last) return m == L.n ? m : -1;
        if (!e.nlit) return p;
        for (int q = p; q <= m; ++q) if (lit_at(P, L, q, e.lit_off, e.lit_len)) return q;
        return -1;
    }
    case EK_TIME_US: return time_us_ok(L, p) ? p + 26 : -1;
    case EK_CLF_IP:
    case EK_IP: {
        int q = ipv4_first(L, p);
        if (q >= 0) return q;
        // IPv6 alternative can only match empty at '-' (no hex/':'), so '-'
        // is exact when the following literal cannot start at p.
        if (e.kind == EK_CLF_IP && p < L.n && L[p] == '-' && e.nlit && P.lit[e.lit_off] != '-') return p + 1;
        return -2;
    }
    }
    return -2;
}

// Next candidate after 'cur' (same priority order).
__host__ __device__ inline int cand_next(const Program& P, const Elem& e, const Line& L, int p, int cur) {
    switch (e.kind) {
    case EK_NOSPACE: return cur - 1 >= p ? cur - 1 : -1;
    case EK_NUMBER: case EK_HEXNUMBER: case EK_NONZERO: return cur - 1 >= p + 1 ? cur - 1 : -1;
    case EK_CLFNUMBER: case EK_CLFHEXNUMBER:
        if (L[p] == '-') return -1;
        return cur - 1 >= p + 1 ? cur - 1 : -1;
    case EK_ANY_GREEDY:
        if (e.last) return -1;
        if (!e.nlit) return cur - 1 >= p ? cur - 1 : -1;
        for (int q = cur - 1; q >= p; --q) if (lit_at(P, L, q, e.lit_off, e.lit_len)) return q;
        return -1;
    case EK_ANY_LAZY: {
        if (e.last) return -1;
        int m = dot_end(L, p);
        if (!e.nlit) return cur + 1 <= m ? cur + 1 : -1;
        for (int q = cur + 1; q <= m; ++q) if (lit_at(P, L, q, e.lit_off, e.lit_len)) return q;
        return -1;
    }
    case EK_TIME_US: return -1;
    case EK_CLF_IP: case EK_IP:
        return (L[p] == '-') ? -1 : -2;  // shorter IPv4 / IPv6 alternatives: not proven here
    }
    return -2;
}

// Backtracking match of "^" elems "$" with java.util.regex priority
// semantics.  caps[k] = span of captured token k.  stk: MAX_STACK scratch.
template <typename Stk>
__host__ __device__ inline int match_line(const Program& P, const Line& L, uint32_t* caps, Stk stk) {
    int i = 0, pos = 0, sp = 0;
    int steps = 0;
    const int budget = 16 * L.n + 256;
    for (;;) {
        if (++steps > budget) return ST_FALLBACK;
        bool ok;
        if (i == P.n_elems) {
            if (pos == L.n) return ST_OK;
            ok = false;
        } else {
            const Elem& e = P.elems[i];
            if (e.kind == EK_LIT) {
                ok = lit_at(P, L, pos, e.lit_off, e.lit_len);
                if (ok) { pos += e.lit_len; ++i; continue; }
            } else {
                int c = cand_first(P, e, L, pos);
                if (c == -2) return ST_FALLBACK;
                ok = c >= 0;
                if (ok) {
                    if (e.cap >= 0) caps[e.cap] = mkspan(pos, c);
                    if (!e.det) {
                        if (sp == MAX_STACK) return ST_FALLBACK;
                        stk[sp++] = (uint32_t)i | ((uint32_t)pos << 6) | ((uint32_t)c << 19);
                    }
                    pos = c;
                    ++i;
                    continue;
                }
            }
        }
        // backtrack to the most recent choice point with another candidate
        for (;;) {
            if (sp == 0) return ST_BAD;
            uint32_t top = stk[sp - 1];
            int j = top & 63, p = (top >> 6) & 8191, cur = (top >> 19) & 8191;
            const Elem& e = P.elems[j];
            int c = cand_next(P, e, L, p, cur);
            if (c == -2) return ST_FALLBACK;
            if (c >= 0) {
                stk[sp - 1] = (uint32_t)j | ((uint32_t)p << 6) | ((uint32_t)c << 19);
                if (e.cap >= 0) caps[e.cap] = mkspan(p, c);
                pos = c;
                i = j + 1;
                break;
            }
            --sp;
        }
    }
}

// ------------------------------------------------------------- calendar
__host__ __device__ inline int64_t days_from_civil(int64_t y, int m, int d) {
    y -= m <= 2;
    const int64_t era = (y >= 0 ? y : y - 399) / 400;
    const int64_t yoe = y - era * 400;
    const int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
    const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    return era * 146097 + doe - 719468;
}
__host__ __device__ inline void civil_from_days(int64_t z, int64_t& y, int& m, int& d) {
    z += 719468;
    const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
    const int64_t doe = z - era * 146097;
    const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
    const int64_t mp = (5 * doy + 2) / 153;
    d = (int)(doy - (153 * mp + 2) / 5 + 1);
    m = (int)(mp < 10 ? mp + 3 : mp - 9);
    y = yoe + era * 400 + (m <= 2);
}
__host__ __device__ inline bool leap(int64_t y) { return (y % 4 == 0 && y % 100 != 0) || y % 400 == 0; }
__host__ __device__ inline int month_len(int64_t y, int m) {
    if (m == 2) return leap(y) ? 29 : 28;
    return (m == 4 || m == 6 || m == 9 || m == 11) ? 30 : 31;
}
__host__ __device__ inline int iso_dow(int64_t days) { return (int)(((days % 7) + 7 + 3) % 7) + 1; }  // Mon=1
// WeekFields.ISO (== WeekFields.of(Locale.UK)): week-based-year and week
__host__ __device__ inline void iso_week(int64_t y, int m, int d, int64_t& wy, int& wk) {
    int64_t days = days_from_civil(y, m, d);
    int wd = iso_dow(days);
    int doy = (int)(days - days_from_civil(y, 1, 1)) + 1;
    int w = (doy - wd + 10) / 7;
    if (w < 1) {
        int64_t py = y - 1;
        int jwd = iso_dow(days_from_civil(py, 1, 1));
        wy = py;
        wk = (jwd == 4 || (jwd == 3 && leap(py))) ? 53 : 52;
        return;
    }
    int jwd = iso_dow(days_from_civil(y, 1, 1));
    int weeks = (jwd == 4 || (jwd == 3 && leap(y))) ? 53 : 52;
    if (w > weeks) { wy = y + 1; wk = 1; return; }
    wy = y;
    wk = w;
}

// DateTimeFormatter "dd/MMM/yyyy:HH:mm:ss ZZ", parseCaseInsensitive,
// Locale.UK, ResolverStyle.SMART (TimeStampDissector.java:46,100-109,418):
// day 1..31 clamped to the month length, 24:00:00 = next day 00:00:00,
// offset sign+HHMM (each <= 59) with |offset| <= 18:00.
__host__ __device__ inline bool parse_apache_time(const uint8_t* c, int64_t& epoch_s, uint64_t& local, uint64_t& utc) {
    int day = (c[0] - '0') * 10 + (c[1] - '0');
    // month name: case-insensitive against the 12 UK short names
    uint32_t m3 = ((uint32_t)(c[3] | 32) << 16) | ((uint32_t)(c[4] | 32) << 8) | (uint32_t)(c[5] | 32);
    int month = 0;
    const uint32_t names[12] = {0x6a616e, 0x666562, 0x6d6172, 0x617072, 0x6d6179, 0x6a756e,
                                0x6a756c, 0x617567, 0x736570, 0x6f6374, 0x6e6f76, 0x646563};
    for (int k = 0; k < 12; ++k) if (names[k] == m3) month = k + 1;
    if (!month) return false;
    int64_t year = (c[7] - '0') * 1000 + (c[8] - '0') * 100 + (c[9] - '0') * 10 + (c[10] - '0');
    int hh = (c[12] - '0') * 10 + (c[13] - '0');
    int mi = (c[15] - '0') * 10 + (c[16] - '0');
    int ss = (c[18] - '0') * 10 + (c[19] - '0');
    int off;
    if (c[21] == '+' && c[22] == '0' && c[23] == '0' && c[24] == '0' && c[25] == '0') off = 0;
    else {
        if (c[21] == '|') return false;
        int oh = (c[22] - '0') * 10 + (c[23] - '0'), om = (c[24] - '0') * 10 + (c[25] - '0');
        if (oh > 59 || om > 59) return false;
        off = (c[21] == '-' ? -1 : 1) * (oh * 3600 + om * 60);
    }
    if (off > 64800 || off < -64800) return false;
    if (day < 1 || day > 31) return false;
    int ml = month_len(year, month);
    if (day > ml) day = ml;
    if (mi > 59) return false;
    int d = day, m = month;
    int64_t y = year;
    if (hh == 24 && mi == 0 && ss == 0) {
        hh = 0;
        civil_from_days(days_from_civil(y, m, d) + 1, y, m, d);
    } else if (hh > 23 || ss > 59) {
        return false;
    }
    int64_t days = days_from_civil(y, m, d);
    epoch_s = days * 86400 + hh * 3600 + mi * 60 + ss - off;
    int64_t wy; int wk;
    iso_week(y, m, d, wy, wk);
    local = pack_cal((uint32_t)y, m, d, hh, mi, ss, (uint32_t)wy, wk);
    int64_t ud = epoch_s >= 0 ? epoch_s / 86400 : -((-epoch_s + 86399) / 86400);
    int64_t rem = epoch_s - ud * 86400;
    int64_t uy; int um, udd;
    civil_from_days(ud, uy, um, udd);
    iso_week(uy, um, udd, wy, wk);
    utc = pack_cal((uint32_t)uy, um, udd, (uint32_t)(rem / 3600), (uint32_t)(rem % 3600 / 60), (uint32_t)(rem % 60),
                   (uint32_t)wy, wk);
    return true;
}

// ----------------------------------------------------------- per-line state
struct LineOut {
    int status;
    uint32_t caps[MAX_TOK];
    uint32_t tok_flags;
    uint32_t fl_kind[MAX_FL], fl_method[MAX_FL], fl_uri[MAX_FL], fl_proto[MAX_FL];
    uint32_t arena_need;
};

__host__ __device__ inline bool prefix_at(const Line& L, int a, int b, const char* lit) {
    int k = 0;
    for (; lit[k]; ++k)
        if (a + k >= b || L[a + k] != (uint8_t)lit[k]) return false;
    return true;
}
__host__ __device__ inline bool value_is_header_name(const Line& L, int a, int b) {
    return (b - a == 17 && prefix_at(L, a, b, "request.firstline")) || prefix_at(L, a, b, "request.header.") ||
           prefix_at(L, a, b, "response.header.");
}

// Source span of URI stage u; returns false when the value is null/absent/empty
__host__ __device__ inline bool uri_source(const Program& P, const LineOut& o, int u, int& a, int& b) {
    const UriStage& U = P.uri[u];
    uint32_t sp;
    if (U.src_tok >= 0) {
        if (o.tok_flags & (1u << U.src_tok)) return false;  // "-" -> null
        sp = o.caps[U.src_tok];
    } else {
        if (o.fl_kind[U.src_fl] == FL_NONE) return false;
        sp = o.fl_uri[U.src_fl];
    }
    a = sp & 0xFFFF;
    b = sp >> 16;
    return b > a;
}

// Phase 1: guard, match, tokens, time, first line; arena need for phase 2.
template <typename Stk, typename Cols>
__host__ __device__ inline void phase1(const Program& P, const Line& L, LineOut& o, Stk stk, Cols& C, int64_t li) {
    o.status = ST_OK;
    o.tok_flags = 0;
    o.arena_need = 0;
    for (int k = 0; k < MAX_FL; ++k) o.fl_kind[k] = FL_NONE;
    if (L.n > MAX_LINE) { o.status = ST_FALLBACK; return; }
    // fast-path guard: printable ASCII + TAB only (no \r, no line
    // terminators, no bytes that need UTF-8 decoding or URIUtil UTF-8 bytes)
    for (int k = 0; k < L.n; ++k) {
        uint32_t c = L[k];
        if ((c < 0x20 && c != '\t') || c >= 0x7F) { o.status = ST_FALLBACK; return; }
    }
    int st = match_line(P, L, o.caps, stk);
    if (st != ST_OK) { o.status = st; return; }
    // decodeExtractedValue: "-" -> null (Apache: ApacheHttpdLogFormatDissector.java:169-196,
    // NGINX: NginxHttpdLogFormatDissector.java:107-119)
    for (int k = 0; k < P.n_tok; ++k) {
        int a = o.caps[k] & 0xFFFF, b = o.caps[k] >> 16;
        if (b - a == 1 && L[a] == '-') o.tok_flags |= 1u << k;
        if (b - a == 1 && L[a] == '0') o.tok_flags |= 1u << (16 + k);
        if (P.apache && b - a >= 15 && value_is_header_name(L, a, b)) {
            // the reference tests the VALUE (not the token name) against
            // "request.firstline" / "request.header." / "response.header." and
            // then unescapes \xhh sequences (ApacheHttpdLogFormatDissector.java:189-193)
            for (int q = a; q < b; ++q) if (L[q] == '\\') { o.status = ST_FALLBACK; return; }
        }
    }
    // TimeStampDissector
    for (int t = 0; t < P.n_time; ++t) {
        int k = P.time[t].tok;
        int a = o.caps[k] & 0xFFFF;
        int64_t ep; uint64_t lo, ut;
        if (!parse_apache_time(L.s + a, ep, lo, ut)) { o.status = ST_BAD; return; }
        C.t_epoch[t][li] = ep * 1000;
        C.t_local[t][li] = lo;
        C.t_utc[t][li] = ut;
    }
    // HttpFirstLineDissector: ^([a-zA-Z-_]+) (.*) (HTTP/[0-9]+\.[0-9]+)$ else ^([a-zA-Z-_]+) (.*)$
    for (int f = 0; f < P.n_fl; ++f) {
        int k = P.fl[f].tok;
        o.fl_kind[f] = FL_NONE;
        if (o.tok_flags & (1u << k)) continue;                // null
        int a = o.caps[k] & 0xFFFF, b = o.caps[k] >> 16;
        if (b <= a) continue;                                 // empty
        int q = a;
        while (q < b && (is_alpha(L[q]) || L[q] == '-' || L[q] == '_')) ++q;
        if (q == a || q >= b || L[q] != ' ') continue;        // neither regex matches
        o.fl_method[f] = mkspan(a, q);
        int us = q + 1;
        // protocol: the last ' ' must be followed by HTTP/d+.d+ up to the end
        int sp = b - 1;
        while (sp >= us && L[sp] != ' ') --sp;
        bool full = false;
        if (sp >= us && b - sp >= 9 && L[sp + 1] == 'H' && L[sp + 2] == 'T' && L[sp + 3] == 'T' && L[sp + 4] == 'P' &&
            L[sp + 5] == '/') {
            int r = sp + 6, d1 = r;
            while (r < b && is_digit(L[r])) ++r;
            if (r > d1 && r < b && L[r] == '.') {
                int d2 = ++r;
                while (r < b && is_digit(L[r])) ++r;
                full = r == b && r > d2;
            }
        }
        if (full) {
            o.fl_kind[f] = FL_FULL;
            o.fl_uri[f] = mkspan(us, sp);
            o.fl_proto[f] = mkspan(sp + 1, b);
        } else {
            o.fl_kind[f] = FL_CHOPPED;
            o.fl_uri[f] = mkspan(us, b);
            o.fl_proto[f] = 0;
        }
    }
    // arena need of the URI / query stages (upper bound of phase-2 writes)
    uint32_t need = 0;
    for (int u = 0; u < P.n_uri; ++u) {
        int a, b;
        if (!uri_source(P, o, u, a, b)) continue;
        uint32_t enc = 0, sep = 0;
        for (int q = a; q < b; ++q) {
            uint32_t c = L[q];
            enc += uri_needs_encode(c);
            sep += (c == '&' || c == '?');
        }
        const UriStage& U = P.uri[u];
        uint32_t ulen = (uint32_t)(b - a), tl = ulen + 2 * enc + 2;
        uint32_t n = 16;
        if (U.want_query) n += tl;
        if (U.want_path) n += ulen;
        if (U.want_ref) n += tl;
        if (U.query_stage >= 0) n += 8 + 16 * (sep + 1) + 2 * tl;
        need += n;
    }
    o.arena_need = (need + 15) & ~15u;
}

// ------------------------------------------------------------ URI stage
struct Arena {
    uint8_t* p;     // this line's region
    uint32_t used;
    uint32_t cap;
    __host__ __device__ uint32_t put(uint32_t c) { p[used] = (uint8_t)c; return used++; }
};

// java.net.URI.Parser.parseIPv4Address/scanIPv4Address on [a,b) of the
// authority (JDK 8); returns end or -1.
__host__ __device__ inline int jdk_ipv4(const Line& L, int a, int b) {
    int m = a;
    while (m < b && (is_digit(L[m]) || L[m] == '.')) ++m;
    if (m <= a) return -1;
    int p = a;
    for (int o = 0; o < 4; ++o) {
        int q = p;
        while (q < m && is_digit(L[q])) ++q;
        if (q <= p) return -1;
        if (q - p > 9) return -1;  // Integer.parseInt would overflow -> NumberFormatException -> -1
        uint32_t v = 0;
        for (int r = p; r < q; ++r) v = v * 10 + (L[r] - '0');
        if (v > 255) return -1;
        p = q;
        if (o < 3) {
            if (p >= m || L[p] != '.') return -1;
            ++p;
        }
    }
    if (p < m) return -1;
    if (p < b && L[p] != ':') return -1;
    return p;
}

// java.net.URI.Parser.parseHostname on [a,b); returns end or -1 (fail)
__host__ __device__ inline int jdk_hostname(const Line& L, int a, int b) {
    int p = a, l = -1;
    do {
        int q = p;
        while (q < b && is_alnum(L[q])) ++q;
        if (q <= p) break;
        l = p;
        p = q;
        q = p;
        while (q < b && (is_alnum(L[q]) || L[q] == '-')) ++q;
        if (q > p) {
            if (L[q - 1] == '-') return -1;
            p = q;
        }
        if (!(p < b && L[p] == '.')) break;
        ++p;
    } while (p < b);
    if (p < b && L[p] != ':') return -1;
    if (l < 0) return -1;
    if (l > a && !is_alpha(L[l])) return -1;
    return p;
}

// strict UTF-8 validation of a decoded byte string
__host__ __device__ inline bool utf8_ok(const uint8_t* b, uint32_t n) {
    for (uint32_t i = 0; i < n;) {
        uint32_t c = b[i];
        if (c < 0x80) { ++i; continue; }
        int need;
        uint32_t cp;
        if (c >= 0xC2 && c <= 0xDF) { need = 1; cp = c & 0x1F; }
        else if (c >= 0xE0 && c <= 0xEF) { need = 2; cp = c & 0x0F; }
        else if (c >= 0xF0 && c <= 0xF4) { need = 3; cp = c & 0x07; }
        else return false;
        if (i + (uint32_t)need >= n) return false;
        for (int r = 1; r <= need; ++r) {
            if ((b[i + r] & 0xC0) != 0x80) return false;
            cp = (cp << 6) | (b[i + r] & 0x3F);
        }
        if (need == 2 && (cp < 0x800 || (cp >= 0xD800 && cp <= 0xDFFF))) return false;
        if (need == 3 && (cp < 0x10000 || cp > 0x10FFFF)) return false;
        i += need + 1;
    }
    return true;
}

// java.net.URI.decode of [a,b) of the line (escapes proven valid):
// returns a ref (line span when nothing to decode), or ~0 on FALLBACK.
__host__ __device__ inline uint64_t decode_span(const Line& L, int a, int b, Arena& A) {
    bool pct = false;
    for (int q = a; q < b; ++q) pct |= L[q] == '%';
    if (!pct) return mkref(a, b - a, false);
    uint32_t start = A.used;
    for (int q = a; q < b;) {
        uint32_t c = L[q];
        if (c == '%') { A.put(hexv(L[q + 1]) * 16 + hexv(L[q + 2])); q += 3; }
        else { A.put(c); ++q; }
    }
    if (!utf8_ok(A.p + start, A.used - start)) return ~0ull;
    return mkref(start, A.used - start, true);
}

__host__ __device__ inline void put_encoded(Arena& A, uint32_t c) {
    const char* HX = "0123456789ABCDEF";
    A.put('%');
    A.put(HX[c >> 4]);
    A.put(HX[c & 15]);
}

// QueryStringFieldDissector on the rawQuery (arena bytes [qa, qb)).
template <typename Cols>
__host__ __device__ inline void query_stage(const Program& P, int qs, Arena& A, uint32_t qa, uint32_t qb, Cols& C, int64_t li) {
    const QueryStage& Q = P.query[qs];
    // count pieces for the table
    uint32_t npieces = 1;
    for (uint32_t q = qa; q < qb; ++q) npieces += A.p[q] == '&';
    uint32_t tab = (A.used + 7) & ~7u;
    A.used = tab + 16 * npieces;
    uint32_t count = 0;
    uint32_t s = qa;
    while (s <= qb) {
        uint32_t e = s;
        while (e < qb && A.p[e] != '&') ++e;
        if (e > s) {
            uint32_t eq = s;
            while (eq < e && A.p[eq] != '=') ++eq;
            uint32_t ne = eq;  // name [s, ne)
            bool upper = false;
            for (uint32_t q = s; q < ne; ++q) upper |= (A.p[q] - 'A') < 26u;
            // requested?  (wantAllFields || requestedParameters.contains(name))
            bool want = Q.want_all;
            for (int k = 0; k < Q.n_names && !want; ++k) {
                if (Q.name_len[k] != ne - s) continue;
                bool same = true;
                for (uint32_t q = 0; q < ne - s; ++q) {
                    uint32_t c = A.p[s + q];
                    if ((c - 'A') < 26u) c |= 32;
                    if (c != P.lit[Q.name_off[k] + q]) { same = false; break; }
                }
                want = same;
            }
            if (want) {
                uint64_t nref;
                if (upper) {
                    uint32_t st = A.used;
                    for (uint32_t q = s; q < ne; ++q) { uint32_t c = A.p[q]; A.put((c - 'A') < 26u ? (c | 32) : c); }
                    nref = mkref(st, ne - s, true);
                } else nref = mkref(s, ne - s, true);
                uint64_t vref;
                if (eq == e) vref = mkref(0, 0, true);  // no '=' -> ""
                else {
                    uint32_t vs = eq + 1;
                    bool plain = true;
                    for (uint32_t q = vs; q < e; ++q) plain &= (A.p[q] != '%' && A.p[q] != '+');
                    if (plain) vref = mkref(vs, e - vs, true);
                    else {
                        // Utils.resilientUrlDecode: every '%' here is followed by two
                        // hex digits (URI stage guard), so each %XX is the Latin-1
                        // char U+00XX (VALID_STANDARD -> %00%XX, UTF-16 decode) and
                        // '+' is a space.  Output UTF-8.
                        uint32_t st = A.used;
                        for (uint32_t q = vs; q < e;) {
                            uint32_t c = A.p[q];
                            if (c == '+') { A.put(' '); ++q; }
                            else if (c == '%') {
                                uint32_t v = hexv(A.p[q + 1]) * 16 + hexv(A.p[q + 2]);
                                if (v < 0x80) A.put(v);
                                else { A.put(0xC0 | (v >> 6)); A.put(0x80 | (v & 0x3F)); }
                                q += 3;
                            } else { A.put(c); ++q; }
                        }
                        vref = mkref(st, A.used - st, true);
                    }
                }
                uint64_t* t = (uint64_t*)(A.p + tab);
                t[2 * count] = nref;
                t[2 * count + 1] = vref;
                ++count;
            }
        }
        s = e + 1;
    }
    C.q_count[qs][li] = count;
    C.q_params[qs][li] = mkref(tab, 16 * count, true);
}

// HttpUriDissector fast path on the line bytes [a,b).  Returns status.
template <typename Cols>
__host__ __device__ inline int uri_stage(const Program& P, int u, const Line& L, int a, int b, Arena& A, Cols& C, int64_t li) {
    const UriStage& U = P.uri[u];
    // ---- guards (FALLBACK when a cleanup step of the reference would change the string)
    int fa = -1, h = -1, nh = 0;
    for (int q = a; q < b; ++q) {
        uint32_t c = L[q];
        if (c == '%') {
            if (q + 2 >= b || !is_hex(L[q + 1]) || !is_hex(L[q + 2])) return ST_FALLBACK;  // BAD_EXCAPE_PATTERN
        } else if (c == '#') {
            ++nh;
            if (h < 0) h = q;
            if (q + 1 < b && (L[q + 1] == '&' || L[q + 1] == '?')) return ST_FALLBACK;     // HASH_AMP
            if (q + 1 < b && L[q + 1] == 'x') return ST_FALLBACK;                          // ALMOST_HTML_ENCODED
            if (q > a && L[q - 1] == '=') return ST_FALLBACK;                              // EQUALS_HASH
        } else if (c == '&' || c == '?') {
            if (fa < 0) fa = q;
            int r = q + 1;                                                                // unescapeHtml4 candidates
            while (r < b && (is_alnum(L[r]) || L[r] == '#')) ++r;
            if (r < b && L[r] == ';') return ST_FALLBACK;
        }
    }
    if (nh > 1) return ST_FALLBACK;                                                       // DOUBLE_HASH
    int pend = b;                              // end of path: first '?'(=fa) or '#'
    if (fa >= 0 && fa < pend) pend = fa;
    if (h >= 0 && h < pend) pend = h;
    uint32_t flags = UF_DONE | UF_PATH;
    int ps;                                    // path start
    int64_t scheme_ref = 0, host_ref = 0;
    int32_t port = -1;
    if (L[a] == '/') {
        ps = a;                                // "dummy-protocol://dummy.host.name" + uri
    } else {
        flags |= UF_IS_URL;
        // scheme: ':' before any of "/?#" (in the normalized string '?' is at fa)
        int p = a;
        while (p < b && L[p] != ':' && L[p] != '/' && L[p] != '#' && p != fa) ++p;
        if (p < b && L[p] == ':') {
            if (p == a || !is_alpha(L[a])) return ST_BAD;                                  // URISyntaxException
            for (int q = a + 1; q < p; ++q) {
                uint32_t c = L[q];
                if (!(is_alnum(c) || c == '+' || c == '-' || c == '.')) return ST_BAD;
            }
            flags |= UF_SCHEME;
            scheme_ref = (int64_t)mkref(a, p - a, false);
            ++p;
            if (!(p < b && L[p] == '/')) return ST_FALLBACK;                              // opaque URI
            if (p + 1 < b && L[p + 1] == '/') {
                int as = p + 2, ae = as;
                while (ae < b && L[ae] != '/' && L[ae] != '#' && ae != fa) ++ae;
                if (ae == as) return ST_FALLBACK;                                          // empty authority
                // chars in both L_SERVER and L_REG_NAME of java.net.URI (no '@'
                // userinfo, no escapes): server parse, else registry (host null)
                for (int q = as; q < ae; ++q) {
                    uint32_t c = L[q];
                    bool ok = is_alnum(c);
                    switch (c) {
                    case '.': case '-': case ':': case '_': case '!': case '~': case '*': case '\'':
                    case '(': case ')': case ';': case '=': case '+': case '$': case ',':
                        ok = true;
                    }
                    if (!ok) return ST_FALLBACK;
                }
                // parseServer; any failure -> registry-based authority (host null)
                int he = jdk_ipv4(L, as, ae);
                if (he <= as) he = jdk_hostname(L, as, ae);
                bool ok = he > as;
                int pt = -1;
                if (ok && he < ae) {
                    // ":" port digits up to the end of the authority
                    int q = he + 1;
                    if (q < ae) {
                        uint64_t v = 0;
                        for (int r = q; r < ae; ++r) {
                            if (!is_digit(L[r])) { ok = false; break; }
                            v = v * 10 + (L[r] - '0');
                            if (v > 0x7FFFFFFFull) { ok = false; break; }
                        }
                        if (ok) pt = (int)v;
                    }
                }
                if (ok) {
                    flags |= UF_HOST;
                    host_ref = (int64_t)mkref(as, he - as, false);
                    if (pt >= 0) { flags |= UF_PORT; port = pt; }
                }
                ps = ae;
            } else {
                ps = p;                                                                    // "scheme:/path"
            }
        } else {
            ps = a;                                                                        // relative, no scheme
        }
    }
    if (pend < ps) pend = ps;
    // ---- outputs
    C.u_scheme[u][li] = (uint64_t)scheme_ref;
    C.u_host[u][li] = (uint64_t)host_ref;
    C.u_port[u][li] = port;
    if (U.want_path) {
        uint64_t r = decode_span(L, ps, pend, A);
        if (r == ~0ull) return ST_FALLBACK;
        C.u_path[u][li] = r;
    }
    if (U.want_query) {
        if (fa >= 0 && (h < 0 || fa < h)) {
            // rawQuery = "&" + normalized text up to '#': '?'->'&', URIUtil escapes
            flags |= UF_QUERY;
            uint32_t st = A.used;
            A.put('&');
            int qe = h >= 0 ? h : b;
            for (int q = fa + 1; q < qe; ++q) {
                uint32_t c = L[q];
                if (c == '?') A.put('&');
                else if (uri_needs_encode(c)) put_encoded(A, c);
                else A.put(c);
            }
            C.u_query[u][li] = mkref(st, A.used - st, true);
            if (U.query_stage >= 0) query_stage(P, U.query_stage, A, st, A.used, C, li);
        } else {
            C.u_query[u][li] = mkref(0, 0, true);
            if (U.query_stage >= 0) { C.q_count[U.query_stage][li] = 0; C.q_params[U.query_stage][li] = 0; }
        }
    }
    if (U.want_ref && h >= 0) {
        flags |= UF_FRAG;
        // fragment = decode(normalized text after '#')
        bool plain = true;
        for (int q = h + 1; q < b; ++q) plain &= !(L[q] == '%' || L[q] == '?' || L[q] == '&');
        if (plain) C.u_frag[u][li] = mkref(h + 1, b - h - 1, false);
        else {
            uint32_t st = A.used;
            for (int q = h + 1; q < b;) {
                uint32_t c = L[q];
                if (q == fa) { A.put('?'); A.put('&'); ++q; }
                else if (c == '?') { A.put('&'); ++q; }
                else if (c == '%') { A.put(hexv(L[q + 1]) * 16 + hexv(L[q + 2])); q += 3; }
                else { A.put(c); ++q; }
            }
            if (!utf8_ok(A.p + st, A.used - st)) return ST_FALLBACK;
            C.u_frag[u][li] = mkref(st, A.used - st, true);
        }
    }
    C.u_flags[u][li] = flags;
    return ST_OK;
}

// Phase 2: URI + query stages into the line's arena region.
template <typename Cols>
__host__ __device__ inline void phase2(const Program& P, const Line& L, LineOut& o, Arena& A, Cols& C, int64_t li) {
    for (int u = 0; u < P.n_uri && o.status == ST_OK; ++u) {
        int a, b;
        if (!uri_source(P, o, u, a, b)) {
            C.u_flags[u][li] = 0;
            if (P.uri[u].query_stage >= 0) { C.q_count[P.uri[u].query_stage][li] = 0; C.q_params[P.uri[u].query_stage][li] = 0; }
            continue;
        }
        int st = uri_stage(P, u, L, a, b, A, C, li);
        if (st != ST_OK) o.status = st;
    }
}

// Final per-line column writes (status, tokens, first line).
template <typename Cols>
__host__ __device__ inline void write_line(const Program& P, const LineOut& o, Cols& C, int64_t li) {
    C.status[li] = (uint8_t)o.status;
    if (o.status != ST_OK) return;
    for (int k = 0; k < P.n_tok; ++k) C.tok_span[k][li] = o.caps[k];
    C.tok_flags[li] = o.tok_flags;
    for (int f = 0; f < P.n_fl; ++f) {
        C.fl_kind[f][li] = o.fl_kind[f];
        C.fl_method[f][li] = o.fl_method[f];
        C.fl_uri[f][li] = o.fl_uri[f];
        C.fl_proto[f][li] = o.fl_proto[f];
    }
}

}  // namespace lp
