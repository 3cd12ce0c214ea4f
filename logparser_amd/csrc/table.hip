// gfx950 kernels of the device table: lp_result_table on a device view
// (include/logparser_amd.h), the ParsedRecord / Hive SerDe output side
// (httpdlog-inputformat/.../ParsedRecord.java:154-214: set(name, value), a
// null ignored, the last value wins; httpdlog-serde/.../ApacheHttpdlogDeserializer.java:
// 224-240, 295-323: STRING / BIGINT / DOUBLE columns, one row per line) built
// from the parse kernels' SoA columns without leaving HBM:
//
//   k_table_values  one lane per row: each column's value from the source the
//                   planner named (lp_table.h), the validity byte, LONG /
//                   DOUBLE values, and each STRING value's length and where
//                   its bytes are (TableArgs::srcw)
//   (scan)          the lengths -> Arrow offsets (hipCUB inclusive sum)
//   k_table_chars   one wave per 64 rows of a STRING column: the column's
//                   bytes of those rows, written 4-byte word by word
//
// What each source delivers mirrors Plan::replay (plan.cpp) case by case.
#include <hip/hip_runtime.h>

#define LP_KERNEL_TU 1  // device column pointers are global-memory pointers (lp_program.h)

#include <hipcub/hipcub.hpp>

#include "kernels.h"
#include "lp_device.h"

namespace lp {

namespace {

constexpr int TB = 256;

// one value: 0 none (null / not delivered), 1 bytes at p (amp: a '&' first),
// 2 a long, 3 bytes in buf
struct TVal {
    int kind = 0;
    const LP_G uint8_t* p = nullptr;
    uint32_t n = 0;
    bool amp = false;
    int64_t l = 0;
    char buf[20];  // formatted values (dates, times, month names, binary IPs)
};

__constant__ char MONTH_TEXT[] = "JanuaryFebruaryMarchAprilMayJuneJulyAugustSeptemberOctoberNovemberDecember";
__constant__ uint8_t MONTH_OFF[13] = {0, 7, 15, 20, 25, 28, 32, 36, 42, 51, 58, 66, 74};

__device__ __forceinline__ void put2(char* b, int64_t v) {
    b[0] = (char)('0' + v / 10);
    b[1] = (char)('0' + v % 10);
}

__device__ __forceinline__ uint32_t digits(int64_t l) {
    uint64_t u = l < 0 ? 0 - (uint64_t)l : (uint64_t)l;
    uint32_t n = 1;
    while (u >= 10) { u /= 10; ++n; }
    return n + (l < 0 ? 1u : 0u);
}

__device__ __forceinline__ void write_long(LP_G uint8_t* d, int64_t l, uint32_t n) {  // n = digits(l)
    uint64_t u = l < 0 ? 0 - (uint64_t)l : (uint64_t)l;
    uint32_t k = n;
    do {
        d[--k] = (uint8_t)('0' + u % 10);
        u /= 10;
    } while (u);
    if (l < 0) d[0] = '-';
}

// Long.parseLong (the host table's java_parse_long)
__device__ bool parse_long(const LP_G uint8_t* p, uint32_t n, bool amp, int64_t& out) {
    if (amp || n == 0) return false;
    uint32_t k = 0;
    bool neg = false;
    if (p[0] == '-' || p[0] == '+') { neg = p[0] == '-'; k = 1; }
    if (k == n) return false;
    uint64_t v = 0;
    for (; k < n; ++k) {
        const uint32_t d = p[k] - '0';
        if (d > 9) return false;
        if (v > (0x8000000000000000ull - d) / 10) return false;  // past 2^63
        v = v * 10 + d;
    }
    if (!neg && v == 0x8000000000000000ull) return false;
    out = neg ? (int64_t)(0 - v) : (int64_t)v;
    return true;
}

// Double.parseDouble of "I.F" (digits '.' digits, each at most 18 digits:
// a SECOND_MILLIS upstream list item, UpstreamModule's element kind):
// correctly rounded, as Java's parse (IEEE round half to even).  S = I *
// 10^f + F and the value is S / 10^f: exact by one IEEE division when S <
// 2^53 and f <= 22 (both operands exact); else the quotient's 54-55
// leading bits by binary long division in 128-bit integers (S < 2^120),
// rounded with the remainder as the sticky bit.
__device__ double decimal_to_double(const LP_G uint8_t* p, uint32_t n) {
    typedef unsigned __int128 u128;
    uint64_t I = 0, F = 0;
    uint32_t q = 0;
    int f = 0;
    for (; q < n && p[q] != '.'; ++q) I = I * 10u + (p[q] - '0');
    for (++q; q < n; ++q, ++f) F = F * 10u + (p[q] - '0');
    u128 D = 1;
    for (int k = 0; k < f; ++k) D *= 10u;
    const u128 S = (u128)I * D + F;
    if (S == 0) return 0.0;
    if (S < ((u128)1 << 53) && f <= 22) return (double)(uint64_t)S / (double)(uint64_t)D;
    auto bitlen = [](u128 x) {
        const uint64_t hi = (uint64_t)(x >> 64), lo = (uint64_t)x;
        return hi ? 128 - __builtin_clzll(hi) : lo ? 64 - __builtin_clzll(lo) : 0;
    };
    const int k = 54 - (bitlen(S) - bitlen(D));  // S * 2^k / D in [2^53, 2^55)
    u128 N = S, Dn = D;
    if (k >= 0) N <<= k;
    else Dn <<= -k;
    uint64_t quo = 0;
    for (int b = 55; b >= 0; --b) {
        const u128 t = Dn << b;
        if (N >= t) {
            N -= t;
            quo |= 1ull << b;
        }
    }
    const int shift = quo >= (1ull << 54) ? 2 : 1;  // keep 53 significant bits
    const uint64_t half = 1ull << (shift - 1), r = quo & ((1ull << shift) - 1);
    uint64_t m = quo >> shift;
    if (r > half || (r == half && (N != 0 || (m & 1u)))) ++m;
    return ldexp((double)m, shift - k);
}

// ResponseSetCookieDissector.dissect (dissectors/ResponseSetCookieDissector.java:86-135) on one
// cookie string [cp, cp + cn) -- the cookie's LAST cookie string (every
// dissection of a name reads the Parsable's cached last value,
// core/Parsable.java:172-183): split(";"), each part trimmed and split("=", 2),
// key and value trimmed; part 0's value is "value", a later part keyed
// "expires" / "domain" / "comment" / "path" delivers that output (the last such
// part wins, ParsedRecord).  Out of line: the table kernels' other columns
// keep their registers.  kind / p / n / l as TVal.
__device__ __noinline__ void setcookie_attr(const LP_G uint8_t* cp, uint32_t cn, int fld, int& kind,
                                            const LP_G uint8_t*& p, uint32_t& n, int64_t& l) {
    auto pk = [](const char* k) {
        uint64_t x = 0;
        for (int q = 0; k[q]; ++q) x |= (uint64_t)(uint8_t)k[q] << (8 * q);
        return x;
    };
    const uint64_t want = fld == SC_DOMAIN ? pk("domain") : fld == SC_COMMENT ? pk("comment") : fld == SC_PATH ? pk("path")
                                                                                                    : pk("expires");
    const uint32_t klen = fld == SC_DOMAIN ? 6u : fld == SC_COMMENT ? 7u : fld == SC_PATH ? 4u : 7u;
    for (uint32_t ps = 0, part = 0; ps <= cn; ++part) {
        uint32_t pe = ps;
        while (pe < cn && cp[pe] != ';') ++pe;
        uint32_t a = ps, b = pe;
        while (a < b && cp[a] <= ' ') ++a;
        while (b > a && cp[b - 1] <= ' ') --b;
        uint32_t x = a;
        while (x < b && cp[x] != '=') ++x;
        uint32_t ka = a, kb = x, va = x < b ? x + 1 : b, vb = b;
        while (kb > ka && cp[kb - 1] <= ' ') --kb;
        while (va < vb && cp[va] <= ' ') ++va;
        if (part == 0) {
            if (fld == SC_VALUE) { kind = 1; p = cp + va; n = vb - va; }
        } else if (fld != SC_VALUE && kb - ka == klen) {
            uint64_t k = 0;
            for (uint32_t q = 0; q < klen; ++q) k |= (uint64_t)cp[ka + q] << (8 * q);
            if (k == want) {
                if (fld == SC_EXPIRES_S || fld == SC_EXPIRES_MS) {
                    // parseExpire: "EEE, dd-MMM-yyyy HH:mm:ss GMT" (the only layout the
                    // phase-1 guard lets through) -> epoch seconds * 1000; STRING:expires
                    // is that / 1000 (ResponseSetCookieDissector.java:104-107, 137-150)
                    const LP_G uint8_t* d = cp + va;
                    int mon = 1;
                    for (int q = 0; q < 12; ++q)
                        if (d[8] == (uint8_t)MONTH_TEXT[MONTH_OFF[q]] && d[9] == (uint8_t)MONTH_TEXT[MONTH_OFF[q] + 1] &&
                            d[10] == (uint8_t)MONTH_TEXT[MONTH_OFF[q] + 2])
                            mon = q + 1;
                    auto d2 = [&](int q) { return (int)(d[q] - '0') * 10 + (int)(d[q + 1] - '0'); };
                    const int64_t days = days_from_civil(d2(12) * 100 + d2(14), mon, d2(5));
                    const int64_t ms = (days * 86400 + d2(17) * 3600 + d2(20) * 60 + d2(23)) * 1000;
                    kind = 2;
                    l = fld == SC_EXPIRES_S ? ms / 1000 : ms;
                } else {
                    kind = 1;
                    p = cp + va;
                    n = vb - va;
                }
            }
        }
        ps = pe + 1;
    }
}

__device__ TVal tvalue(const Program& P, const Columns& C, const TableArgs& T, const TableSrc& s, int64_t i,
                       const LP_G uint8_t* line, const LP_G uint8_t* region) {
    TVal v;
    auto bytes = [&](const LP_G uint8_t* p, uint32_t n) {
        v.kind = 1;
        v.p = p;
        v.n = n;
    };
    auto span = [&](uint32_t sp) { bytes(line + (sp & 0xFFFFu), (sp >> 16) - (sp & 0xFFFFu)); };
    auto ref = [&](uint64_t r) {
        bytes((ref_arena(r) ? region : line) + ref_off(r), ref_len(r));
        v.amp = ref_amp(r);
    };
    auto along = [&](int64_t l) {
        v.kind = 2;
        v.l = l;
    };
    switch (s.kind) {
    case TC_TOKEN: case TC_CLF2NUM: case TC_NUM2CLF: {
        const bool null = (C.tok_flags[i] >> s.a) & 1u;
        if (null) {
            if (s.kind == TC_CLF2NUM) along(0);  // ConvertCLFIntoNumber: null -> 0L
            return v;
        }
        span(C.tok_span[s.a][i]);
        if (s.kind == TC_NUM2CLF && v.n == 1 && v.p[0] == '0') v.kind = 0;  // "0" -> null
        return v;
    }
    case TC_TIME: {
        const TimeStage& TS = P.time[s.a];
        const uint32_t sp = C.tok_span[TS.tok][i];
        if (((C.tok_flags[i] >> TS.tok) & 1u) || (sp >> 16) <= (sp & 0xFFFFu)) return v;  // null / empty: no dissection
        if (s.b == TF_EPOCH) { along(C.t_epoch[s.a][i]); return v; }
        const uint64_t w = s.c ? C.t_utc[s.a][i] : C.t_local[s.a][i];
        const int64_t Y = w & 0xFFFF, MO = (w >> 16) & 15, D = (w >> 20) & 31, H = (w >> 25) & 31, MI = (w >> 30) & 63,
                      S = (w >> 36) & 63, WY = (w >> 42) & 0xFFFF, WK = (w >> 58) & 63;
        const int64_t nanos = TS.kind == TK_STRF ? (int64_t)C.t_nano[s.a][i] : 0;
        switch (s.b) {
        case TF_DAY: along(D); break;
        case TF_MONTH: along(MO); break;
        case TF_WEEK: along(WK); break;
        case TF_WEEKYEAR: along(WY); break;
        case TF_YEAR: along(Y); break;
        case TF_HOUR: along(H); break;
        case TF_MINUTE: along(MI); break;
        case TF_SECOND: along(S); break;
        case TF_MILLI: along(nanos / 1000000); break;
        case TF_MICRO: along(nanos / 1000); break;
        case TF_NANO: along(nanos); break;
        case TF_MONTHNAME:
            v.kind = 3;
            v.n = MONTH_OFF[MO] - MONTH_OFF[MO - 1];
            for (uint32_t k = 0; k < v.n; ++k) v.buf[k] = MONTH_TEXT[MONTH_OFF[MO - 1] + k];
            break;
        case TF_DATE:  // "%04d-%02d-%02d"
            v.kind = 3;
            v.n = 10;
            put2(v.buf, Y / 100);
            put2(v.buf + 2, Y % 100);
            v.buf[4] = '-';
            put2(v.buf + 5, MO);
            v.buf[7] = '-';
            put2(v.buf + 8, D);
            break;
        case TF_TIME:  // "%02d:%02d:%02d"
            v.kind = 3;
            v.n = 8;
            put2(v.buf, H);
            v.buf[2] = ':';
            put2(v.buf + 3, MI);
            v.buf[5] = ':';
            put2(v.buf + 6, S);
            break;
        default: break;
        }
        return v;
    }
    case TC_FL: {
        const uint32_t kind = C.fl_kind[s.a][i];
        if (kind == FL_NONE) return v;
        if (s.b == 0) span(C.fl_method[s.a][i]);
        else if (s.b == 1) span(C.fl_uri[s.a][i]);
        else if (kind == FL_FULL) span(C.fl_proto[s.a][i]);  // a chopped line's protocol is null
        return v;
    }
    case TC_PROTO: {  // HttpFirstLineProtocolDissector: "HTTP/x.y".split("/", 2)
        if (C.fl_kind[s.a][i] != FL_FULL) return v;
        span(C.fl_proto[s.a][i]);
        if (v.n == 0 || (v.n == 1 && v.p[0] == '-')) { v.kind = 0; return v; }
        uint32_t sl = 0;
        while (sl < v.n && v.p[sl] != '/') ++sl;
        if (sl == v.n) { v.kind = 0; return v; }  // no '/': both null
        if (s.b == 0) v.n = sl;
        else { v.p += sl + 1; v.n -= sl + 1; }
        return v;
    }
    case TC_URI: {
        const uint32_t f = C.u_flags[s.a][i];
        if (!(f & UF_DONE)) return v;
        switch (s.b) {
        case UP_QUERY: ref(C.u_query[s.a][i]); break;
        case UP_PATH: ref(C.u_path[s.a][i]); break;
        case UP_REF: if (f & UF_FRAG) ref(C.u_frag[s.a][i]); break;
        case UP_PROTOCOL: if ((f & UF_IS_URL) && (f & UF_SCHEME)) ref(C.u_scheme[s.a][i]); break;
        case UP_HOST: if ((f & UF_IS_URL) && (f & UF_HOST)) ref(C.u_host[s.a][i]); break;
        case UP_PORT: if ((f & UF_IS_URL) && (f & UF_PORT)) along(C.u_port[s.a][i]); break;
        default: break;
        }
        return v;
    }
    case TC_SECMS:  // ConvertSecondsWithMillisStringDissector (+ ConvertMillisecondsIntoMicroseconds)
        if (!((C.tok_flags[i] >> P.secms[s.a].tok) & 1u)) along(s.b ? (int64_t)((uint64_t)C.sm_ms[s.a][i] * 1000u) : C.sm_ms[s.a][i]);
        return v;
    case TC_BINIP: {  // BinaryIPDissector: "%d.%d.%d.%d" of the signed bytes
        const uint32_t sp = C.tok_span[P.binip[s.a].tok][i];
        if ((sp >> 16) - (sp & 0xFFFFu) != 16u) return v;
        const uint32_t x = C.bip[s.a][i];
        v.kind = 3;
        v.n = 0;
        for (int k = 0; k < 4; ++k) {
            int b = (int)(int8_t)((x >> (8 * k)) & 0xFF);
            if (k) v.buf[v.n++] = '.';
            if (b < 0) { v.buf[v.n++] = '-'; b = -b; }
            if (b >= 100) v.buf[v.n++] = (char)('0' + b / 100);
            if (b >= 10) v.buf[v.n++] = (char)('0' + (b / 10) % 10);
            v.buf[v.n++] = (char)('0' + b % 10);
        }
        return v;
    }
    case TC_LIST: case TC_LIST_MS: {  // UpstreamListDissector item b (its table in the line's region)
        if ((uint32_t)s.b >= C.l_count[s.a][i]) return v;
        const uint32_t ent = P.list[s.a].secms ? LIST_ENT_MS : LIST_ENT;
        const LP_G uint8_t* e = region + ref_off(C.l_tab[s.a][i]) + (uint32_t)s.b * ent;
        if (s.kind == TC_LIST) {
            span(reinterpret_cast<const LP_G uint32_t*>(e)[s.c & 1]);
        } else {
            const int64_t ms = reinterpret_cast<const LP_G int64_t*>(e + 8)[s.c & 1];
            along((s.c & 2) ? (int64_t)((uint64_t)ms * 1000u) : ms);
        }
        return v;
    }
    case TC_PAIR: {  // the cookie / parameter's last occurrence in the pair stage's piece table
        const uint32_t cnt = C.p_count[s.a][i];
        const LP_G uint64_t* t = reinterpret_cast<const LP_G uint64_t*>(region + ref_off(C.p_tab[s.a][i]));
        for (uint32_t k = 0; k < cnt; ++k) {
            const uint64_t nref = t[2 * k];
            if (ref_len(nref) != (uint32_t)s.c) continue;
            const LP_G uint8_t* np = (ref_arena(nref) ? region : line) + ref_off(nref);
            bool same = true;
            for (int q = 0; q < s.c && same; ++q) same = np[q] == T.names[s.b + q];
            if (same) ref(t[2 * k + 1]);
        }
        return v;
    }
    case TC_SETC: {
        const int j = s.a & 0xFF;
        const uint32_t cnt = C.p_count[j][i];
        const LP_G uint64_t* t = reinterpret_cast<const LP_G uint64_t*>(region + ref_off(C.p_tab[j][i]));
        uint64_t cref = 0;
        bool found = false;
        for (uint32_t k = 0; k < cnt; ++k) {
            const uint64_t nref = t[2 * k];
            if (ref_len(nref) != (uint32_t)s.c) continue;
            const LP_G uint8_t* np = (ref_arena(nref) ? region : line) + ref_off(nref);
            bool same = true;
            for (int q = 0; q < s.c && same; ++q) same = np[q] == T.names[s.b + q];
            if (same) { cref = t[2 * k + 1]; found = true; }
        }
        if (found) setcookie_attr((ref_arena(cref) ? region : line) + ref_off(cref), ref_len(cref), s.a >> 8, v.kind, v.p, v.n, v.l);
        return v;
    }
    case TC_QP: {  // the parameter's last occurrence (ParsedRecord: the last value wins)
        const uint32_t cnt = C.q_count[s.a][i];
        if (cnt == 0) return v;
        const LP_G uint64_t* t = reinterpret_cast<const LP_G uint64_t*>(region + ref_off(C.q_params[s.a][i]));
        for (uint32_t k = 0; k < cnt; ++k) {
            const uint64_t nref = t[2 * k];
            if (nref == REF_SKIP || ref_len(nref) != (uint32_t)s.c) continue;
            const LP_G uint8_t* np = (ref_arena(nref) ? region : line) + ref_off(nref);
            bool same = true;
            for (int q = 0; q < s.c && same; ++q) same = np[q] == T.names[s.b + q];
            if (same) ref(t[2 * k + 1]);
        }
        return v;
    }
    default:  // TC_NONE, TC_NULL
        return v;
    }
}

// the row's line and arena region (a program without URI stages writes no
// region: nothing refers to one)
__device__ __forceinline__ bool row_view(const Program& P, const Columns& C, const uint8_t* buf, int64_t i,
                                         const LP_G uint8_t*& line, const LP_G uint8_t*& region) {
    if (C.status[i] != ST_OK) return false;
    line = (const LP_G uint8_t*)buf + C.line_off[i];
    region = P.has_phase2() ? C.arena + C.arena_base[i] : C.arena;
    return true;
}

__global__ __launch_bounds__(TB) void k_table_values(const DeviceArgs* __restrict__ args,
                                                     const TableArgs* __restrict__ targs, const uint8_t* buf) {
    const Program& P = args->prog;
    const Columns& C = args->cols;
    const TableArgs& T = *targs;
    const int64_t k = (int64_t)blockIdx.x * TB + threadIdx.x;
    if (k >= T.count) return;
    const int64_t i = T.first + k;
    const LP_G uint8_t *line = nullptr, *region = nullptr;
    const bool ok = row_view(P, C, buf, i, line, region);
    const int fmt = ok && P.n_fmt > 1 ? (int)C.fmt_id[i] : 0;
    for (int c = 0, rank = 0; c < T.n_cols; ++c) {
        const TableCol& col = T.cols[c];
        bool valid = false;
        int64_t x = 0;
        double d = 0.0;
        uint64_t w = 0;
        // the later delivery, then (a value that is none for the column) the earlier
        for (int pass = 0; pass < 2 && ok && !valid; ++pass) {
            const TableSrc& sc = pass ? col.alt[fmt] : col.src[fmt];
            if (pass && sc.kind == TC_NONE) break;
            const TVal v = tvalue(P, C, T, sc, i, line, region);
            valid = v.kind != 0;
            if (col.kind == 1) {  // STRING: its length now, its bytes after the scan
                x = v.kind == 2 ? digits(v.l) : v.n + (v.amp ? 1u : 0u);
                // where k_table_chars finds them (lp_table.h SW_*)
                const uint64_t pa = (uint64_t)(uintptr_t)v.p;
                if (v.kind == 1 && pa < SW_AMP) w = pa | (v.amp ? SW_AMP : 0ull);
                else if (v.kind == 2 && v.l >= -(int64_t)SW_AMP && v.l < (int64_t)SW_AMP)
                    w = SW_LONG | ((uint64_t)v.l & (SW_LONG - 1));
                else w = SW_SLOW;
            } else if (col.kind == 2) {
                x = v.l;
                if (v.kind == 1) valid = parse_long(v.p, v.n, v.amp, x);
                else if (v.kind == 3) valid = false;  // month names, dates: not numbers
            } else {
                // the planner admits long-valued sources and SECOND_MILLIS list items here
                if (v.kind == 1 && sc.kind == TC_LIST) d = decimal_to_double(v.p, v.n);
                else if (v.kind == 2) d = (double)v.l;
                else valid = false;
            }
        }
        if (col.kind == 1) {
            col.i64[k + 1] = valid ? x : 0;
            if (k == 0) col.i64[0] = 0;
            T.srcw[(int64_t)rank++ * T.count + k] = valid ? w : 0;
        } else if (col.kind == 2) {
            if (valid) col.i64[k] = x;
        } else if (valid) {
            col.f64[k] = d;
        }
        col.valid[k] = valid ? 1 : 0;
    }
}

// The STRING columns' bytes, destination-major: one wave per 64 rows of one
// STRING column (grid y = the column's rank among the STRING columns).  The
// wave's rows fill one contiguous byte range of the column ([off[k0],
// off[k0 + 64]), Arrow offsets), so the wave walks that range 256 bytes per
// step, lane l on its 4-byte word: each byte's row by a binary search over
// the rows' offsets in LDS, its source byte from the input / arena (a value's
// bytes), the wave's LDS scratch (formatted longs, dates, binary IPs) or the
// '&' of a raw query string, and one aligned 4-byte store per full word
// (byte stores only at the range's two ends, whose words the neighbouring
// waves share).  Consecutive lanes read consecutive source bytes of a row and
// write consecutive words: the traffic is coalesced both ways.
constexpr int CW = 4;    // waves per block
constexpr int FMTB = 24; // scratch bytes per row (a long's 20 characters at most)

__global__ __launch_bounds__(64 * CW) void k_table_chars(const DeviceArgs* __restrict__ args,
                                                         const TableArgs* __restrict__ targs, const uint8_t* buf) {
    const Program& P = args->prog;
    const Columns& C = args->cols;
    const TableArgs& T = *targs;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    __shared__ uint32_t s_off[CW][65];
    __shared__ uint32_t s_flag[CW][64];
    __shared__ uint64_t s_src[CW][64];
    __shared__ uint8_t s_fmt[CW][64 * FMTB];
    // the column: the blockIdx.y-th STRING column
    int c = -1;
    for (int j = 0, r = 0; j < T.n_cols; ++j)
        if (T.cols[j].kind == 1 && r++ == (int)blockIdx.y) c = j;
    const int64_t k0 = ((int64_t)blockIdx.x * CW + wv) * 64;
    if (c < 0 || k0 >= T.count) return;  // wave-uniform; only wave-level LDS sharing below
    const TableCol& col = T.cols[c];
    const int64_t kend = k0 + 64 < T.count ? k0 + 64 : T.count;
    const int nrows = (int)(kend - k0);
    const int64_t k = k0 + lane;
    const uint64_t D0 = (uint64_t)col.i64[k0], D1 = (uint64_t)col.i64[kend];
    uint32_t flag = 0;  // bit 0: bytes in the scratch; bit 1: a leading '&'
    uint64_t src = 0;
    // the row's value as k_table_values found it (one coalesced word: no
    // status -> line -> span chain here); a long is formatted into the wave's
    // scratch, a SW_SLOW value derived again
    const uint64_t w = k < kend ? T.srcw[(int64_t)blockIdx.y * T.count + k] : 0;
    if (k < kend && col.valid[k]) {
        uint8_t* f = &s_fmt[wv][lane * FMTB];
        TVal v;
        if ((w >> 62) == 0) {
            v.kind = 1;
            v.p = reinterpret_cast<const LP_G uint8_t*>((uintptr_t)(w & (SW_AMP - 1)));
            v.amp = (w & SW_AMP) != 0;
        } else if ((w >> 62) == 1) {
            v.kind = 2;
            v.l = (int64_t)(w << 2) >> 2;
        } else {
            const LP_G uint8_t *line = nullptr, *region = nullptr;
            if (row_view(P, C, buf, T.first + k, line, region)) {
                const int fmt = P.n_fmt > 1 ? (int)C.fmt_id[T.first + k] : 0;
                v = tvalue(P, C, T, col.src[fmt], T.first + k, line, region);
                if (v.kind == 0) v = tvalue(P, C, T, col.alt[fmt], T.first + k, line, region);  // the earlier delivery
            }
        }
        if (v.kind == 2) {
            uint64_t u = v.l < 0 ? 0 - (uint64_t)v.l : (uint64_t)v.l;
            const uint32_t n = digits(v.l);
            uint32_t q = n;
            do {
                f[--q] = (uint8_t)('0' + u % 10);
                u /= 10;
            } while (u);
            if (v.l < 0) f[0] = '-';
            flag = 1;
        } else if (v.kind == 3) {
            for (uint32_t q = 0; q < v.n; ++q) f[q] = (uint8_t)v.buf[q];
            flag = 1;
        } else {
            src = (uint64_t)(uintptr_t)v.p;
            flag = v.amp ? 2u : 0u;
        }
    }
    if (lane < nrows) {
        s_off[wv][lane] = (uint32_t)((uint64_t)col.i64[k] - D0);
        s_flag[wv][lane] = flag;
        s_src[wv][lane] = src;
    }
    if (lane == 0) s_off[wv][nrows] = (uint32_t)(D1 - D0);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (D1 == D0) return;
    const uint32_t total = (uint32_t)(D1 - D0);
    const uint32_t* off = s_off[wv];
    // 4-byte words of the destination: offsets congruent to -mis mod 4
    const uint32_t mis = (uint32_t)((uintptr_t)col.chars & 3u);
    const uint64_t A0 = D0 - ((D0 + mis) & 3u);
    LP_G uint8_t* const out = col.chars;
    // U words per lane per step: every source byte load of the step is in
    // flight before the first store
    constexpr int U = 4;
    for (uint64_t a0 = A0; a0 < D1; a0 += 256 * U) {
        uint32_t word[U], have[U];
        uint8_t bv[U][4];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t d = a0 + 256ull * u + 4ull * (uint64_t)lane;
            have[u] = 0;
            if (!(d < D1 && d + 4 > D0)) continue;
            const uint32_t t0 = d < D0 ? (uint32_t)(D0 - d) : 0u;
            const uint32_t x0 = (uint32_t)(d + t0 - D0);  // the first byte in range, relative
            int r = 0;
            for (int st = 32; st; st >>= 1)
                if (r + st < nrows && off[r + st] <= x0) r += st;
            uint32_t nxt = off[r + 1], beg = off[r], fl = s_flag[wv][r];
            uint64_t sp = s_src[wv][r];
#pragma unroll
            for (uint32_t t = 0; t < 4; ++t) {
                const uint32_t x = x0 + t - t0;
                if (t < t0 || x >= total) continue;
                while (x >= nxt) {  // the next non-empty row
                    ++r;
                    beg = nxt;
                    nxt = off[r + 1];
                    fl = s_flag[wv][r];
                    sp = s_src[wv][r];
                }
                const uint32_t o = x - beg;
                if (fl & 1u) bv[u][t] = s_fmt[wv][r * FMTB + o];
                else if ((fl & 2u) && o == 0) bv[u][t] = '&';
                else bv[u][t] = reinterpret_cast<const LP_G uint8_t*>((uintptr_t)sp)[o - (fl >> 1)];
                have[u] |= 1u << t;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t d = a0 + 256ull * u + 4ull * (uint64_t)lane;
            word[u] = 0;
#pragma unroll
            for (uint32_t t = 0; t < 4; ++t)
                if ((have[u] >> t) & 1u) word[u] |= (uint32_t)bv[u][t] << (8 * t);
            if (have[u] == 15u) {
                *reinterpret_cast<LP_G uint32_t*>(out + d) = word[u];
            } else if (have[u]) {
                for (uint32_t t = 0; t < 4; ++t)
                    if ((have[u] >> t) & 1u) out[d + t] = (uint8_t)(word[u] >> (8 * t));
            }
        }
    }
}

}  // namespace

// scratch: the scan's temporary storage, its sums, the STRING value words
size_t table_srcw_offset(int64_t count) {
    size_t tmp = 0;
    hipcub::DeviceScan::InclusiveSum(nullptr, tmp, (const int64_t*)nullptr, (int64_t*)nullptr, (int)count);
    return ((tmp + 255) & ~(size_t)255) + ((8 * (size_t)count + 255) & ~(size_t)255);
}

size_t table_scratch_bytes(int64_t count, int n_str) {
    return table_srcw_offset(count) + 8 * (size_t)count * (size_t)n_str + 256;
}

int launch_table_values(const DeviceArgs* d_args, const TableArgs* d_targs, const TableArgs& ta, const uint8_t* buf,
                        void* scratch, size_t scratch_bytes, hipStream_t s, hipEvent_t mid) {
    if (ta.count > 0x7FFFFFFF) return -1;  // the scan's item count is an int
    const int64_t n = ta.count;
    if (n == 0) {
        for (int c = 0; c < ta.n_cols; ++c)
            if (ta.cols[c].kind == 1 && hipMemsetAsync(ta.cols[c].i64, 0, 8, s) != hipSuccess) return -1;
        return 0;
    }
    hipLaunchKernelGGL(k_table_values, dim3((unsigned)((n + TB - 1) / TB)), dim3(TB), 0, s, d_args, d_targs, buf);
    if (mid) hipEventRecord(mid, s);  // the values kernel done: the scans follow
    size_t tmp = 0;
    hipcub::DeviceScan::InclusiveSum(nullptr, tmp, (const int64_t*)nullptr, (int64_t*)nullptr, (int)n);
    const size_t tmp_al = (tmp + 255) & ~(size_t)255;
    if (tmp_al + 8 * (size_t)n > scratch_bytes) return -1;
    int64_t* sums = reinterpret_cast<int64_t*>((char*)scratch + tmp_al);
    for (int c = 0; c < ta.n_cols; ++c) {
        if (ta.cols[c].kind != 1) continue;
        int64_t* off = (int64_t*)ta.cols[c].i64;
        size_t t = tmp;
        if (hipcub::DeviceScan::InclusiveSum(scratch, t, off + 1, sums, (int)n, s) != hipSuccess) return -1;
        if (hipMemcpyAsync(off + 1, sums, 8 * (size_t)n, hipMemcpyDeviceToDevice, s) != hipSuccess) return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_table_chars(const DeviceArgs* d_args, const TableArgs* d_targs, const TableArgs& ta, const uint8_t* buf,
                       hipStream_t s) {
    int n_str = 0;
    for (int c = 0; c < ta.n_cols; ++c) n_str += ta.cols[c].kind == 1 ? 1 : 0;
    if (ta.count == 0 || n_str == 0) return 0;
    const int64_t waves = (ta.count + 63) / 64;
    hipLaunchKernelGGL(k_table_chars, dim3((unsigned)((waves + CW - 1) / CW), (unsigned)n_str), dim3(64 * CW), 0, s,
                       d_args, d_targs, buf);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace lp
