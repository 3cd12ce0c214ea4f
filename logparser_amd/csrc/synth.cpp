// Deterministic synthetic access-log generators for BASELINE.json configs
// 2, 3, 4 and 5: every line i is a pure function
// of (seed, i), so any range of lines can be generated independently (and in
// parallel) and re-generated bit-identically for parity checks.
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "../../include/logparser_amd.h"

namespace {

struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed) {}
    uint64_t next() {  // splitmix64
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    uint32_t below(uint32_t n) { return (uint32_t)((next() >> 32) * (uint64_t)n >> 32); }
    bool pct(uint32_t p) { return below(100) < p; }
};

struct Out {
    char* p;
    size_t n, cap;
    bool ok = true;
    void c(char ch) { if (n < cap) p[n++] = ch; else ok = false; }
    void s(const char* x) { while (*x) c(*x++); }
    void u(uint64_t v, int width = 0) {
        char b[24];
        int k = 0;
        do { b[k++] = (char)('0' + v % 10); v /= 10; } while (v);
        while (k < width) b[k++] = '0';
        while (k) c(b[--k]);
    }
};

const char* ALNUM = "abcdefghijklmnopqrstuvwxyz0123456789";
const char* SEGCH = "abcdefghijklmnopqrstuvwxyz0123456789._-";
const char* MONTHS[] = {"Jan", "Feb", "Mar", "Apr", "May", "Jun", "Jul", "Aug", "Sep", "Oct", "Nov", "Dec"};
const char* OFFSETS[] = {"+0000", "+0100", "+0200", "-0500", "-0700", "+0530", "+0930"};
const int STATUS[] = {200, 200, 200, 200, 200, 304, 301, 302, 404, 403, 500, 206};
const char* TLDS[] = {"com", "net", "org", "nl", "de", "io"};
const char* WORDS[] = {"www", "shop", "blog", "news", "api", "static", "images", "example", "basjes", "howto", "mail", "search"};

const char* UA_BROWSER[] = {
    "Mozilla/5.0 (%s) Gecko/20100101 Firefox/%d.0",
    "Mozilla/5.0 (%s) AppleWebKit/537.36 (KHTML, like Gecko) Chrome/%d.0.4472.124 Safari/537.36",
    "Mozilla/5.0 (%s) AppleWebKit/605.1.15 (KHTML, like Gecko) Version/%d.1 Safari/605.1.15",
    "Mozilla/5.0 (%s) AppleWebKit/537.36 (KHTML, like Gecko) Chrome/%d.0.0.0 Safari/537.36 Edg/%d.0.0.0",
    "curl/7.%d.0"};
const char* UA_OS[] = {"Windows NT 10.0; Win64; x64", "Macintosh; Intel Mac OS X 10_15_7", "X11; Linux x86_64",
                       "X11; Ubuntu; Linux x86_64", "iPhone; CPU iPhone OS 14_6 like Mac OS X"};

// the ~50 fixed user agents (5 templates x 5 platforms x 2 versions)
const char* user_agent(uint32_t k) {
    struct Table {
        char t[50][200];
        Table() {
            for (int i = 0; i < 50; ++i) {
                int b = i % 5, os = (i / 5) % 5, v = 60 + 7 * (i / 25) + b;
                if (b == 4) snprintf(t[i], sizeof t[i], UA_BROWSER[b], v);
                else snprintf(t[i], sizeof t[i], UA_BROWSER[b], UA_OS[os], v, v);
            }
        }
    };
    static const Table table;  // thread-safe initialisation
    return table.t[k % 50];
}

void word(Out& o, Rng& r, const char* set, uint32_t setn, uint32_t lo, uint32_t hi) {
    uint32_t n = lo + r.below(hi - lo + 1);
    for (uint32_t i = 0; i < n; ++i) o.c(set[r.below(setn)]);
}

void hostname(Out& o, Rng& r) {
    o.s(WORDS[r.below(12)]);
    o.c('.');
    word(o, r, ALNUM, 26, 3, 9);
    o.c('.');
    o.s(TLDS[r.below(6)]);
}

void query(Out& o, Rng& r) {
    uint32_t np = 1 + r.below(8);
    for (uint32_t p = 0; p < np; ++p) {
        o.c(p == 0 ? '?' : '&');
        word(o, r, ALNUM, 26, 1, 8);
        o.c('=');
        uint32_t vl = 1 + r.below(10);
        bool pctv = r.pct(20), plus = r.pct(5);
        for (uint32_t k = 0; k < vl; ++k) {
            if (pctv && r.pct(25)) {
                static const char* HX = "0123456789ABCDEF";
                uint32_t v = r.pct(50) ? 0x20 + r.below(0x5F) : 0xA0 + r.below(0x60);  // ASCII or Latin-1
                o.c('%');
                o.c(HX[v >> 4]);
                o.c(HX[v & 15]);
            } else if (plus && r.pct(15)) {
                o.c('+');
            } else {
                o.c(ALNUM[r.below(36)]);
            }
        }
    }
}

void path(Out& o, Rng& r) {
    uint32_t ns = 1 + r.below(6);
    for (uint32_t s = 0; s < ns; ++s) {
        o.c('/');
        word(o, r, SEGCH, 39, 1, 12);
    }
}

struct Civil { int d, m; int64_t y; };

// uniform day in 2010-01-01 .. 2025-12-31 (days_from_civil inverse)
Civil civil_day(Rng& r) {
    uint64_t days = r.below(5844);
    int64_t z = 14610 + (int64_t)days + 719468;  // 2010-01-01 = day 14610
    int64_t era = z / 146097, doe = z - era * 146097;
    int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100), mp = (5 * doy + 2) / 153;
    Civil c;
    c.d = (int)(doy - (153 * mp + 2) / 5 + 1);
    c.m = (int)(mp < 10 ? mp + 3 : mp - 9);
    c.y = yoe + era * 400 + (c.m <= 2);
    return c;
}

void ipv4(Out& o, Rng& r) {
    for (int k = 0; k < 4; ++k) {
        if (k) o.c('.');
        o.u(r.below(256));
    }
}

// dd/MMM/yyyy:HH:mm:ss (sep = ':' for %t, ' ' for strftime %d/%b/%Y %T)
void stamp(Out& o, Rng& r, char sep, const char* month_override = nullptr, bool day00 = false) {
    Civil c = civil_day(r);
    o.u(day00 ? 0 : c.d, 2);
    o.c('/');
    o.s(month_override ? month_override : MONTHS[c.m - 1]);
    o.c('/');
    o.u((uint64_t)c.y, 4);
    o.c(sep);
    o.u(r.below(24), 2);
    o.c(':');
    o.u(r.below(60), 2);
    o.c(':');
    o.u(r.below(60), 2);
}

void request(Out& o, Rng& r) {
    uint32_t mth = r.below(100);
    static const char* OTHER[] = {"HEAD", "PUT", "DELETE", "OPTIONS", "HEAD"};
    o.s(mth < 80 ? "GET" : mth < 95 ? "POST" : OTHER[r.below(5)]);
    o.c(' ');
    path(o, r);
    if (r.pct(35)) query(o, r);
    uint32_t pv = r.below(3);
    o.s(pv == 0 ? " HTTP/1.0" : pv == 1 ? " HTTP/1.1" : " HTTP/2.0");
}

void referer(Out& o, Rng& r) {
    if (r.pct(40)) o.c('-');
    else {
        o.s(r.pct(50) ? "https://" : "http://");
        hostname(o, r);
        path(o, r);
        if (r.pct(30)) query(o, r);
    }
}

// %h %l %u: host, logname, user
void who(Out& o, Rng& r) {
    if (r.pct(5)) hostname(o, r); else ipv4(o, r);
    o.c(' ');
    if (r.pct(99)) o.c('-'); else o.u(1 + r.below(65535));
    o.c(' ');
    if (r.pct(90)) o.c('-'); else word(o, r, ALNUM, 26, 3, 10);
}

Rng line_rng(uint64_t seed, int64_t i) {
    Rng r(seed * 0x2545F4914F6CDD1Dull ^ (uint64_t)i * 0x9E3779B97F4A7C15ull);
    r.next();
    return r;
}

// config 2: Apache 'combined'
void combined_line(Out& o, uint64_t seed, int64_t i) {
    Rng r = line_rng(seed, i);
    who(o, r);
    o.s(" [");
    stamp(o, r, ':');
    o.c(' ');
    o.s(OFFSETS[r.below(7)]);
    o.s("] \"");
    request(o, r);
    o.s("\" ");
    o.u(STATUS[r.below(12)]);
    o.c(' ');
    if (r.pct(95)) o.u(r.below(200000)); else o.c('-');
    o.s(" \"");
    referer(o, r);
    o.s("\" \"");
    o.s(user_agent(r.below(50)));
    o.s("\"\n");
}

// config 3: '%h %l %u [%{%d/%b/%Y %T}t.%{msec_frac}t] "%r" %>s %b
// "%{Referer}i" "%{User-Agent}i" %I %O' with 5 % malformed lines, uniform over
// {truncated, missing closing quote, month Foo, day 00, non-numeric %b,
// extra field}
void strftime_line(Out& o, uint64_t seed, int64_t i) {
    Rng r = line_rng(seed, i);
    const size_t start = o.n;
    const int bad = r.pct(5) ? 1 + (int)r.below(6) : 0;
    who(o, r);
    o.s(" [");
    stamp(o, r, ' ', bad == 3 ? "Foo" : nullptr, bad == 4);
    o.c('.');
    o.u(r.below(1000), 3);
    o.s("] \"");
    request(o, r);
    o.s(bad == 2 ? " " : "\" ");
    o.u(STATUS[r.below(12)]);
    o.c(' ');
    if (bad == 5) o.s("12x");
    else if (r.pct(95)) o.u(r.below(200000));
    else o.c('-');
    o.s(" \"");
    referer(o, r);
    o.s("\" \"");
    o.s(user_agent(r.below(50)));
    o.s("\" ");
    o.u(200 + r.below(4000));
    o.c(' ');
    o.u(200 + r.below(200000));
    if (bad == 6) o.s(" extra");
    if (bad == 1 && o.ok) o.n = start + 1 + (o.n - start - 1) * (20 + r.below(70)) / 100;  // truncated
    o.c('\n');
}

// config 4: NGINX log_format of hpt/nginxmodules/NginxUpstreamTest.java:94
// '$remote_addr - $remote_user [$time_local] "$request" $status
// $body_bytes_sent "$http_referer" "$http_user_agent" "$http_x_forwarded_for"
// $request_time $upstream_response_time $pipe'
void nginx_line(Out& o, uint64_t seed, int64_t i) {
    Rng r = line_rng(seed, i);
    ipv4(o, r);
    o.s(" - ");
    if (r.pct(90)) o.c('-'); else word(o, r, ALNUM, 26, 3, 10);
    o.s(" [");
    stamp(o, r, ':');
    o.c(' ');
    o.s(OFFSETS[r.below(7)]);
    o.s("] \"");
    request(o, r);
    o.s("\" ");
    o.u(STATUS[r.below(12)]);
    o.c(' ');
    o.u(r.below(200000));
    o.s(" \"");
    referer(o, r);
    o.s("\" \"");
    o.s(user_agent(r.below(50)));
    o.s("\" \"");
    if (r.pct(70)) o.c('-');
    else {
        ipv4(o, r);
        if (r.pct(30)) { o.s(", "); ipv4(o, r); }
    }
    o.s("\" ");
    auto secs = [&]() { o.u(r.below(r.pct(90) ? 2 : 100)); o.c('.'); o.u(r.below(1000), 3); };
    secs();
    o.c(' ');
    secs();
    if (r.pct(10)) {  // 2-3 upstreams: "X, X" or "X, X : X" (UpstreamModule.upstreamListOf)
        o.s(", ");
        secs();
        if (r.pct(50)) {
            o.s(r.pct(50) ? ", " : " : ");
            secs();
        }
    }
    o.c(' ');
    o.c(r.pct(20) ? 'p' : '.');
    o.c('\n');
}

// Apache 'common' ('%h %l %u %t "%r" %>s %b'): a combined line without the
// referer and user agent
void common_line(Out& o, uint64_t seed, int64_t i) {
    Rng r = line_rng(seed, i);
    who(o, r);
    o.s(" [");
    stamp(o, r, ':');
    o.c(' ');
    o.s(OFFSETS[r.below(7)]);
    o.s("] \"");
    request(o, r);
    o.s("\" ");
    o.u(STATUS[r.below(12)]);
    o.c(' ');
    if (r.pct(95)) o.u(r.below(200000)); else o.c('-');
    o.c('\n');
}

// config 5: mixed-format corpus, 40 % config-2 'combined', 30 % config-4
// NGINX, 30 % 'common' lines.  The three formats are
// mutually exclusive (a combined line ends in '"', an NGINX line in its $pipe
// byte after a time, a common line in %b), so the sticky active-format state
// of HttpdLogFormatDissector is history-independent and every line is
// decided by its own format.
void mixed_line(Out& o, uint64_t seed, int64_t i) {
    Rng r(seed ^ 0xA5A5A5A55A5A5A5Aull);
    r.s += (uint64_t)i * 0xD1B54A32D192ED03ull;
    const uint32_t k = r.below(10);
    if (k < 4) combined_line(o, seed, i);
    else if (k < 7) nginx_line(o, seed, i);
    else common_line(o, seed, i);
}

}  // namespace

extern "C" int64_t lp_synth(int workload, uint64_t seed, int64_t first_line, int64_t max_lines, char* out,
                            size_t cap, int64_t* n_lines) {
    void (*gen)(Out&, uint64_t, int64_t) = workload == LP_SYNTH_COMBINED   ? combined_line
                                           : workload == LP_SYNTH_STRFTIME ? strftime_line
                                           : workload == LP_SYNTH_NGINX    ? nginx_line
                                           : workload == LP_SYNTH_MIXED    ? mixed_line
                                                                           : nullptr;
    if (!gen) return LP_E_INVALID;
    Out o{out, 0, cap};
    int64_t k = 0;
    for (; k < max_lines; ++k) {
        size_t mark = o.n;
        gen(o, seed, first_line + k);
        if (!o.ok) { o.n = mark; break; }
    }
    if (n_lines) *n_lines = k;
    return (int64_t)o.n;
}

extern "C" int64_t lp_synth_combined(uint64_t seed, int64_t first_line, int64_t max_lines, char* out, size_t cap,
                                     int64_t* n_lines) {
    return lp_synth(LP_SYNTH_COMBINED, seed, first_line, max_lines, out, cap, n_lines);
}
