/*
 * ORACLE / TEST INFRASTRUCTURE ONLY -- see oracle.h for scope and the list of
 * reference files restated here.  Never linked into the product.
 *
 * All reference paths below are relative to /root/reference:
 *   core/ = parser-core/src/main/java/nl/basjes/parse/core/
 *   hp/   = httpdlog/httpdlog-parser/src/main/java/nl/basjes/parse/httpdlog/
 */
#include "oracle.h"

#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "jregex.h"
#include "ostr.h"

void oracle_md5_hex(const unsigned char *msg, size_t len, char out[33]);

/* ================================================================ utils */
static void *xmalloc(size_t n) {
    void *p = calloc(1, n ? n : 1);
    if (!p) { fprintf(stderr, "oracle: out of memory\n"); abort(); }
    return p;
}
static char *xstrdup(const char *s) {
    size_t n = strlen(s);
    char *d = (char *)xmalloc(n + 1);
    memcpy(d, s, n + 1);
    return d;
}
static char *xfmt(const char *f, ...) {
    va_list ap;
    va_start(ap, f);
    char tmp[4096];
    vsnprintf(tmp, sizeof tmp, f, ap);
    va_end(ap);
    return xstrdup(tmp);
}

typedef struct { char **v; int n, cap; } slist;
static void sl_add(slist *l, const char *s) {
    if (l->n == l->cap) { l->cap = l->cap ? l->cap * 2 : 8; l->v = (char **)realloc(l->v, sizeof(char *) * (size_t)l->cap); }
    l->v[l->n++] = xstrdup(s);
}
static int sl_has(const slist *l, const char *s) {
    for (int i = 0; i < l->n; i++) if (strcmp(l->v[i], s) == 0) return 1;
    return 0;
}
static void sl_add_unique(slist *l, const char *s) { if (!sl_has(l, s)) sl_add(l, s); }
static void sl_free(slist *l) {
    for (int i = 0; i < l->n; i++) free(l->v[i]);
    free(l->v);
    l->v = NULL; l->n = l->cap = 0;
}

static void ascii_lower(char *s) { for (; *s; s++) if (*s >= 'A' && *s <= 'Z') *s += 32; }
static void ascii_upper(char *s) { for (; *s; s++) if (*s >= 'a' && *s <= 'z') *s -= 32; }

/* code points <-> UTF-8 for setup-time strings */
static int *cp_of(const char *s, int *n) {
    int len = (int)strlen(s);
    int *cp = (int *)xmalloc(sizeof(int) * (size_t)(len + 1));
    int k = 0;
    const unsigned char *u = (const unsigned char *)s;
    for (int i = 0; i < len;) {
        unsigned c = u[i];
        if (c < 0x80) { cp[k++] = (int)c; i++; }
        else if ((c >> 5) == 6 && i + 1 < len) { cp[k++] = (int)(((c & 0x1F) << 6) | (u[i + 1] & 0x3F)); i += 2; }
        else if ((c >> 4) == 14 && i + 2 < len) { cp[k++] = (int)(((c & 0x0F) << 12) | ((u[i + 1] & 0x3F) << 6) | (u[i + 2] & 0x3F)); i += 3; }
        else if ((c >> 3) == 30 && i + 3 < len) { cp[k++] = (int)(((c & 0x07) << 18) | ((u[i + 1] & 0x3F) << 12) | ((u[i + 2] & 0x3F) << 6) | (u[i + 3] & 0x3F)); i += 4; }
        else { cp[k++] = 0xFFFD; i++; }
    }
    *n = k;
    return cp;
}
static char *utf8_of(const int *cp, int n) {
    char *o = (char *)xmalloc((size_t)n * 4 + 1);
    int k = 0;
    for (int i = 0; i < n; i++) {
        unsigned c = (unsigned)cp[i];
        if (c < 0x80) o[k++] = (char)c;
        else if (c < 0x800) { o[k++] = (char)(0xC0 | (c >> 6)); o[k++] = (char)(0x80 | (c & 0x3F)); }
        else if (c < 0x10000) { o[k++] = (char)(0xE0 | (c >> 12)); o[k++] = (char)(0x80 | ((c >> 6) & 0x3F)); o[k++] = (char)(0x80 | (c & 0x3F)); }
        else { o[k++] = (char)(0xF0 | (c >> 18)); o[k++] = (char)(0x80 | ((c >> 12) & 0x3F)); o[k++] = (char)(0x80 | ((c >> 6) & 0x3F)); o[k++] = (char)(0x80 | (c & 0x3F)); }
    }
    o[k] = 0;
    return o;
}

static jre *must_compile(const char *pat) {
    char err[256];
    jre *r = jre_compile(pat, err, sizeof err);
    if (!r) { fprintf(stderr, "oracle: internal regex '%s' failed: %s\n", pat, err); abort(); }
    return r;
}

/* setup-time regex replaceAll on UTF-8 strings (replacement is literal
 * except $n) */
static char *re_replace_all_s(const char *pat, const char *s, const char *repl) {
    arena a = {0};
    jre *re = must_compile(pat);
    js in = js_lit(&a, s);
    js out = js_replace_all(&a, re, in, repl);
    char *r = utf8_of(out.c, out.n);
    jre_free(re);
    ar_free(&a);
    return r;
}

/* ====================================================== token parsers */
/* Casts bitmask */
#define C_S 1
#define C_L 2
#define C_D 4
#define STRING_ONLY C_S
#define STRING_OR_LONG (C_S | C_L)
#define STRING_OR_LONG_OR_DOUBLE (C_S | C_L | C_D)

/* hp/dissectors/tokenformat/TokenParser.java:35-59 */
#define FORMAT_DIGIT "[0-9]"
#define FORMAT_NUMBER FORMAT_DIGIT "+"
#define FORMAT_CLF_NUMBER FORMAT_NUMBER "|-"
#define FORMAT_HEXDIGIT "[0-9a-fA-F]"
#define FORMAT_HEXNUMBER FORMAT_HEXDIGIT "+"
#define FORMAT_CLF_HEXNUMBER FORMAT_HEXNUMBER "|-"
#define FORMAT_NON_ZERO_NUMBER "[1-9][0-9]*"
#define FORMAT_EIGHT_BIT_DECIMAL "(?:25[0-5]|2[0-4][0-9]|[01]?[0-9][0-9]?)"
#define FORMAT_IPV4 "(?:" FORMAT_EIGHT_BIT_DECIMAL "\\.){3}" FORMAT_EIGHT_BIT_DECIMAL
#define FORMAT_IPV6 ":?(?:" FORMAT_HEXDIGIT "{1,4}(?::|.)?){0,8}(?::|::)?(?:" FORMAT_HEXDIGIT "{1,4}(?::|.)?){0,8}"
#define FORMAT_IP FORMAT_IPV4 "|" FORMAT_IPV6
#define FORMAT_CLF_IP FORMAT_IP "|-"
#define FORMAT_STRING ".*?"
#define FORMAT_NO_SPACE_STRING "[^\\s]*"
#define FORMAT_STANDARD_TIME_US "[0-3][0-9]/(?:[a-zA-Z][a-zA-Z][a-zA-Z])/[1-9][0-9][0-9][0-9]:[0-9][0-9]:[0-9][0-9]:[0-9][0-9] [\\+|\\-][0-9][0-9][0-9][0-9]"
#define FIRSTLINE_REGEX ".*" /* hp/dissectors/HttpFirstLineDissector.java:56-57 */

enum { TP_PLAIN, TP_FIXED, TP_NAMED, TP_PARAM };
enum { CUSTOM_NONE = 0, CUSTOM_STRFTIME = 1 };

typedef struct { char *type, *name; int casts; } ofield;

typedef struct {
    int kind;
    char *tok;      /* literal token (PLAIN/FIXED) or pattern (NAMED/PARAM) */
    char *regex;
    int prio;
    ofield outs[4];
    int nouts;
    int custom;
    jre *pat;
} tparser;

typedef struct { tparser *v; int n, cap; } tplist;

static tparser *tp_add(tplist *l, int kind, const char *tok, const char *regex, int prio) {
    if (l->n == l->cap) { l->cap = l->cap ? l->cap * 2 : 64; l->v = (tparser *)realloc(l->v, sizeof(tparser) * (size_t)l->cap); }
    tparser *t = &l->v[l->n++];
    memset(t, 0, sizeof *t);
    t->kind = kind;
    t->tok = xstrdup(tok);
    t->regex = xstrdup(regex);
    t->prio = prio;
    if (kind == TP_NAMED || kind == TP_PARAM) t->pat = must_compile(tok);
    return t;
}
/* TokenOutputField lowercases the name (tokenformat/TokenOutputField.java:39-44) */
static void tp_out(tparser *t, const char *type, const char *name, int casts) {
    char *n = xstrdup(name);
    ascii_lower(n);
    t->outs[t->nouts].type = xstrdup(type);
    t->outs[t->nouts].name = n;
    t->outs[t->nouts].casts = casts;
    t->nouts++;
}

/* ApacheHttpdLogFormatDissector.createFirstAndLastTokenParsers (:651-714) */
static void first_last(tplist *l, const char *token, const char *name, const char *type, int casts, const char *regex, int prio) {
    tparser *t = tp_add(l, TP_PLAIN, token, regex, prio);
    const char *orig_tokens[] = {"%s", "%U", "%T", "%{us}T", "%{ms}T", "%{s}T", "%D", "%r", NULL};
    int orig = 0;
    for (int i = 0; orig_tokens[i]; i++) if (strcmp(orig_tokens[i], token) == 0) orig = 1;
    char buf[256];
    tp_out(t, type, name, casts);
    snprintf(buf, sizeof buf, "%s%s", name, orig ? ".original" : ".last");
    tp_out(t, type, buf, casts);
    /* replaceFirst("%", "%<") */
    char tk[128];
    const char *pc = strchr(token, '%');
    snprintf(tk, sizeof tk, "%.*s%%<%s", (int)(pc - token), token, pc + 1);
    t = tp_add(l, TP_PLAIN, tk, regex, prio);
    snprintf(buf, sizeof buf, "%s.original", name);
    tp_out(t, type, buf, casts);
    snprintf(tk, sizeof tk, "%.*s%%>%s", (int)(pc - token), token, pc + 1);
    t = tp_add(l, TP_PLAIN, tk, regex, prio);
    snprintf(buf, sizeof buf, "%s.last", name);
    tp_out(t, type, buf, casts);
}
static void fl(tplist *l, const char *token, const char *name, const char *type, int casts, const char *regex) {
    first_last(l, token, name, type, casts, regex, 0);
}
/* addExtraOutput (:640-649): first parser with exactly this token */
static void extra_out(tplist *l, const char *token, const char *type, const char *name, int casts) {
    for (int i = 0; i < l->n; i++)
        if (strcmp(l->v[i].tok, token) == 0) { tp_out(&l->v[i], type, name, casts); return; }
}

/* ApacheHttpdLogFormatDissector.createAllTokenParsers (:199-638) */
static void apache_token_parsers(tplist *l) {
    tp_add(l, TP_FIXED, "%%", "%", 0);
    fl(l, "%a", "connection.client.ip", "IP", STRING_ONLY, FORMAT_CLF_IP);
    fl(l, "%{c}a", "connection.client.peerip", "IP", STRING_ONLY, FORMAT_CLF_IP);
    fl(l, "%A", "connection.server.ip", "IP", STRING_ONLY, FORMAT_CLF_IP);
    fl(l, "%B", "response.body.bytes", "BYTES", STRING_OR_LONG, FORMAT_NUMBER);
    fl(l, "%b", "response.body.bytes", "BYTESCLF", STRING_OR_LONG, FORMAT_CLF_NUMBER);
    extra_out(l, "%b", "BYTES", "response.body.bytesclf", STRING_OR_LONG);
    tp_out(tp_add(l, TP_NAMED, "\\%\\{([a-z0-9\\-_]*)\\}C", FORMAT_STRING, 0), "HTTP.COOKIE", "request.cookies.", STRING_ONLY);
    tp_out(tp_add(l, TP_NAMED, "\\%\\{([a-z0-9\\-_]*)\\}e", FORMAT_STRING, 0), "VARIABLE", "server.environment.", STRING_ONLY);
    fl(l, "%f", "server.filename", "FILENAME", STRING_ONLY, FORMAT_STRING);
    fl(l, "%h", "connection.client.host", "IP", STRING_ONLY, FORMAT_NO_SPACE_STRING);
    fl(l, "%H", "request.protocol", "PROTOCOL", STRING_ONLY, FORMAT_NO_SPACE_STRING);
    tp_out(tp_add(l, TP_NAMED, "\\%\\{([a-z0-9\\-_]*)\\}i", FORMAT_STRING, 0), "HTTP.HEADER", "request.header.", STRING_ONLY);
    tp_out(tp_add(l, TP_NAMED, "\\%\\{([a-z0-9\\-_]*)\\}\\^ti", FORMAT_STRING, 0), "HTTP.TRAILER", "request.trailer.", STRING_ONLY);
    fl(l, "%k", "connection.keepalivecount", "NUMBER", STRING_OR_LONG, FORMAT_NUMBER);
    fl(l, "%l", "connection.client.logname", "NUMBER", STRING_OR_LONG, FORMAT_CLF_NUMBER);
    fl(l, "%L", "request.errorlogid", "STRING", STRING_ONLY, FORMAT_NO_SPACE_STRING);
    fl(l, "%m", "request.method", "HTTP.METHOD", STRING_ONLY, FORMAT_NO_SPACE_STRING);
    tp_out(tp_add(l, TP_NAMED, "\\%\\{([a-z0-9\\-_]*)\\}n", FORMAT_STRING, 0), "STRING", "server.module_note.", STRING_ONLY);
    tp_out(tp_add(l, TP_NAMED, "\\%\\{([a-z0-9\\-]*)\\}o", FORMAT_STRING, 0), "HTTP.HEADER", "response.header.", STRING_ONLY);
    tp_out(tp_add(l, TP_NAMED, "\\%\\{([a-z0-9\\-_]*)\\}\\^to", FORMAT_STRING, 0), "HTTP.TRAILER", "response.trailer.", STRING_ONLY);
    fl(l, "%p", "request.server.port.canonical", "PORT", STRING_OR_LONG, FORMAT_NUMBER);
    fl(l, "%{canonical}p", "connection.server.port.canonical", "PORT", STRING_OR_LONG, FORMAT_NUMBER);
    fl(l, "%{local}p", "connection.server.port", "PORT", STRING_OR_LONG, FORMAT_NUMBER);
    fl(l, "%{remote}p", "connection.client.port", "PORT", STRING_OR_LONG, FORMAT_NUMBER);
    fl(l, "%P", "connection.server.child.processid", "NUMBER", STRING_OR_LONG, FORMAT_NUMBER);
    fl(l, "%{pid}P", "connection.server.child.processid", "NUMBER", STRING_OR_LONG, FORMAT_NUMBER);
    fl(l, "%{tid}P", "connection.server.child.threadid", "NUMBER", STRING_OR_LONG, FORMAT_NUMBER);
    fl(l, "%{hextid}P", "connection.server.child.hexthreadid", "NUMBER", STRING_OR_LONG, FORMAT_CLF_HEXNUMBER);
    fl(l, "%q", "request.querystring", "HTTP.QUERYSTRING", STRING_ONLY, FORMAT_NO_SPACE_STRING);
    fl(l, "%r", "request.firstline", "HTTP.FIRSTLINE", STRING_ONLY, FIRSTLINE_REGEX);
    fl(l, "%R", "request.handler", "STRING", STRING_ONLY, FORMAT_STRING);
    first_last(l, "%s", "request.status", "STRING", STRING_ONLY, FORMAT_NO_SPACE_STRING, 0);
    fl(l, "%t", "request.receive.time", "TIME.STAMP", STRING_ONLY, FORMAT_STANDARD_TIME_US);
    tparser *t;
    t = tp_add(l, TP_PARAM, "\\%\\{([^\\}]*%[^\\}]*)\\}t", FORMAT_STRING, -1);
    tp_out(t, "TIME.STRFTIME_", "request.receive.time", STRING_ONLY);
    t->custom = CUSTOM_STRFTIME;
    t = tp_add(l, TP_PARAM, "\\%\\{begin:([^\\}]*%[^\\}]*)\\}t", FORMAT_STRING, 0);
    tp_out(t, "TIME.STRFTIME_", "request.receive.time.begin", STRING_ONLY);
    t->custom = CUSTOM_STRFTIME;
    t = tp_add(l, TP_PARAM, "\\%\\{end:([^\\}]*%[^\\}]*)\\}t", FORMAT_STRING, 0);
    tp_out(t, "TIME.STRFTIME_", "request.receive.time.end", STRING_ONLY);
    t->custom = CUSTOM_STRFTIME;
    fl(l, "%{sec}t", "request.receive.time.sec", "TIME.SECONDS", STRING_OR_LONG, FORMAT_NUMBER);
    fl(l, "%{begin:sec}t", "request.receive.time.begin.sec", "TIME.SECONDS", STRING_OR_LONG, FORMAT_NUMBER);
    fl(l, "%{end:sec}t", "request.receive.time.end.sec", "TIME.SECONDS", STRING_OR_LONG, FORMAT_NUMBER);
    fl(l, "%{msec}t", "request.receive.time.msec", "TIME.EPOCH", STRING_OR_LONG, FORMAT_NUMBER);
    extra_out(l, "%{msec}t", "TIME.EPOCH", "request.receive.time.begin.msec", STRING_OR_LONG);
    fl(l, "%{begin:msec}t", "request.receive.time.begin.msec", "TIME.EPOCH", STRING_OR_LONG, FORMAT_NUMBER);
    fl(l, "%{end:msec}t", "request.receive.time.end.msec", "TIME.EPOCH", STRING_OR_LONG, FORMAT_NUMBER);
    fl(l, "%{usec}t", "request.receive.time.usec", "TIME.EPOCH.USEC", STRING_OR_LONG, FORMAT_NUMBER);
    extra_out(l, "%{usec}t", "TIME.EPOCH.USEC", "request.receive.time.begin.usec", STRING_OR_LONG);
    fl(l, "%{begin:usec}t", "request.receive.time.begin.usec", "TIME.EPOCH.USEC", STRING_OR_LONG, FORMAT_NUMBER);
    fl(l, "%{end:usec}t", "request.receive.time.end.usec", "TIME.EPOCH.USEC", STRING_OR_LONG, FORMAT_NUMBER);
    fl(l, "%{msec_frac}t", "request.receive.time.msec_frac", "TIME.EPOCH", STRING_OR_LONG, FORMAT_NUMBER);
    extra_out(l, "%{msec_frac}t", "TIME.EPOCH", "request.receive.time.begin.msec_frac", STRING_OR_LONG);
    fl(l, "%{begin:msec_frac}t", "request.receive.time.begin.msec_frac", "TIME.EPOCH", STRING_OR_LONG, FORMAT_NUMBER);
    fl(l, "%{end:msec_frac}t", "request.receive.time.end.msec_frac", "TIME.EPOCH", STRING_OR_LONG, FORMAT_NUMBER);
    fl(l, "%{usec_frac}t", "request.receive.time.usec_frac", "TIME.EPOCH.USEC_FRAC", STRING_OR_LONG, FORMAT_NUMBER);
    extra_out(l, "%{usec_frac}t", "TIME.EPOCH.USEC_FRAC", "request.receive.time.begin.usec_frac", STRING_OR_LONG);
    fl(l, "%{begin:usec_frac}t", "request.receive.time.begin.usec_frac", "TIME.EPOCH.USEC_FRAC", STRING_OR_LONG, FORMAT_NUMBER);
    fl(l, "%{end:usec_frac}t", "request.receive.time.end.usec_frac", "TIME.EPOCH.USEC_FRAC", STRING_OR_LONG, FORMAT_NUMBER);
    fl(l, "%T", "response.server.processing.time", "SECONDS", STRING_OR_LONG, FORMAT_NUMBER);
    fl(l, "%D", "response.server.processing.time", "MICROSECONDS", STRING_OR_LONG, FORMAT_NUMBER);
    extra_out(l, "%D", "MICROSECONDS", "server.process.time", STRING_OR_LONG);
    fl(l, "%{us}T", "response.server.processing.time", "MICROSECONDS", STRING_OR_LONG, FORMAT_NUMBER);
    fl(l, "%{ms}T", "response.server.processing.time", "MILLISECONDS", STRING_OR_LONG, FORMAT_NUMBER);
    fl(l, "%{s}T", "response.server.processing.time", "SECONDS", STRING_OR_LONG, FORMAT_NUMBER);
    fl(l, "%u", "connection.client.user", "STRING", STRING_ONLY, FORMAT_NO_SPACE_STRING);
    fl(l, "%U", "request.urlpath", "URI", STRING_ONLY, FORMAT_NO_SPACE_STRING);
    fl(l, "%v", "connection.server.name.canonical", "STRING", STRING_ONLY, FORMAT_NO_SPACE_STRING);
    fl(l, "%V", "connection.server.name", "STRING", STRING_ONLY, FORMAT_NO_SPACE_STRING);
    fl(l, "%X", "response.connection.status", "HTTP.CONNECTSTATUS", STRING_ONLY, FORMAT_NO_SPACE_STRING);
    fl(l, "%I", "request.bytes", "BYTES", STRING_OR_LONG, FORMAT_CLF_NUMBER);
    fl(l, "%O", "response.bytes", "BYTES", STRING_OR_LONG, FORMAT_CLF_NUMBER);
    fl(l, "%S", "total.bytes", "BYTES", STRING_OR_LONG, FORMAT_NON_ZERO_NUMBER);
    first_last(l, "%{cookie}i", "request.cookies", "HTTP.COOKIES", STRING_ONLY, FORMAT_STRING, 1);
    first_last(l, "%{set-cookie}o", "response.cookies", "HTTP.SETCOOKIES", STRING_ONLY, FORMAT_STRING, 1);
    first_last(l, "%{user-agent}i", "request.user-agent", "HTTP.USERAGENT", STRING_ONLY, FORMAT_STRING, 1);
    first_last(l, "%{referer}i", "request.referer", "HTTP.URI", STRING_ONLY, FORMAT_STRING, 1);
}

/* ---------------------------------------------------------------- NGINX
 * NginxHttpdLogFormatDissector.createAllTokenParsers (hp/NginxHttpdLogFormatDissector.java:121-142):
 * the token parsers of every module, in module order.  TokenParser's default
 * prio is 10 (tokenformat/TokenParser.java:81-88), NamedTokenParser's 0
 * (tokenformat/NamedTokenParser.java:34-41). */
#define FORMAT_STANDARD_TIME_ISO8601 "[1-9][0-9][0-9][0-9]-[0-1][0-9]-[0-3][0-9]T[0-9][0-9]:[0-9][0-9]:[0-9][0-9][\\+|\\-][0-9][0-9]:[0-9][0-9]"
#define FORMAT_NUMBER_DECIMAL FORMAT_NUMBER "\\." FORMAT_NUMBER
#define FORMAT_NUMBER_OPTIONAL_DECIMAL FORMAT_NUMBER "(?:\\." FORMAT_NUMBER ")?"
/* UpstreamModule.upstreamListOf (nginxmodules/UpstreamModule.java:42-44) */
#define UPSTREAM_LIST(X) X "(?: *, *" X "(?: *: *" X ")?)*"

static void ng(tplist *l, const char *tok, const char *name, const char *type, int casts, const char *regex, int prio) {
    tp_out(tp_add(l, TP_PLAIN, tok, regex, prio), type, name, casts);
}
static void ng_named(tplist *l, const char *pat, const char *name, const char *type, int casts, const char *regex, int prio) {
    tp_out(tp_add(l, TP_NAMED, pat, regex, prio), type, name, casts);
}
/* TokenFormatDissector.NotImplementedTokenParser (tokenformat/TokenFormatDissector.java:89-103) */
static void ng_notimpl(tplist *l, const char *tok, const char *prefix, const char *regex, int prio) {
    char name[256];
    int k = snprintf(name, sizeof name, "%s_", prefix);
    for (const char *p = tok; *p && k < 250; p++) {
        char c = (*p >= 'A' && *p <= 'Z') ? (char)(*p + 32) : *p;
        name[k++] = ((c >= 'a' && c <= 'z') || (c >= '0' && c <= '9') || c == '_') ? c : '_';
    }
    name[k] = 0;
    ng(l, tok, name, "NOT_IMPLEMENTED", STRING_ONLY, regex, prio);
}

static void nginx_token_parsers(tplist *l) {
    /* CoreLogModule (nginxmodules/CoreLogModule.java:45-489) */
    ng(l, "$bytes_sent", "response.bytes", "BYTES", STRING_OR_LONG, FORMAT_NUMBER, 10);
    ng(l, "$bytes_received", "request.bytes", "BYTES", STRING_OR_LONG, FORMAT_NUMBER, 10);
    ng(l, "$connection", "connection.serial_number", "NUMBER", STRING_OR_LONG, FORMAT_CLF_NUMBER, -1);
    ng(l, "$connection_requests", "connection.requestnr", "NUMBER", STRING_OR_LONG, FORMAT_CLF_NUMBER, 10);
    ng(l, "$msec", "request.receive.time.epoch", "TIME.EPOCH_SECOND_MILLIS", STRING_ONLY, "[0-9]+\\.[0-9][0-9][0-9]", 10);
    ng(l, "$status", "request.status.last", "STRING", STRING_ONLY, FORMAT_NO_SPACE_STRING, 10);
    ng(l, "$time_iso8601", "request.receive.time", "TIME.ISO8601", STRING_ONLY, FORMAT_STANDARD_TIME_ISO8601, 10);
    ng(l, "$time_local", "request.receive.time", "TIME.STAMP", STRING_ONLY, FORMAT_STANDARD_TIME_US, 10);
    ng_named(l, "\\$arg_([a-z0-9\\-\\_]*)", "request.firstline.uri.query.", "STRING", STRING_ONLY, FORMAT_STRING, 0);
    ng(l, "$is_args", "request.firstline.uri.is_args", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$args", "request.firstline.uri.query", "HTTP.QUERYSTRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$query_string", "request.firstline.uri.query", "HTTP.QUERYSTRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$body_bytes_sent", "response.body.bytes", "BYTES", STRING_OR_LONG, FORMAT_NUMBER, 10);
    ng(l, "$content_length", "request.header.content_length", "HTTP.HEADER", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$content_type", "request.header.content_type", "HTTP.HEADER", STRING_ONLY, FORMAT_STRING, 10);
    ng_named(l, "\\$cookie_([a-z0-9\\-_]*)", "request.cookies.", "HTTP.COOKIE", STRING_ONLY, FORMAT_STRING, 0);
    ng(l, "$document_root", "request.firstline.document_root", "STRING", STRING_ONLY, FORMAT_NO_SPACE_STRING, 10);
    ng(l, "$realpath_root", "request.firstline.realpath_root", "STRING", STRING_ONLY, FORMAT_NO_SPACE_STRING, 10);
    ng(l, "$host", "connection.server.name", "STRING", STRING_ONLY, FORMAT_NO_SPACE_STRING, -1);
    ng(l, "$hostname", "connection.client.host", "STRING", STRING_ONLY, FORMAT_NO_SPACE_STRING, 10);
    ng_named(l, "\\$http_([a-z0-9\\-_]*)", "request.header.", "HTTP.HEADER", STRING_ONLY, FORMAT_STRING, 0);
    ng(l, "$http_user_agent", "request.user-agent", "HTTP.USERAGENT", STRING_ONLY, FORMAT_STRING, 1);
    ng(l, "$http_referer", "request.referer", "HTTP.URI", STRING_ONLY, FORMAT_NO_SPACE_STRING, 1);
    ng(l, "$https", "connection.https", "STRING", STRING_ONLY, FORMAT_NO_SPACE_STRING, 10);
    ng_notimpl(l, "$limit_rate", "nginx_parameter_not_intended_for_logging", FORMAT_NO_SPACE_STRING, 0);
    ng(l, "$nginx_version", "server.nginx.version", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$pid", "connection.server.child.processid", "NUMBER", STRING_OR_LONG, FORMAT_NUMBER, 10);
    ng(l, "$protocol", "connection.protocol", "STRING", STRING_ONLY, FORMAT_NO_SPACE_STRING, 10);
    ng(l, "$pipe", "connection.nginx.pipe", "STRING", STRING_ONLY, ".", 10);
    ng(l, "$proxy_protocol_addr", "connection.client.proxy.host", "IP", STRING_OR_LONG, FORMAT_CLF_IP, 10);
    ng(l, "$proxy_protocol_port", "connection.client.proxy.port", "PORT", STRING_OR_LONG, FORMAT_CLF_NUMBER, 10);
    ng(l, "$remote_addr", "connection.client.host", "IP", STRING_OR_LONG, FORMAT_CLF_IP, 10);
    ng(l, "$binary_remote_addr", "connection.client.host", "IP_BINARY", STRING_OR_LONG,
       "\\\\x" FORMAT_HEXDIGIT FORMAT_HEXDIGIT "\\\\x" FORMAT_HEXDIGIT FORMAT_HEXDIGIT
       "\\\\x" FORMAT_HEXDIGIT FORMAT_HEXDIGIT "\\\\x" FORMAT_HEXDIGIT FORMAT_HEXDIGIT, 10);
    ng(l, "$remote_port", "connection.client.port", "PORT", STRING_OR_LONG, FORMAT_NUMBER, 10);
    ng(l, "$remote_user", "connection.client.user", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$request", "request.firstline", "HTTP.FIRSTLINE", STRING_ONLY,
       FORMAT_NO_SPACE_STRING " " FORMAT_NO_SPACE_STRING " " FORMAT_NO_SPACE_STRING, -2);
    ng_notimpl(l, "$request_body", "nginx_parameter_not_intended_for_logging", FORMAT_STRING, -1);
    ng_notimpl(l, "$request_body_file", "nginx_parameter_not_intended_for_logging", FORMAT_STRING, -1);
    ng(l, "$request_completion", "request.completion", "STRING", STRING_ONLY, FORMAT_NO_SPACE_STRING, 10);
    ng(l, "$request_filename", "server.filename", "FILENAME", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$request_length", "request.bytes", "BYTES", STRING_OR_LONG, FORMAT_CLF_NUMBER, 10);
    ng(l, "$request_method", "request.firstline.method", "HTTP.METHOD", STRING_ONLY, FORMAT_NO_SPACE_STRING, 10);
    ng(l, "$request_time", "response.server.processing.time", "SECOND_MILLIS", STRING_ONLY, FORMAT_NUMBER_DECIMAL, 10);
    ng(l, "$request_uri", "request.firstline.uri", "HTTP.URI", STRING_ONLY, FORMAT_NO_SPACE_STRING, 10);
    ng(l, "$request_id", "request.id", "STRING", STRING_ONLY, FORMAT_HEXNUMBER, 10);
    ng(l, "$uri", "request.firstline.uri.normalized", "HTTP.URI", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$document_uri", "request.firstline.uri.normalized", "HTTP.URI", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$scheme", "request.firstline.uri.protocol", "HTTP.PROTOCOL", STRING_ONLY, FORMAT_NO_SPACE_STRING, 10);
    ng_named(l, "\\$sent_http_([a-z0-9\\-_]*)", "response.header.", "HTTP.HEADER", STRING_ONLY, FORMAT_STRING, 0);
    ng_named(l, "\\$sent_trailer_([a-z0-9\\-_]*)", "response.trailer.", "HTTP.TRAILER", STRING_ONLY, FORMAT_STRING, 0);
    ng(l, "$server_addr", "connection.server.ip", "IP", STRING_OR_LONG, FORMAT_CLF_IP, 10);
    ng(l, "$server_name", "connection.server.name", "STRING", STRING_ONLY, FORMAT_NO_SPACE_STRING, 10);
    ng(l, "$server_port", "connection.server.port", "PORT", STRING_OR_LONG, FORMAT_NUMBER, 10);
    ng(l, "$server_protocol", "request.firstline.protocol", "HTTP.PROTOCOL_VERSION", STRING_OR_LONG, FORMAT_NO_SPACE_STRING, 10);
    ng(l, "$session_time", "connection.session.time", "SECOND_MILLIS", STRING_ONLY, FORMAT_NUMBER_DECIMAL, 10);
    ng(l, "$tcpinfo_rtt", "connection.tcpinfo.rtt", "MICROSECONDS", STRING_OR_LONG, FORMAT_NUMBER, -1);
    ng(l, "$tcpinfo_rttvar", "connection.tcpinfo.rttvar", "MICROSECONDS", STRING_OR_LONG, FORMAT_NUMBER, 10);
    ng(l, "$tcpinfo_snd_cwnd", "connection.tcpinfo.send.cwnd", "BYTES", STRING_OR_LONG, FORMAT_NUMBER, 10);
    ng(l, "$tcpinfo_rcv_space", "connection.tcpinfo.receive.space", "BYTES", STRING_OR_LONG, FORMAT_NUMBER, 10);
    ng_named(l, "\\$([a-z0-9\\-\\_]*)", "nginx.unknown.", "UNKNOWN_NGINX_VARIABLE", STRING_ONLY, FORMAT_NO_SPACE_STRING, -10);
    /* UpstreamModule (nginxmodules/UpstreamModule.java:46-160) */
#define UP "nginxmodule.upstream"
    ng(l, "$upstream_addr", UP ".addr", "UPSTREAM_ADDR_LIST", STRING_ONLY, UPSTREAM_LIST(FORMAT_NO_SPACE_STRING), 10);
    ng(l, "$upstream_bytes_received", UP ".bytes.received", "UPSTREAM_BYTES_LIST", STRING_ONLY, UPSTREAM_LIST(FORMAT_NUMBER), 10);
    ng(l, "$upstream_bytes_sent", UP ".bytes.sent", "UPSTREAM_BYTES_LIST", STRING_ONLY, UPSTREAM_LIST(FORMAT_NUMBER), 10);
    ng(l, "$upstream_cache_status", UP ".cache.status", "UPSTREAM_CACHE_STATUS", STRING_ONLY,
       "(?:MISS|BYPASS|EXPIRED|STALE|UPDATING|REVALIDATED|HIT)", 10);
    ng(l, "$upstream_connect_time", UP ".connect.time", "UPSTREAM_SECOND_MILLIS_LIST", STRING_ONLY, UPSTREAM_LIST(FORMAT_NUMBER_DECIMAL), 10);
    ng_named(l, "\\$upstream_cookie_([a-z0-9\\-_]*)", UP ".response.cookies.", "HTTP.COOKIE", STRING_ONLY, FORMAT_STRING, 0);
    ng(l, "$upstream_header_time", UP ".header.time", "UPSTREAM_SECOND_MILLIS_LIST", STRING_ONLY, UPSTREAM_LIST(FORMAT_NUMBER_DECIMAL), 10);
    ng_named(l, "\\$upstream_http_([a-z0-9\\-_]*)", UP ".header.", "HTTP.HEADER", STRING_ONLY, FORMAT_STRING, 0);
    ng(l, "$upstream_queue_time", UP ".queue.time", "UPSTREAM_SECOND_MILLIS_LIST", STRING_ONLY, UPSTREAM_LIST(FORMAT_NUMBER_DECIMAL), 10);
    ng(l, "$upstream_response_length", UP ".response.length", "UPSTREAM_BYTES_LIST", STRING_ONLY, UPSTREAM_LIST(FORMAT_NUMBER), 10);
    ng(l, "$upstream_response_time", UP ".response.time", "UPSTREAM_SECOND_MILLIS_LIST", STRING_ONLY, UPSTREAM_LIST(FORMAT_NUMBER_DECIMAL), 10);
    ng(l, "$upstream_status", UP ".status", "UPSTREAM_STATUS_LIST", STRING_ONLY, UPSTREAM_LIST(FORMAT_NO_SPACE_STRING), 10);
    ng_named(l, "\\$upstream_trailer_([a-z0-9\\-_]*)", UP ".trailer.", "HTTP.TRAILER", STRING_ONLY, FORMAT_STRING, 0);
    ng(l, "$upstream_first_byte_time", UP ".first_byte.time", "UPSTREAM_SECOND_MILLIS_LIST", STRING_ONLY, UPSTREAM_LIST(FORMAT_NUMBER_DECIMAL), 10);
    ng(l, "$upstream_session_time", UP ".session.time", "UPSTREAM_SECOND_MILLIS_LIST", STRING_ONLY, UPSTREAM_LIST(FORMAT_NUMBER_DECIMAL), 10);
#undef UP
    /* SslModule (nginxmodules/SslModule.java:37-200) */
#define SSL "nginxmodule.ssl"
    ng(l, "$ssl_cipher", SSL ".cipher", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$ssl_ciphers", SSL ".client.ciphers", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$ssl_client_escaped_cert", SSL ".client.cert", "PEM_CERT_URLENCODED", STRING_ONLY, FORMAT_NO_SPACE_STRING, 10);
    ng(l, "$ssl_client_cert", SSL ".client.cert", "PEM_CERT", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$ssl_client_raw_cert", SSL ".client.cert", "PEM_CERT_RAW", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$ssl_client_fingerprint", SSL ".client.cert.fingerprint", "SHA1", STRING_ONLY, FORMAT_NO_SPACE_STRING, 10);
    ng(l, "$ssl_client_i_dn", SSL ".client.cert.issuer_dn", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$ssl_client_i_dn_legacy", SSL ".client.cert.issuer_dn.legacy", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$ssl_client_s_dn", SSL ".client.cert.subject_dn", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$ssl_client_s_dn_legacy", SSL ".client.cert.subject_dn.legacy", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$ssl_client_serial", SSL ".client.cert.serial", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$ssl_client_v_end", SSL ".client.cert.end_date", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$ssl_client_v_remain", SSL ".client.cert.remain_days", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$ssl_client_v_start", SSL ".client.cert.start_date", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$ssl_client_verify", SSL ".client.cert.verify", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$ssl_curves", SSL ".client.curves", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$ssl_early_data", SSL ".early_data", "STRING", STRING_ONLY, "1?", 10);
    ng(l, "$ssl_protocol", SSL ".protocol", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$ssl_server_name", SSL ".server_name", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$ssl_session_id", SSL ".session.id", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$ssl_session_reused", SSL ".session.reused", "STRING", STRING_ONLY, "(r|.)", 10);
    ng(l, "$ssl_preread_protocol", SSL ".preread.protocol", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$ssl_preread_server_name", SSL ".preread.server_name", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$ssl_preread_alpn_protocols", SSL ".preread.alpn_protocols", "STRING", STRING_ONLY, FORMAT_STRING, 10);
#undef SSL
    /* GeoIPModule (nginxmodules/GeoIPModule.java:35-104) */
#define GEO "nginxmodule.geoip"
    ng(l, "$geoip_country_code", GEO ".country.code", "STRING", STRING_ONLY, FORMAT_NO_SPACE_STRING, 10);
    ng(l, "$geoip_country_code3", GEO ".country.code3", "STRING", STRING_ONLY, FORMAT_NO_SPACE_STRING, 10);
    ng(l, "$geoip_country_name", GEO ".country.name", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$geoip_area_code", GEO ".area.code", "STRING", STRING_ONLY, FORMAT_NO_SPACE_STRING, 10);
    ng(l, "$geoip_city_continent_code", GEO ".continent.code", "STRING", STRING_ONLY, FORMAT_NO_SPACE_STRING, 10);
    ng(l, "$geoip_city_country_code", GEO ".country.code", "STRING", STRING_ONLY, FORMAT_NO_SPACE_STRING, 10);
    ng(l, "$geoip_city_country_code3", GEO ".country.code3", "STRING", STRING_ONLY, FORMAT_NO_SPACE_STRING, 10);
    ng(l, "$geoip_city_country_name", GEO ".country.name", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$geoip_dma_code", GEO ".dma.code", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$geoip_latitude", GEO ".location.latitude", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$geoip_longitude", GEO ".location.longitude", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$geoip_region", GEO ".region.code", "STRING", STRING_ONLY, FORMAT_NO_SPACE_STRING, 10);
    ng(l, "$geoip_region_name", GEO ".region.name", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$geoip_city", GEO ".city", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$geoip_postal_code", GEO ".postal.code", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$geoip_org", GEO ".organization", "STRING", STRING_ONLY, FORMAT_STRING, 10);
#undef GEO
    /* VariousModule (nginxmodules/VariousModule.java:37-212) */
#define VAR "nginxmodule"
    ng(l, "$secure_link", VAR ".secure_link.status", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$session_log_id", VAR ".session_log.id", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$slice_range", VAR ".slice_range", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$proxy_host", VAR ".proxy.host", "STRING", STRING_ONLY, FORMAT_NO_SPACE_STRING, 10);
    ng(l, "$proxy_port", VAR ".proxy.port", "STRING", STRING_ONLY, FORMAT_NO_SPACE_STRING, 10);
    ng(l, "$proxy_add_x_forwarded_for", VAR ".proxy.add_x_forwarded_for", "STRING", STRING_ONLY, FORMAT_NO_SPACE_STRING, 10);
    ng(l, "$uid_got", VAR ".userid.uid_got", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$uid_reset", VAR ".userid.uid_reset", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$uid_set", VAR ".userid.uid_set", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$modern_browser", VAR ".browser.modern", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$ancient_browser", VAR ".browser.ancient", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$msie", VAR ".browser.msie", "STRING", STRING_ONLY, FORMAT_NO_SPACE_STRING, 10);
    ng(l, "$connections_active", VAR ".stub_status.connections.active", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$connections_reading", VAR ".stub_status.connections.reading", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$connections_writing", VAR ".stub_status.connections.writing", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$connections_waiting", VAR ".stub_status.connections.waiting", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$date_local", VAR ".date.local", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$date_gmt", VAR ".date.gmt", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$fastcgi_script_name", VAR ".fastcgi.script_name", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$fastcgi_path_info", VAR ".fastcgi.path_info", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$gzip_ratio", VAR ".gzip.ratio", "STRING", STRING_ONLY, FORMAT_NUMBER_OPTIONAL_DECIMAL, 10);
    ng(l, "$spdy", VAR ".spdy.version", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$spdy_request_priority", VAR ".spdy.request_priority", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$http2", VAR ".http2.negotiated_protocol", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$invalid_referer", VAR ".referer.invalid", "STRING", STRING_ONLY, "1?", 10);
    ng_named(l, "\\$jwt_header_([a-z0-9\\-_]*)", VAR ".jwt.header.", "STRING", STRING_ONLY, FORMAT_STRING, 0);
    ng_named(l, "\\$jwt_claim_([a-z0-9\\-_]*)", VAR ".jwt.claim.", "STRING", STRING_ONLY, FORMAT_STRING, 0);
    ng(l, "$memcached_key", VAR ".memcached.key", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$realip_remote_addr", VAR ".realip.remote_addr", "IP", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$realip_remote_port", VAR ".realip.remote_port", "PORT", STRING_OR_LONG, FORMAT_STRING, 10);
#undef VAR
    /* KubernetesIngressModule (nginxmodules/KubernetesIngressModule.java:35-68) */
#define K8S "nginxmodule.kubernetes"
    ng(l, "$the_real_ip", K8S ".the_real_ip", "IP", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$proxy_upstream_name", K8S ".proxy_upstream_name", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$req_id", K8S ".req_id", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$namespace", K8S ".namespace", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$ingress_name", K8S ".ingress_name", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$service_name", K8S ".service.name", "STRING", STRING_ONLY, FORMAT_STRING, 10);
    ng(l, "$service_port", K8S ".service.port", "PORT", STRING_ONLY, FORMAT_STRING, 10);
#undef K8S
}

/* =============================================================== tokens */
typedef struct {
    int fixed;          /* FixedStringToken */
    char *regex;        /* fixed: the literal text */
    int start, len, prio;
    ofield outs[4];
    int nouts;
    int custom;
    char *custom_type, *custom_param;
} token;

typedef struct { token *v; int n, cap; } toklist;
static token *tk_push(toklist *l) {
    if (l->n == l->cap) { l->cap = l->cap ? l->cap * 2 : 32; l->v = (token *)realloc(l->v, sizeof(token) * (size_t)l->cap); }
    token *t = &l->v[l->n++];
    memset(t, 0, sizeof *t);
    return t;
}

/* ParameterizedTokenParser.tokenParameterToTypeName (:99-105) */
static char *param_type_name(const char *base_type, const char *param) {
    char clean[512];
    int k = 0;
    for (const char *p = param; *p && k < 500; p++)
        if ((*p >= 'A' && *p <= 'Z') || (*p >= 'a' && *p <= 'z') || (*p >= '0' && *p <= '9')) clean[k++] = *p;
    clean[k] = 0;
    char md5[33];
    oracle_md5_hex((const unsigned char *)param, strlen(param), md5);
    char *r = xfmt("%s%s_%s", base_type, clean, md5);
    ascii_upper(r);
    return r;
}

/* TokenParser/NamedTokenParser/ParameterizedTokenParser.getNextToken and
 * TokenParser.getTokens (TokenParser.java:569-614, NamedTokenParser.java:43-77,
 * ParameterizedTokenParser.java:58-95) */
static void collect_tokens(const tparser *tp, const char *fmt, const int *fcp, int fn, toklist *out) {
    /* StringUtils.isBlank */
    int blank = 1;
    for (const char *p = fmt; *p; p++) if (!(*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r' || *p == '\f' || *p == 0x0B)) blank = 0;
    if (blank) return;
    int offset = 0;
    for (;;) {
        int start, len;
        char *fieldname = NULL;
        if (tp->kind == TP_PLAIN || tp->kind == TP_FIXED) {
            int tn;
            int *tcp = cp_of(tp->tok, &tn);
            int pos = -1;
            for (int i = offset; i + tn <= fn; i++)
                if (memcmp(fcp + i, tcp, sizeof(int) * (size_t)tn) == 0) { pos = i; break; }
            free(tcp);
            if (pos < 0) return;
            start = pos;
            len = tn;
        } else {
            int caps[2 * 8];
            if (!jre_find(tp->pat, fcp, fn, offset, caps)) return;
            start = caps[0];
            len = caps[1] - caps[0];
            if (jre_ngroups(tp->pat) > 0 && caps[2] >= 0) fieldname = utf8_of(fcp + caps[2], caps[3] - caps[2]);
            else fieldname = xstrdup("");
        }
        token *t = tk_push(out);
        t->fixed = tp->kind == TP_FIXED;
        t->regex = xstrdup(tp->regex);
        t->start = start;
        t->len = len;
        t->prio = tp->kind == TP_FIXED ? 0 : tp->prio;
        for (int i = 0; i < tp->nouts; i++) {
            ofield o = tp->outs[i];
            if (tp->kind == TP_NAMED) {
                char *nm = xfmt("%s%s", o.name, fieldname);
                ascii_lower(nm); /* new TokenOutputField lowercases */
                t->outs[i].type = xstrdup(o.type);
                t->outs[i].name = nm;
            } else if (tp->kind == TP_PARAM) {
                t->outs[i].type = param_type_name(o.type, fieldname);
                t->outs[i].name = xstrdup(o.name);
            } else {
                t->outs[i].type = xstrdup(o.type);
                t->outs[i].name = xstrdup(o.name);
            }
            t->outs[i].casts = o.casts;
        }
        t->nouts = tp->nouts;
        if (tp->custom) {
            t->custom = tp->custom;
            t->custom_type = xstrdup(t->outs[0].type);
            t->custom_param = xstrdup(fieldname);
        }
        free(fieldname);
        offset = start + len;
    }
}

static int tok_cmp(const token *a, const token *b) { /* TokenSorterByStartPos */
    if (a->start != b->start) return a->start < b->start ? -1 : 1;
    if (a->len != b->len) return a->len < b->len ? -1 : 1;
    if (a->prio != b->prio) return a->prio > b->prio ? -1 : 1;
    return 0;
}

/* ============================================================= formats */
enum { FMT_APACHE = 1, FMT_NGINX = 2 };

typedef struct {
    int kind;
    char *logformat;      /* as registered (after alias mapping) */
    char *cleaned;
    token *tokens;        /* in order, incl. fixed strings */
    int ntokens;
    slist output_types;   /* "TYPE:name" */
    slist requested;      /* requestedFields (output names) */
    /* prepared */
    char *regex;
    jre *re;
    int *used;            /* group -> token index */
    int nused;
    int unsupported;      /* reason flag */
} fmtd;

/* TokenFormatDissector.parseTokenLogFileDefinition (:294-379) */
static void parse_token_def(fmtd *f, const tplist *tps) {
    int fn;
    int *fcp = cp_of(f->cleaned, &fn);
    toklist all = {0};
    for (int i = 0; i < tps->n; i++) collect_tokens(&tps->v[i], f->cleaned, fcp, fn, &all);
    /* stable sort */
    for (int i = 1; i < all.n; i++) {
        token t = all.v[i];
        int j = i - 1;
        while (j >= 0 && tok_cmp(&all.v[j], &t) > 0) { all.v[j + 1] = all.v[j]; j--; }
        all.v[j + 1] = t;
    }
    char *kick = (char *)xmalloc((size_t)all.n + 1);
    int prev = -1;
    for (int i = 0; i < all.n; i++) {
        token *tk = &all.v[i];
        if (prev < 0) { prev = i; continue; }
        token *pv = &all.v[prev];
        if (pv->start == tk->start) {
            if (pv->len == tk->len) {
                if (pv->prio < tk->prio) kick[prev] = 1; else kick[i] = 1;
            } else {
                if (pv->len < tk->len) kick[prev] = 1; else kick[i] = 1;
            }
        } else {
            if (pv->start + pv->len > tk->start) { kick[i] = 1; continue; }
        }
        prev = i;
    }
    toklist res = {0};
    int tend = 0;
    for (int i = 0; i < all.n; i++) {
        if (kick[i]) continue;
        token *tk = &all.v[i];
        if (tk->start - tend > 0) {
            token *fx = tk_push(&res);
            fx->fixed = 1;
            fx->regex = utf8_of(fcp + tend, tk->start - tend);
            fx->start = tk->start;
            fx->len = tk->start - tend;
        }
        *tk_push(&res) = *tk;
        tend = tk->start + tk->len;
    }
    if (tend < fn) {
        token *fx = tk_push(&res);
        fx->fixed = 1;
        fx->regex = utf8_of(fcp + tend, fn - tend);
        fx->start = tend;
        fx->len = fn - tend;
    }
    free(kick);
    free(all.v);
    free(fcp);
    f->tokens = res.v;
    f->ntokens = res.n;
    for (int i = 0; i < f->ntokens; i++) {
        token *t = &f->tokens[i];
        if (t->fixed) continue;
        for (int k = 0; k < t->nouts; k++) {
            char *s = xfmt("%s:%s", t->outs[k].type, t->outs[k].name);
            sl_add(&f->output_types, s);
            free(s);
        }
    }
}

/* ApacheHttpdLogFormatDissector.cleanupLogFormat (:121-167) */
static char *apache_cleanup(const char *fmt) {
    char *a = re_replace_all_s("%!?[0-9]{3}(?:,[0-9]{3})*", fmt, "%");
    /* makeHeaderNamesLowercaseInLogFormat: %{X}c (c != 't') -> lowercase X */
    arena ar = {0};
    jre *re = must_compile("%\\{([^}]*)}([^t])");
    js in = js_lit(&ar, a);
    int caps[6];
    int from = 0, last = 0;
    int *ob = (int *)xmalloc(sizeof(int) * (size_t)(in.n * 2 + 8));
    int on = 0;
    while (from <= in.n && jre_find(re, in.c, in.n, from, caps)) {
        for (int k = last; k < caps[0]; k++) ob[on++] = in.c[k];
        ob[on++] = '%';
        ob[on++] = '{';
        for (int k = caps[2]; k < caps[3]; k++) {
            int c = in.c[k];
            ob[on++] = (c >= 'A' && c <= 'Z') ? c + 32 : c;
        }
        ob[on++] = '}';
        ob[on++] = in.c[caps[4]];
        last = caps[1];
        from = caps[1] > caps[0] ? caps[1] : caps[1] + 1;
    }
    for (int k = last; k < in.n; k++) ob[on++] = in.c[k];
    char *b = utf8_of(ob, on);
    free(ob);
    jre_free(re);
    ar_free(&ar);
    free(a);
    char *c = re_replace_all_s("%t", b, "[%t]");
    free(b);
    return c;
}

static int ieq(const char *a, const char *b) {
    for (; *a && *b; a++, b++) {
        int x = *a, y = *b;
        if (x >= 'A' && x <= 'Z') x += 32;
        if (y >= 'A' && y <= 'Z') y += 32;
        if (x != y) return 0;
    }
    return *a == *b;
}

/* ApacheHttpdLogFormatDissector.setLogFormat alias mapping (:73-101) */
static const char *apache_alias(const char *f) {
    if (ieq(f, "common")) return "%h %l %u %t \"%r\" %>s %b";
    if (ieq(f, "combined")) return "%h %l %u %t \"%r\" %>s %b \"%{Referer}i\" \"%{User-Agent}i\"";
    if (ieq(f, "combinedio")) return "%h %l %u %t \"%r\" %>s %b \"%{Referer}i\" \"%{User-Agent}i\" %I %O";
    if (ieq(f, "referer")) return "%{Referer}i -> %U";
    if (ieq(f, "agent")) return "%{User-agent}i";
    return f;
}
static int looks_apache(const char *f) {
    return strchr(f, '%') != NULL || ieq(f, "common") || ieq(f, "combined") || ieq(f, "combinedio") || ieq(f, "referer") || ieq(f, "agent");
}
static int looks_nginx(const char *f) { return strchr(f, '$') != NULL || ieq(f, "combined"); }

static tplist g_apache_tps, g_nginx_tps;
static pthread_once_t g_tps_once = PTHREAD_ONCE_INIT;
static void init_tps(void) {
    apache_token_parsers(&g_apache_tps);
    nginx_token_parsers(&g_nginx_tps);
}

/* NginxHttpdLogFormatDissector.setLogFormat alias (hp/NginxHttpdLogFormatDissector.java:75-92) */
static const char *nginx_alias(const char *f) {
    if (ieq(f, "combined"))
        return "$remote_addr - $remote_user [$time_local] \"$request\" $status $body_bytes_sent \"$http_referer\" \"$http_user_agent\"";
    return f;
}

static fmtd *fmt_new(int kind, const char *logformat) {
    pthread_once(&g_tps_once, init_tps);
    fmtd *f = (fmtd *)xmalloc(sizeof(fmtd));
    f->kind = kind;
    if (kind == FMT_APACHE) {
        f->logformat = xstrdup(apache_alias(logformat));
        f->cleaned = apache_cleanup(f->logformat);
        parse_token_def(f, &g_apache_tps);
    } else {
        /* NGINX: no cleanup step (TokenFormatDissector.cleanupLogFormat default) */
        f->logformat = xstrdup(nginx_alias(logformat));
        f->cleaned = xstrdup(f->logformat);
        parse_token_def(f, &g_nginx_tps);
    }
    return f;
}

static fmtd *fmt_clone(const fmtd *src) { return fmt_new(src->kind, src->logformat); }

/* TokenFormatDissector.prepareForDissect (:162-174) */
static int fmt_prepare_for_dissect(fmtd *f, const char *outname) {
    sl_add_unique(&f->requested, outname);
    for (int i = 0; i < f->ntokens; i++)
        for (int k = 0; k < f->tokens[i].nouts; k++)
            if (strcmp(outname, f->tokens[i].outs[k].name) == 0) return f->tokens[i].outs[k].casts;
    return STRING_ONLY;
}

/* Pattern.quote */
static void append_quote(char **dst, size_t *dn, size_t *dcap, const char *s) {
#define APP(str) do { size_t l_ = strlen(str); while (*dn + l_ + 1 > *dcap) { *dcap *= 2; *dst = (char *)realloc(*dst, *dcap); } memcpy(*dst + *dn, str, l_); *dn += l_; (*dst)[*dn] = 0; } while (0)
    const char *e = strstr(s, "\\E");
    if (!e) { APP("\\Q"); APP(s); APP("\\E"); return; }
    APP("\\Q");
    const char *cur = s;
    while ((e = strstr(cur, "\\E")) != NULL) {
        char tmp[4096];
        snprintf(tmp, sizeof tmp, "%.*s", (int)(e - cur), cur);
        APP(tmp);
        cur = e + 2;
        APP("\\E\\\\E\\Q");
    }
    APP(cur);
    APP("\\E");
}

/* TokenFormatDissector.prepareForRun (:178-213) */
static void fmt_prepare_for_run(fmtd *f) {
    size_t cap = 256, n = 0;
    char *r = (char *)xmalloc(cap);
    r[0] = 0;
    f->used = (int *)xmalloc(sizeof(int) * (size_t)(f->ntokens + 1));
    f->nused = 0;
#define APPL(str) do { size_t l_ = strlen(str); while (n + l_ + 1 > cap) { cap *= 2; r = (char *)realloc(r, cap); } memcpy(r + n, str, l_); n += l_; r[n] = 0; } while (0)
    APPL("^");
    for (int i = 0; i < f->ntokens; i++) {
        token *t = &f->tokens[i];
        if (t->fixed) { append_quote(&r, &n, &cap, t->regex); continue; }
        int wanted = 0;
        for (int k = 0; k < t->nouts; k++) if (sl_has(&f->requested, t->outs[k].name)) wanted = 1;
        if (wanted) {
            f->used[f->nused++] = i;
            APPL("("); APPL(t->regex); APPL(")");
        } else {
            APPL("(?:"); APPL(t->regex); APPL(")");
        }
    }
    APPL("$");
#undef APPL
#undef APP
    f->regex = r;
    char err[256];
    f->re = jre_compile(r, err, sizeof err);
    if (!f->re) { fprintf(stderr, "oracle: format regex failed: %s\n%s\n", err, r); f->unsupported = 1; }
    else if (jre_ngroups(f->re) != f->nused) f->unsupported = 1; /* capturing groups inside token regexes */
}

/* ========================================================= dissectors */
enum {
    D_ROOT, D_TIMESTAMP, D_TIMESTAMP_ISO, D_FIRSTLINE, D_PROTOCOL, D_URI, D_QUERY,
    D_COOKIES, D_SETCOOKIES, D_SETCOOKIE, D_UNIQUEID, D_CLF2NUM, D_NUM2CLF,
    D_STRFTIME, D_LOCALIZED,
    D_BINIP, D_SECMILLIS, D_MS2US, D_UPSTREAM  /* NGINX createAdditionalDissectors */
};

typedef struct {
    int cls;
    char *in_type;
    char *param;         /* D_STRFTIME: the strftime pattern */
    slist outs;          /* "TYPE:name" */
    char *out_type;      /* converters */
    /* root */
    fmtd **fmts;
    int nfmts;
} dissector;

static const char *TS_OUTS[] = {
    "TIME.DAY:day", "TIME.MONTHNAME:monthname", "TIME.MONTH:month", "TIME.WEEK:weekofweekyear",
    "TIME.YEAR:weekyear", "TIME.YEAR:year", "TIME.HOUR:hour", "TIME.MINUTE:minute",
    "TIME.SECOND:second", "TIME.MILLISECOND:millisecond", "TIME.MICROSECOND:microsecond",
    "TIME.NANOSECOND:nanosecond", "TIME.DATE:date", "TIME.TIME:time", "TIME.ZONE:timezone",
    "TIME.EPOCH:epoch", "TIME.DAY:day_utc", "TIME.MONTHNAME:monthname_utc", "TIME.MONTH:month_utc",
    "TIME.WEEK:weekofweekyear_utc", "TIME.YEAR:weekyear_utc", "TIME.YEAR:year_utc",
    "TIME.HOUR:hour_utc", "TIME.MINUTE:minute_utc", "TIME.SECOND:second_utc",
    "TIME.MILLISECOND:millisecond_utc", "TIME.MICROSECOND:microsecond_utc",
    "TIME.NANOSECOND:nanosecond_utc", "TIME.DATE:date_utc", "TIME.TIME:time_utc", NULL};

static dissector *dis_new(int cls, const char *in_type) {
    dissector *d = (dissector *)xmalloc(sizeof(dissector));
    d->cls = cls;
    d->in_type = xstrdup(in_type);
    switch (cls) {
    case D_TIMESTAMP: case D_TIMESTAMP_ISO: case D_STRFTIME:
        for (int i = 0; TS_OUTS[i]; i++) sl_add(&d->outs, TS_OUTS[i]);
        break;
    case D_FIRSTLINE:
        sl_add(&d->outs, "HTTP.METHOD:method"); sl_add(&d->outs, "HTTP.URI:uri"); sl_add(&d->outs, "HTTP.PROTOCOL_VERSION:protocol");
        break;
    case D_PROTOCOL:
        sl_add(&d->outs, "HTTP.PROTOCOL:"); sl_add(&d->outs, "HTTP.PROTOCOL.VERSION:version");
        break;
    case D_URI: {
        const char *o[] = {"HTTP.PROTOCOL:protocol", "HTTP.USERINFO:userinfo", "HTTP.HOST:host", "HTTP.PORT:port",
                           "HTTP.PATH:path", "HTTP.QUERYSTRING:query", "HTTP.REF:ref", NULL};
        for (int i = 0; o[i]; i++) sl_add(&d->outs, o[i]);
        break;
    }
    case D_QUERY: sl_add(&d->outs, "STRING:*"); break;
    case D_COOKIES: sl_add(&d->outs, "HTTP.COOKIE:*"); break;
    case D_SETCOOKIES: sl_add(&d->outs, "HTTP.SETCOOKIE:*"); break;
    case D_SETCOOKIE: {
        const char *o[] = {"STRING:value", "STRING:expires", "TIME.EPOCH:expires", "STRING:path", "STRING:domain", "STRING:comment", NULL};
        for (int i = 0; o[i]; i++) sl_add(&d->outs, o[i]);
        break;
    }
    case D_UNIQUEID: {
        const char *o[] = {"TIME.EPOCH:epoch", "IP:ip", "PROCESSID:processid", "COUNTER:counter", "THREAD_INDEX:threadindex", NULL};
        for (int i = 0; o[i]; i++) sl_add(&d->outs, o[i]);
        break;
    }
    case D_LOCALIZED: sl_add(&d->outs, "TIME.LOCALIZEDSTRING:"); break;
    default: break;
    }
    return d;
}

/* TypeConvertBaseDissector (translate/TypeConvertBaseDissector.java:42-46): one
 * output "OUT:" */
static dissector *dis_conv(int cls, const char *in_type, const char *out_type) {
    dissector *d = dis_new(cls, in_type);
    d->out_type = xstrdup(out_type);
    char *o = xfmt("%s:", out_type);
    sl_add(&d->outs, o);
    free(o);
    return d;
}
/* UpstreamListDissector.getPossibleOutput (nginxmodules/UpstreamListDissector.java:127-135):
 * N.value and N.redirected for N < 32 (same type for both in every use) */
static dissector *dis_upstream(const char *in_type, const char *out_type) {
    dissector *d = dis_new(D_UPSTREAM, in_type);
    d->out_type = xstrdup(out_type);
    for (int i = 0; i < 32; i++) {
        char *o = xfmt("%s:%d.value", out_type, i);
        sl_add(&d->outs, o);
        free(o);
        o = xfmt("%s:%d.redirected", out_type, i);
        sl_add(&d->outs, o);
        free(o);
    }
    return d;
}

/* ===================================================== planner state */
typedef struct instance {
    dissector *d;
    slist requested;  /* extractFieldName(input, output) */
    /* root: own formats (getNewInstance re-registers them) */
    fmtd **fmts;
    int nfmts;
    int active;       /* sticky active format (HttpdLogFormatDissector.java:180-202) */
    int want_all;     /* query */
} instance;

typedef struct { char *id; instance **ph; int n; } centry;

struct orc_parser {
    dissector **dis;
    int ndis;
    char *root_type;
    slist needed;     /* cleaned targets */
    centry *compiled;
    int ncompiled;
    slist useful;     /* usefulIntermediateFields (names) */
    slist located;
    slist rm_in, rm_type;  /* typeRemappings as (input name, new type) pairs (core/Parser.java:639-677) */
    int unsupported;
    char unsupported_why[256];
    /* for cloning */
    char *logformat_arg;
    slist field_args;
    arena ar;
};

static centry *c_get(orc_parser *p, const char *id) {
    for (int i = 0; i < p->ncompiled; i++) if (strcmp(p->compiled[i].id, id) == 0) return &p->compiled[i];
    return NULL;
}
static centry *c_put(orc_parser *p, const char *id) {
    p->compiled = (centry *)realloc(p->compiled, sizeof(centry) * (size_t)(p->ncompiled + 1));
    centry *c = &p->compiled[p->ncompiled++];
    c->id = xstrdup(id);
    c->ph = NULL;
    c->n = 0;
    return c;
}

/* Dissector.extractFieldName (core/Dissector.java:147-157) */
static char *extract_field_name(const char *in, const char *out) {
    if (strcmp(in, out) == 0) return xstrdup("");
    if (in[0]) return xstrdup(out + strlen(in) + 1);
    return xstrdup(out);
}

static instance *inst_new(dissector *d) {
    instance *in = (instance *)xmalloc(sizeof(instance));
    in->d = d;
    if (d->cls == D_ROOT) {
        in->nfmts = d->nfmts;
        in->fmts = (fmtd **)xmalloc(sizeof(fmtd *) * (size_t)(d->nfmts + 1));
        for (int i = 0; i < d->nfmts; i++) in->fmts[i] = fmt_clone(d->fmts[i]);
        in->active = -1;
    }
    return in;
}

/* ---------------------------------------------------------- strftime
 * StrfTimeToDateTimeFormatter (hp/dissectors/StrfTimeToDateTimeFormatter.java
 * :140-432, grammar StrfTime.g4:40-89) restated as the DateTimeFormatterBuilder
 * elements each conversion appends, parsed as JDK 8's DateTimeFormatter parses
 * them (parseCaseInsensitive, strict, default locale en_US) and resolved as
 * JDK 8's java.time.format.Parsed.resolve does (ResolverStyle.SMART), see
 * strf_parse below.  E / O modifiers are ignored (StrfTime.g4 MOD).
 *   %a %A   DAY_OF_WEEK text SHORT / FULL        %b %h %B  MONTH_OF_YEAR text
 *   %d %m   DAY_OF_MONTH / MONTH_OF_YEAR, 2       %Y       YEAR, 4
 *   %y      YEAR reduced (2 digits, base 2000)    %D       %m/%d/%y
 *   %e      padNext(2,' ') DAY_OF_MONTH           %F       %Y-%m-%d
 *   %H      CLOCK_HOUR_OF_DAY, 2                  %k       padNext(2,' ') CLOCK_HOUR_OF_DAY
 *   %I      CLOCK_HOUR_OF_AMPM, 2                 %l       padNext(2,' ') CLOCK_HOUR_OF_AMPM
 *   %p      AMPM_OF_DAY text "AM"/"PM"            %P       AMPM_OF_DAY text "am"/"pm"
 *   %M %S   MINUTE_OF_HOUR / SECOND_OF_MINUTE, 2  %T %R    HOUR_OF_DAY:%M[:%S]
 *   %r      %I:%M:%S %p                           %j       DAY_OF_YEAR, 3
 *   %s      INSTANT_SECONDS, 1..19 digits         %u       WeekFields.ISO.dayOfWeek(), 1
 *   %V %W   WeekFields.ISO.weekOfYear(), 1..19 / 2
 *   %G %g   WeekFields.of(en_US).weekBasedYear(), 4 / reduced 2 (base 2000)
 *   %z      appendOffset("+HHMM", "+0000")        %Z       appendZoneText(SHORT)
 *   [%]msec_frac / [%]usec_frac  MILLI_ / MICRO_OF_SECOND, 3 / 6
 * %c %C %U %w %x %X %+ throw UnsupportedStrfField in the reference (the
 * parser cannot be built): outside the restatement (ORC_UNSUPPORTED), as is
 * a variable-width number directly followed by another number (JDK adjacent
 * value parsing).  No %z / %Z: the formatter is withZone(UTC) (:97-105). */
enum { SF_YEAR, SF_MONTH, SF_DOM, SF_DOW, SF_ISODOW, SF_DOY, SF_WBY, SF_WOY, SF_HOD, SF_CHOD, SF_CHAP, SF_AMPM,
       SF_MIN, SF_SEC, SF_MILLI, SF_MICRO, SF_INSTANT, SF_OFFSET, SF_NFIELDS };
/* elements: literal char, fixed-width number, 1..19-digit number,
 * padNext(2,' ') + 1..19-digit number, 2-digit reduced value (base 2000),
 * text table, offset +HHMM, zone text */
enum { SE_LIT, SE_NUM, SE_NUMV, SE_PAD2, SE_RED2, SE_TEXT, SE_OFF, SE_ZONE };
enum { TT_MON_SHORT, TT_MON_FULL, TT_DOW_SHORT, TT_DOW_FULL, TT_AMPM_UP, TT_AMPM_LOW };
typedef struct { unsigned char kind, field, width, arg; } strf_el;
typedef struct { strf_el el[96]; int nel, zone; } strf_prog;

static int strf_add(strf_prog *sp, int kind, int field, int width, int arg) {
    if (sp->nel >= 96) return 0;
    strf_el *e = &sp->el[sp->nel++];
    e->kind = (unsigned char)kind; e->field = (unsigned char)field; e->width = (unsigned char)width; e->arg = (unsigned char)arg;
    return 1;
}

static int strf_compile(const char *f, strf_prog *sp) {
    memset(sp, 0, sizeof *sp);
    size_t n = strlen(f);
#define NUM(fl, w) strf_add(sp, SE_NUM, fl, w, 0)
#define LIT(c) strf_add(sp, SE_LIT, 0, 1, (unsigned char)(c))
    for (size_t i = 0; i < n;) {
        /* MsecFrac / UsecFrac : '%'? 'msec_frac' (longest match wins over LITERAL) */
        size_t j = i + (f[i] == '%');
        if (n - j >= 9 && (!strncmp(f + j, "msec_frac", 9) || !strncmp(f + j, "usec_frac", 9))) {
            if (!(f[j] == 'm' ? NUM(SF_MILLI, 3) : NUM(SF_MICRO, 6))) return 0;
            i = j + 9;
            continue;
        }
        if (f[i] != '%') { if (!LIT(f[i])) return 0; i++; continue; }
        if (i + 1 >= n) return 0;
        char c = f[i + 1];
        if (c == '%') { if (!LIT('%')) return 0; i += 2; continue; }
        if (c == 't') { if (!LIT('\t')) return 0; i += 2; continue; }
        if (c == 'n') { if (!LIT('\n')) return 0; i += 2; continue; }
        size_t k = i + 1;
        if (c == 'E' || c == 'O') { if (i + 2 >= n) return 0; c = f[i + 2]; k++; }
        int ok = 1;
        switch (c) {
        case 'a': ok = strf_add(sp, SE_TEXT, SF_DOW, 0, TT_DOW_SHORT); break;
        case 'A': ok = strf_add(sp, SE_TEXT, SF_DOW, 0, TT_DOW_FULL); break;
        case 'b': case 'h': ok = strf_add(sp, SE_TEXT, SF_MONTH, 0, TT_MON_SHORT); break;
        case 'B': ok = strf_add(sp, SE_TEXT, SF_MONTH, 0, TT_MON_FULL); break;
        case 'd': ok = NUM(SF_DOM, 2); break;
        case 'D': ok = NUM(SF_MONTH, 2) && LIT('/') && NUM(SF_DOM, 2) && LIT('/') && strf_add(sp, SE_RED2, SF_YEAR, 2, 0); break;
        case 'e': ok = strf_add(sp, SE_PAD2, SF_DOM, 2, 0); break;
        case 'F': ok = NUM(SF_YEAR, 4) && LIT('-') && NUM(SF_MONTH, 2) && LIT('-') && NUM(SF_DOM, 2); break;
        case 'G': ok = NUM(SF_WBY, 4); break;
        case 'g': ok = strf_add(sp, SE_RED2, SF_WBY, 2, 0); break;
        case 'H': ok = NUM(SF_CHOD, 2); break;
        case 'I': ok = NUM(SF_CHAP, 2); break;
        case 'j': ok = NUM(SF_DOY, 3); break;
        case 'k': ok = strf_add(sp, SE_PAD2, SF_CHOD, 2, 0); break;
        case 'l': ok = strf_add(sp, SE_PAD2, SF_CHAP, 2, 0); break;
        case 'm': ok = NUM(SF_MONTH, 2); break;
        case 'M': ok = NUM(SF_MIN, 2); break;
        case 'p': ok = strf_add(sp, SE_TEXT, SF_AMPM, 0, TT_AMPM_UP); break;
        case 'P': ok = strf_add(sp, SE_TEXT, SF_AMPM, 0, TT_AMPM_LOW); break;
        case 'r': ok = NUM(SF_CHAP, 2) && LIT(':') && NUM(SF_MIN, 2) && LIT(':') && NUM(SF_SEC, 2) && LIT(' ') &&
                       strf_add(sp, SE_TEXT, SF_AMPM, 0, TT_AMPM_UP); break;
        case 'R': ok = NUM(SF_HOD, 2) && LIT(':') && NUM(SF_MIN, 2); break;
        case 's': ok = strf_add(sp, SE_NUMV, SF_INSTANT, 19, 0); break;
        case 'S': ok = NUM(SF_SEC, 2); break;
        case 'T': ok = NUM(SF_HOD, 2) && LIT(':') && NUM(SF_MIN, 2) && LIT(':') && NUM(SF_SEC, 2); break;
        case 'u': ok = NUM(SF_ISODOW, 1); break;
        case 'V': ok = strf_add(sp, SE_NUMV, SF_WOY, 19, 0); break;
        case 'W': ok = NUM(SF_WOY, 2); break;
        case 'y': ok = strf_add(sp, SE_RED2, SF_YEAR, 2, 0); break;
        case 'Y': ok = NUM(SF_YEAR, 4); break;
        case 'z': ok = strf_add(sp, SE_OFF, SF_OFFSET, 5, 0); sp->zone = 1; break;
        case 'Z': ok = strf_add(sp, SE_ZONE, 0, 0, 0); sp->zone = 1; break;
        default: return 0; /* %c %C %U %w %x %X %+ (UnsupportedStrfField) or a syntax error */
        }
        if (!ok) return 0;
        i = k + 1;
    }
#undef NUM
#undef LIT
    /* adjacent value parsing (DateTimeFormatterBuilder.appendValue): a
     * variable-width number directly followed by another number */
    for (int e = 0; e + 1 < sp->nel; e++) {
        const int k0 = sp->el[e].kind, k1 = sp->el[e + 1].kind;
        const int num1 = k1 == SE_NUM || k1 == SE_NUMV || k1 == SE_PAD2 || k1 == SE_RED2;
        if ((k0 == SE_NUMV || k0 == SE_PAD2) && num1) return 0;
    }
    return 1;
}

static void inst_prepare(orc_parser *p, instance *in, const char *subroot, const char *check) {
    char *name = extract_field_name(subroot, check);
    sl_add_unique(&in->requested, name);
    if (in->d->cls == D_ROOT)
        for (int i = 0; i < in->nfmts; i++) fmt_prepare_for_dissect(in->fmts[i], check);
    switch (in->d->cls) {
    case D_STRFTIME: {
        strf_prog sp;
        if (!strf_compile(in->d->param, &sp) && !p->unsupported) {
            p->unsupported = 1;
            snprintf(p->unsupported_why, sizeof p->unsupported_why, "strftime pattern outside the restated subset: %s",
                     in->d->param);
        }
        break;
    }
    case D_LOCALIZED: break;
    case D_UNIQUEID:
        if (!p->unsupported) {
            p->unsupported = 1;
            snprintf(p->unsupported_why, sizeof p->unsupported_why, "unsupported dissector for input type %s", in->d->in_type);
        }
        break;
    default: break;
    }
    free(name);
}

/* Parser.findUsefulDissectorsFromField (core/Parser.java:360-458) */
static void find_useful(orc_parser *p, slist *possible, const char *sr_type, const char *sr_name, int is_root) {
    char *srid = xfmt("%s:%s", sr_type, sr_name);
    if (sl_has(&p->located, srid)) { free(srid); return; }
    sl_add(&p->located, srid);
    for (int di = 0; di < p->ndis; di++) {
        dissector *d = p->dis[di];
        if (strcmp(d->in_type, sr_type) != 0) continue;
        for (int oi = 0; oi < d->outs.n; oi++) {
            const char *out = d->outs.v[oi];
            const char *colon = strchr(out, ':');
            char *otype = xfmt("%.*s", (int)(colon - out), out);
            const char *oname = colon + 1;
            slist checks = {0};
            if (strcmp(oname, "*") == 0) {
                char *pre = xfmt("%s.", sr_name);
                for (int k = 0; k < possible->n; k++)
                    if (strncmp(possible->v[k], pre, strlen(pre)) == 0) sl_add_unique(&checks, possible->v[k]);
                free(pre);
            } else if (is_root) {
                sl_add(&checks, oname);
            } else if (oname[0] == 0) {
                sl_add(&checks, sr_name);
            } else {
                char *c = xfmt("%s.%s", sr_name, oname);
                sl_add(&checks, c);
                free(c);
            }
            for (int k = 0; k < checks.n; k++) {
                const char *cf = checks.v[k];
                char *cid = xfmt("%s:%s", otype, cf);
                if (sl_has(possible, cf) && !c_get(p, cid)) {
                    centry *ce = c_get(p, srid);
                    if (!ce) { ce = c_put(p, srid); sl_add_unique(&p->useful, sr_name); }
                    instance *in = NULL;
                    for (int q = 0; q < ce->n; q++) if (ce->ph[q]->d->cls == d->cls) in = ce->ph[q];
                    if (!in) {
                        in = inst_new(d);
                        ce = c_get(p, srid);
                        ce->ph = (instance **)realloc(ce->ph, sizeof(instance *) * (size_t)(ce->n + 1));
                        ce->ph[ce->n++] = in;
                    }
                    inst_prepare(p, in, sr_name, cf);
                    find_useful(p, possible, otype, cf, 0);
                }
                free(cid);
            }
            sl_free(&checks);
            free(otype);
        }
    }
    /* the new types of a remapped name get their dissectors (core/Parser.java:447-455) */
    for (int k = 0; k < p->rm_in.n; k++) {
        if (strcmp(p->rm_in.v[k], sr_name) != 0) continue;
        char *mid = xfmt("%s:%s", p->rm_type.v[k], sr_name);
        if (!c_get(p, mid)) find_useful(p, possible, p->rm_type.v[k], sr_name, 0);
        free(mid);
    }
    free(srid);
}

/* Parser.cleanupFieldValue (core/Parser.java:681-691) */
static char *cleanup_field(const char *f) {
    const char *c = strchr(f, ':');
    char *r = xstrdup(f);
    if (!c) { ascii_lower(r); return r; }
    size_t k = (size_t)(c - f);
    for (size_t i = 0; i < k; i++) if (r[i] >= 'a' && r[i] <= 'z') r[i] -= 32;
    ascii_lower(r + k + 1);
    return r;
}

/* HttpdLoglineParser.setupDissectors + HttpdLogFormatDissector ctor */
static int build_dissectors(orc_parser *p, const char *logformat, char *err, int errlen) {
    dissector *root = dis_new(D_ROOT, "HTTPLOGLINE");
    /* addMultipleLogFormats: split("\\r?\\n") */
    char *copy = xstrdup(logformat);
    slist formats = {0};
    int jetty = 0;
    char *s = copy;
    for (;;) {
        char *nl = strchr(s, '\n');
        if (nl) { *nl = 0; if (nl > s && nl[-1] == '\r') nl[-1] = 0; }
        /* addLogFormat (:110-140) */
        int blank = 1;
        for (char *q = s; *q; q++) if (!(*q == ' ' || *q == '\t' || *q == '\r' || *q == '\n' || *q == '\f' || *q == 0x0B)) blank = 0;
        if (!blank) {
            char *up = xstrdup(s);
            ascii_upper(up);
            char *t = up; while (*t == ' ' || *t == '\t') t++;
            char *e = t + strlen(t); while (e > t && (e[-1] == ' ' || e[-1] == '\t')) *--e = 0;
            if (strcmp(t, "ENABLE JETTY FIX") == 0) jetty = 1;
            else if (!sl_has(&formats, s)) sl_add(&formats, s);
            free(up);
        }
        if (!nl) break;
        s = nl + 1;
    }
    free(copy);
    if (jetty) {
        /* addAdditionalLogFormatsToHandleJettyUseragentProblem
         * (hp/HttpdLogFormatDissector.java:72-92): over getAllLogFormats() (the
         * alias-expanded format of every registered dissector, :254-262),
         * first "\"%{User-Agent}i\"" -> "\"%{User-Agent}i\" ", then (over
         * the grown list) "%u" -> " %u "; String.replace = every occurrence;
         * addLogFormat skips a format string already registered */
        static const char *from[2] = {"\"%{User-Agent}i\"", "%u"}, *to[2] = {"\"%{User-Agent}i\" ", " %u "};
        for (int pass = 0; pass < 2; pass++) {
            int n0 = formats.n;
            for (int i = 0; i < n0; i++) {
                int kind = looks_apache(formats.v[i]) ? FMT_APACHE : looks_nginx(formats.v[i]) ? FMT_NGINX : 0;
                if (!kind) continue;
                const char *lf = kind == FMT_APACHE ? apache_alias(formats.v[i]) : nginx_alias(formats.v[i]);
                if (!strstr(lf, from[pass])) continue;
                size_t fl = strlen(from[pass]), tl = strlen(to[pass]), n = 0;
                char *out = (char *)xmalloc(strlen(lf) * 3 + 8);
                for (const char *q = lf; *q;) {
                    if (!strncmp(q, from[pass], fl)) { memcpy(out + n, to[pass], tl); n += tl; q += fl; }
                    else out[n++] = *q++;
                }
                out[n] = 0;
                if (!sl_has(&formats, out)) sl_add(&formats, out);
                free(out);
            }
        }
    }
    root->fmts = (fmtd **)xmalloc(sizeof(fmtd *) * (size_t)(formats.n + 1));
    for (int i = 0; i < formats.n; i++) {
        int kind = looks_apache(formats.v[i]) ? FMT_APACHE : looks_nginx(formats.v[i]) ? FMT_NGINX : 0;
        if (!kind) continue;
        fmtd *f = fmt_new(kind, formats.v[i]);
        root->fmts[root->nfmts++] = f;
        for (int k = 0; k < f->output_types.n; k++) sl_add_unique(&root->outs, f->output_types.v[k]);
    }
    sl_free(&formats);
    int nd = 0;
    p->dis = (dissector **)xmalloc(sizeof(dissector *) * 64);
    p->dis[nd++] = root;
    p->dis[nd++] = dis_new(D_TIMESTAMP, "TIME.STAMP");
    p->dis[nd++] = dis_new(D_TIMESTAMP_ISO, "TIME.ISO8601");
    p->dis[nd++] = dis_new(D_FIRSTLINE, "HTTP.FIRSTLINE");
    p->dis[nd++] = dis_new(D_PROTOCOL, "HTTP.PROTOCOL_VERSION");
    p->dis[nd++] = dis_new(D_URI, "HTTP.URI");
    p->dis[nd++] = dis_new(D_QUERY, "HTTP.QUERYSTRING");
    p->dis[nd++] = dis_new(D_COOKIES, "HTTP.COOKIES");
    p->dis[nd++] = dis_new(D_SETCOOKIES, "HTTP.SETCOOKIES");
    p->dis[nd++] = dis_new(D_SETCOOKIE, "HTTP.SETCOOKIE");
    p->dis[nd++] = dis_new(D_UNIQUEID, "MOD_UNIQUE_ID");
    dissector *c2n = dis_new(D_CLF2NUM, "BYTESCLF");
    c2n->out_type = xstrdup("BYTES");
    sl_add(&c2n->outs, "BYTES:");
    p->dis[nd++] = c2n;
    dissector *n2c = dis_new(D_NUM2CLF, "BYTES");
    n2c->out_type = xstrdup("BYTESCLF");
    sl_add(&n2c->outs, "BYTESCLF:");
    p->dis[nd++] = n2c;
    /* NginxHttpdLogFormatDissector.createAdditionalDissectors
     * (hp/NginxHttpdLogFormatDissector.java:144-152 + UpstreamModule.getDissectors,
     * nginxmodules/UpstreamModule.java:163-198), once for any NGINX format */
    int any_nginx = 0;
    for (int i = 0; i < root->nfmts; i++) any_nginx |= root->fmts[i]->kind == FMT_NGINX;
    if (any_nginx) {
        dissector *b = dis_new(D_BINIP, "IP_BINARY");
        sl_add(&b->outs, "IP:");
        p->dis[nd++] = b;
        p->dis[nd++] = dis_conv(D_SECMILLIS, "SECOND_MILLIS", "MILLISECONDS");
        p->dis[nd++] = dis_conv(D_SECMILLIS, "TIME.EPOCH_SECOND_MILLIS", "TIME.EPOCH");
        p->dis[nd++] = dis_conv(D_MS2US, "MILLISECONDS", "MICROSECONDS");
        p->dis[nd++] = dis_upstream("UPSTREAM_ADDR_LIST", "UPSTREAM_ADDR");
        p->dis[nd++] = dis_upstream("UPSTREAM_BYTES_LIST", "BYTES");
        p->dis[nd++] = dis_upstream("UPSTREAM_SECOND_MILLIS_LIST", "SECOND_MILLIS");
        p->dis[nd++] = dis_upstream("UPSTREAM_STATUS_LIST", "UPSTREAM_STATUS");
    }
    /* createAdditionalDissectors (core/Parser.java:281-292): token custom
     * dissectors (StrfTimeStampDissector) + LocalizedTimeDissector */
    for (int i = 0; i < root->nfmts; i++) {
        fmtd *f = root->fmts[i];
        for (int k = 0; k < f->ntokens; k++) {
            if (f->tokens[k].custom == CUSTOM_STRFTIME && nd < 60) {
                p->dis[nd] = dis_new(D_STRFTIME, f->tokens[k].custom_type);
                p->dis[nd++]->param = xstrdup(f->tokens[k].custom_param);
                p->dis[nd++] = dis_new(D_LOCALIZED, f->tokens[k].custom_type);
            }
        }
    }
    p->ndis = nd;
    p->root_type = xstrdup("HTTPLOGLINE");
    return 0;
}

/* ============================================================ runtime */
enum { V_STRING = 0, V_LONG = 1 };
typedef struct { int filled; js s; int64_t l; int lnull; } val;

static val vstr(js s) { val v; memset(&v, 0, sizeof v); v.filled = V_STRING; v.s = s; return v; }
static val vlong(int64_t l) { val v; memset(&v, 0, sizeof v); v.filled = V_LONG; v.l = l; return v; }

/* Value.getString (core/Value.java:48-57) */
static js v_getstring(arena *a, val v) {
    if (v.filled == V_STRING) return v.s;
    if (v.lnull) return js_null();
    char b[32];
    snprintf(b, sizeof b, "%lld", (long long)v.l);
    return js_lit(a, b);
}

typedef struct { char *type; char *name; val v; } pfield;
typedef struct { char *name; val v; int seq; } rentry;

typedef struct {
    orc_parser *p;
    arena *a;
    pfield *cache; int ncache, capcache;
    pfield *todo; int ntodo, captodo;
    rentry *rec; int nrec, caprec;
    int failed;
    int unsupported;
} parsable;

static void cache_put(parsable *ps, const char *type, const char *name, val v) {
    for (int i = 0; i < ps->ncache; i++)
        if (strcmp(ps->cache[i].type, type) == 0 && strcmp(ps->cache[i].name, name) == 0) { ps->cache[i].v = v; return; }
    if (ps->ncache == ps->capcache) { ps->capcache = ps->capcache ? ps->capcache * 2 : 32; ps->cache = (pfield *)realloc(ps->cache, sizeof(pfield) * (size_t)ps->capcache); }
    char *t = (char *)ar_alloc(ps->a, strlen(type) + 1); strcpy(t, type);
    char *n = (char *)ar_alloc(ps->a, strlen(name) + 1); strcpy(n, name);
    ps->cache[ps->ncache].type = t;
    ps->cache[ps->ncache].name = n;
    ps->cache[ps->ncache].v = v;
    ps->ncache++;
}
static val *cache_get(parsable *ps, const char *type, const char *name) {
    for (int i = 0; i < ps->ncache; i++)
        if (strcmp(ps->cache[i].type, type) == 0 && strcmp(ps->cache[i].name, name) == 0) return &ps->cache[i].v;
    return NULL;
}
static void todo_add(parsable *ps, const char *type, const char *name) {
    if (ps->ntodo == ps->captodo) { ps->captodo = ps->captodo ? ps->captodo * 2 : 32; ps->todo = (pfield *)realloc(ps->todo, sizeof(pfield) * (size_t)ps->captodo); }
    char *t = (char *)ar_alloc(ps->a, strlen(type) + 1); strcpy(t, type);
    char *n = (char *)ar_alloc(ps->a, strlen(name) + 1); strcpy(n, name);
    ps->todo[ps->ntodo].type = t;
    ps->todo[ps->ntodo].name = n;
    ps->ntodo++;
}
static void rec_add(parsable *ps, const char *name, val v) {
    if (ps->nrec == ps->caprec) { ps->caprec = ps->caprec ? ps->caprec * 2 : 64; ps->rec = (rentry *)realloc(ps->rec, sizeof(rentry) * (size_t)ps->caprec); }
    char *n = (char *)ar_alloc(ps->a, strlen(name) + 1); strcpy(n, name);
    ps->rec[ps->nrec].name = n;
    ps->rec[ps->nrec].v = v;
    ps->rec[ps->nrec].seq = ps->nrec;
    ps->nrec++;
}

/* Parsable.addDissection (core/Parsable.java:142-193): with recursion 0, a
 * remapped name's value is first added again under each new type
 * (:160-176; the same type is a DissectionFailure) */
static void add_dissection_r(parsable *ps, const char *base, const char *type, const char *name, val v, int recursion);
static void add_dissection(parsable *ps, const char *base, const char *type, const char *name, val v) {
    add_dissection_r(ps, base, type, name, v, 0);
}
static void add_dissection_r(parsable *ps, const char *base, const char *type, const char *name, val v, int recursion) {
    char complete[1024], wild[1024], needed[1024];
    if (base[0] == 0) {
        snprintf(complete, sizeof complete, "%s", name);
        snprintf(wild, sizeof wild, "%s:*", type);
    } else {
        if (name[0] == 0) snprintf(complete, sizeof complete, "%s", base);
        else snprintf(complete, sizeof complete, "%s.%s", base, name);
        snprintf(wild, sizeof wild, "%s:%s.*", type, base);
    }
    snprintf(needed, sizeof needed, "%s:%s", type, complete);
    if (!recursion)
        for (int k = 0; k < ps->p->rm_in.n; k++) {
            if (strcmp(ps->p->rm_in.v[k], complete) != 0) continue;
            if (strcmp(ps->p->rm_type.v[k], type) == 0) { ps->failed = 1; return; }
            add_dissection_r(ps, base, ps->p->rm_type.v[k], name, v, 1);
        }
    if (sl_has(&ps->p->useful, complete)) {
        cache_put(ps, type, complete, v);
        todo_add(ps, type, complete);
    }
    if (sl_has(&ps->p->needed, needed)) rec_add(ps, needed, v);
    if (sl_has(&ps->p->needed, wild)) rec_add(ps, needed, v);
}

static void add_str(parsable *ps, const char *base, const char *type, const char *name, js s) {
    add_dissection(ps, base, type, name, vstr(s));
}
static void add_long(parsable *ps, const char *base, const char *type, const char *name, int64_t l) {
    add_dissection(ps, base, type, name, vlong(l));
}
static char *js_cstr(parsable *ps, js s) { return js_to_utf8(ps->a, s, NULL); }

/* ------------------------------------------------------ root / format */
/* ApacheHttpdLogFormatDissector.decodeExtractedValue (:169-196): note the
 * condition tests the VALUE (not the token name), as the reference does. */
static int apache_decode(parsable *ps, js value, js *out) {
    if (value.null || value.n == 0) { *out = value; return 0; }
    if (js_eq_lit(value, "-")) { *out = js_null(); return 0; }
    if (js_eq_lit(value, "request.firstline") || js_starts_lit(value, "request.header.") || js_starts_lit(value, "response.header.")) {
        if (js_index_of_char(value, '\\', 0) >= 0) { ps->unsupported = 1; return -1; }
    }
    *out = value;
    return 0;
}

/* TokenFormatDissector.dissect (:243-275); returns 1 on match */
static int fmt_dissect(parsable *ps, fmtd *f, js line, const char *inputname) {
    if (f->unsupported) { ps->unsupported = 1; return 0; }
    int caps[2 * 128];
    if (f->nused >= 127) { ps->unsupported = 1; return 0; }
    if (!jre_find(f->re, line.c, line.n, 0, caps)) return 0;
    for (int g = 1; g <= f->nused; g++) {
        token *t = &f->tokens[f->used[g - 1]];
        js grp = caps[2 * g] < 0 ? js_null() : js_sub(line, caps[2 * g], caps[2 * g + 1]);
        for (int k = 0; k < t->nouts; k++) {
            js dec;
            if (f->kind == FMT_APACHE) { if (apache_decode(ps, grp, &dec) < 0) return 1; }
            else dec = js_eq_lit(grp, "-") ? js_null() : grp; /* NginxHttpdLogFormatDissector.java:107-119 */
            add_str(ps, inputname, t->outs[k].type, t->outs[k].name, dec);
        }
    }
    return 1;
}

/* HttpdLogFormatDissector.dissect (:173-204) */
static void d_root(parsable *ps, instance *in, const char *inputname) {
    val *v = cache_get(ps, "HTTPLOGLINE", inputname);
    js line = v_getstring(ps->a, *v);
    if (in->nfmts == 0) { ps->failed = 1; return; }
    if (in->active < 0) in->active = 0;
    if (fmt_dissect(ps, in->fmts[in->active], line, inputname)) return;
    if (ps->unsupported) return;
    if (in->nfmts > 1) {
        for (int i = 0; i < in->nfmts; i++) {
            if (fmt_dissect(ps, in->fmts[i], line, inputname)) { in->active = i; return; }
            if (ps->unsupported) return;
        }
    }
    ps->failed = 1;
}

/* ------------------------------------------------------------- time */
static int64_t days_from_civil(int64_t y, int m, int d) {
    y -= m <= 2;
    const int64_t era = (y >= 0 ? y : y - 399) / 400;
    const int64_t yoe = y - era * 400;
    const int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
    const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    return era * 146097 + doe - 719468;
}
static void civil_from_days(int64_t z, int64_t *y, int *m, int *d) {
    z += 719468;
    const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
    const int64_t doe = z - era * 146097;
    const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    const int64_t yy = yoe + era * 400;
    const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
    const int64_t mp = (5 * doy + 2) / 153;
    *d = (int)(doy - (153 * mp + 2) / 5 + 1);
    *m = (int)(mp < 10 ? mp + 3 : mp - 9);
    *y = yy + (*m <= 2);
}
static int is_leap(int64_t y) { return (y % 4 == 0 && y % 100 != 0) || y % 400 == 0; }
static int month_len(int64_t y, int m) {
    static const int ml[] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
    return m == 2 ? (is_leap(y) ? 29 : 28) : ml[m - 1];
}
/* ISO-8601 week fields (WeekFields.ISO == WeekFields.of(Locale.UK)) */
static void iso_week(int64_t y, int m, int d, int64_t *wy, int *wk) {
    int64_t days = days_from_civil(y, m, d);
    int wd = (int)(((days % 7) + 7 + 3) % 7) + 1; /* 1970-01-01 = Thursday; Mon=1 */
    int doy = (int)(days - days_from_civil(y, 1, 1)) + 1;
    int w = (doy - wd + 10) / 7;
    if (w < 1) {
        int64_t py = y - 1;
        int64_t jan1 = days_from_civil(py, 1, 1);
        int jwd = (int)(((jan1 % 7) + 7 + 3) % 7) + 1;
        int weeks = (jwd == 4 || (jwd == 3 && is_leap(py))) ? 53 : 52;
        *wy = py; *wk = weeks;
        return;
    }
    int64_t jan1 = days_from_civil(y, 1, 1);
    int jwd = (int)(((jan1 % 7) + 7 + 3) % 7) + 1;
    int weeks = (jwd == 4 || (jwd == 3 && is_leap(y))) ? 53 : 52;
    if (w > weeks) { *wy = y + 1; *wk = 1; return; }
    *wy = y; *wk = w;
}

static const char *MONTH_SHORT[] = {"Jan", "Feb", "Mar", "Apr", "May", "Jun", "Jul", "Aug", "Sep", "Oct", "Nov", "Dec"};
static const char *MONTH_FULL[] = {"January", "February", "March", "April", "May", "June", "July", "August", "September", "October", "November", "December"};

static int dig(int c) { return c >= '0' && c <= '9' ? c - '0' : -1; }

/* DateTimeFormatter "dd/MMM/yyyy:HH:mm:ss ZZ" (parseCaseInsensitive,
 * Locale.UK, SMART resolver) -- TimeStampDissector.java:46,100-109,418.
 * Returns 0 ok, 1 DateTimeParseException. */
static int parse_apache_time(js s, int64_t *ly, int *lm, int *ld, int *lh, int *lmi, int *ls, int *offset_secs) {
    if (s.n != 26) return 1;
    const int *c = s.c;
    int d1 = dig(c[0]), d2 = dig(c[1]);
    if (d1 < 0 || d2 < 0 || c[2] != '/') return 1;
    int day = d1 * 10 + d2;
    int month = -1;
    for (int m = 0; m < 12; m++) {
        int ok = 1;
        for (int k = 0; k < 3; k++) {
            int x = c[3 + k], y = MONTH_SHORT[m][k];
            if (x >= 'a' && x <= 'z') x -= 32;
            if (y >= 'a' && y <= 'z') y -= 32;
            if (x != y) ok = 0;
        }
        if (ok) { month = m + 1; break; }
    }
    if (month < 0 || c[6] != '/') return 1;
    int64_t year = 0;
    for (int k = 0; k < 4; k++) { int v = dig(c[7 + k]); if (v < 0) return 1; year = year * 10 + v; }
    if (c[11] != ':') return 1;
    int hh = dig(c[12]) * 10 + dig(c[13]);
    if (dig(c[12]) < 0 || dig(c[13]) < 0 || c[14] != ':') return 1;
    int mi = dig(c[15]) * 10 + dig(c[16]);
    if (dig(c[15]) < 0 || dig(c[16]) < 0 || c[17] != ':') return 1;
    int ss = dig(c[18]) * 10 + dig(c[19]);
    if (dig(c[18]) < 0 || dig(c[19]) < 0 || c[20] != ' ') return 1;
    /* OffsetIdPrinterParser("+HHMM","+0000") */
    int off;
    if (c[21] == '+' && c[22] == '0' && c[23] == '0' && c[24] == '0' && c[25] == '0') off = 0;
    else {
        if (c[21] != '+' && c[21] != '-') return 1;
        int oh1 = dig(c[22]), oh2 = dig(c[23]), om1 = dig(c[24]), om2 = dig(c[25]);
        if (oh1 < 0 || oh2 < 0 || om1 < 0 || om2 < 0) return 1;
        int oh = oh1 * 10 + oh2, om = om1 * 10 + om2;
        if (oh > 59 || om > 59) return 1;
        off = (c[21] == '-' ? -1 : 1) * (oh * 3600 + om * 60);
    }
    /* resolve: ZoneOffset.ofTotalSeconds range */
    if (off > 18 * 3600 || off < -18 * 3600) return 1;
    /* resolveDate: DAY_OF_MONTH 1..31, MONTH 1..12; SMART clamps to month length */
    if (day < 1 || day > 31) return 1;
    int ml = month_len(year, month);
    if (day > ml) day = ml;
    /* resolveTime: MINUTE 0..59, SMART 24:00:00 = end of day */
    if (mi > 59) return 1;
    int plus_day = 0;
    if (hh == 24 && mi == 0 && ss == 0) { hh = 0; plus_day = 1; }
    else {
        if (hh > 23) return 1;
        if (ss > 59) return 1;
    }
    if (plus_day) {
        int64_t days = days_from_civil(year, month, day) + 1;
        civil_from_days(days, &year, &month, &day);
    }
    *ly = year; *lm = month; *ld = day; *lh = hh; *lmi = mi; *ls = ss; *offset_secs = off;
    return 0;
}

/* TimeStampDissector("TIME.ISO8601", "yyyy-MM-dd'T'HH:mm:ssXXX") (hp/HttpdLoglineParser.java:110,
 * TimeStampDissector.java:100-108): parseCaseInsensitive + appendPattern, SMART
 * resolver.  YEAR_OF_ERA 4+ digits (the token regex gives exactly 4),
 * MONTH_OF_YEAR / DAY_OF_MONTH / HOUR_OF_DAY / MINUTE / SECOND two digits,
 * appendOffset("+HH:MM", "Z") (each number <= 59, total within +-18:00);
 * resolution as in parse_apache_time (month 1..12, day 1..31 clamped to the
 * month, 24:00:00 = next day). */
static int parse_iso_time(js s, int64_t *ly, int *lm, int *ld, int *lh, int *lmi, int *ls, int *offset_secs) {
    if (s.n != 25) return 1;
    const int *c = s.c;
    int64_t year = 0;
    for (int k = 0; k < 4; k++) { int v = dig(c[k]); if (v < 0) return 1; year = year * 10 + v; }
    if (c[4] != '-' || c[7] != '-' || c[10] != 'T' || c[13] != ':' || c[16] != ':' || c[22] != ':') return 1;
    const int idx[] = {5, 8, 11, 14, 17, 20, 23};
    int v[7];
    for (int k = 0; k < 7; k++) {
        int a = dig(c[idx[k]]), b = dig(c[idx[k] + 1]);
        if (a < 0 || b < 0) return 1;
        v[k] = a * 10 + b;
    }
    if (c[19] != '+' && c[19] != '-') return 1;
    if (v[5] > 59 || v[6] > 59) return 1;
    int off = (c[19] == '-' ? -1 : 1) * (v[5] * 3600 + v[6] * 60);
    if (off > 18 * 3600 || off < -18 * 3600) return 1;
    int month = v[0], day = v[1], hh = v[2], mi = v[3], ss = v[4];
    if (month < 1 || month > 12) return 1;
    if (day < 1 || day > 31) return 1;
    int ml = month_len(year, month);
    if (day > ml) day = ml;
    if (mi > 59) return 1;
    int plus_day = 0;
    if (hh == 24 && mi == 0 && ss == 0) { hh = 0; plus_day = 1; }
    else {
        if (hh > 23) return 1;
        if (ss > 59) return 1;
    }
    if (plus_day) {
        int64_t days = days_from_civil(year, month, day) + 1;
        civil_from_days(days, &year, &month, &day);
    }
    *ly = year; *lm = month; *ld = day; *lh = hh; *lmi = mi; *ls = ss; *offset_secs = off;
    return 0;
}

static int has_req(instance *in, const char *n) { return sl_has(&in->requested, n); }

static js fmt2(parsable *ps, const char *f, int64_t a, int b, int c) {
    char buf[64];
    snprintf(buf, sizeof buf, f, (long long)a, b, c);
    return js_lit(ps->a, buf);
}

/* ---- strftime parsing: JDK 8 DateTimeFormatter.parse(text, ZonedDateTime::from)
 * with the elements above, restated step by step.  Returns 0 ok (local
 * date-time, nanos, offset seconds), 1 DateTimeParseException (the dissector
 * throws DissectionFailure), 2 outside the restatement (ORC_UNSUPPORTED). */
static const char *DOW_SHORT[] = {"Mon", "Tue", "Wed", "Thu", "Fri", "Sat", "Sun"};
static const char *DOW_FULL[] = {"Monday", "Tuesday", "Wednesday", "Thursday", "Friday", "Saturday", "Sunday"};
static const char *AMPM_UP[] = {"AM", "PM"};
static const char *AMPM_LOW[] = {"am", "pm"};
static int lower_c(int c) { return c >= 'A' && c <= 'Z' ? c + 32 : c; }

/* WeekFields (java.time.temporal.WeekFields.ComputedDayOfField) of a date:
 * first day of week sow (1 Monday .. 7 Sunday), minimal days in week 1 */
static int dow_of(int64_t days) { return (int)(((days % 7) + 7 + 3) % 7) + 1; } /* ISO, Monday 1 */
static int wf_start_offset(int day, int ldow, int mind) {
    int week_start = ((day - ldow) % 7 + 7) % 7;
    return week_start + 1 > mind ? 7 - week_start : -week_start;
}
static int wf_week(int offset, int day) { return (7 + offset + (day - 1)) / 7; }
static int wf_ldow(int64_t days, int sow) { return ((dow_of(days) - sow) % 7 + 7) % 7 + 1; }
/* weekOfYear (rangeUnit YEARS) */
static int wf_week_of_year(int64_t y, int m, int d, int sow, int mind) {
    int64_t days = days_from_civil(y, m, d);
    int doy = (int)(days - days_from_civil(y, 1, 1)) + 1;
    return wf_week(wf_start_offset(doy, wf_ldow(days, sow), mind), doy);
}
/* weekBasedYear */
static int64_t wf_week_based_year(int64_t y, int m, int d, int sow, int mind) {
    int64_t days = days_from_civil(y, m, d);
    int doy = (int)(days - days_from_civil(y, 1, 1)) + 1;
    int offset = wf_start_offset(doy, wf_ldow(days, sow), mind);
    int week = wf_week(offset, doy);
    if (week == 0) return y - 1;
    int ylen = is_leap(y) ? 366 : 365;
    if (week >= wf_week(offset, ylen + mind)) return y + 1;
    return y;
}

typedef struct { int64_t v[SF_NFIELDS]; int has[SF_NFIELDS]; } strf_fields;
/* DateTimeParseContext.setParsedField: a field parsed twice must agree */
static int strf_set(strf_fields *f, int field, int64_t v) {
    if (f->has[field] && f->v[field] != v) return 0;
    f->has[field] = 1;
    f->v[field] = v;
    return 1;
}

static int strf_parse(const strf_prog *sp, js s, int64_t *ly, int *lm, int *ld, int *lh, int *lmi, int *ls,
                      int *nanos, int *offset_secs) {
    strf_fields F;
    memset(&F, 0, sizeof F);
    const int *c = s.c;
    int pos = 0, zone_utc = 0;
    for (int e = 0; e < sp->nel; e++) {
        const strf_el *el = &sp->el[e];
        switch (el->kind) {
        case SE_LIT: /* CharLiteralPrinterParser, case-insensitive */
            if (pos >= s.n || lower_c(c[pos]) != lower_c(el->arg)) return 1;
            pos++;
            break;
        case SE_NUM: case SE_RED2: { /* NumberPrinterParser fixed width, NOT_NEGATIVE (no sign) */
            int64_t v = 0;
            if (pos + el->width > s.n) return 1;
            for (int q = 0; q < el->width; q++) { int d = dig(c[pos + q]); if (d < 0) return 1; v = v * 10 + d; }
            pos += el->width;
            /* ReducedPrinterParser.setValue: base 2000, range 100 -> 2000 + v */
            if (el->kind == SE_RED2) v += 2000;
            if (!strf_set(&F, el->field, v)) return 1;
            break;
        }
        case SE_NUMV: { /* 1..19 digits; a sign (NORMAL for %V) is left to the reference */
            if (pos < s.n && (c[pos] == '+' || c[pos] == '-')) return 2;
            int q = pos;
            int64_t v = 0;
            while (q < s.n && q - pos < 19 && dig(c[q]) >= 0) { v = v * 10 + dig(c[q]); q++; }
            if (q == pos) return 1;
            if (q - pos == 19) return 2; /* 19 digits may exceed a long: outside the restatement */
            pos = q;
            if (!strf_set(&F, el->field, v)) return 1;
            break;
        }
        case SE_PAD2: { /* PadPrinterParserDecorator(2, ' ') around a 1..19 digit number, strict */
            if (pos >= s.n || pos + 2 > s.n) return 1;
            int q = pos, end = pos + 2;
            while (q < end && c[q] == ' ') q++;
            if (q < end && (c[q] == '+' || c[q] == '-')) return 2;
            int64_t v = 0;
            int r = q;
            while (r < end && dig(c[r]) >= 0) { v = v * 10 + dig(c[r]); r++; }
            if (r == q || r != end) return 1;
            pos = end;
            if (!strf_set(&F, el->field, v)) return 1;
            break;
        }
        case SE_TEXT: { /* TextPrinterParser: the longest entry that matches, case-insensitive */
            const char **tab; int nt;
            switch (el->arg) {
            case TT_MON_SHORT: tab = MONTH_SHORT; nt = 12; break;
            case TT_MON_FULL: tab = MONTH_FULL; nt = 12; break;
            case TT_DOW_SHORT: tab = DOW_SHORT; nt = 7; break;
            case TT_DOW_FULL: tab = DOW_FULL; nt = 7; break;
            case TT_AMPM_UP: tab = AMPM_UP; nt = 2; break;
            default: tab = AMPM_LOW; nt = 2; break;
            }
            int best = -1, blen = 0;
            for (int t = 0; t < nt; t++) {
                int L = (int)strlen(tab[t]), ok = pos + L <= s.n;
                for (int q = 0; ok && q < L; q++) ok = lower_c(c[pos + q]) == lower_c(tab[t][q]);
                if (ok && L > blen) { best = t; blen = L; }
            }
            if (best < 0) return 1;
            pos += blen;
            /* values: months 1..12, days of week 1..7 (Monday 1), AM 0 / PM 1 */
            int64_t v = (el->arg == TT_AMPM_UP || el->arg == TT_AMPM_LOW) ? best : best + 1;
            if (!strf_set(&F, el->field, v)) return 1;
            break;
        }
        case SE_OFF: { /* OffsetIdPrinterParser("+HHMM", "+0000") */
            if (pos + 5 > s.n) return 1;
            const int *p = c + pos;
            int off;
            if (p[0] == '+' && p[1] == '0' && p[2] == '0' && p[3] == '0' && p[4] == '0') off = 0;
            else {
                if (p[0] != '+' && p[0] != '-') return 1;
                int a1 = dig(p[1]), a2 = dig(p[2]), b1 = dig(p[3]), b2 = dig(p[4]);
                if (a1 < 0 || a2 < 0 || b1 < 0 || b2 < 0) return 1;
                int oh = a1 * 10 + a2, om = b1 * 10 + b2;
                if (oh > 59 || om > 59) return 1;
                off = (p[0] == '-' ? -1 : 1) * (oh * 3600 + om * 60);
            }
            pos += 5;
            if (!strf_set(&F, SF_OFFSET, off)) return 1;
            break;
        }
        case SE_ZONE: { /* ZoneTextPrinterParser: "UTC" / "GMT" (not followed by an offset) only */
            if (pos + 3 > s.n) return 2;
            const int *p = c + pos;
            int utc = lower_c(p[0]) == 'u' && lower_c(p[1]) == 't' && lower_c(p[2]) == 'c';
            int gmt = lower_c(p[0]) == 'g' && lower_c(p[1]) == 'm' && lower_c(p[2]) == 't';
            if (!utc && !gmt) return 2;
            if (pos + 3 < s.n && (p[3] == '+' || p[3] == '-')) return 2;
            pos += 3;
            zone_utc = 1;
            break;
        }
        }
    }
    if (pos != s.n) return 1; /* unparsed text */
    /* ---- Parsed.resolve (JDK 8), SMART */
    int has_date = 0, has_time = 0, plus_day = 0;
    int64_t dy = 0; int dm = 0, dd = 0;
    int th = 0, tmi = 0, tsec = 0, tnano = 0;
    int64_t sod = -1; /* SECOND_OF_DAY from the instant */
    /* resolveInstantFields: the zone is the parsed one, else the formatter's
     * UTC (no %z / %Z), else OFFSET_SECONDS */
    if (F.has[SF_INSTANT]) {
        int64_t off;
        if (zone_utc || !sp->zone) off = 0;
        else if (F.has[SF_OFFSET]) off = F.v[SF_OFFSET];
        else return 2;
        if (off > 18 * 3600 || off < -18 * 3600) return 1;
        const int64_t t = F.v[SF_INSTANT] + off;
        if (F.v[SF_INSTANT] > 253402300799LL) return 2; /* beyond year 9999: outside the restatement */
        int64_t days = t >= 0 ? t / 86400 : -((-t + 86399) / 86400);
        civil_from_days(days, &dy, &dm, &dd);
        has_date = 1;
        sod = t - days * 86400;
    }
    /* resolveDateFields: IsoChronology.resolveDate (YEAR + MONTH_OF_YEAR +
     * DAY_OF_MONTH, else YEAR + DAY_OF_YEAR; fields it does not consume stay
     * for the cross-check) */
    if (F.has[SF_YEAR] && ((F.has[SF_MONTH] && F.has[SF_DOM]) || F.has[SF_DOY])) {
        int64_t y = F.v[SF_YEAR];
        int64_t ry; int rm, rd;
        if (y < -999999999 || y > 999999999) return 1;
        if (F.has[SF_MONTH] && F.has[SF_DOM]) { /* resolveYMD */
            int64_t mo = F.v[SF_MONTH], dom = F.v[SF_DOM];
            if (mo < 1 || mo > 12 || dom < 1 || dom > 31) return 1;
            if (y < 1 || y > 9999) return 2; /* the calendar is restated for years 1..9999 */
            int ml = month_len(y, (int)mo);
            if (dom > ml) dom = ml; /* SMART clamps to the month's length */
            ry = y; rm = (int)mo; rd = (int)dom;
            F.has[SF_MONTH] = F.has[SF_DOM] = 0;
        } else { /* resolveYD */
            int64_t doy = F.v[SF_DOY];
            if (doy < 1 || doy > 366) return 1;
            if (y < 1 || y > 9999) return 2;
            if (doy == 366 && !is_leap(y)) return 1; /* LocalDate.ofYearDay */
            civil_from_days(days_from_civil(y, 1, 1) + doy - 1, &ry, &rm, &rd);
            F.has[SF_DOY] = 0;
        }
        F.has[SF_YEAR] = 0;
        if (has_date && (ry != dy || rm != dm || rd != dd)) return 1; /* updateCheckConflict(date) */
        dy = ry; dm = rm; dd = rd; has_date = 1;
    }
    /* a week-of-year with the YEAR left: WeekFields resolves a date from it
     * (resolveWoY): outside the restatement */
    if (F.has[SF_WOY] && F.has[SF_YEAR]) return 2;
    /* resolveTimeFields */
    int64_t hod = -1, hap = -1;
    if (F.has[SF_HOD]) hod = F.v[SF_HOD];
#define CONFLICT_HOD(val) do { int64_t v_ = (val); if (hod >= 0 && hod != v_) return 1; hod = v_; } while (0)
    if (F.has[SF_CHOD]) { /* SMART allows 0-24, 24 -> 0 */
        int64_t ch = F.v[SF_CHOD];
        if (ch != 0 && (ch < 1 || ch > 24)) return 1;
        CONFLICT_HOD(ch == 24 ? 0 : ch);
    }
    if (F.has[SF_CHAP]) { /* SMART allows 0-12, 12 -> 0 */
        int64_t ch = F.v[SF_CHAP];
        if (ch != 0 && (ch < 1 || ch > 12)) return 1;
        hap = ch == 12 ? 0 : ch;
    }
    int ampm_used = 0;
    if (F.has[SF_AMPM] && hap >= 0) {
        CONFLICT_HOD(F.v[SF_AMPM] * 12 + hap);
        ampm_used = 1;
    }
    if (sod >= 0) { /* SECOND_OF_DAY from the instant -> HOUR_OF_DAY, MINUTE, SECOND */
        CONFLICT_HOD(sod / 3600);
        if (F.has[SF_MIN] && F.v[SF_MIN] != (sod / 60) % 60) return 1;
        if (F.has[SF_SEC] && F.v[SF_SEC] != sod % 60) return 1;
        F.v[SF_MIN] = (sod / 60) % 60; F.has[SF_MIN] = 1;
        F.v[SF_SEC] = sod % 60; F.has[SF_SEC] = 1;
    }
#undef CONFLICT_HOD
    /* the localized day-of-week (%u) replaces DAY_OF_WEEK (ComputedDayOfField.resolve, no conflict check) */
    if (F.has[SF_ISODOW]) {
        if (F.v[SF_ISODOW] < 1 || F.v[SF_ISODOW] > 7) return 1;
        F.v[SF_DOW] = F.v[SF_ISODOW]; F.has[SF_DOW] = 1;
    }
    /* resolveTimeLenient: milli / micro to nano, hour with defaults */
    int64_t nos = -1;
    if (F.has[SF_MILLI] && F.has[SF_MICRO]) return 2;
    if (F.has[SF_MILLI]) nos = F.v[SF_MILLI] * 1000000;
    if (F.has[SF_MICRO]) nos = F.v[SF_MICRO] * 1000;
    if (hod >= 0) {
        int64_t moh = F.has[SF_MIN] ? F.v[SF_MIN] : -1, som = F.has[SF_SEC] ? F.v[SF_SEC] : -1;
        if (!((moh < 0 && (som >= 0 || nos >= 0)) || (moh >= 0 && som < 0 && nos >= 0))) {
            if (moh < 0) moh = 0;
            if (som < 0) som = 0;
            if (nos < 0) nos = 0;
            /* resolveTime: MINUTE and NANO checked, 24:00 = end of day, then HOUR / SECOND */
            if (moh > 59) return 1;
            if (hod == 24 && moh == 0 && som == 0 && nos == 0) { th = 0; plus_day = 1; }
            else { if (hod > 23 || som > 59) return 1; th = (int)hod; }
            tmi = (int)moh; tsec = (int)som; tnano = (int)nos;
            has_time = 1;
        }
    }
    if (!has_date || !has_time) return 1; /* LocalDateTime.from: no date or no time */
    if (plus_day) { int64_t dd2 = days_from_civil(dy, dm, dd) + 1; civil_from_days(dd2, &dy, &dm, &dd); }
    /* crossCheck: the fields left against the resolved date and time */
    const int64_t days = days_from_civil(dy, dm, dd);
    if (F.has[SF_DOW] && F.v[SF_DOW] != dow_of(days)) return 1;
    if (F.has[SF_DOY] && F.v[SF_DOY] != days - days_from_civil(dy, 1, 1) + 1) return 1;
    if (F.has[SF_WOY] && F.v[SF_WOY] != wf_week_of_year(dy, dm, dd, 1, 4)) return 1;
    if (F.has[SF_WBY] && F.v[SF_WBY] != wf_week_based_year(dy, dm, dd, 7, 1)) return 1;
    if (F.has[SF_AMPM] && !ampm_used && F.v[SF_AMPM] != th / 12) return 1;
    if (hap >= 0 && !ampm_used && hap != th % 12) return 1;
    if (F.has[SF_MONTH] || F.has[SF_DOM] || F.has[SF_YEAR]) {
        /* date fields the date did not come from (e.g. YEAR with an instant) */
        if (F.has[SF_MONTH] && F.v[SF_MONTH] != dm) return 1;
        if (F.has[SF_DOM] && F.v[SF_DOM] != dd) return 1;
        if (F.has[SF_YEAR] && F.v[SF_YEAR] != dy) return 1;
    }
    /* ZonedDateTime.from: the zone (ZoneOffset.ofTotalSeconds when %z) */
    int off = 0;
    if (!zone_utc && sp->zone) {
        if (!F.has[SF_OFFSET]) return 1;
        off = (int)F.v[SF_OFFSET];
        if (off > 18 * 3600 || off < -18 * 3600) return 1;
    }
    if (dy < 1 || dy > 9999) return 2;
    *ly = dy; *lm = dm; *ld = dd; *lh = th; *lmi = tmi; *ls = tsec; *nanos = tnano; *offset_secs = off;
    return 0;
}

/* TimeStampDissector.dissect (:404-564) */
static void emit_time(parsable *ps, instance *in, const char *inputname, int64_t y, int m, int d, int h, int mi,
                      int sec, int nanos, int off);
static void d_timestamp(parsable *ps, instance *in, const char *inputname) {
    val *vp = cache_get(ps, in->d->in_type, inputname);
    js s = v_getstring(ps->a, *vp);
    if (s.null || s.n == 0) return;
    int64_t y; int m, d, h, mi, sec, off;
    const int bad = in->d->cls == D_TIMESTAMP_ISO ? parse_iso_time(s, &y, &m, &d, &h, &mi, &sec, &off)
                                                  : parse_apache_time(s, &y, &m, &d, &h, &mi, &sec, &off);
    if (bad) { ps->failed = 1; return; }
    emit_time(ps, in, inputname, y, m, d, h, mi, sec, 0, off);
}

/* StrfTimeStampDissector.dissect (StrfTimeStampDissector.java:66-70): the
 * TimeStampDissector with the converted formatter */
static void d_strftime(parsable *ps, instance *in, const char *inputname) {
    val *vp = cache_get(ps, in->d->in_type, inputname);
    js s = v_getstring(ps->a, *vp);
    if (s.null || s.n == 0) return;
    strf_prog sp;
    strf_compile(in->d->param, &sp);
    int64_t y; int m, d, h, mi, sec, nanos, off;
    const int st = strf_parse(&sp, s, &y, &m, &d, &h, &mi, &sec, &nanos, &off);
    if (st == 2) { ps->unsupported = 1; return; }
    if (st) { ps->failed = 1; return; }
    emit_time(ps, in, inputname, y, m, d, h, mi, sec, nanos, off);
}

/* StrfTimeStampDissector.LocalizedTimeDissector.dissect (:117-120): the raw value */
static void d_localized(parsable *ps, instance *in, const char *inputname) {
    val *vp = cache_get(ps, in->d->in_type, inputname);
    if (has_req(in, "")) add_str(ps, inputname, "TIME.LOCALIZEDSTRING", "", v_getstring(ps->a, *vp));
}

/* the outputs of TimeStampDissector.dissect (:425-564) for a parsed
 * date-time (local fields as parsed, nanos, offset seconds) */
static void emit_time(parsable *ps, instance *in, const char *inputname, int64_t y, int m, int d, int h, int mi,
                      int sec, int nanos, int off) {
    int64_t epoch_s = days_from_civil(y, m, d) * 86400 + h * 3600 + mi * 60 + sec - off;
    int any_tz = has_req(in, "timezone") || has_req(in, "epoch");
    if (any_tz) {
        /* timezone: emitted as TIME.TIMEZONE but advertised as TIME.ZONE ->
         * never stored (:429); only epoch matters */
        if (has_req(in, "epoch")) add_long(ps, inputname, "TIME.EPOCH", "epoch", epoch_s * 1000 + nanos / 1000000);
    }
    const char *asp[] = {"day", "monthname", "month", "weekofweekyear", "weekyear", "year", "hour", "minute", "second",
                         "millisecond", "microsecond", "nanosecond", "date", "time", NULL};
    int any_local = 0, any_utc = 0;
    for (int i = 0; asp[i]; i++) {
        char u[64];
        snprintf(u, sizeof u, "%s_utc", asp[i]);
        if (has_req(in, asp[i])) any_local = 1;
        if (has_req(in, u)) any_utc = 1;
    }
    for (int pass = 0; pass < 2; pass++) {
        if (pass == 0 && !any_local) continue;
        if (pass == 1 && !any_utc) continue;
        int64_t Y = y; int M = m, D = d, H = h, MI = mi, S = sec;
        if (pass == 1) {
            int64_t days = epoch_s >= 0 ? epoch_s / 86400 : -((-epoch_s + 86399) / 86400);
            int64_t rem = epoch_s - days * 86400;
            civil_from_days(days, &Y, &M, &D);
            H = (int)(rem / 3600); MI = (int)(rem % 3600 / 60); S = (int)(rem % 60);
        }
        const char *sfx = pass == 1 ? "_utc" : "";
        char nm[64];
#define WANT(base) (snprintf(nm, sizeof nm, "%s%s", base, sfx), has_req(in, nm))
        int64_t wy; int wk;
        iso_week(Y, M, D, &wy, &wk);
        if (WANT("day")) add_long(ps, inputname, "TIME.DAY", nm, D);
        if (WANT("monthname")) add_str(ps, inputname, "TIME.MONTHNAME", nm, js_lit(ps->a, MONTH_FULL[M - 1]));
        if (WANT("month")) add_long(ps, inputname, "TIME.MONTH", nm, M);
        if (WANT("weekofweekyear")) add_long(ps, inputname, "TIME.WEEK", nm, wk);
        if (WANT("weekyear")) add_long(ps, inputname, "TIME.YEAR", nm, wy);
        if (WANT("year")) add_long(ps, inputname, "TIME.YEAR", nm, Y);
        if (WANT("hour")) add_long(ps, inputname, "TIME.HOUR", nm, H);
        if (WANT("minute")) add_long(ps, inputname, "TIME.MINUTE", nm, MI);
        if (WANT("second")) add_long(ps, inputname, "TIME.SECOND", nm, S);
        if (WANT("millisecond")) add_long(ps, inputname, "TIME.MILLISECOND", nm, nanos / 1000000);
        if (WANT("microsecond")) add_long(ps, inputname, "TIME.MICROSECOND", nm, nanos / 1000);
        if (WANT("nanosecond")) add_long(ps, inputname, "TIME.NANOSECOND", nm, nanos);
        if (WANT("date")) add_str(ps, inputname, "TIME.DATE", nm, fmt2(ps, "%04lld-%02d-%02d", Y, M, D));
        if (WANT("time")) add_str(ps, inputname, "TIME.TIME", nm, fmt2(ps, "%02lld:%02d:%02d", H, MI, S));
#undef WANT
    }
}

/* ------------------------------------------------------- first line */
static jre *g_fl1, *g_fl2, *g_bad_escape, *g_almost_html, *g_eq_hash, *g_hash_amp, *g_double_hash;
static jre *g_q_question, *g_q_amp, *g_valid_std, *g_chopped_std, *g_valid_nonstd, *g_chopped_nonstd;
static pthread_once_t g_re_once = PTHREAD_ONCE_INIT;
static void init_res(void) {
    g_fl1 = must_compile("^([a-zA-Z-_]+) (.*) (HTTP/[0-9]+\\.[0-9]+)$");   /* HttpFirstLineDissector.java:59-60 */
    g_fl2 = must_compile("^([a-zA-Z-_]+) (.*)$");                            /* :62-63 */
    g_bad_escape = must_compile("%([^0-9a-fA-F]|[0-9a-fA-F][^0-9a-fA-F]|.$|$)"); /* HttpUriDissector.java:123 */
    g_almost_html = must_compile("([^&])(#x[0-9a-fA-F][0-9a-fA-F];)");     /* :127 */
    g_eq_hash = must_compile("=#");
    g_hash_amp = must_compile("#&");
    g_double_hash = must_compile("#(.*)#");
    g_q_question = must_compile("\\?");
    g_q_amp = must_compile("&");
    g_valid_std = must_compile("%([0-9A-Fa-f]{2})");                        /* Utils.java:27-30 */
    g_chopped_std = must_compile("%[0-9A-Fa-f]?$");
    g_valid_nonstd = must_compile("%u([0-9A-Fa-f][0-9A-Fa-f])([0-9A-Fa-f][0-9A-Fa-f])");
    g_chopped_nonstd = must_compile("%u[0-9A-Fa-f]{0,3}$");
}

/* HttpFirstLineDissector.dissect (:86-122) */
static void d_firstline(parsable *ps, instance *in, const char *inputname) {
    val *vp = cache_get(ps, "HTTP.FIRSTLINE", inputname);
    js s = v_getstring(ps->a, *vp);
    if (s.null || s.n == 0 || js_eq_lit(s, "-")) return;
    int caps[8];
    if (jre_find(g_fl1, s.c, s.n, 0, caps)) {
        if (has_req(in, "method")) add_str(ps, inputname, "HTTP.METHOD", "method", js_sub(s, caps[2], caps[3]));
        if (has_req(in, "uri")) add_str(ps, inputname, "HTTP.URI", "uri", js_sub(s, caps[4], caps[5]));
        if (has_req(in, "protocol")) add_str(ps, inputname, "HTTP.PROTOCOL_VERSION", "protocol", js_sub(s, caps[6], caps[7]));
        return;
    }
    if (jre_find(g_fl2, s.c, s.n, 0, caps)) {
        if (has_req(in, "method")) add_str(ps, inputname, "HTTP.METHOD", "method", js_sub(s, caps[2], caps[3]));
        if (has_req(in, "uri")) add_str(ps, inputname, "HTTP.URI", "uri", js_sub(s, caps[4], caps[5]));
        add_str(ps, inputname, "HTTP.PROTOCOL_VERSION", "protocol", js_null());
    }
}

/* HttpFirstLineProtocolDissector.dissect (:56-77) */
static void d_protocol(parsable *ps, instance *in, const char *inputname) {
    val *vp = cache_get(ps, "HTTP.PROTOCOL_VERSION", inputname);
    js s = v_getstring(ps->a, *vp);
    if (s.null || s.n == 0 || js_eq_lit(s, "-")) return;
    js *parts;
    int np = js_split_char_limit(ps->a, s, '/', 2, &parts);
    if (np == 2) {
        if (has_req(in, "")) add_str(ps, inputname, "HTTP.PROTOCOL", "", parts[0]);
        if (has_req(in, "version")) add_str(ps, inputname, "HTTP.PROTOCOL.VERSION", "version", parts[1]);
        return;
    }
    add_str(ps, inputname, "HTTP.PROTOCOL", "", js_null());
    add_str(ps, inputname, "HTTP.PROTOCOL.VERSION", "version", js_null());
}

/* ------------------------------------------------------------- URI */
/* commons-httpclient 3.1 URIUtil.encode(s, allowed, "UTF-8") with the
 * HttpUriDissector badUriChars set (HttpUriDissector.java:111-120):
 * allowed = 0..254 minus URI.unwise {}|\^[]` , space, control (0-0x1F,0x7F),
 * and <>".  Bytes >= 0x80 stay raw and then decode as US-ASCII -> U+FFFD. */
static int uri_allowed(int b) {
    if (b == 255) return 0;
    if (b <= 0x20 || b == 0x7F) return 0;
    switch (b) {
    case '{': case '}': case '|': case '\\': case '^': case '[': case ']': case '`':
    case '<': case '>': case '"': return 0;
    }
    return 1;
}
static js uriutil_encode(parsable *ps, js s) {
    int blen;
    char *u8 = js_to_utf8(ps->a, s, &blen);
    int *o = (int *)ar_alloc(ps->a, sizeof(int) * (size_t)(blen * 3 + 1));
    int k = 0;
    static const char *HX = "0123456789ABCDEF";
    for (int i = 0; i < blen; i++) {
        int b = (unsigned char)u8[i];
        if (uri_allowed(b)) o[k++] = b >= 0x80 ? 0xFFFD : b;
        else { o[k++] = '%'; o[k++] = HX[b >> 4]; o[k++] = HX[b & 15]; }
    }
    js r = {o, k, 0};
    return r;
}

/* commons-lang3 3.8.1 StringEscapeUtils.unescapeHtml4 restated for the
 * BASIC + ISO8859_1 tables and NumericEntityUnescaper(semiColonRequired).
 * Any other '&name;' sequence -> UNSUPPORTED (HTML40 extended table not
 * restated). */
static const char *LAT1[] = {"nbsp", "iexcl", "cent", "pound", "curren", "yen", "brvbar", "sect", "uml", "copy", "ordf", "laquo", "not", "shy", "reg", "macr",
                             "deg", "plusmn", "sup2", "sup3", "acute", "micro", "para", "middot", "cedil", "sup1", "ordm", "raquo", "frac14", "frac12", "frac34", "iquest",
                             "Agrave", "Aacute", "Acirc", "Atilde", "Auml", "Aring", "AElig", "Ccedil", "Egrave", "Eacute", "Ecirc", "Euml", "Igrave", "Iacute", "Icirc", "Iuml",
                             "ETH", "Ntilde", "Ograve", "Oacute", "Ocirc", "Otilde", "Ouml", "times", "Oslash", "Ugrave", "Uacute", "Ucirc", "Uuml", "Yacute", "THORN", "szlig",
                             "agrave", "aacute", "acirc", "atilde", "auml", "aring", "aelig", "ccedil", "egrave", "eacute", "ecirc", "euml", "igrave", "iacute", "icirc", "iuml",
                             "eth", "ntilde", "ograve", "oacute", "ocirc", "otilde", "ouml", "divide", "oslash", "ugrave", "uacute", "ucirc", "uuml", "yacute", "thorn", "yuml"};
static int is_hexc(int c) { return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'); }
static int is_alnum(int c) { return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }

static js unescape_html4(parsable *ps, js s) {
    int *o = (int *)ar_alloc(ps->a, sizeof(int) * (size_t)(s.n + 1));
    int k = 0, changed = 0;
    for (int i = 0; i < s.n;) {
        int c = s.c[i];
        if (c == '&') {
            /* Lookup translators: longest key first; keys are &name; */
            int j = i + 1;
            while (j < s.n && is_alnum(s.c[j]) && j - i <= 10) j++;
            if (j < s.n && s.c[j] == ';' && j > i + 1) {
                char nm[16];
                int L = j - i - 1;
                for (int q = 0; q < L; q++) nm[q] = (char)s.c[i + 1 + q];
                nm[L] = 0;
                int val = -1;
                if (!strcmp(nm, "quot")) val = '"';
                else if (!strcmp(nm, "amp")) val = '&';
                else if (!strcmp(nm, "lt")) val = '<';
                else if (!strcmp(nm, "gt")) val = '>';
                else for (int q = 0; q < 96; q++) if (!strcmp(nm, LAT1[q])) { val = 160 + q; break; }
                if (val >= 0) { o[k++] = val; i = j + 1; changed = 1; continue; }
                ps->unsupported = 1; /* possibly an HTML40-extended entity */
                return s;
            }
            /* NumericEntityUnescaper */
            if (i < s.n - 2 && s.c[i + 1] == '#') {
                int start = i + 2, hex = 0;
                if (s.c[start] == 'x' || s.c[start] == 'X') { start++; hex = 1; if (start == s.n) goto copy; }
                int end = start;
                while (end < s.n && is_hexc(s.c[end])) end++;
                int semi = end != s.n && s.c[end] == ';';
                if (!semi) goto copy;
                if (end == start) goto copy; /* parseInt("") -> NFE -> 0 */
                long long v = 0;
                int bad = 0;
                for (int q = start; q < end; q++) {
                    int dv = s.c[q] <= '9' ? s.c[q] - '0' : (s.c[q] | 32) - 'a' + 10;
                    if (!hex && dv > 9) { bad = 1; break; }
                    v = v * (hex ? 16 : 10) + dv;
                    if (v > 0x7FFFFFFF) { bad = 1; break; }
                }
                if (bad) goto copy;
                if (v > 0x10FFFF || (v >= 0xD800 && v <= 0xDFFF)) { ps->unsupported = 1; return s; }
                o[k++] = (int)v;
                i = end + 1;
                changed = 1;
                continue;
            }
        }
    copy:
        o[k++] = c;
        i++;
    }
    if (!changed) return s;
    js r = {o, k, 0};
    return r;
}

/* java.net.URI.decode (UTF-8 with REPLACE); invalid UTF-8 -> UNSUPPORTED */
static js uri_decode(parsable *ps, js s) {
    if (s.null || s.n == 0 || js_index_of_char(s, '%', 0) < 0) return s;
    int *o = (int *)ar_alloc(ps->a, sizeof(int) * (size_t)(s.n + 1));
    int k = 0, between = 0;
    for (int i = 0; i < s.n;) {
        int c = s.c[i];
        if (c == '[') between = 1;
        else if (between && c == ']') between = 0;
        if (c != '%' || between) { o[k++] = c; i++; continue; }
        unsigned char bytes[4096];
        int nb = 0;
        while (i < s.n && s.c[i] == '%') {
            if (i + 2 >= s.n) { ps->unsupported = 1; return s; }
            int h1 = s.c[i + 1], h2 = s.c[i + 2];
            int v1 = h1 <= '9' ? h1 - '0' : (h1 | 32) - 'a' + 10;
            int v2 = h2 <= '9' ? h2 - '0' : (h2 | 32) - 'a' + 10;
            if (nb < 4096) bytes[nb++] = (unsigned char)(v1 * 16 + v2);
            i += 3;
        }
        /* strict UTF-8 decode */
        for (int q = 0; q < nb;) {
            unsigned b = bytes[q];
            int need, cp;
            if (b < 0x80) { need = 0; cp = (int)b; }
            else if (b >= 0xC2 && b <= 0xDF) { need = 1; cp = (int)(b & 0x1F); }
            else if (b >= 0xE0 && b <= 0xEF) { need = 2; cp = (int)(b & 0x0F); }
            else if (b >= 0xF0 && b <= 0xF4) { need = 3; cp = (int)(b & 0x07); }
            else { ps->unsupported = 1; return s; }
            if (need > 0 && q + need >= nb) { ps->unsupported = 1; return s; }
            for (int r = 1; r <= need; r++) {
                if ((bytes[q + r] & 0xC0) != 0x80) { ps->unsupported = 1; return s; }
                cp = (cp << 6) | (bytes[q + r] & 0x3F);
            }
            if ((need == 2 && (cp < 0x800 || (cp >= 0xD800 && cp <= 0xDFFF))) || (need == 3 && (cp < 0x10000 || cp > 0x10FFFF))) {
                ps->unsupported = 1;
                return s;
            }
            o[k++] = cp;
            q += need + 1;
        }
    }
    js r = {o, k, 0};
    return r;
}

/* java.net.URI parser (RFC 2396 as implemented by JDK 8 java.net.URI.Parser) */
#define CL_ALPHA 1
#define CL_DIGIT 2
#define CL_MARK 4      /* -_.!~*'() */
#define CL_RESERVED 8  /* ;/?:@&=+$,[] */
static int ccls(int c) {
    int r = 0;
    if ((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z')) r |= CL_ALPHA;
    if (c >= '0' && c <= '9') r |= CL_DIGIT;
    if (c && strchr("-_.!~*'()", c) && c < 128) r |= CL_MARK;
    if (c && strchr(";/?:@&=+$,[]", c) && c < 128) r |= CL_RESERVED;
    return r;
}
typedef struct {
    js s;
    js scheme, userinfo, host, path, query, fragment;
    int port;
    int fail;
} urip;

enum { K_URIC, K_PATH, K_SCHEME, K_USERINFO, K_SERVER, K_REGNAME };
static int char_ok(int k, int c) {
    int cl = ccls(c);
    int unreserved = cl & (CL_ALPHA | CL_DIGIT | CL_MARK);
    switch (k) {
    case K_URIC: return unreserved || (cl & CL_RESERVED);
    case K_PATH: return unreserved || (c && c < 128 && strchr(":@&=+$,;/", c));
    case K_SCHEME: return (cl & (CL_ALPHA | CL_DIGIT)) || c == '+' || c == '-' || c == '.';
    case K_USERINFO: return unreserved || (c && c < 128 && strchr(";:&=+$,", c));
    case K_SERVER: return unreserved || (c && c < 128 && strchr(";:&=+$,", c)) || (cl & (CL_ALPHA | CL_DIGIT)) || c == '-' || (c && c < 128 && strchr(".:@[]", c));
    case K_REGNAME: return unreserved || (c && c < 128 && strchr("$,;:@&=+", c));
    }
    return 0;
}
/* scan while chars match class k, allowing escapes (and non-ASCII "other") */
static int u_scan_cls(urip *u, int p, int n, int k, int escapes) {
    while (p < n) {
        int c = u->s.c[p];
        if (char_ok(k, c)) { p++; continue; }
        if (escapes) {
            if (c == '%') {
                if (p + 3 <= n && is_hexc(u->s.c[p + 1]) && is_hexc(u->s.c[p + 2])) { p += 3; continue; }
                u->fail = 1; /* Malformed escape pair */
                return p;
            }
            if (c > 128) { u->fail = 2; return p; } /* "other" chars: not restated */
        }
        break;
    }
    return p;
}
static int u_scan_stop(urip *u, int p, int n, const char *err, const char *stop) {
    while (p < n) {
        int c = u->s.c[p];
        if (c < 128 && c && strchr(err, c)) return -1;
        if (c < 128 && c && strchr(stop, c)) break;
        p++;
    }
    return p;
}
static int u_check(urip *u, int p, int q, int k) {
    int r = u_scan_cls(u, p, q, k, 1);
    if (u->fail) return 0;
    if (r < q) { u->fail = 1; return 0; }
    return 1;
}
static int u_at(urip *u, int p, int n, int c) { return p < n && u->s.c[p] == c; }

static int u_scan_byte(urip *u, int p, int n) {
    int q = p;
    while (q < n && u->s.c[q] >= '0' && u->s.c[q] <= '9') q++;
    if (q <= p) return q;
    long long v = 0;
    for (int i = p; i < q; i++) { v = v * 10 + (u->s.c[i] - '0'); if (v > 100000) break; }
    if (v > 255) return p;
    return q;
}
/* parseIPv4Address: returns end or -1 */
static int u_ipv4(urip *u, int start, int n) {
    int p = start, m = start;
    while (m < n && ((u->s.c[m] >= '0' && u->s.c[m] <= '9') || u->s.c[m] == '.')) m++;
    if (m <= p) return -1;
    int q;
    int ok = 0;
    for (;;) {
        if ((q = u_scan_byte(u, p, m)) <= p) break; p = q;
        if (!u_at(u, p, m, '.')) break; p++;
        if ((q = u_scan_byte(u, p, m)) <= p) break; p = q;
        if (!u_at(u, p, m, '.')) break; p++;
        if ((q = u_scan_byte(u, p, m)) <= p) break; p = q;
        if (!u_at(u, p, m, '.')) break; p++;
        if ((q = u_scan_byte(u, p, m)) <= p) break; p = q;
        if (q < m) break;
        ok = 1;
        break;
    }
    if (!ok) return -1;
    if (p > start && p < n && u->s.c[p] != ':') return -1;
    if (p > start) u->host = js_sub(u->s, start, p);
    return p;
}
static int u_hostname(urip *u, int start, int n) {
    int p = start, q, l = -1;
    do {
        q = p;
        while (q < n && (ccls(u->s.c[q]) & (CL_ALPHA | CL_DIGIT))) q++;
        if (q <= p) break;
        l = p;
        p = q;
        q = p;
        while (q < n && ((ccls(u->s.c[q]) & (CL_ALPHA | CL_DIGIT)) || u->s.c[q] == '-')) q++;
        if (q > p) {
            if (u->s.c[q - 1] == '-') { u->fail = 1; return -1; }
            p = q;
        }
        if (!u_at(u, p, n, '.')) break;
        p++;
    } while (p < n);
    if (p < n && !u_at(u, p, n, ':')) { u->fail = 1; return -1; }
    if (l < 0) { u->fail = 1; return -1; }
    if (l > start && !(ccls(u->s.c[l]) & CL_ALPHA)) { u->fail = 1; return -1; }
    u->host = js_sub(u->s, start, p);
    return p;
}
static int u_server(urip *u, int start, int n) {
    int p = start, q;
    q = u_scan_stop(u, p, n, "/?#", "@");
    if (q >= p && u_at(u, q, n, '@')) {
        if (!u_check(u, p, q, K_USERINFO)) return -1;
        u->userinfo = js_sub(u->s, p, q);
        p = q + 1;
    }
    if (u_at(u, p, n, '[')) { u->fail = 2; return -1; } /* IPv6 literal: not restated */
    q = u_ipv4(u, p, n);
    if (q <= p) {
        q = u_hostname(u, p, n);
        if (u->fail) return -1;
    }
    p = q;
    if (u_at(u, p, n, ':')) {
        p++;
        q = u_scan_stop(u, p, n, "", "/");
        if (q > p) {
            for (int i = p; i < q; i++) if (!(u->s.c[i] >= '0' && u->s.c[i] <= '9')) { u->fail = 1; return -1; }
            long long v = 0;
            for (int i = p; i < q; i++) { v = v * 10 + (u->s.c[i] - '0'); if (v > 0x7FFFFFFF) { u->fail = 1; return -1; } }
            u->port = (int)v;
            p = q;
        }
    }
    if (p < n) { u->fail = 1; return -1; }
    return p;
}
static int u_authority(urip *u, int p, int n) {
    int server_chars, reg_chars;
    int q = p;
    for (q = p; q < n && char_ok(K_SERVER, u->s.c[q]); q++) {}
    /* JDK: scan(p, n, "]") > p  ->  authority starts with ']' (never for our inputs) */
    server_chars = (q == n);
    int r = p;
    while (r < n) {
        int c = u->s.c[r];
        if (char_ok(K_REGNAME, c)) { r++; continue; }
        if (c == '%' && r + 3 <= n && is_hexc(u->s.c[r + 1]) && is_hexc(u->s.c[r + 2])) { r += 3; continue; }
        if (c == '%') { u->fail = 1; return n; }
        if (c > 128) { u->fail = 2; return n; }
        break;
    }
    reg_chars = (r == n);
    if (reg_chars && !server_chars) return n; /* registry-based */
    int failed = 0;
    q = p;
    if (server_chars) {
        urip save = *u;
        int e = u_server(u, p, n);
        if (u->fail == 2) return n;
        if (u->fail || e < n) {
            *u = save;
            u->userinfo = js_null(); u->host = js_null(); u->port = -1;
            u->fail = 0;
            failed = 1;
            q = p;
        } else q = n;
    }
    if (q < n) {
        if (reg_chars) return n;
        (void)failed;
        u->fail = 1;
    }
    return n;
}
static int u_hier(urip *u, int start, int n) {
    int p = start;
    if (u_at(u, p, n, '/') && u_at(u, p + 1, n, '/')) {
        p += 2;
        int q = u_scan_stop(u, p, n, "", "/?#");
        if (q > p) p = u_authority(u, p, q);
        else if (q < n) { /* empty authority allowed */ }
        else { u->fail = 1; return n; }
        if (u->fail) return n;
    }
    int q = u_scan_stop(u, p, n, "", "?#");
    if (!u_check(u, p, q, K_PATH)) return n;
    u->path = js_sub(u->s, p, q);
    p = q;
    if (u_at(u, p, n, '?')) {
        p++;
        q = u_scan_stop(u, p, n, "", "#");
        if (!u_check(u, p, q, K_URIC)) return n;
        u->query = js_sub(u->s, p, q);
        p = q;
    }
    return p;
}
static void u_parse(urip *u) {
    int n = u->s.n;
    u->scheme = u->userinfo = u->host = u->path = u->query = u->fragment = js_null();
    u->port = -1;
    u->fail = 0;
    int p = u_scan_stop(u, 0, n, "/?#", ":");
    if (p >= 0 && u_at(u, p, n, ':')) {
        if (p == 0) { u->fail = 1; return; }
        if (!(ccls(u->s.c[0]) & CL_ALPHA)) { u->fail = 1; return; }
        for (int i = 1; i < p; i++) if (!char_ok(K_SCHEME, u->s.c[i])) { u->fail = 1; return; }
        u->scheme = js_sub(u->s, 0, p);
        p++;
        if (u_at(u, p, n, '/')) {
            p = u_hier(u, p, n);
            if (u->fail) return;
        } else {
            int q = u_scan_stop(u, p, n, "", "#");
            if (q <= p) { u->fail = 1; return; }
            if (!u_check(u, p, q, K_URIC)) return;
            p = q; /* opaque: path/query stay null */
        }
    } else {
        p = u_hier(u, 0, n);
        if (u->fail) return;
    }
    if (u_at(u, p, n, '#')) {
        if (!u_check(u, p + 1, n, K_URIC)) return;
        u->fragment = js_sub(u->s, p + 1, n);
        p = n;
    }
    if (p < n) u->fail = 1;
}

/* HttpUriDissector.dissect (:130-233) */
static void d_uri(parsable *ps, instance *in, const char *inputname) {
    val *vp = cache_get(ps, "HTTP.URI", inputname);
    js s = v_getstring(ps->a, *vp);
    if (s.null || s.n == 0) return;
    for (int i = 0; i < s.n; i++) if (s.c[i] >= 0xD800 && s.c[i] <= 0xDFFF) { ps->unsupported = 1; return; }
    s = uriutil_encode(ps, s);
    int fq = js_index_of_char(s, '?', 0), fa = js_index_of_char(s, '&', 0);
    if (fq != -1 || fa != -1) {
        s = js_replace_all(ps->a, g_q_question, s, "&");
        s = js_replace_first(ps->a, g_q_amp, s, "?&");
    }
    s = js_replace_all(ps->a, g_bad_escape, s, "%25$1");
    s = js_replace_all(ps->a, g_bad_escape, s, "%25$1");
    s = js_replace_all(ps->a, g_almost_html, s, "$1&$2");
    s = unescape_html4(ps, s);
    if (ps->unsupported) return;
    s = js_replace_all(ps->a, g_eq_hash, s, "=");
    s = js_replace_all(ps->a, g_hash_amp, s, "&");
    for (;;) {
        int caps[4];
        if (!jre_find(g_double_hash, s.c, s.n, 0, caps)) break;
        s = js_replace_all(ps->a, g_double_hash, s, "~$1#");
    }
    if (s.n == 0) { ps->unsupported = 1; return; } /* charAt(0) on "" -> StringIndexOutOfBounds */
    int is_url = 1;
    urip u;
    memset(&u, 0, sizeof u);
    if (s.c[0] == '/') {
        u.s = js_cat(ps->a, js_lit(ps->a, "dummy-protocol://dummy.host.name"), s);
        is_url = 0;
    } else u.s = s;
    for (int i = 0; i < u.s.n; i++) if (u.s.c[i] >= 0xD800 && u.s.c[i] <= 0xDFFF) { ps->unsupported = 1; return; }
    u_parse(&u);
    if (u.fail == 2) { ps->unsupported = 1; return; }
    if (u.fail) { ps->failed = 1; return; }
    if (has_req(in, "query") || has_req(in, "path") || has_req(in, "ref")) {
        if (has_req(in, "query")) add_str(ps, inputname, "HTTP.QUERYSTRING", "query", u.query.null ? js_lit(ps->a, "") : u.query);
        if (has_req(in, "path")) {
            js d = uri_decode(ps, u.path);
            if (ps->unsupported) return;
            add_str(ps, inputname, "HTTP.PATH", "path", d);
        }
        if (has_req(in, "ref")) {
            js d = uri_decode(ps, u.fragment);
            if (ps->unsupported) return;
            add_str(ps, inputname, "HTTP.REF", "ref", d);
        }
    }
    if (is_url) {
        if (has_req(in, "protocol")) add_str(ps, inputname, "HTTP.PROTOCOL", "protocol", u.scheme);
        if (has_req(in, "userinfo")) {
            js d = uri_decode(ps, u.userinfo);
            if (ps->unsupported) return;
            add_str(ps, inputname, "HTTP.USERINFO", "userinfo", d);
        }
        if (has_req(in, "host")) add_str(ps, inputname, "HTTP.HOST", "host", u.host);
        if (has_req(in, "port") && u.port != -1) add_long(ps, inputname, "HTTP.PORT", "port", u.port);
    }
}

/* ----------------------------------------------------------- query */
/* URLDecoder.decode(s, "UTF-16") (JDK 8).  Returns 0, or 1 on
 * IllegalArgumentException, 2 unsupported. */
static int url_decode_utf16(parsable *ps, js s, js *out) {
    int *o = (int *)ar_alloc(ps->a, sizeof(int) * (size_t)(s.n + 1));
    int k = 0, changed = 0;
    for (int i = 0; i < s.n;) {
        int c = s.c[i];
        if (c == '+') { o[k++] = ' '; i++; changed = 1; continue; }
        if (c != '%') { o[k++] = c; i++; continue; }
        unsigned char bytes[8192];
        int nb = 0;
        while (i + 2 < s.n && c == '%') {
            int a = s.c[i + 1], b = s.c[i + 2];
            /* Integer.parseInt(x, 16): optional sign then hex digits */
            int sign = 1, v;
            if (a == '+' || a == '-') {
                if (!is_hexc(b)) return 1;
                if (a == '-') sign = -1;
                v = b <= '9' ? b - '0' : (b | 32) - 'a' + 10;
            } else {
                if (a >= 128 || b >= 128) return 2; /* Character.digit on non-ASCII: not restated */
                if (!is_hexc(a) || !is_hexc(b)) return 1;
                v = (a <= '9' ? a - '0' : (a | 32) - 'a' + 10) * 16 + (b <= '9' ? b - '0' : (b | 32) - 'a' + 10);
            }
            v *= sign;
            if (v < 0) return 1;
            if (nb < 8192) bytes[nb++] = (unsigned char)v;
            i += 3;
            if (i < s.n) c = s.c[i];
        }
        if (i < s.n && c == '%') return 1; /* Incomplete trailing escape */
        /* new String(bytes, "UTF-16"): BOM sniffing, BE default */
        int q = 0, le = 0;
        if (nb >= 2 && bytes[0] == 0xFE && bytes[1] == 0xFF) q = 2;
        else if (nb >= 2 && bytes[0] == 0xFF && bytes[1] == 0xFE) { q = 2; le = 1; }
        while (q + 1 < nb) {
            int unit = le ? (bytes[q] | (bytes[q + 1] << 8)) : ((bytes[q] << 8) | bytes[q + 1]);
            q += 2;
            if (unit >= 0xD800 && unit <= 0xDBFF) {
                if (q + 1 < nb) {
                    int u2 = le ? (bytes[q] | (bytes[q + 1] << 8)) : ((bytes[q] << 8) | bytes[q + 1]);
                    if (u2 >= 0xDC00 && u2 <= 0xDFFF) {
                        o[k++] = 0x10000 + ((unit - 0xD800) << 10) + (u2 - 0xDC00);
                        q += 2;
                        continue;
                    }
                }
                return 2; /* malformed surrogate: replacement rules not restated */
            }
            if (unit >= 0xDC00 && unit <= 0xDFFF) return 2;
            o[k++] = unit;
        }
        if (q < nb) return 2; /* odd trailing byte */
        changed = 1;
    }
    (void)changed;
    js r = {o, k, 0};
    *out = r;
    return 0;
}

/* Utils.resilientUrlDecode (Utils.java:38-65) */
static int resilient_url_decode(parsable *ps, js in, js *out) {
    js cooked = in;
    if (js_index_of_char(cooked, '%', 0) > -1) {
        cooked = js_replace_all(ps->a, g_valid_std, cooked, "%00%$1");
        cooked = js_replace_all(ps->a, g_chopped_std, cooked, "");
        js pu = js_lit(ps->a, "%u");
        if (js_index_of(cooked, pu, 0) >= 0) {
            cooked = js_replace_all(ps->a, g_valid_nonstd, cooked, "%$1%$2");
            cooked = js_replace_all(ps->a, g_chopped_nonstd, cooked, "");
        }
    }
    return url_decode_utf16(ps, cooked, out);
}

/* QueryStringFieldDissector.dissect (:76-108) */
static void d_query(parsable *ps, instance *in, const char *inputname) {
    val *vp = cache_get(ps, "HTTP.QUERYSTRING", inputname);
    js s = v_getstring(ps->a, *vp);
    if (s.null || s.n == 0) return;
    int want_all = has_req(in, "*");
    js *parts;
    int np = js_split_char(ps->a, s, '&', &parts);
    for (int i = 0; i < np; i++) {
        js v = parts[i];
        int eq = js_index_of_char(v, '=', 0);
        if (eq == -1) {
            if (v.n != 0) {
                js name = js_lower(ps->a, v);
                char *nm = js_cstr(ps, name);
                if (want_all || has_req(in, nm)) add_str(ps, inputname, "STRING", nm, js_lit(ps->a, ""));
            }
        } else {
            js name = js_lower(ps->a, js_sub(v, 0, eq));
            char *nm = js_cstr(ps, name);
            if (want_all || has_req(in, nm)) {
                js dec;
                int r = resilient_url_decode(ps, js_sub(v, eq + 1, v.n), &dec);
                if (r == 1) { ps->failed = 1; return; }
                if (r == 2) { ps->unsupported = 1; return; }
                add_str(ps, inputname, "STRING", nm, dec);
            }
        }
    }
}

/* ------------------------------------------------------ converters */
/* ConvertCLFIntoNumber.dissect (translate/ConvertCLFIntoNumber.java:33-40) */
static void d_clf2num(parsable *ps, instance *in, const char *inputname) {
    val *vp = cache_get(ps, in->d->in_type, inputname);
    js sv = v_getstring(ps->a, *vp);
    if (sv.null || js_eq_lit(sv, "-")) add_long(ps, inputname, in->d->out_type, "", 0);
    else add_dissection(ps, inputname, in->d->out_type, "", *vp);
}
/* ConvertNumberIntoCLF.dissect (translate/ConvertNumberIntoCLF.java:33-39) */
static void d_num2clf(parsable *ps, instance *in, const char *inputname) {
    val *vp = cache_get(ps, in->d->in_type, inputname);
    js sv = v_getstring(ps->a, *vp);
    if (js_eq_lit(sv, "0")) add_str(ps, inputname, in->d->out_type, "", js_null());
    else add_dissection(ps, inputname, in->d->out_type, "", *vp);
}

/* Java Long.parseLong of an all-digit string; 0 on overflow
 * (NumberFormatException, a RuntimeException: not restated). */
static int parse_long_digits(js s, int a, int b, int64_t *out) {
    if (b <= a) return 0;
    uint64_t v = 0;
    for (int i = a; i < b; i++) {
        int c = s.c[i];
        if (c < '0' || c > '9') return 0;
        if (v > (uint64_t)(INT64_MAX - (c - '0')) / 10) return 0;
        v = v * 10 + (uint64_t)(c - '0');
    }
    *out = (int64_t)v;
    return 1;
}

/* ConvertSecondsWithMillisStringDissector.dissect (translate/ConvertSecondsWithMillisStringDissector.java:33-40):
 * split("\\.", 2), both halves Long.parseLong, seconds * 1000 + millis (the
 * fraction is read as an integer: "1.5" -> 1005).  A null value
 * (NullPointerException), a missing or non-numeric half
 * (ArrayIndexOutOfBounds / NumberFormatException) are runtime exceptions of
 * the reference: not restated. */
static void d_secmillis(parsable *ps, instance *in, const char *inputname) {
    val *vp = cache_get(ps, in->d->in_type, inputname);
    js sv = v_getstring(ps->a, *vp);
    if (sv.null) { ps->unsupported = 1; return; }
    int dot = js_index_of_char(sv, '.', 0);
    int64_t sec, ms;
    if (dot < 0 || !parse_long_digits(sv, 0, dot, &sec) || !parse_long_digits(sv, dot + 1, sv.n, &ms)) {
        ps->unsupported = 1;
        return;
    }
    add_long(ps, inputname, in->d->out_type, "", (int64_t)((uint64_t)sec * 1000u + (uint64_t)ms));  /* long wraps */
}

/* ConvertMillisecondsIntoMicroseconds.dissect (translate/ConvertMillisecondsIntoMicroseconds.java:33-35):
 * value.getLong() * 1000; a null Long is a NullPointerException (not restated) */
static void d_ms2us(parsable *ps, instance *in, const char *inputname) {
    val *vp = cache_get(ps, in->d->in_type, inputname);
    int64_t l;
    if (vp->filled == V_LONG) {
        if (vp->lnull) { ps->unsupported = 1; return; }
        l = vp->l;
    } else {
        js sv = vp->s;  /* Value.getLong: Long.parseLong, null on NumberFormatException */
        int neg = sv.n > 0 && sv.c[0] == '-';
        if (sv.null || !parse_long_digits(sv, neg || (sv.n > 0 && sv.c[0] == '+'), sv.n, &l)) { ps->unsupported = 1; return; }
        if (neg) l = -l;
    }
    add_long(ps, inputname, in->d->out_type, "", (int64_t)((uint64_t)l * 1000u));
}

/* NginxHttpdLogFormatDissector.BinaryIPDissector (hp/NginxHttpdLogFormatDissector.java:151-178):
 * \\xHH x4 (matches() the whole value) -> the SIGNED bytes joined by '.' */
static void d_binip(parsable *ps, instance *in, const char *inputname) {
    val *vp = cache_get(ps, in->d->in_type, inputname);
    js sv = v_getstring(ps->a, *vp);
    if (sv.null) { ps->unsupported = 1; return; }
    if (sv.n != 16) return;
    int b[4];
    for (int k = 0; k < 4; k++) {
        const int *c = sv.c + 4 * k;
        if (c[0] != '\\' || c[1] != 'x' || !is_hexc(c[2]) || !is_hexc(c[3])) return;
        int v = 0;
        for (int j = 2; j < 4; j++) v = v * 16 + (c[j] <= '9' ? c[j] - '0' : (c[j] | 32) - 'a' + 10);
        b[k] = v >= 128 ? v - 256 : v;  /* (byte) */
    }
    char out[64];
    snprintf(out, sizeof out, "%d.%d.%d.%d", b[0], b[1], b[2], b[3]);
    add_str(ps, inputname, "IP", "", js_lit(ps->a, out));
}

/* Java String.split(sep) for a two-char literal separator: pieces [start,
 * end) into v; trailing empty pieces removed (limit 0).  Returns the count. */
static int java_split2(js s, int a, int b, int c0, int c1, int *st, int *en, int cap) {
    int n = 0, from = a;
    for (int i = a; i + 1 < b; i++) {
        if (s.c[i] == c0 && s.c[i + 1] == c1) {
            if (n < cap) { st[n] = from; en[n] = i; }
            n++;
            from = i + 2;
            i++;
        }
    }
    if (n < cap) { st[n] = from; en[n] = b; }
    n++;
    if (n > cap) return -1;
    if (n == 1) return 1;  /* no match: the whole input, even when empty */
    while (n > 0 && en[n - 1] == st[n - 1]) n--;
    return n;
}
/* String.trim(): strip chars <= ' ' at both ends */
static js js_trim(js s, int a, int b) {
    while (a < b && s.c[a] <= ' ') a++;
    while (b > a && s.c[b - 1] <= ' ') b--;
    return js_sub(s, a, b);
}

/* RequestCookieListDissector.dissect (dissectors/RequestCookieListDissector.java:79-110):
 * Pattern("; ").split (trailing empty pieces dropped); a piece without '='
 * (and not empty) is a name with value ""; else name = trim + lower-case of
 * the part before the first '=', value = Utils.resilientUrlDecode of the
 * trimmed rest (IllegalArgumentException -> DissectionFailure).  Only
 * requested names ("*" = all) are delivered, as HTTP.COOKIE:<name>. */
static void d_cookies(parsable *ps, instance *in, const char *inputname) {
    val *vp = cache_get(ps, "HTTP.COOKIES", inputname);
    js s = v_getstring(ps->a, *vp);
    if (s.null || s.n == 0) return;
    const int want_all = has_req(in, "*");
    int st[512], en[512];
    const int np = java_split2(s, 0, s.n, ';', ' ', st, en, 512);
    if (np < 0) { ps->unsupported = 1; return; }
    for (int k = 0; k < np; k++) {
        js v = js_sub(s, st[k], en[k]);
        const int eq = js_index_of_char(v, '=', 0);
        if (eq == -1) {
            if (v.n == 0) continue;
            js name = js_lower(ps->a, js_trim(v, 0, v.n));
            char *nm = js_cstr(ps, name);
            if (want_all || has_req(in, nm)) add_str(ps, inputname, "HTTP.COOKIE", nm, js_lit(ps->a, ""));
        } else {
            js name = js_lower(ps->a, js_trim(v, 0, eq));
            char *nm = js_cstr(ps, name);
            if (!(want_all || has_req(in, nm))) continue;
            js dec;
            const int r = resilient_url_decode(ps, js_trim(v, eq + 1, v.n), &dec);
            if (r == 1) { ps->failed = 1; return; }
            if (r == 2) { ps->unsupported = 1; return; }
            add_str(ps, inputname, "HTTP.COOKIE", nm, dec);
        }
    }
}

/* ---- Set-Cookie (ResponseSetCookieListDissector.java:79-110 with JDK 8
 * java.net.HttpCookie.parse, ResponseSetCookieDissector.java:78-151).
 * Restated on the subset where HttpCookie.parse takes its Netscape
 * (version 0) branch: printable ASCII without '"', '\\' and '$', and none of
 * "max-age", "version", "set-cookie" (any case) -- guessCookieVersion then
 * returns 0 and parseInternal reads the whole string as one cookie.  Inputs
 * outside it, and inputs on which the reference throws out of the parser
 * (IllegalArgumentException from HttpCookie, DateTimeParseException from
 * parseExpire), are UNSUPPORTED. */
static int sc_subset(parsable *ps, js s) {
    for (int i = 0; i < s.n; i++) {
        const int c = s.c[i];
        if (c < 0x20 || c > 0x7E || c == '"' || c == '\\' || c == '$') return 0;
    }
    js low = js_lower(ps->a, s);
    return js_index_of(low, js_lit(ps->a, "max-age"), 0) < 0 && js_index_of(low, js_lit(ps->a, "version"), 0) < 0 &&
           js_index_of(low, js_lit(ps->a, "set-cookie"), 0) < 0;
}

/* HttpCookie.parseInternal's name of cookie string v (StringTokenizer(";")
 * first token, split at its first '=', trimmed; the HttpCookie constructor's
 * isToken / '$' checks): 1 and *name, or 0 when the reference throws.  Names
 * that older JDKs reserve (isReserved) are refused too. */
static int sc_name(parsable *ps, js v, js *name) {
    int q = 0;
    while (q < v.n && v.c[q] == ';') q++;
    if (q == v.n) return 0;  /* "Empty cookie header string" */
    int te = q;
    while (te < v.n && v.c[te] != ';') te++;
    int eq = -1;
    for (int i = q; i < te; i++) if (v.c[i] == '=') { eq = i; break; }
    if (eq < 0) return 0;  /* "Invalid cookie name-value pair" */
    js nm = js_trim(v, q, eq);
    if (nm.n == 0 || nm.c[0] == '$') return 0;
    for (int i = 0; i < nm.n; i++) {
        const int c = nm.c[i];
        if (c < 0x20 || c >= 0x7F || c == ',' || c == ';' || c == ' ') return 0;  /* isToken */
    }
    static const char *const reserved[] = {"comment", "commenturl", "discard", "domain", "expires", "max-age",
                                           "path", "port", "secure", "version", NULL};
    js low = js_lower(ps->a, nm);
    for (int k = 0; reserved[k]; k++) if (js_eq_lit(low, reserved[k])) return 0;
    *name = nm;
    return 1;
}

static void d_setcookies(parsable *ps, instance *in, const char *inputname) {
    val *vp = cache_get(ps, "HTTP.SETCOOKIES", inputname);
    js s = v_getstring(ps->a, *vp);
    if (s.null || s.n == 0) return;
    if (!sc_subset(ps, s)) { ps->unsupported = 1; return; }
    const int want_all = has_req(in, "*");
    int st[512], en[512];
    const int np = java_split2(s, 0, s.n, ',', ' ', st, en, 512);  /* fieldValue.split(", ") */
    if (np < 0) { ps->unsupported = 1; return; }
    int prev = -1;
    for (int k = 0; k < np; k++) {
        js part = js_sub(s, st[k], en[k]);
        const int ei = js_index_of(js_lower(ps->a, part), js_lit(ps->a, "expires="), 0);
        if (ei != -1 && part.n - 15 < ei) { prev = k; continue; }  /* "expires=XXXXXXX".length() */
        /* previous + ", " + part: the parts are contiguous in s */
        js value = prev >= 0 ? js_sub(s, st[prev], en[k]) : part;
        prev = -1;
        js name;
        if (!sc_name(ps, value, &name)) { ps->unsupported = 1; return; }
        js low = js_lower(ps->a, name);
        char *nm = js_cstr(ps, low);
        if (want_all || has_req(in, nm)) add_str(ps, inputname, "HTTP.SETCOOKIE", nm, value);
    }
}

/* ResponseSetCookieDissector.parseExpire (:138-151): only its first pattern
 * "EEE',' dd-MMM-yyyy HH:mm:ss zzz" can ever succeed (a DateTimeParseException
 * is not the IllegalArgumentException the loop catches).  Restated for the
 * zone "GMT", 4-digit years, in-range fields and a matching day name; anything
 * else UNSUPPORTED.  1 and *ms on success. */
static int sc_expire(js v, int64_t *ms) {
    static const char *const days[] = {"Mon", "Tue", "Wed", "Thu", "Fri", "Sat", "Sun"};
    static const char *const mons[] = {"Jan", "Feb", "Mar", "Apr", "May", "Jun",
                                       "Jul", "Aug", "Sep", "Oct", "Nov", "Dec"};
    if (v.n != 29) return 0;
    const char *shape = "AAA, 00-AAA-0000 00:00:00 GMT";
    for (int i = 0; i < 29; i++) {
        const int c = v.c[i], t = shape[i];
        if (t == 'A') { if (!((c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z'))) return 0; }
        else if (t == '0') { if (c < '0' || c > '9') return 0; }
        else if (c != t) return 0;
    }
    int dow = -1, mon = -1;
    for (int k = 0; k < 7; k++) if (v.c[0] == days[k][0] && v.c[1] == days[k][1] && v.c[2] == days[k][2]) dow = k;
    for (int k = 0; k < 12; k++) if (v.c[8] == mons[k][0] && v.c[9] == mons[k][1] && v.c[10] == mons[k][2]) mon = k + 1;
    if (dow < 0 || mon < 0) return 0;
#define D2(i) ((v.c[i] - '0') * 10 + (v.c[i + 1] - '0'))
    const int d = D2(5), y = D2(12) * 100 + D2(14), h = D2(17), mi = D2(20), se = D2(23);
#undef D2
    static const int ml[] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
    const int leap = (y % 4 == 0 && y % 100 != 0) || y % 400 == 0;
    const int mlen = ml[mon - 1] + (mon == 2 && leap);
    if (y < 1 || d < 1 || d > mlen || h > 23 || mi > 59 || se > 59) return 0;
    const int64_t days_ = days_from_civil(y, mon, d);
    const int iso = (int)(((days_ % 7) + 7 + 3) % 7);  /* 1970-01-01 was a Thursday (ISO 4 -> index 3) */
    if (iso != dow) return 0;
    *ms = (days_ * 86400 + h * 3600 + mi * 60 + se) * 1000;
    return 1;
}

static void d_setcookie(parsable *ps, instance *in, const char *inputname) {
    (void)in;
    val *vp = cache_get(ps, "HTTP.SETCOOKIE", inputname);
    js s = v_getstring(ps->a, *vp);
    if (s.null || s.n == 0) return;
    js *parts;
    const int np = js_split_char(ps->a, s, ';', &parts);
    for (int i = 0; i < np; i++) {
        js part = js_trim(parts[i], 0, parts[i].n);
        js *kv;
        const int nkv = js_split_char_limit(ps->a, part, '=', 2, &kv);
        js key = js_trim(kv[0], 0, kv[0].n);
        js value = nkv == 2 ? js_trim(kv[1], 0, kv[1].n) : js_lit(ps->a, "");
        if (i == 0) {
            add_str(ps, inputname, "STRING", "value", value);
        } else if (js_eq_lit(key, "expires")) {
            int64_t ms;
            if (!sc_expire(value, &ms)) { ps->unsupported = 1; return; }
            add_long(ps, inputname, "STRING", "expires", ms / 1000);
            add_long(ps, inputname, "TIME.EPOCH", "expires", ms);
        } else if (js_eq_lit(key, "domain") || js_eq_lit(key, "comment") || js_eq_lit(key, "path")) {
            char *nm = js_cstr(ps, key);
            add_str(ps, inputname, "STRING", nm, value);
        }
    }
}

/* UpstreamListDissector.dissect (nginxmodules/UpstreamListDissector.java:79-125):
 * split(", ") into servers, each split(": ") into original / redirected,
 * both trimmed; N.value and N.redirected per server. */
static void d_upstream(parsable *ps, instance *in, const char *inputname) {
    val *vp = cache_get(ps, in->d->in_type, inputname);
    js sv = v_getstring(ps->a, *vp);
    if (sv.null) { ps->unsupported = 1; return; }  /* NullPointerException */
    int ss[256], se[256];
    int ns = java_split2(sv, 0, sv.n, ',', ' ', ss, se, 256);
    if (ns < 0) { ps->unsupported = 1; return; }
    for (int k = 0; k < ns; k++) {
        int ps_[256], pe[256];
        int np = java_split2(sv, ss[k], se[k], ':', ' ', ps_, pe, 256);
        if (np <= 0) { ps->unsupported = 1; return; }  /* parts[0] of an empty array */
        char nm[64];
        js orig = js_trim(sv, ps_[0], pe[0]);
        js redir = np == 1 ? orig : js_trim(sv, ps_[1], pe[1]);
        snprintf(nm, sizeof nm, "%d.value", k);
        add_str(ps, inputname, in->d->out_type, nm, orig);
        snprintf(nm, sizeof nm, "%d.redirected", k);
        add_str(ps, inputname, in->d->out_type, nm, redir);
    }
}

static void run_instance(parsable *ps, instance *in, const char *name) {
    switch (in->d->cls) {
    case D_ROOT: d_root(ps, in, name); break;
    case D_TIMESTAMP: case D_TIMESTAMP_ISO: d_timestamp(ps, in, name); break;
    case D_STRFTIME: d_strftime(ps, in, name); break;
    case D_LOCALIZED: d_localized(ps, in, name); break;
    case D_FIRSTLINE: d_firstline(ps, in, name); break;
    case D_PROTOCOL: d_protocol(ps, in, name); break;
    case D_URI: d_uri(ps, in, name); break;
    case D_QUERY: d_query(ps, in, name); break;
    case D_CLF2NUM: d_clf2num(ps, in, name); break;
    case D_NUM2CLF: d_num2clf(ps, in, name); break;
    case D_BINIP: d_binip(ps, in, name); break;
    case D_SECMILLIS: d_secmillis(ps, in, name); break;
    case D_MS2US: d_ms2us(ps, in, name); break;
    case D_UPSTREAM: d_upstream(ps, in, name); break;
    case D_COOKIES: d_cookies(ps, in, name); break;
    case D_SETCOOKIES: d_setcookies(ps, in, name); break;
    case D_SETCOOKIE: d_setcookie(ps, in, name); break;
    default: ps->unsupported = 1; break;
    }
}

/* =================================================================== API */
static orc_parser *build(const char *logformat, const char *const *fields, int nfields, const char *const *rm_in,
                         const char *const *rm_type, int n_rm, char *err, int errlen, int for_paths) {
    pthread_once(&g_re_once, init_res);
    orc_parser *p = (orc_parser *)xmalloc(sizeof(orc_parser));
    p->logformat_arg = xstrdup(logformat);
    /* Parser.addTypeRemapping (core/Parser.java:664-677): input trimmed +
     * lower-cased, type trimmed + upper-cased, each pair once */
    for (int k = 0; k < n_rm; k++) {
        char *in = xstrdup(rm_in[k]), *ty = xstrdup(rm_type[k]);
        for (char **x = (char *[]){in, ty, NULL}; *x; x++) {
            char *a = *x, *b = a + strlen(a);
            while (*a && (unsigned char)*a <= ' ') a++;
            while (b > a && (unsigned char)b[-1] <= ' ') b--;
            memmove(*x, a, (size_t)(b - a));
            (*x)[b - a] = 0;
        }
        ascii_lower(in);
        for (char *c = ty; *c; c++) if (*c >= 'a' && *c <= 'z') *c -= 32;
        int dup = 0;
        for (int j = 0; j < p->rm_in.n; j++) dup |= !strcmp(p->rm_in.v[j], in) && !strcmp(p->rm_type.v[j], ty);
        if (!dup) { sl_add(&p->rm_in, in); sl_add(&p->rm_type, ty); }
        free(in);
        free(ty);
    }
    for (int i = 0; i < nfields; i++) sl_add(&p->field_args, fields[i]);
    if (build_dissectors(p, logformat, err, errlen)) { return NULL; }
    if (for_paths) return p;
    for (int i = 0; i < nfields; i++) {
        char *c = cleanup_field(fields[i]);
        sl_add_unique(&p->needed, c);
        free(c);
    }
    /* Parser.assembleDissectors (core/Parser.java:300-356) */
    for (int i = 0; i < p->ndis; i++)
        if (p->dis[i]->outs.n == 0) {
            snprintf(err, errlen, "InvalidDissectorException: Dissector cannot create any outputs (%s)", p->dis[i]->in_type);
            return NULL;
        }
    slist needed = {0};
    for (int i = 0; i < p->needed.n; i++) sl_add(&needed, p->needed.v[i]);
    char *rootneed = xfmt("%s:", p->root_type);
    sl_add(&needed, rootneed);
    free(rootneed);
    slist possible = {0};
    for (int i = 0; i < needed.n; i++) {
        const char *nm = strchr(needed.v[i], ':') + 1;
        char sb[1024];
        sb[0] = 0;
        size_t sbl = 0;
        const char *s = nm;
        for (;;) {
            const char *dot = strchr(s, '.');
            size_t pl = dot ? (size_t)(dot - s) : strlen(s);
            if (sbl == 0 || pl == 0) { memcpy(sb + sbl, s, pl); sbl += pl; }
            else { sb[sbl++] = '.'; memcpy(sb + sbl, s, pl); sbl += pl; }
            sb[sbl] = 0;
            sl_add_unique(&possible, sb);
            if (!dot) break;
            s = dot + 1;
        }
    }
    find_useful(p, &possible, p->root_type, "", 1);
    sl_free(&needed);
    sl_free(&possible);
    /* prepareForRun on every phase */
    for (int i = 0; i < p->ncompiled; i++)
        for (int k = 0; k < p->compiled[i].n; k++) {
            instance *in = p->compiled[i].ph[k];
            if (in->d->cls == D_ROOT) {
                if (in->nfmts == 0) { snprintf(err, errlen, "InvalidDissectorException: Cannot run without logformats"); return NULL; }
                for (int f = 0; f < in->nfmts; f++) {
                    fmt_prepare_for_run(in->fmts[f]);
                    if (in->fmts[f]->unsupported && !p->unsupported) {
                        p->unsupported = 1;
                        snprintf(p->unsupported_why, sizeof p->unsupported_why, "logformat not restated: %s", in->fmts[f]->logformat);
                    }
                }
            }
        }
    if (p->ncompiled == 0) { snprintf(err, errlen, "MissingDissectorsException: There are no dissectors at all"); return NULL; }
    /* getTheMissingFields (core/Parser.java:472-490) */
    for (int i = 0; i < p->needed.n; i++) {
        const char *t = p->needed.v[i];
        if (sl_has(&p->located, t)) continue;
        size_t L = strlen(t);
        if (L && t[L - 1] == '*') {
            if (L >= 2 && t[L - 2] == '.') {
                char *pre = xfmt("%.*s", (int)(L - 2), t);
                int ok = sl_has(&p->located, pre);
                free(pre);
                if (!ok) { snprintf(err, errlen, "MissingDissectorsException: %s", t); return NULL; }
            }
        } else { snprintf(err, errlen, "MissingDissectorsException: %s", t); return NULL; }
    }
    if (p->unsupported) { snprintf(err, errlen, "unsupported: %s", p->unsupported_why); return NULL; }
    return p;
}

orc_parser *orc_new(const char *logformat, const char *const *fields, int nfields, char *err, int errlen) {
    if (err && errlen) err[0] = 0;
    return build(logformat, fields, nfields, NULL, NULL, 0, err, errlen, 0);
}

orc_parser *orc_new_remapped(const char *logformat, const char *const *fields, int nfields, const char *const *rm_in,
                             const char *const *rm_type, int n_rm, char *err, int errlen) {
    if (err && errlen) err[0] = 0;
    return build(logformat, fields, nfields, rm_in, rm_type, n_rm, err, errlen, 0);
}

void orc_free(orc_parser *p) {
    /* the oracle is short-lived test code; formats/dissectors are leaked */
    if (!p) return;
    ar_free(&p->ar);
    free(p);
}

int orc_format_regex(orc_parser *p, int i, char *out, int out_cap) {
    centry *ce = c_get(p, "HTTPLOGLINE:");
    if (!ce || ce->n == 0) return -1;
    instance *in = ce->ph[0];
    if (i < 0 || i >= in->nfmts || !in->fmts[i]->regex) return -1;
    int L = (int)strlen(in->fmts[i]->regex);
    if (L + 1 > out_cap) return -1;
    memcpy(out, in->fmts[i]->regex, (size_t)L + 1);
    return L;
}

/* JSON output helpers */
typedef struct { char *b; int n, cap; int overflow; } ob;
static void ob_put(ob *o, const char *s, int n) {
    if (o->n + n + 1 > o->cap) { o->overflow = 1; return; }
    memcpy(o->b + o->n, s, (size_t)n);
    o->n += n;
    o->b[o->n] = 0;
}
static void ob_s(ob *o, const char *s) { ob_put(o, s, (int)strlen(s)); }
static void ob_json_str(ob *o, const char *s, int n) {
    ob_put(o, "\"", 1);
    for (int i = 0; i < n; i++) {
        unsigned char c = (unsigned char)s[i];
        char e[8];
        if (c == '"') ob_put(o, "\\\"", 2);
        else if (c == '\\') ob_put(o, "\\\\", 2);
        else if (c < 0x20) { snprintf(e, sizeof e, "\\u%04x", c); ob_put(o, e, 6); }
        else ob_put(o, (const char *)&c, 1);
    }
    ob_put(o, "\"", 1);
}

int orc_token_table(int nginx, char *out, int out_cap) {
    pthread_once(&g_tps_once, init_tps);
    const tplist *l = nginx ? &g_nginx_tps : &g_apache_tps;
    ob o = {out, 0, out_cap, 0};
    if (out_cap > 0) out[0] = 0;
    ob_s(&o, "[");
    for (int k = 0; k < l->n; k++) {
        const tparser *t = &l->v[k];
        const char *kind = t->kind == TP_FIXED ? "fixed" : t->kind == TP_NAMED ? "named" : t->kind == TP_PARAM ? "param" : "plain";
        ob_s(&o, k ? ",\n{\"kind\":" : "{\"kind\":");
        ob_json_str(&o, kind, (int)strlen(kind));
        ob_s(&o, ",\"token\":");
        ob_json_str(&o, t->tok, (int)strlen(t->tok));
        ob_s(&o, ",\"regex\":");
        ob_json_str(&o, t->regex, (int)strlen(t->regex));
        char b[64];
        snprintf(b, sizeof b, ",\"prio\":%d,\"custom\":", t->prio);
        ob_s(&o, b);
        ob_s(&o, t->custom == CUSTOM_STRFTIME ? "\"StrfTimeStampDissector\"" : "null");
        ob_s(&o, ",\"outs\":[");
        for (int j = 0; j < t->nouts; j++) {
            const ofield *u = &t->outs[j];
            ob_s(&o, j ? ",[" : "[");
            ob_json_str(&o, u->type, (int)strlen(u->type));
            ob_s(&o, ",");
            ob_json_str(&o, u->name, (int)strlen(u->name));
            int first = 1;
            ob_s(&o, ",[");
            if (u->casts & C_S) { ob_s(&o, "\"STRING\""); first = 0; }
            if (u->casts & C_L) { ob_s(&o, first ? "\"LONG\"" : ",\"LONG\""); first = 0; }
            if (u->casts & C_D) ob_s(&o, first ? "\"DOUBLE\"" : ",\"DOUBLE\"");
            ob_s(&o, "]]");
        }
        ob_s(&o, "]}");
    }
    ob_s(&o, "]");
    return o.overflow ? -1 : o.n;
}

static int rcmp(const void *a, const void *b) {
    const rentry *x = (const rentry *)a, *y = (const rentry *)b;
    int c = strcmp(x->name, y->name);
    if (c) return c;
    return x->seq - y->seq;
}

int orc_parse(orc_parser *p, const char *line, int len, char *out, int out_cap) {
    parsable ps;
    memset(&ps, 0, sizeof ps);
    ps.p = p;
    ar_reset(&p->ar);
    ps.a = &p->ar;
    js l = js_from_utf8(ps.a, line, len);
    /* reject invalid UTF-8 input (callers decode bytes with replacement;
     * that decoding is outside the restated path) */
    {
        const unsigned char *u = (const unsigned char *)line;
        for (int i = 0; i < len;) {
            unsigned c = u[i];
            int need = c < 0x80 ? 0 : (c >= 0xC2 && c <= 0xDF) ? 1 : (c >= 0xE0 && c <= 0xEF) ? 2 : (c >= 0xF0 && c <= 0xF4) ? 3 : -1;
            if (need < 0) return ORC_UNSUPPORTED;
            unsigned cp = need == 1 ? (c & 0x1F) : need == 2 ? (c & 0x0F) : (c & 0x07);
            for (int k = 1; k <= need; k++) {
                if (i + k >= len || (u[i + k] & 0xC0) != 0x80) return ORC_UNSUPPORTED;
                cp = (cp << 6) | (u[i + k] & 0x3F);
            }
            /* overlong forms, surrogates and code points past U+10FFFF decode to U+FFFD */
            if ((need == 2 && (cp < 0x800 || (cp >= 0xD800 && cp <= 0xDFFF))) || (need == 3 && (cp < 0x10000 || cp > 0x10FFFF)))
                return ORC_UNSUPPORTED;
            i += need + 1;
        }
    }
    cache_put(&ps, p->root_type, "", vstr(l));
    todo_add(&ps, p->root_type, "");
    /* Parser.parse(Parsable) worklist (core/Parser.java:726-756) */
    int guard = 0;
    while (ps.ntodo > 0 && !ps.failed && !ps.unsupported) {
        int n = ps.ntodo;
        pfield *batch = (pfield *)malloc(sizeof(pfield) * (size_t)n);
        memcpy(batch, ps.todo, sizeof(pfield) * (size_t)n);
        ps.ntodo = 0;
        for (int i = 0; i < n && !ps.failed && !ps.unsupported; i++) {
            char id[1024];
            snprintf(id, sizeof id, "%s:%s", batch[i].type, batch[i].name);
            centry *ce = c_get(p, id);
            if (!ce) continue;
            for (int k = 0; k < ce->n && !ps.failed && !ps.unsupported; k++) run_instance(&ps, ce->ph[k], batch[i].name);
        }
        free(batch);
        if (++guard > 64) { ps.unsupported = 1; break; }
    }
    int status = ps.unsupported ? ORC_UNSUPPORTED : ps.failed ? ORC_BAD : ORC_OK;
    if (status == ORC_OK && out) {
        if (ps.nrec > 1) qsort(ps.rec, (size_t)ps.nrec, sizeof(rentry), rcmp);
        ob o = {out, 0, out_cap, 0};
        out[0] = 0;
        ob_s(&o, "{");
        for (int i = 0; i < ps.nrec;) {
            if (i) ob_s(&o, ",");
            ob_json_str(&o, ps.rec[i].name, (int)strlen(ps.rec[i].name));
            ob_s(&o, ":[");
            int j = i;
            for (; j < ps.nrec && strcmp(ps.rec[j].name, ps.rec[i].name) == 0; j++) {
                if (j > i) ob_s(&o, ",");
                val v = ps.rec[j].v;
                if (v.filled == V_LONG) {
                    char b[48];
                    if (v.lnull) snprintf(b, sizeof b, "{\"l\":null}");
                    else snprintf(b, sizeof b, "{\"l\":%lld}", (long long)v.l);
                    ob_s(&o, b);
                } else if (v.s.null) ob_s(&o, "null");
                else {
                    int bl;
                    char *u8 = js_to_utf8(ps.a, v.s, &bl);
                    ob_json_str(&o, u8, bl);
                }
            }
            ob_s(&o, "]");
            i = j;
        }
        ob_s(&o, "}");
        if (o.overflow) status = -1;
    }
    free(ps.cache);
    free(ps.todo);
    free(ps.rec);
    return status;
}

/* Parser.getPossiblePaths (core/Parser.java:914-1012) */
static void find_paths(orc_parser *p, slist *paths, const char *base, const char *btype, int depth) {
    if (depth == 0) return;
    for (int di = 0; di < p->ndis; di++) {
        dissector *d = p->dis[di];
        if (strcmp(d->in_type, btype) != 0) continue;
        for (int oi = 0; oi < d->outs.n; oi++) {
            const char *o = d->outs.v[oi];
            const char *colon = strchr(o, ':');
            char *ctype = xfmt("%.*s", (int)(colon - o), o);
            const char *cname = colon + 1;
            char *cbase;
            if (base[0] == 0) cbase = xstrdup(cname);
            else if (cname[0] == 0) cbase = xstrdup(base);
            else cbase = xfmt("%s.%s", base, cname);
            char *np = xfmt("%s:%s", ctype, cbase);
            if (!sl_has(paths, np)) {
                sl_add(paths, np);
                find_paths(p, paths, cbase, ctype, depth - 1);
            }
            free(np);
            free(cbase);
            free(ctype);
        }
    }
}

static int scmp(const void *a, const void *b) { return strcmp(*(char *const *)a, *(char *const *)b); }

int orc_possible_paths(const char *logformat, int max_depth, char *out, int out_cap) {
    char err[256];
    pthread_once(&g_re_once, init_res);
    orc_parser *p = build(logformat, NULL, 0, NULL, NULL, 0, err, sizeof err, 1);
    if (!p) return -1;
    slist paths = {0};
    find_paths(p, &paths, "", p->root_type, max_depth);
    qsort(paths.v, (size_t)paths.n, sizeof(char *), scmp);
    int n = 0;
    for (int i = 0; i < paths.n; i++) {
        int L = (int)strlen(paths.v[i]);
        if (n + L + 2 > out_cap) { sl_free(&paths); return -1; }
        memcpy(out + n, paths.v[i], (size_t)L);
        n += L;
        out[n++] = '\n';
    }
    out[n] = 0;
    sl_free(&paths);
    return n;
}

int orc_resilient_url_decode(const char *in, int len, char *out, int out_cap) {
    pthread_once(&g_re_once, init_res);
    arena a = {0};
    parsable ps;
    memset(&ps, 0, sizeof ps);
    ps.a = &a;
    js s = js_from_utf8(&a, in, len);
    js r;
    int st = resilient_url_decode(&ps, s, &r);
    int n = -1;
    if (st == 0) {
        int bl;
        char *u8 = js_to_utf8(&a, r, &bl);
        if (bl + 1 <= out_cap) { memcpy(out, u8, (size_t)bl + 1); n = bl; }
    } else n = st == 1 ? -2 : -3;
    ar_free(&a);
    return n;
}

/* ------------------------------------------------------------- bench */
typedef struct {
    const char *logformat;
    const char *const *fields;
    int nfields;
    const char *buf;
    size_t from, to;
    int64_t lines, ok, bad, unsup;
} bench_job;

static void *bench_thread(void *arg) {
    bench_job *j = (bench_job *)arg;
    char err[256];
    orc_parser *p = orc_new(j->logformat, j->fields, j->nfields, err, sizeof err);
    if (!p) return NULL;
    static __thread char out[1 << 16];
    size_t i = j->from;
    while (i < j->to) {
        const char *nl = (const char *)memchr(j->buf + i, '\n', j->to - i);
        size_t e = nl ? (size_t)(nl - j->buf) : j->to;
        int st = orc_parse(p, j->buf + i, (int)(e - i), out, sizeof out);
        j->lines++;
        if (st == ORC_OK) j->ok++; else if (st == ORC_BAD) j->bad++; else j->unsup++;
        i = e + 1;
    }
    orc_free(p);
    return NULL;
}

double orc_bench(const char *logformat, const char *const *fields, int nfields,
                 const char *buf, size_t nbytes, int nthreads, int64_t *out4) {
    if (nthreads < 1) nthreads = 1;
    bench_job *jobs = (bench_job *)xmalloc(sizeof(bench_job) * (size_t)nthreads);
    pthread_t *th = (pthread_t *)xmalloc(sizeof(pthread_t) * (size_t)nthreads);
    /* newline-aligned contiguous ranges, one parser per thread */
    size_t start = 0;
    for (int t = 0; t < nthreads; t++) {
        size_t end = t == nthreads - 1 ? nbytes : (nbytes * (size_t)(t + 1)) / (size_t)nthreads;
        if (end < start) end = start;
        while (end < nbytes && end > 0 && buf[end - 1] != '\n') end++;
        jobs[t].logformat = logformat;
        jobs[t].fields = fields;
        jobs[t].nfields = nfields;
        jobs[t].buf = buf;
        jobs[t].from = start;
        jobs[t].to = end;
        start = end;
    }
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, bench_thread, &jobs[t]);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &b);
    int64_t tot[4] = {0, 0, 0, 0};
    for (int t = 0; t < nthreads; t++) { tot[0] += jobs[t].lines; tot[1] += jobs[t].ok; tot[2] += jobs[t].bad; tot[3] += jobs[t].unsup; }
    if (out4) memcpy(out4, tot, sizeof tot);
    free(jobs);
    free(th);
    return (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
}
