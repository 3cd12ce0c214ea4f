// Host setup: LogFormat compilation, dissection-tree planning and device
// Program construction, plus the per-line replay of device results.
//
// Restates (reference paths; hp/ = httpdlog/httpdlog-parser/src/main/java/nl/basjes/parse/httpdlog/,
// core/ = parser-core/src/main/java/nl/basjes/parse/core/):
//   ApacheHttpdLogFormatDissector.setLogFormat / cleanupLogFormat / createAllTokenParsers
//                                         hp/ApacheHttpdLogFormatDissector.java:73-167, 199-714
//   TokenParser / NamedTokenParser / ParameterizedTokenParser .getNextToken / getTokens
//                                         hp/dissectors/tokenformat/*.java
//   TokenFormatDissector.parseTokenLogFileDefinition (sort, kick, fixed-string gaps)
//                                         hp/dissectors/tokenformat/TokenFormatDissector.java:294-379
//   HttpdLogFormatDissector.addLogFormat  hp/HttpdLogFormatDissector.java:99-140
//   HttpdLoglineParser.setupDissectors    hp/HttpdLoglineParser.java:104-126
//   Parser.assembleDissectors / findUsefulDissectorsFromField / getTheMissingFields / getPossiblePaths
//                                         core/Parser.java:237-490, 904-1012
//   Parsable.addDissection                core/Parsable.java:142-193 (replay)
#include "plan.h"

#include <atomic>
#include <unordered_map>

namespace {
std::atomic<uint64_t> g_plan_gen{1};  // Plan build ids (the replay memo's key)
}  // namespace
#include "lp_device.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <deque>
#include <functional>

#include "../../include/logparser_amd.h"

namespace lp {

namespace {

// --------------------------------------------------------------- regexes
// hp/dissectors/tokenformat/TokenParser.java:35-59
const std::string R_DIGIT = "[0-9]";
const std::string R_NUMBER = R_DIGIT + "+";
const std::string R_CLF_NUMBER = R_NUMBER + "|-";
const std::string R_HEXDIGIT = "[0-9a-fA-F]";
const std::string R_HEXNUMBER = R_HEXDIGIT + "+";
const std::string R_CLF_HEXNUMBER = R_HEXNUMBER + "|-";
const std::string R_NON_ZERO = "[1-9][0-9]*";
const std::string R_8BIT = "(?:25[0-5]|2[0-4][0-9]|[01]?[0-9][0-9]?)";
const std::string R_IPV4 = "(?:" + R_8BIT + "\\.){3}" + R_8BIT;
const std::string R_IPV6 = ":?(?:" + R_HEXDIGIT + "{1,4}(?::|.)?){0,8}(?::|::)?(?:" + R_HEXDIGIT + "{1,4}(?::|.)?){0,8}";
const std::string R_IP = R_IPV4 + "|" + R_IPV6;
const std::string R_CLF_IP = R_IP + "|-";
const std::string R_STRING = ".*?";
const std::string R_NO_SPACE = "[^\\s]*";
const std::string R_TIME_US =
    "[0-3][0-9]/(?:[a-zA-Z][a-zA-Z][a-zA-Z])/[1-9][0-9][0-9][0-9]:[0-9][0-9]:[0-9][0-9]:[0-9][0-9] [\\+|\\-][0-9][0-9][0-9][0-9]";
const std::string R_FIRSTLINE = ".*";  // hp/dissectors/HttpFirstLineDissector.java:56-57
const std::string R_TIME_ISO8601 =
    "[1-9][0-9][0-9][0-9]-[0-1][0-9]-[0-3][0-9]T[0-9][0-9]:[0-9][0-9]:[0-9][0-9][\\+|\\-][0-9][0-9]:[0-9][0-9]";
const std::string R_NUMBER_DECIMAL = R_NUMBER + "\\." + R_NUMBER;
const std::string R_NUMBER_OPT_DECIMAL = R_NUMBER + "(?:\\." + R_NUMBER + ")?";
const std::string R_MSEC = "[0-9]+\\.[0-9][0-9][0-9]";      // nginxmodules/CoreLogModule.java:56-58
const std::string R_NOSPACE3 = R_NO_SPACE + " " + R_NO_SPACE + " " + R_NO_SPACE;  // $request (CoreLogModule.java:296-300)
// $binary_remote_addr (CoreLogModule.java): four "\\x" + 2 hex digits
const std::string R_BINIP = "\\\\x" + R_HEXDIGIT + R_HEXDIGIT + "\\\\x" + R_HEXDIGIT + R_HEXDIGIT + "\\\\x" + R_HEXDIGIT +
                            R_HEXDIGIT + "\\\\x" + R_HEXDIGIT + R_HEXDIGIT;
// UpstreamModule.upstreamListOf (nginxmodules/UpstreamModule.java:42-44)
std::string upstream_list(const std::string& x) { return x + "(?: *, *" + x + "(?: *: *" + x + ")?)*"; }

int elem_kind_of(const std::string& r) {
    if (r == R_NO_SPACE) return EK_NOSPACE;
    if (r == R_NUMBER) return EK_NUMBER;
    if (r == R_CLF_NUMBER) return EK_CLFNUMBER;
    if (r == R_HEXNUMBER) return EK_HEXNUMBER;
    if (r == R_CLF_HEXNUMBER) return EK_CLFHEXNUMBER;
    if (r == R_NON_ZERO) return EK_NONZERO;
    if (r == R_FIRSTLINE) return EK_ANY_GREEDY;
    if (r == R_STRING) return EK_ANY_LAZY;
    if (r == R_TIME_US) return EK_TIME_US;
    if (r == R_CLF_IP) return EK_CLF_IP;
    if (r == R_IP) return EK_IP;
    if (r == ".") return EK_ANYCHAR;
    if (r == R_NUMBER_DECIMAL) return EK_DECIMAL;
    if (r == R_MSEC) return EK_MSEC;
    if (r == R_NOSPACE3) return EK_NOSPACE3;
    if (r == upstream_list(R_NUMBER_DECIMAL)) return EK_UPLIST_DEC;
    if (r == upstream_list(R_NUMBER)) return EK_UPLIST_NUM;
    if (r == upstream_list(R_NO_SPACE)) return EK_UPLIST_NS;
    if (r == R_BINIP) return EK_BINIP;
    if (r == R_TIME_ISO8601) return EK_TIME_ISO;
    if (r == "(?:MISS|BYPASS|EXPIRED|STALE|UPDATING|REVALIDATED|HIT)") return EK_CACHE_STATUS;  // UpstreamModule.java
    return -1;
}

// ----------------------------------------------------------- token table
enum TpKind { TP_PLAIN, TP_FIXED, TP_NAMED, TP_PARAM, TP_DOLLAR };

struct TParser {
    TpKind kind;
    std::string tok;   // PLAIN/FIXED literal token; NAMED/PARAM: id of the pattern
    std::string regex;
    int prio = 0;
    std::vector<TokOut> outs;
    bool strftime = false;
    // NAMED pattern: "%{" NAMECLASS* "}" suffix ; PARAM: "%{" prefix [^}]*%[^}]* "}t"
    std::string suffix;     // NAMED suffix after '}' (e.g. "i", "^ti")
    bool underscore = true; // NAMED class includes '_'
    std::string pprefix;    // PARAM prefix inside braces ("", "begin:", "end:"); DOLLAR: "$" + name prefix
};

std::string lower(std::string s) {
    for (auto& c : s) if (c >= 'A' && c <= 'Z') c = char(c + 32);
    return s;
}
std::string upper(std::string s) {
    for (auto& c : s) if (c >= 'a' && c <= 'z') c = char(c - 32);
    return s;
}

struct TokenTable {
    std::vector<TParser> v;
    TParser& add(TpKind k, const std::string& tok, const std::string& re, int prio) {
        v.push_back(TParser{k, tok, re, prio, {}, false, "", true, ""});
        return v.back();
    }
    static void out(TParser& t, const std::string& type, const std::string& name, int casts) {
        t.outs.push_back(TokOut{type, lower(name), casts});  // TokenOutputField lowercases (TokenOutputField.java:39-44)
    }
    // createFirstAndLastTokenParsers (ApacheHttpdLogFormatDissector.java:651-714)
    void fl(const std::string& token, const std::string& name, const std::string& type, int casts,
            const std::string& re, int prio = 0) {
        static const char* orig[] = {"%s", "%U", "%T", "%{us}T", "%{ms}T", "%{s}T", "%D", "%r"};
        bool o = false;
        for (auto* x : orig) if (token == x) o = true;
        auto& a = add(TP_PLAIN, token, re, prio);
        out(a, type, name, casts);
        out(a, type, name + (o ? ".original" : ".last"), casts);
        size_t pc = token.find('%');
        auto& b = add(TP_PLAIN, token.substr(0, pc) + "%<" + token.substr(pc + 1), re, prio);
        out(b, type, name + ".original", casts);
        auto& c = add(TP_PLAIN, token.substr(0, pc) + "%>" + token.substr(pc + 1), re, prio);
        out(c, type, name + ".last", casts);
    }
    void extra(const std::string& token, const std::string& type, const std::string& name, int casts) {
        for (auto& t : v)
            if (t.tok == token) { out(t, type, name, casts); return; }
    }
    void named(const std::string& suffix, bool underscore, const std::string& name, const std::string& type) {
        auto& t = add(TP_NAMED, "named:" + suffix, R_STRING, 0);
        t.suffix = suffix;
        t.underscore = underscore;
        out(t, type, name, CAST_S);
    }
    // NGINX (nginxmodules/*.java): TokenParser (default prio 10), NamedTokenParser
    // "\\$prefix([a-z0-9\\-_]*)" (default prio 0), NotImplementedTokenParser
    void ng(const std::string& token, const std::string& name, const std::string& type, int casts,
            const std::string& re, int prio) {
        out(add(TP_PLAIN, token, re, prio), type, name, casts);
    }
    void ngnamed(const std::string& pattern, const std::string& name, const std::string& type, int casts,
                 const std::string& re, int prio) {
        auto& t = add(TP_DOLLAR, pattern, re, prio);
        t.pprefix = "$" + pattern.substr(2, pattern.find('(') - 2);  // "\\$http_(...)" -> "$http_"
        out(t, type, name, casts);
    }
    void ngnotimpl(const std::string& token, const std::string& prefix, const std::string& re, int prio) {
        std::string n = prefix + "_";  // TokenFormatDissector.java:95-102
        for (char c : lower(token)) n += ((c >= 'a' && c <= 'z') || (c >= '0' && c <= '9') || c == '_') ? c : '_';
        out(add(TP_PLAIN, token, re, prio), "NOT_IMPLEMENTED", n, CAST_S);
    }
    void param(const std::string& prefix, const std::string& name, int prio) {
        auto& t = add(TP_PARAM, "param:" + prefix, R_STRING, prio);
        t.pprefix = prefix;
        t.strftime = true;
        out(t, "TIME.STRFTIME_", name, CAST_S);
    }
};

// StrfTimeToDateTimeFormatter (hp/dissectors/StrfTimeToDateTimeFormatter.java
// :140-432, grammar StrfTime.g4:40-89): the DateTimeFormatterBuilder
// elements of each conversion (E / O modifiers ignored).  %c %C %U %w %x %X
// %+ throw UnsupportedStrfField in the reference (no parser can be built),
// and a variable-width number directly followed by another number switches
// JDK's adjacent value parsing on: those stay off the device.
static bool strf_compile(const std::string& f, TimeStage& T) {
    T.n_ops = 0;
    T.zone = 0;
    auto add = [&](int kind, int field, int width, int arg) {
        if (T.n_ops >= MAX_SF_OPS) return false;
        T.op[T.n_ops++] = (uint32_t)kind | ((uint32_t)field << 8) | ((uint32_t)width << 16) | ((uint32_t)(uint8_t)arg << 24);
        return true;
    };
    auto num = [&](int field, int w) { return add(SE_NUM, field, w, 0); };
    auto lit = [&](int c) { return add(SE_LIT, 0, 1, c); };
    const size_t n = f.size();
    for (size_t i = 0; i < n;) {
        const size_t j = i + (f[i] == '%');
        if (n - j >= 9 && (f.compare(j, 9, "msec_frac") == 0 || f.compare(j, 9, "usec_frac") == 0)) {
            if (!(f[j] == 'm' ? num(SF_MILLI, 3) : num(SF_MICRO, 6))) return false;
            i = j + 9;
            continue;
        }
        if (f[i] != '%') {
            if (!lit((uint8_t)f[i])) return false;
            ++i;
            continue;
        }
        if (i + 1 >= n) return false;
        char c = f[i + 1];
        size_t k = i + 1;
        if (c == '%' || c == 't' || c == 'n') {
            if (!lit(c == '%' ? '%' : c == 't' ? '\t' : '\n')) return false;
            i += 2;
            continue;
        }
        if (c == 'E' || c == 'O') {
            if (i + 2 >= n) return false;
            c = f[i + 2];
            ++k;
        }
        bool ok;
        switch (c) {
        case 'a': ok = add(SE_TEXT, SF_DOW, 0, ST_DOW_SHORT); break;
        case 'A': ok = add(SE_TEXT, SF_DOW, 0, ST_DOW_FULL); break;
        case 'b': case 'h': ok = add(SE_TEXT, SF_MONTH, 0, ST_MON_SHORT); break;
        case 'B': ok = add(SE_TEXT, SF_MONTH, 0, ST_MON_FULL); break;
        case 'd': ok = num(SF_DOM, 2); break;
        case 'D': ok = num(SF_MONTH, 2) && lit('/') && num(SF_DOM, 2) && lit('/') && add(SE_RED2, SF_YEAR, 2, 0); break;
        case 'e': ok = add(SE_PAD2, SF_DOM, 2, 0); break;
        case 'F': ok = num(SF_YEAR, 4) && lit('-') && num(SF_MONTH, 2) && lit('-') && num(SF_DOM, 2); break;
        case 'G': ok = num(SF_WBY, 4); break;
        case 'g': ok = add(SE_RED2, SF_WBY, 2, 0); break;
        case 'H': ok = num(SF_CHOD, 2); break;
        case 'I': ok = num(SF_CHAP, 2); break;
        case 'j': ok = num(SF_DOY, 3); break;
        case 'k': ok = add(SE_PAD2, SF_CHOD, 2, 0); break;
        case 'l': ok = add(SE_PAD2, SF_CHAP, 2, 0); break;
        case 'm': ok = num(SF_MONTH, 2); break;
        case 'M': ok = num(SF_MIN, 2); break;
        case 'p': ok = add(SE_TEXT, SF_AMPM, 0, ST_AMPM_UP); break;
        case 'P': ok = add(SE_TEXT, SF_AMPM, 0, ST_AMPM_LOW); break;
        case 'r': ok = num(SF_CHAP, 2) && lit(':') && num(SF_MIN, 2) && lit(':') && num(SF_SEC, 2) && lit(' ') &&
                       add(SE_TEXT, SF_AMPM, 0, ST_AMPM_UP); break;
        case 'R': ok = num(SF_HOD, 2) && lit(':') && num(SF_MIN, 2); break;
        case 's': ok = add(SE_NUMV, SF_INSTANT, 19, 0); break;
        case 'S': ok = num(SF_SEC, 2); break;
        case 'T': ok = num(SF_HOD, 2) && lit(':') && num(SF_MIN, 2) && lit(':') && num(SF_SEC, 2); break;
        case 'u': ok = num(SF_ISODOW, 1); break;
        case 'V': ok = add(SE_NUMV, SF_WOY, 19, 0); break;
        case 'W': ok = num(SF_WOY, 2); break;
        case 'y': ok = add(SE_RED2, SF_YEAR, 2, 0); break;
        case 'Y': ok = num(SF_YEAR, 4); break;
        case 'z': ok = add(SE_OFF, SF_OFFSET, 5, 0); T.zone = 1; break;
        case 'Z': ok = add(SE_ZONE, 0, 0, 0); T.zone = 1; break;
        default: ok = false; break;
        }
        if (!ok) return false;
        i = k + 1;
    }
    for (int e = 0; e + 1 < T.n_ops; ++e) {  // adjacent value parsing
        const int k0 = T.op[e] & 0xFF, k1 = T.op[e + 1] & 0xFF;
        const bool num1 = k1 == SE_NUM || k1 == SE_NUMV || k1 == SE_PAD2 || k1 == SE_RED2;
        if ((k0 == SE_NUMV || k0 == SE_PAD2) && num1) return false;
    }
    // a layout of fixed-width elements only (e.g. %d/%b/%Y %T): the device
    // parses a value of exactly that width from registers (strf_fixed)
    T.fixed_w = 0;
    int w = 0;
    for (int e = 0; e < T.n_ops && w >= 0; ++e) {
        const int kind = T.op[e] & 0xFF, width = (T.op[e] >> 16) & 0xFF, arg = T.op[e] >> 24;
        switch (kind) {
        case SE_LIT: w += 1; break;
        case SE_NUM: case SE_RED2: w += width; break;
        case SE_TEXT: w = arg == ST_MON_SHORT || arg == ST_DOW_SHORT ? w + 3 : arg == ST_AMPM_UP || arg == ST_AMPM_LOW ? w + 2 : -1; break;
        case SE_OFF: w += 5; break;
        default: w = -1; break;
        }
    }
    if (w > 0 && w <= 32) T.fixed_w = w;
    // ... and as byte masks + field offsets (strf_fixed): a value of that
    // width whose literals, digits and fields all check is the general loop's
    // parse, any failing check its ST_BAD; a field given twice (the general
    // loop's "must agree" check) keeps the general loop
    T.fx_n = 0;
    T.fx_has = 0;
    for (int j = 0; j < 8; ++j) T.fx_lit[j] = T.fx_litm[j] = T.fx_fold[j] = T.fx_dig[j] = 0;
    if (T.fixed_w > 0) {
        int off = 0, nf = 0;
        bool ok = true;
        auto put = [&](uint32_t* a, int i, uint32_t byte) { a[i >> 2] |= byte << (8 * (i & 3)); };
        for (int e = 0; e < T.n_ops && ok; ++e) {
            const int kind = T.op[e] & 0xFF, field = (T.op[e] >> 8) & 0xFF, width = (T.op[e] >> 16) & 0xFF;
            const int arg = T.op[e] >> 24;
            if (kind == SE_LIT) {
                const bool letter = ((arg | 0x20) - 'a') < 26;
                put(T.fx_lit, off, letter ? (uint32_t)(arg | 0x20) : (uint32_t)arg);
                put(T.fx_litm, off, 0xFF);
                if (letter) put(T.fx_fold, off, 0x20);
                ++off;
                continue;
            }
            int code, n;
            switch (kind) {
            case SE_NUM: case SE_RED2: code = kind == SE_NUM ? FX_NUM : FX_RED2; n = width; break;
            case SE_TEXT: code = FX_TEXT | (arg << 4); n = arg == ST_MON_SHORT || arg == ST_DOW_SHORT ? 3 : 2; break;
            default: code = FX_OFF; n = 5; break;  // SE_OFF (fixed_w admits no other kind)
            }
            if (nf >= MAX_FX || (T.fx_has >> field) & 1u || n > 8) { ok = false; break; }
            for (int q = 0; q < n; ++q)
                if ((code == FX_NUM || code == FX_RED2) || (code == FX_OFF && q > 0)) put(T.fx_dig, off + q, 0xFF);
            T.fx_f[nf++] = (uint32_t)off | (uint32_t)n << 8 | (uint32_t)field << 16 | (uint32_t)code << 24;
            T.fx_has |= 1u << field;
            off += n;
        }
        if (ok && off == T.fixed_w) T.fx_n = nf;
    }
    return true;
}

// ApacheHttpdLogFormatDissector.createAllTokenParsers (:199-638)
const TokenTable& apache_table() {
    static TokenTable T = [] {
        TokenTable t;
        const int S = CAST_S, SL = CAST_S | CAST_L;
        t.add(TP_FIXED, "%%", "%", 0);
        t.fl("%a", "connection.client.ip", "IP", S, R_CLF_IP);
        t.fl("%{c}a", "connection.client.peerip", "IP", S, R_CLF_IP);
        t.fl("%A", "connection.server.ip", "IP", S, R_CLF_IP);
        t.fl("%B", "response.body.bytes", "BYTES", SL, R_NUMBER);
        t.fl("%b", "response.body.bytes", "BYTESCLF", SL, R_CLF_NUMBER);
        t.extra("%b", "BYTES", "response.body.bytesclf", SL);
        t.named("C", true, "request.cookies.", "HTTP.COOKIE");
        t.named("e", true, "server.environment.", "VARIABLE");
        t.fl("%f", "server.filename", "FILENAME", S, R_STRING);
        t.fl("%h", "connection.client.host", "IP", S, R_NO_SPACE);
        t.fl("%H", "request.protocol", "PROTOCOL", S, R_NO_SPACE);
        t.named("i", true, "request.header.", "HTTP.HEADER");
        t.named("^ti", true, "request.trailer.", "HTTP.TRAILER");
        t.fl("%k", "connection.keepalivecount", "NUMBER", SL, R_NUMBER);
        t.fl("%l", "connection.client.logname", "NUMBER", SL, R_CLF_NUMBER);
        t.fl("%L", "request.errorlogid", "STRING", S, R_NO_SPACE);
        t.fl("%m", "request.method", "HTTP.METHOD", S, R_NO_SPACE);
        t.named("n", true, "server.module_note.", "STRING");
        t.named("o", false, "response.header.", "HTTP.HEADER");
        t.named("^to", true, "response.trailer.", "HTTP.TRAILER");
        t.fl("%p", "request.server.port.canonical", "PORT", SL, R_NUMBER);
        t.fl("%{canonical}p", "connection.server.port.canonical", "PORT", SL, R_NUMBER);
        t.fl("%{local}p", "connection.server.port", "PORT", SL, R_NUMBER);
        t.fl("%{remote}p", "connection.client.port", "PORT", SL, R_NUMBER);
        t.fl("%P", "connection.server.child.processid", "NUMBER", SL, R_NUMBER);
        t.fl("%{pid}P", "connection.server.child.processid", "NUMBER", SL, R_NUMBER);
        t.fl("%{tid}P", "connection.server.child.threadid", "NUMBER", SL, R_NUMBER);
        t.fl("%{hextid}P", "connection.server.child.hexthreadid", "NUMBER", SL, R_CLF_HEXNUMBER);
        t.fl("%q", "request.querystring", "HTTP.QUERYSTRING", S, R_NO_SPACE);
        t.fl("%r", "request.firstline", "HTTP.FIRSTLINE", S, R_FIRSTLINE);
        t.fl("%R", "request.handler", "STRING", S, R_STRING);
        t.fl("%s", "request.status", "STRING", S, R_NO_SPACE, 0);
        t.fl("%t", "request.receive.time", "TIME.STAMP", S, R_TIME_US);
        t.param("", "request.receive.time", -1);
        t.param("begin:", "request.receive.time.begin", 0);
        t.param("end:", "request.receive.time.end", 0);
        t.fl("%{sec}t", "request.receive.time.sec", "TIME.SECONDS", SL, R_NUMBER);
        t.fl("%{begin:sec}t", "request.receive.time.begin.sec", "TIME.SECONDS", SL, R_NUMBER);
        t.fl("%{end:sec}t", "request.receive.time.end.sec", "TIME.SECONDS", SL, R_NUMBER);
        t.fl("%{msec}t", "request.receive.time.msec", "TIME.EPOCH", SL, R_NUMBER);
        t.extra("%{msec}t", "TIME.EPOCH", "request.receive.time.begin.msec", SL);
        t.fl("%{begin:msec}t", "request.receive.time.begin.msec", "TIME.EPOCH", SL, R_NUMBER);
        t.fl("%{end:msec}t", "request.receive.time.end.msec", "TIME.EPOCH", SL, R_NUMBER);
        t.fl("%{usec}t", "request.receive.time.usec", "TIME.EPOCH.USEC", SL, R_NUMBER);
        t.extra("%{usec}t", "TIME.EPOCH.USEC", "request.receive.time.begin.usec", SL);
        t.fl("%{begin:usec}t", "request.receive.time.begin.usec", "TIME.EPOCH.USEC", SL, R_NUMBER);
        t.fl("%{end:usec}t", "request.receive.time.end.usec", "TIME.EPOCH.USEC", SL, R_NUMBER);
        t.fl("%{msec_frac}t", "request.receive.time.msec_frac", "TIME.EPOCH", SL, R_NUMBER);
        t.extra("%{msec_frac}t", "TIME.EPOCH", "request.receive.time.begin.msec_frac", SL);
        t.fl("%{begin:msec_frac}t", "request.receive.time.begin.msec_frac", "TIME.EPOCH", SL, R_NUMBER);
        t.fl("%{end:msec_frac}t", "request.receive.time.end.msec_frac", "TIME.EPOCH", SL, R_NUMBER);
        t.fl("%{usec_frac}t", "request.receive.time.usec_frac", "TIME.EPOCH.USEC_FRAC", SL, R_NUMBER);
        t.extra("%{usec_frac}t", "TIME.EPOCH.USEC_FRAC", "request.receive.time.begin.usec_frac", SL);
        t.fl("%{begin:usec_frac}t", "request.receive.time.begin.usec_frac", "TIME.EPOCH.USEC_FRAC", SL, R_NUMBER);
        t.fl("%{end:usec_frac}t", "request.receive.time.end.usec_frac", "TIME.EPOCH.USEC_FRAC", SL, R_NUMBER);
        t.fl("%T", "response.server.processing.time", "SECONDS", SL, R_NUMBER);
        t.fl("%D", "response.server.processing.time", "MICROSECONDS", SL, R_NUMBER);
        t.extra("%D", "MICROSECONDS", "server.process.time", SL);
        t.fl("%{us}T", "response.server.processing.time", "MICROSECONDS", SL, R_NUMBER);
        t.fl("%{ms}T", "response.server.processing.time", "MILLISECONDS", SL, R_NUMBER);
        t.fl("%{s}T", "response.server.processing.time", "SECONDS", SL, R_NUMBER);
        t.fl("%u", "connection.client.user", "STRING", S, R_NO_SPACE);
        t.fl("%U", "request.urlpath", "URI", S, R_NO_SPACE);
        t.fl("%v", "connection.server.name.canonical", "STRING", S, R_NO_SPACE);
        t.fl("%V", "connection.server.name", "STRING", S, R_NO_SPACE);
        t.fl("%X", "response.connection.status", "HTTP.CONNECTSTATUS", S, R_NO_SPACE);
        t.fl("%I", "request.bytes", "BYTES", SL, R_CLF_NUMBER);
        t.fl("%O", "response.bytes", "BYTES", SL, R_CLF_NUMBER);
        t.fl("%S", "total.bytes", "BYTES", SL, R_NON_ZERO);
        t.fl("%{cookie}i", "request.cookies", "HTTP.COOKIES", S, R_STRING, 1);
        t.fl("%{set-cookie}o", "response.cookies", "HTTP.SETCOOKIES", S, R_STRING, 1);
        t.fl("%{user-agent}i", "request.user-agent", "HTTP.USERAGENT", S, R_STRING, 1);
        t.fl("%{referer}i", "request.referer", "HTTP.URI", S, R_STRING, 1);
        return t;
    }();
    return T;
}

// NginxHttpdLogFormatDissector.createAllTokenParsers (hp/NginxHttpdLogFormatDissector.java:121-142):
// the token parsers of every NGINX module, in module order
const TokenTable& nginx_table() {
    static TokenTable T;
    static bool init = false;
    if (init) return T;
    init = true;
    const int CAST_SL = CAST_S | CAST_L;
    (void)CAST_SL;

    /* CoreLogModule (nginxmodules/CoreLogModule.java:45-489) */
    T.ng("$bytes_sent", "response.bytes", "BYTES", CAST_SL, R_NUMBER, 10);
    T.ng("$bytes_received", "request.bytes", "BYTES", CAST_SL, R_NUMBER, 10);
    T.ng("$connection", "connection.serial_number", "NUMBER", CAST_SL, R_CLF_NUMBER, -1);
    T.ng("$connection_requests", "connection.requestnr", "NUMBER", CAST_SL, R_CLF_NUMBER, 10);
    T.ng("$msec", "request.receive.time.epoch", "TIME.EPOCH_SECOND_MILLIS", CAST_S, "[0-9]+\\.[0-9][0-9][0-9]", 10);
    T.ng("$status", "request.status.last", "STRING", CAST_S, R_NO_SPACE, 10);
    T.ng("$time_iso8601", "request.receive.time", "TIME.ISO8601", CAST_S, R_TIME_ISO8601, 10);
    T.ng("$time_local", "request.receive.time", "TIME.STAMP", CAST_S, R_TIME_US, 10);
    T.ngnamed("\\$arg_([a-z0-9\\-\\_]*)", "request.firstline.uri.query.", "STRING", CAST_S, R_STRING, 0);
    T.ng("$is_args", "request.firstline.uri.is_args", "STRING", CAST_S, R_STRING, 10);
    T.ng("$args", "request.firstline.uri.query", "HTTP.QUERYSTRING", CAST_S, R_STRING, 10);
    T.ng("$query_string", "request.firstline.uri.query", "HTTP.QUERYSTRING", CAST_S, R_STRING, 10);
    T.ng("$body_bytes_sent", "response.body.bytes", "BYTES", CAST_SL, R_NUMBER, 10);
    T.ng("$content_length", "request.header.content_length", "HTTP.HEADER", CAST_S, R_STRING, 10);
    T.ng("$content_type", "request.header.content_type", "HTTP.HEADER", CAST_S, R_STRING, 10);
    T.ngnamed("\\$cookie_([a-z0-9\\-_]*)", "request.cookies.", "HTTP.COOKIE", CAST_S, R_STRING, 0);
    T.ng("$document_root", "request.firstline.document_root", "STRING", CAST_S, R_NO_SPACE, 10);
    T.ng("$realpath_root", "request.firstline.realpath_root", "STRING", CAST_S, R_NO_SPACE, 10);
    T.ng("$host", "connection.server.name", "STRING", CAST_S, R_NO_SPACE, -1);
    T.ng("$hostname", "connection.client.host", "STRING", CAST_S, R_NO_SPACE, 10);
    T.ngnamed("\\$http_([a-z0-9\\-_]*)", "request.header.", "HTTP.HEADER", CAST_S, R_STRING, 0);
    T.ng("$http_user_agent", "request.user-agent", "HTTP.USERAGENT", CAST_S, R_STRING, 1);
    T.ng("$http_referer", "request.referer", "HTTP.URI", CAST_S, R_NO_SPACE, 1);
    T.ng("$https", "connection.https", "STRING", CAST_S, R_NO_SPACE, 10);
    T.ngnotimpl("$limit_rate", "nginx_parameter_not_intended_for_logging", R_NO_SPACE, 0);
    T.ng("$nginx_version", "server.nginx.version", "STRING", CAST_S, R_STRING, 10);
    T.ng("$pid", "connection.server.child.processid", "NUMBER", CAST_SL, R_NUMBER, 10);
    T.ng("$protocol", "connection.protocol", "STRING", CAST_S, R_NO_SPACE, 10);
    T.ng("$pipe", "connection.nginx.pipe", "STRING", CAST_S, ".", 10);
    T.ng("$proxy_protocol_addr", "connection.client.proxy.host", "IP", CAST_SL, R_CLF_IP, 10);
    T.ng("$proxy_protocol_port", "connection.client.proxy.port", "PORT", CAST_SL, R_CLF_NUMBER, 10);
    T.ng("$remote_addr", "connection.client.host", "IP", CAST_SL, R_CLF_IP, 10);
    T.ng("$binary_remote_addr", "connection.client.host", "IP_BINARY", CAST_SL, std::string("\\\\x") + R_HEXDIGIT + R_HEXDIGIT + "\\\\x" + R_HEXDIGIT + R_HEXDIGIT + "\\\\x" + R_HEXDIGIT + R_HEXDIGIT + "\\\\x" + R_HEXDIGIT + R_HEXDIGIT, 10);
    T.ng("$remote_port", "connection.client.port", "PORT", CAST_SL, R_NUMBER, 10);
    T.ng("$remote_user", "connection.client.user", "STRING", CAST_S, R_STRING, 10);
    T.ng("$request", "request.firstline", "HTTP.FIRSTLINE", CAST_S, R_NO_SPACE + " " + R_NO_SPACE + " " + R_NO_SPACE, -2);
    T.ngnotimpl("$request_body", "nginx_parameter_not_intended_for_logging", R_STRING, -1);
    T.ngnotimpl("$request_body_file", "nginx_parameter_not_intended_for_logging", R_STRING, -1);
    T.ng("$request_completion", "request.completion", "STRING", CAST_S, R_NO_SPACE, 10);
    T.ng("$request_filename", "server.filename", "FILENAME", CAST_S, R_STRING, 10);
    T.ng("$request_length", "request.bytes", "BYTES", CAST_SL, R_CLF_NUMBER, 10);
    T.ng("$request_method", "request.firstline.method", "HTTP.METHOD", CAST_S, R_NO_SPACE, 10);
    T.ng("$request_time", "response.server.processing.time", "SECOND_MILLIS", CAST_S, R_NUMBER_DECIMAL, 10);
    T.ng("$request_uri", "request.firstline.uri", "HTTP.URI", CAST_S, R_NO_SPACE, 10);
    T.ng("$request_id", "request.id", "STRING", CAST_S, R_HEXNUMBER, 10);
    T.ng("$uri", "request.firstline.uri.normalized", "HTTP.URI", CAST_S, R_STRING, 10);
    T.ng("$document_uri", "request.firstline.uri.normalized", "HTTP.URI", CAST_S, R_STRING, 10);
    T.ng("$scheme", "request.firstline.uri.protocol", "HTTP.PROTOCOL", CAST_S, R_NO_SPACE, 10);
    T.ngnamed("\\$sent_http_([a-z0-9\\-_]*)", "response.header.", "HTTP.HEADER", CAST_S, R_STRING, 0);
    T.ngnamed("\\$sent_trailer_([a-z0-9\\-_]*)", "response.trailer.", "HTTP.TRAILER", CAST_S, R_STRING, 0);
    T.ng("$server_addr", "connection.server.ip", "IP", CAST_SL, R_CLF_IP, 10);
    T.ng("$server_name", "connection.server.name", "STRING", CAST_S, R_NO_SPACE, 10);
    T.ng("$server_port", "connection.server.port", "PORT", CAST_SL, R_NUMBER, 10);
    T.ng("$server_protocol", "request.firstline.protocol", "HTTP.PROTOCOL_VERSION", CAST_SL, R_NO_SPACE, 10);
    T.ng("$session_time", "connection.session.time", "SECOND_MILLIS", CAST_S, R_NUMBER_DECIMAL, 10);
    T.ng("$tcpinfo_rtt", "connection.tcpinfo.rtt", "MICROSECONDS", CAST_SL, R_NUMBER, -1);
    T.ng("$tcpinfo_rttvar", "connection.tcpinfo.rttvar", "MICROSECONDS", CAST_SL, R_NUMBER, 10);
    T.ng("$tcpinfo_snd_cwnd", "connection.tcpinfo.send.cwnd", "BYTES", CAST_SL, R_NUMBER, 10);
    T.ng("$tcpinfo_rcv_space", "connection.tcpinfo.receive.space", "BYTES", CAST_SL, R_NUMBER, 10);
    T.ngnamed("\\$([a-z0-9\\-\\_]*)", "nginx.unknown.", "UNKNOWN_NGINX_VARIABLE", CAST_S, R_NO_SPACE, -10);
    /* UpstreamModule (nginxmodules/UpstreamModule.java:46-160) */
const std::string UP = "nginxmodule.upstream";
    T.ng("$upstream_addr", UP + ".addr", "UPSTREAM_ADDR_LIST", CAST_S, upstream_list(R_NO_SPACE), 10);
    T.ng("$upstream_bytes_received", UP + ".bytes.received", "UPSTREAM_BYTES_LIST", CAST_S, upstream_list(R_NUMBER), 10);
    T.ng("$upstream_bytes_sent", UP + ".bytes.sent", "UPSTREAM_BYTES_LIST", CAST_S, upstream_list(R_NUMBER), 10);
    T.ng("$upstream_cache_status", UP + ".cache.status", "UPSTREAM_CACHE_STATUS", CAST_S, "(?:MISS|BYPASS|EXPIRED|STALE|UPDATING|REVALIDATED|HIT)", 10);
    T.ng("$upstream_connect_time", UP + ".connect.time", "UPSTREAM_SECOND_MILLIS_LIST", CAST_S, upstream_list(R_NUMBER_DECIMAL), 10);
    T.ngnamed("\\$upstream_cookie_([a-z0-9\\-_]*)", UP + ".response.cookies.", "HTTP.COOKIE", CAST_S, R_STRING, 0);
    T.ng("$upstream_header_time", UP + ".header.time", "UPSTREAM_SECOND_MILLIS_LIST", CAST_S, upstream_list(R_NUMBER_DECIMAL), 10);
    T.ngnamed("\\$upstream_http_([a-z0-9\\-_]*)", UP + ".header.", "HTTP.HEADER", CAST_S, R_STRING, 0);
    T.ng("$upstream_queue_time", UP + ".queue.time", "UPSTREAM_SECOND_MILLIS_LIST", CAST_S, upstream_list(R_NUMBER_DECIMAL), 10);
    T.ng("$upstream_response_length", UP + ".response.length", "UPSTREAM_BYTES_LIST", CAST_S, upstream_list(R_NUMBER), 10);
    T.ng("$upstream_response_time", UP + ".response.time", "UPSTREAM_SECOND_MILLIS_LIST", CAST_S, upstream_list(R_NUMBER_DECIMAL), 10);
    T.ng("$upstream_status", UP + ".status", "UPSTREAM_STATUS_LIST", CAST_S, upstream_list(R_NO_SPACE), 10);
    T.ngnamed("\\$upstream_trailer_([a-z0-9\\-_]*)", UP + ".trailer.", "HTTP.TRAILER", CAST_S, R_STRING, 0);
    T.ng("$upstream_first_byte_time", UP + ".first_byte.time", "UPSTREAM_SECOND_MILLIS_LIST", CAST_S, upstream_list(R_NUMBER_DECIMAL), 10);
    T.ng("$upstream_session_time", UP + ".session.time", "UPSTREAM_SECOND_MILLIS_LIST", CAST_S, upstream_list(R_NUMBER_DECIMAL), 10);

    /* SslModule (nginxmodules/SslModule.java:37-200) */
const std::string SSL = "nginxmodule.ssl";
    T.ng("$ssl_cipher", SSL + ".cipher", "STRING", CAST_S, R_STRING, 10);
    T.ng("$ssl_ciphers", SSL + ".client.ciphers", "STRING", CAST_S, R_STRING, 10);
    T.ng("$ssl_client_escaped_cert", SSL + ".client.cert", "PEM_CERT_URLENCODED", CAST_S, R_NO_SPACE, 10);
    T.ng("$ssl_client_cert", SSL + ".client.cert", "PEM_CERT", CAST_S, R_STRING, 10);
    T.ng("$ssl_client_raw_cert", SSL + ".client.cert", "PEM_CERT_RAW", CAST_S, R_STRING, 10);
    T.ng("$ssl_client_fingerprint", SSL + ".client.cert.fingerprint", "SHA1", CAST_S, R_NO_SPACE, 10);
    T.ng("$ssl_client_i_dn", SSL + ".client.cert.issuer_dn", "STRING", CAST_S, R_STRING, 10);
    T.ng("$ssl_client_i_dn_legacy", SSL + ".client.cert.issuer_dn.legacy", "STRING", CAST_S, R_STRING, 10);
    T.ng("$ssl_client_s_dn", SSL + ".client.cert.subject_dn", "STRING", CAST_S, R_STRING, 10);
    T.ng("$ssl_client_s_dn_legacy", SSL + ".client.cert.subject_dn.legacy", "STRING", CAST_S, R_STRING, 10);
    T.ng("$ssl_client_serial", SSL + ".client.cert.serial", "STRING", CAST_S, R_STRING, 10);
    T.ng("$ssl_client_v_end", SSL + ".client.cert.end_date", "STRING", CAST_S, R_STRING, 10);
    T.ng("$ssl_client_v_remain", SSL + ".client.cert.remain_days", "STRING", CAST_S, R_STRING, 10);
    T.ng("$ssl_client_v_start", SSL + ".client.cert.start_date", "STRING", CAST_S, R_STRING, 10);
    T.ng("$ssl_client_verify", SSL + ".client.cert.verify", "STRING", CAST_S, R_STRING, 10);
    T.ng("$ssl_curves", SSL + ".client.curves", "STRING", CAST_S, R_STRING, 10);
    T.ng("$ssl_early_data", SSL + ".early_data", "STRING", CAST_S, "1?", 10);
    T.ng("$ssl_protocol", SSL + ".protocol", "STRING", CAST_S, R_STRING, 10);
    T.ng("$ssl_server_name", SSL + ".server_name", "STRING", CAST_S, R_STRING, 10);
    T.ng("$ssl_session_id", SSL + ".session.id", "STRING", CAST_S, R_STRING, 10);
    T.ng("$ssl_session_reused", SSL + ".session.reused", "STRING", CAST_S, "(r|.)", 10);
    T.ng("$ssl_preread_protocol", SSL + ".preread.protocol", "STRING", CAST_S, R_STRING, 10);
    T.ng("$ssl_preread_server_name", SSL + ".preread.server_name", "STRING", CAST_S, R_STRING, 10);
    T.ng("$ssl_preread_alpn_protocols", SSL + ".preread.alpn_protocols", "STRING", CAST_S, R_STRING, 10);

    /* GeoIPModule (nginxmodules/GeoIPModule.java:35-104) */
const std::string GEO = "nginxmodule.geoip";
    T.ng("$geoip_country_code", GEO + ".country.code", "STRING", CAST_S, R_NO_SPACE, 10);
    T.ng("$geoip_country_code3", GEO + ".country.code3", "STRING", CAST_S, R_NO_SPACE, 10);
    T.ng("$geoip_country_name", GEO + ".country.name", "STRING", CAST_S, R_STRING, 10);
    T.ng("$geoip_area_code", GEO + ".area.code", "STRING", CAST_S, R_NO_SPACE, 10);
    T.ng("$geoip_city_continent_code", GEO + ".continent.code", "STRING", CAST_S, R_NO_SPACE, 10);
    T.ng("$geoip_city_country_code", GEO + ".country.code", "STRING", CAST_S, R_NO_SPACE, 10);
    T.ng("$geoip_city_country_code3", GEO + ".country.code3", "STRING", CAST_S, R_NO_SPACE, 10);
    T.ng("$geoip_city_country_name", GEO + ".country.name", "STRING", CAST_S, R_STRING, 10);
    T.ng("$geoip_dma_code", GEO + ".dma.code", "STRING", CAST_S, R_STRING, 10);
    T.ng("$geoip_latitude", GEO + ".location.latitude", "STRING", CAST_S, R_STRING, 10);
    T.ng("$geoip_longitude", GEO + ".location.longitude", "STRING", CAST_S, R_STRING, 10);
    T.ng("$geoip_region", GEO + ".region.code", "STRING", CAST_S, R_NO_SPACE, 10);
    T.ng("$geoip_region_name", GEO + ".region.name", "STRING", CAST_S, R_STRING, 10);
    T.ng("$geoip_city", GEO + ".city", "STRING", CAST_S, R_STRING, 10);
    T.ng("$geoip_postal_code", GEO + ".postal.code", "STRING", CAST_S, R_STRING, 10);
    T.ng("$geoip_org", GEO + ".organization", "STRING", CAST_S, R_STRING, 10);

    /* VariousModule (nginxmodules/VariousModule.java:37-212) */
const std::string VAR = "nginxmodule";
    T.ng("$secure_link", VAR + ".secure_link.status", "STRING", CAST_S, R_STRING, 10);
    T.ng("$session_log_id", VAR + ".session_log.id", "STRING", CAST_S, R_STRING, 10);
    T.ng("$slice_range", VAR + ".slice_range", "STRING", CAST_S, R_STRING, 10);
    T.ng("$proxy_host", VAR + ".proxy.host", "STRING", CAST_S, R_NO_SPACE, 10);
    T.ng("$proxy_port", VAR + ".proxy.port", "STRING", CAST_S, R_NO_SPACE, 10);
    T.ng("$proxy_add_x_forwarded_for", VAR + ".proxy.add_x_forwarded_for", "STRING", CAST_S, R_NO_SPACE, 10);
    T.ng("$uid_got", VAR + ".userid.uid_got", "STRING", CAST_S, R_STRING, 10);
    T.ng("$uid_reset", VAR + ".userid.uid_reset", "STRING", CAST_S, R_STRING, 10);
    T.ng("$uid_set", VAR + ".userid.uid_set", "STRING", CAST_S, R_STRING, 10);
    T.ng("$modern_browser", VAR + ".browser.modern", "STRING", CAST_S, R_STRING, 10);
    T.ng("$ancient_browser", VAR + ".browser.ancient", "STRING", CAST_S, R_STRING, 10);
    T.ng("$msie", VAR + ".browser.msie", "STRING", CAST_S, R_NO_SPACE, 10);
    T.ng("$connections_active", VAR + ".stub_status.connections.active", "STRING", CAST_S, R_STRING, 10);
    T.ng("$connections_reading", VAR + ".stub_status.connections.reading", "STRING", CAST_S, R_STRING, 10);
    T.ng("$connections_writing", VAR + ".stub_status.connections.writing", "STRING", CAST_S, R_STRING, 10);
    T.ng("$connections_waiting", VAR + ".stub_status.connections.waiting", "STRING", CAST_S, R_STRING, 10);
    T.ng("$date_local", VAR + ".date.local", "STRING", CAST_S, R_STRING, 10);
    T.ng("$date_gmt", VAR + ".date.gmt", "STRING", CAST_S, R_STRING, 10);
    T.ng("$fastcgi_script_name", VAR + ".fastcgi.script_name", "STRING", CAST_S, R_STRING, 10);
    T.ng("$fastcgi_path_info", VAR + ".fastcgi.path_info", "STRING", CAST_S, R_STRING, 10);
    T.ng("$gzip_ratio", VAR + ".gzip.ratio", "STRING", CAST_S, R_NUMBER_OPT_DECIMAL, 10);
    T.ng("$spdy", VAR + ".spdy.version", "STRING", CAST_S, R_STRING, 10);
    T.ng("$spdy_request_priority", VAR + ".spdy.request_priority", "STRING", CAST_S, R_STRING, 10);
    T.ng("$http2", VAR + ".http2.negotiated_protocol", "STRING", CAST_S, R_STRING, 10);
    T.ng("$invalid_referer", VAR + ".referer.invalid", "STRING", CAST_S, "1?", 10);
    T.ngnamed("\\$jwt_header_([a-z0-9\\-_]*)", VAR + ".jwt.header.", "STRING", CAST_S, R_STRING, 0);
    T.ngnamed("\\$jwt_claim_([a-z0-9\\-_]*)", VAR + ".jwt.claim.", "STRING", CAST_S, R_STRING, 0);
    T.ng("$memcached_key", VAR + ".memcached.key", "STRING", CAST_S, R_STRING, 10);
    T.ng("$realip_remote_addr", VAR + ".realip.remote_addr", "IP", CAST_S, R_STRING, 10);
    T.ng("$realip_remote_port", VAR + ".realip.remote_port", "PORT", CAST_SL, R_STRING, 10);

    /* KubernetesIngressModule (nginxmodules/KubernetesIngressModule.java:35-68) */
const std::string K8S = "nginxmodule.kubernetes";
    T.ng("$the_real_ip", K8S + ".the_real_ip", "IP", CAST_S, R_STRING, 10);
    T.ng("$proxy_upstream_name", K8S + ".proxy_upstream_name", "STRING", CAST_S, R_STRING, 10);
    T.ng("$req_id", K8S + ".req_id", "STRING", CAST_S, R_STRING, 10);
    T.ng("$namespace", K8S + ".namespace", "STRING", CAST_S, R_STRING, 10);
    T.ng("$ingress_name", K8S + ".ingress_name", "STRING", CAST_S, R_STRING, 10);
    T.ng("$service_name", K8S + ".service.name", "STRING", CAST_S, R_STRING, 10);
    T.ng("$service_port", K8S + ".service.port", "PORT", CAST_S, R_STRING, 10);


    return T;
}

// commons-codec Hex(MD5) for ParameterizedTokenParser.tokenParameterToTypeName
std::string md5_hex(const std::string& msg) {
    static const uint32_t K[64] = {
        0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501, 0x698098d8,
        0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821, 0xf61e2562, 0xc040b340,
        0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8, 0x21e1cde6, 0xc33707d6, 0xf4d50d87,
        0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a, 0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c,
        0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70, 0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039,
        0xe6db99e5, 0x1fa27cf8, 0xc4ac5665, 0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92,
        0xffeff47d, 0x85845dd1, 0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb,
        0xeb86d391};
    static const int R[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 5, 9, 14, 20, 5, 9,
                              14, 20, 5, 9, 14, 20, 5, 9, 14, 20, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                              4, 11, 16, 23, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};
    std::vector<uint8_t> m(msg.begin(), msg.end());
    uint64_t bits = (uint64_t)m.size() * 8;
    m.push_back(0x80);
    while (m.size() % 64 != 56) m.push_back(0);
    for (int i = 0; i < 8; i++) m.push_back((uint8_t)(bits >> (8 * i)));
    uint32_t h[4] = {0x67452301, 0xefcdab89, 0x98badcfe, 0x10325476};
    for (size_t off = 0; off < m.size(); off += 64) {
        uint32_t w[16];
        for (int i = 0; i < 16; i++)
            w[i] = m[off + 4 * i] | (m[off + 4 * i + 1] << 8) | (m[off + 4 * i + 2] << 16) | ((uint32_t)m[off + 4 * i + 3] << 24);
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
        for (int i = 0; i < 64; i++) {
            uint32_t f;
            int g;
            if (i < 16) { f = (b & c) | (~b & d); g = i; }
            else if (i < 32) { f = (d & b) | (~d & c); g = (5 * i + 1) % 16; }
            else if (i < 48) { f = b ^ c ^ d; g = (3 * i + 5) % 16; }
            else { f = c ^ (b | ~d); g = (7 * i) % 16; }
            uint32_t t = d;
            d = c;
            c = b;
            uint32_t x = a + f + K[i] + w[g];
            b = b + ((x << R[i]) | (x >> (32 - R[i])));
            a = t;
        }
        h[0] += a; h[1] += b; h[2] += c; h[3] += d;
    }
    static const char* hx = "0123456789abcdef";
    std::string out;
    for (int i = 0; i < 4; i++)
        for (int k = 0; k < 4; k++) {
            unsigned byte = (h[i] >> (8 * k)) & 0xff;
            out += hx[byte >> 4];
            out += hx[byte & 15];
        }
    return out;
}

// Leftmost match of a NAMED / PARAM token pattern at or after 'from'
// (NamedTokenParser.java:43-77; ParameterizedTokenParser.java:58-95 with
// the patterns \%\{([a-z0-9\-_]*)\}X and \%\{PREFIX([^\}]*%[^\}]*)\}t).
bool find_pattern(const TParser& tp, const std::string& s, size_t from, size_t& start, size_t& end,
                  std::string& field) {
    if (tp.kind == TP_DOLLAR) {  // \$prefix([a-z0-9\-_]*): leftmost prefix, greedy name
        size_t p = s.find(tp.pprefix, from);
        if (p == std::string::npos) return false;
        size_t q = p + tp.pprefix.size();
        while (q < s.size() && ((s[q] >= 'a' && s[q] <= 'z') || (s[q] >= '0' && s[q] <= '9') || s[q] == '-' || s[q] == '_')) ++q;
        field = s.substr(p + tp.pprefix.size(), q - p - tp.pprefix.size());
        start = p;
        end = q;
        return true;
    }
    for (size_t p = from; p + 1 < s.size(); ++p) {
        if (s[p] != '%' || s[p + 1] != '{') continue;
        size_t q = p + 2;
        if (tp.kind == TP_NAMED) {
            while (q < s.size()) {
                char c = s[q];
                bool ok = (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9') || c == '-' || (tp.underscore && c == '_');
                if (!ok) break;
                ++q;
            }
            if (q >= s.size() || s[q] != '}') continue;
            if (s.compare(q + 1, tp.suffix.size(), tp.suffix) != 0) continue;
            field = s.substr(p + 2, q - p - 2);
            start = p;
            end = q + 1 + tp.suffix.size();
            return true;
        }
        // PARAM
        if (s.compare(q, tp.pprefix.size(), tp.pprefix) != 0) continue;
        q += tp.pprefix.size();
        size_t close = s.find('}', q);
        if (close == std::string::npos) continue;
        std::string inner = s.substr(q, close - q);
        if (inner.find('%') == std::string::npos) continue;
        if (close + 1 >= s.size() || s[close + 1] != 't') continue;
        field = inner;
        start = p;
        end = close + 2;
        return true;
    }
    return false;
}

void collect_tokens(const TParser& tp, const std::string& fmt, std::vector<Token>& out) {
    bool blank = true;  // StringUtils.isBlank
    for (char c : fmt) if (!(c == ' ' || (c >= 9 && c <= 13))) blank = false;
    if (blank) return;
    size_t offset = 0;
    for (;;) {
        size_t start, end;
        std::string field;
        if (tp.kind == TP_PLAIN || tp.kind == TP_FIXED) {
            size_t pos = fmt.find(tp.tok, offset);
            if (pos == std::string::npos) return;
            start = pos;
            end = pos + tp.tok.size();
        } else if (!find_pattern(tp, fmt, offset, start, end, field)) {
            return;
        }
        Token t;
        t.fixed = tp.kind == TP_FIXED;
        t.regex = tp.regex;
        t.start = (int)start;
        t.len = (int)(end - start);
        t.prio = t.fixed ? 0 : tp.prio;
        for (const auto& o : tp.outs) {
            TokOut x = o;
            if (tp.kind == TP_NAMED || tp.kind == TP_DOLLAR) x.name = lower(o.name + field);
            if (tp.kind == TP_PARAM) {
                std::string clean;
                for (char c : field) if (isalnum((unsigned char)c)) clean += c;
                x.type = upper(o.type + clean + "_" + md5_hex(field));
            }
            t.outs.push_back(x);
        }
        if (tp.strftime) {
            t.strftime = true;
            t.custom_type = t.outs[0].type;
            t.custom_param = field;
        }
        out.push_back(t);
        offset = end;
    }
}

// cleanupLogFormat (:121-167)
std::string apache_cleanup(const std::string& in) {
    // removeModifiersFromLogformat: "%!?[0-9]{3}(?:,[0-9]{3})*" -> "%"
    std::string a;
    for (size_t i = 0; i < in.size();) {
        if (in[i] == '%') {
            size_t j = i + 1;
            if (j < in.size() && in[j] == '!') ++j;
            auto three = [&](size_t k) {
                return k + 3 <= in.size() && isdigit((unsigned char)in[k]) && isdigit((unsigned char)in[k + 1]) &&
                       isdigit((unsigned char)in[k + 2]);
            };
            if (three(j)) {
                j += 3;
                while (j < in.size() && in[j] == ',' && three(j + 1)) j += 4;
                a += '%';
                i = j;
                continue;
            }
        }
        a += in[i++];
    }
    // makeHeaderNamesLowercaseInLogFormat: find loop of "%\{([^}]*)}([^t])"
    // ([^}]* stops at the first '}'; [^t] is any char but 't', newline included)
    std::string b;
    size_t last = 0, from = 0;
    for (;;) {
        size_t p = a.find("%{", from);
        if (p == std::string::npos) break;
        size_t c = a.find('}', p + 2);
        if (c == std::string::npos || c + 1 >= a.size() || a[c + 1] == 't') {
            from = p + 1;
            continue;
        }
        b += a.substr(last, p - last);
        b += "%{" + lower(a.substr(p + 2, c - p - 2)) + "}" + a[c + 1];
        last = c + 2;
        from = c + 2;
    }
    b += a.substr(last);
    // fixTimestampFormat: "%t" -> "[%t]"
    std::string c;
    for (size_t i = 0; i < b.size();) {
        if (b.compare(i, 2, "%t") == 0) { c += "[%t]"; i += 2; }
        else c += b[i++];
    }
    return c;
}

bool ieq(const std::string& a, const char* b) {
    if (a.size() != strlen(b)) return false;
    for (size_t i = 0; i < a.size(); ++i)
        if (tolower((unsigned char)a[i]) != b[i]) return false;
    return true;
}

std::string apache_alias(const std::string& f) {
    if (ieq(f, "common")) return "%h %l %u %t \"%r\" %>s %b";
    if (ieq(f, "combined")) return "%h %l %u %t \"%r\" %>s %b \"%{Referer}i\" \"%{User-Agent}i\"";
    if (ieq(f, "combinedio")) return "%h %l %u %t \"%r\" %>s %b \"%{Referer}i\" \"%{User-Agent}i\" %I %O";
    if (ieq(f, "referer")) return "%{Referer}i -> %U";
    if (ieq(f, "agent")) return "%{User-agent}i";
    return f;
}
bool looks_apache(const std::string& f) {
    return f.find('%') != std::string::npos || ieq(f, "common") || ieq(f, "combined") || ieq(f, "combinedio") ||
           ieq(f, "referer") || ieq(f, "agent");
}
bool looks_nginx(const std::string& f) { return f.find('$') != std::string::npos || ieq(f, "combined"); }

// TokenFormatDissector.parseTokenLogFileDefinition (:294-379)
void parse_token_def(Format& f, const TokenTable& T) {
    std::vector<Token> all;
    for (const auto& tp : T.v) collect_tokens(tp, f.cleaned, all);
    std::stable_sort(all.begin(), all.end(), [](const Token& a, const Token& b) {
        if (a.start != b.start) return a.start < b.start;
        if (a.len != b.len) return a.len < b.len;
        return a.prio > b.prio;
    });
    std::vector<char> kick(all.size(), 0);
    int prev = -1;
    for (int i = 0; i < (int)all.size(); ++i) {
        if (prev < 0) { prev = i; continue; }
        const Token& pv = all[prev];
        const Token& tk = all[i];
        if (pv.start == tk.start) {
            if (pv.len == tk.len) { if (pv.prio < tk.prio) kick[prev] = 1; else kick[i] = 1; }
            else { if (pv.len < tk.len) kick[prev] = 1; else kick[i] = 1; }
        } else if (pv.start + pv.len > tk.start) {
            kick[i] = 1;
            continue;
        }
        prev = i;
    }
    int tend = 0;
    for (size_t i = 0; i < all.size(); ++i) {
        if (kick[i]) continue;
        const Token& tk = all[i];
        if (tk.start - tend > 0) {
            Token fx;
            fx.fixed = true;
            fx.regex = f.cleaned.substr(tend, tk.start - tend);
            fx.start = tk.start;
            fx.len = tk.start - tend;
            f.tokens.push_back(fx);
        }
        f.tokens.push_back(tk);
        tend = tk.start + tk.len;
    }
    if (tend < (int)f.cleaned.size()) {
        Token fx;
        fx.fixed = true;
        fx.regex = f.cleaned.substr(tend);
        fx.start = tend;
        fx.len = (int)f.cleaned.size() - tend;
        f.tokens.push_back(fx);
    }
    for (const auto& t : f.tokens) {
        if (t.fixed) continue;
        for (const auto& o : t.outs) {
            std::string s = o.type + ":" + o.name;
            if (std::find(f.output_types.begin(), f.output_types.end(), s) == f.output_types.end())
                f.output_types.push_back(s);
        }
    }
}

const char* TS_OUTS[] = {
    "TIME.DAY:day", "TIME.MONTHNAME:monthname", "TIME.MONTH:month", "TIME.WEEK:weekofweekyear", "TIME.YEAR:weekyear",
    "TIME.YEAR:year", "TIME.HOUR:hour", "TIME.MINUTE:minute", "TIME.SECOND:second", "TIME.MILLISECOND:millisecond",
    "TIME.MICROSECOND:microsecond", "TIME.NANOSECOND:nanosecond", "TIME.DATE:date", "TIME.TIME:time",
    "TIME.ZONE:timezone", "TIME.EPOCH:epoch", "TIME.DAY:day_utc", "TIME.MONTHNAME:monthname_utc",
    "TIME.MONTH:month_utc", "TIME.WEEK:weekofweekyear_utc", "TIME.YEAR:weekyear_utc", "TIME.YEAR:year_utc",
    "TIME.HOUR:hour_utc", "TIME.MINUTE:minute_utc", "TIME.SECOND:second_utc", "TIME.MILLISECOND:millisecond_utc",
    "TIME.MICROSECOND:microsecond_utc", "TIME.NANOSECOND:nanosecond_utc", "TIME.DATE:date_utc", "TIME.TIME:time_utc"};

std::unique_ptr<Dissector> mkdis(int cls, const std::string& in) {
    auto d = std::make_unique<Dissector>();
    d->cls = cls;
    d->in_type = in;
    switch (cls) {
    case D_TIMESTAMP: case D_TIMESTAMP_ISO: case D_STRFTIME:
        for (auto* s : TS_OUTS) d->outs.push_back(s);
        break;
    case D_FIRSTLINE: d->outs = {"HTTP.METHOD:method", "HTTP.URI:uri", "HTTP.PROTOCOL_VERSION:protocol"}; break;
    case D_PROTOCOL: d->outs = {"HTTP.PROTOCOL:", "HTTP.PROTOCOL.VERSION:version"}; break;
    case D_URI:
        d->outs = {"HTTP.PROTOCOL:protocol", "HTTP.USERINFO:userinfo", "HTTP.HOST:host", "HTTP.PORT:port",
                   "HTTP.PATH:path", "HTTP.QUERYSTRING:query", "HTTP.REF:ref"};
        break;
    case D_QUERY: d->outs = {"STRING:*"}; break;
    case D_COOKIES: d->outs = {"HTTP.COOKIE:*"}; break;
    case D_SETCOOKIES: d->outs = {"HTTP.SETCOOKIE:*"}; break;
    case D_SETCOOKIE:
        d->outs = {"STRING:value", "STRING:expires", "TIME.EPOCH:expires", "STRING:path", "STRING:domain", "STRING:comment"};
        break;
    case D_UNIQUEID:
        d->outs = {"TIME.EPOCH:epoch", "IP:ip", "PROCESSID:processid", "COUNTER:counter", "THREAD_INDEX:threadindex"};
        break;
    case D_LOCALIZED: d->outs = {"TIME.LOCALIZEDSTRING:"}; break;
    default: break;
    }
    return d;
}

// Utils.resilientUrlDecode (hp/Utils.java:27-65) of a value whose every '%'
// is followed by two hex digits (the device's guard_pct proved it): each %XX
// is the Latin-1 char U+00XX (VALID_STANDARD -> %00%XX, a UTF-16 decode), '+'
// a space; UTF-8 out
std::string latin1_url_decode(const uint8_t* s, uint32_t n) {
    std::string val;
    auto hv = [](uint8_t x) { return x <= '9' ? x - '0' : (x | 32) - 'a' + 10; };
    for (uint32_t q = 0; q < n;) {
        const uint8_t ch = s[q];
        if (ch == '%' && q + 2 < n) {
            const int x = hv(s[q + 1]) * 16 + hv(s[q + 2]);
            if (x < 0x80) val += char(x);
            else { val += char(0xC0 | (x >> 6)); val += char(0x80 | (x & 0x3F)); }
            q += 3;
        } else {
            val += ch == '+' ? ' ' : char(ch);
            ++q;
        }
    }
    return val;
}

std::string extract_field_name(const std::string& in, const std::string& out) {
    if (in == out) return "";
    if (!in.empty()) return out.substr(in.size() + 1);
    return out;
}

std::string cleanup_field(const std::string& f) {  // Parser.cleanupFieldValue
    size_t c = f.find(':');
    if (c == std::string::npos) return lower(f);
    return upper(f.substr(0, c)) + ":" + lower(f.substr(c + 1));
}

}  // namespace

// ============================================================== planning
int Plan::build_dissectors(const std::string& logformats, std::string& err) {
    auto root = std::make_unique<Dissector>();
    root->cls = D_ROOT;
    root->in_type = root_type_;
    std::vector<std::string> list;
    bool jetty = false;
    size_t s = 0;
    for (;;) {  // split("\\r?\\n")
        size_t nl = logformats.find('\n', s);
        std::string line = logformats.substr(s, nl == std::string::npos ? std::string::npos : nl - s);
        if (!line.empty() && line.back() == '\r' && nl != std::string::npos) line.pop_back();
        bool blank = true;
        for (char c : line) if (!(c == ' ' || (c >= 9 && c <= 13))) blank = false;
        if (!blank) {
            std::string up = upper(line);
            size_t a = up.find_first_not_of(" \t"), b = up.find_last_not_of(" \t");
            if (up.substr(a, b - a + 1) == "ENABLE JETTY FIX") jetty = true;
            else if (std::find(list.begin(), list.end(), line) == list.end()) list.push_back(line);
        }
        if (nl == std::string::npos) break;
        s = nl + 1;
    }
    if (jetty) {
        // addAdditionalLogFormatsToHandleJettyUseragentProblem (hp/HttpdLogFormatDissector.java:72-92)
        // over getAllLogFormats() (alias-expanded, :254-262): "\"%{User-Agent}i\"" ->
        // "\"%{User-Agent}i\" ", then over the grown list "%u" -> " %u " (every occurrence);
        // addLogFormat skips a string already registered
        const char* from[2] = {"\"%{User-Agent}i\"", "%u"};
        const char* to[2] = {"\"%{User-Agent}i\" ", " %u "};
        for (int pass = 0; pass < 2; ++pass) {
            const size_t n0 = list.size();
            for (size_t i = 0; i < n0; ++i) {
                const std::string f = list[i];
                std::string lf;
                if (looks_apache(f)) lf = apache_alias(f);
                else if (looks_nginx(f)) lf = ieq(f, "combined") ? "$remote_addr - $remote_user [$time_local] \"$request\" $status "
                                                                  "$body_bytes_sent \"$http_referer\" \"$http_user_agent\""
                                                                : f;
                else continue;
                if (lf.find(from[pass]) == std::string::npos) continue;
                std::string out;
                for (size_t q = 0; q < lf.size();) {
                    if (lf.compare(q, strlen(from[pass]), from[pass]) == 0) { out += to[pass]; q += strlen(from[pass]); }
                    else out += lf[q++];
                }
                if (std::find(list.begin(), list.end(), out) == list.end()) list.push_back(out);
            }
        }
    }
    for (const auto& f : list) {
        int kind = looks_apache(f) ? FMT_APACHE : looks_nginx(f) ? FMT_NGINX : 0;
        if (!kind) continue;
        auto fm = std::make_unique<Format>();
        fm->kind = kind;
        if (kind == FMT_APACHE) {
            fm->logformat = apache_alias(f);
            fm->cleaned = apache_cleanup(fm->logformat);
            parse_token_def(*fm, apache_table());
        } else {
            // NginxHttpdLogFormatDissector.setLogFormat (hp/NginxHttpdLogFormatDissector.java:75-92):
            // the "combined" alias, no cleanup
            fm->logformat = ieq(f, "combined") ? "$remote_addr - $remote_user [$time_local] \"$request\" $status "
                                                 "$body_bytes_sent \"$http_referer\" \"$http_user_agent\""
                                               : f;
            fm->cleaned = fm->logformat;
            parse_token_def(*fm, nginx_table());
        }
        for (const auto& o : fm->output_types)
            if (std::find(root->outs.begin(), root->outs.end(), o) == root->outs.end()) root->outs.push_back(o);
        formats_.push_back(std::move(fm));
    }
    dis_.push_back(std::move(root));
    dis_.push_back(mkdis(D_TIMESTAMP, "TIME.STAMP"));
    dis_.push_back(mkdis(D_TIMESTAMP_ISO, "TIME.ISO8601"));
    dis_.push_back(mkdis(D_FIRSTLINE, "HTTP.FIRSTLINE"));
    dis_.push_back(mkdis(D_PROTOCOL, "HTTP.PROTOCOL_VERSION"));
    dis_.push_back(mkdis(D_URI, "HTTP.URI"));
    dis_.push_back(mkdis(D_QUERY, "HTTP.QUERYSTRING"));
    dis_.push_back(mkdis(D_COOKIES, "HTTP.COOKIES"));
    dis_.push_back(mkdis(D_SETCOOKIES, "HTTP.SETCOOKIES"));
    dis_.push_back(mkdis(D_SETCOOKIE, "HTTP.SETCOOKIE"));
    dis_.push_back(mkdis(D_UNIQUEID, "MOD_UNIQUE_ID"));
    auto c2n = mkdis(D_CLF2NUM, "BYTESCLF");
    c2n->out_type = "BYTES";
    c2n->outs = {"BYTES:"};
    dis_.push_back(std::move(c2n));
    auto n2c = mkdis(D_NUM2CLF, "BYTES");
    n2c->out_type = "BYTESCLF";
    n2c->outs = {"BYTESCLF:"};
    dis_.push_back(std::move(n2c));
    // NginxHttpdLogFormatDissector.createAdditionalDissectors (hp/NginxHttpdLogFormatDissector.java:144-152)
    // and UpstreamModule.getDissectors (nginxmodules/UpstreamModule.java:163-198)
    bool any_nginx = false;
    for (const auto& f : formats_) any_nginx |= f->kind == FMT_NGINX;
    if (any_nginx) {
        auto conv = [&](int cls, const char* in, const char* out) {
            auto d = mkdis(cls, in);
            d->out_type = out;
            d->outs = {std::string(out) + ":"};
            dis_.push_back(std::move(d));
        };
        conv(D_BINIP, "IP_BINARY", "IP");
        conv(D_SECMILLIS, "SECOND_MILLIS", "MILLISECONDS");
        conv(D_SECMILLIS, "TIME.EPOCH_SECOND_MILLIS", "TIME.EPOCH");
        conv(D_MS2US, "MILLISECONDS", "MICROSECONDS");
        auto up = [&](const char* in, const char* out) {
            auto d = mkdis(D_UPSTREAM, in);
            d->out_type = out;
            for (int k = 0; k < 32; ++k) {  // UpstreamListDissector.getPossibleOutput (:127-135)
                d->outs.push_back(std::string(out) + ":" + std::to_string(k) + ".value");
                d->outs.push_back(std::string(out) + ":" + std::to_string(k) + ".redirected");
            }
            dis_.push_back(std::move(d));
        };
        up("UPSTREAM_ADDR_LIST", "UPSTREAM_ADDR");
        up("UPSTREAM_BYTES_LIST", "BYTES");
        up("UPSTREAM_SECOND_MILLIS_LIST", "SECOND_MILLIS");
        up("UPSTREAM_STATUS_LIST", "UPSTREAM_STATUS");
    }
    for (const auto& f : formats_)
        for (const auto& t : f->tokens)
            if (t.strftime) {
                dis_.push_back(mkdis(D_STRFTIME, t.custom_type));
                dis_.push_back(mkdis(D_LOCALIZED, t.custom_type));
            }
    (void)err;
    return LP_OK;
}

// Dissector.prepareForDissect(inputname, outputname) of dissector d for the
// output `otype:cf` below input `in_name`: the casts Parser records in
// castsOfTargets (core/Parser.java:438-439)
int Plan::casts_of(const Dissector& d, const std::string& otype, const std::string& in_name,
                   const std::string& cf) const {
    const std::string n = d.cls == D_ROOT ? cf : extract_field_name(in_name, cf);
    constexpr int SO = CAST_S, SL = CAST_S | CAST_L, SLD = CAST_S | CAST_L | CAST_D, NONE = 0;
    switch (d.cls) {
    case D_ROOT: {
        // HttpdLogFormatDissector.prepareForDissect (:226-235): the union over
        // the LogFormats of TokenFormatDissector's first output named cf (:163-174)
        int r = 0;
        for (const auto& f : formats_) {
            int c = SO;
            bool found = false;
            for (const auto& t : f->tokens) {
                for (const auto& o : t.outs)
                    if (o.name == cf) { c = o.casts; found = true; break; }
                if (found) break;
            }
            r |= c;
        }
        return r;
    }
    case D_TIMESTAMP: case D_TIMESTAMP_ISO: case D_STRFTIME: {  // TimeStampDissector.java:223-352
        static const char* const so[] = {"monthname", "date", "time", "timezone", "monthname_utc", "date_utc",
                                         "time_utc"};
        static const char* const sl[] = {"day", "month", "weekofweekyear", "weekyear", "year", "hour", "minute",
                                         "second", "millisecond", "microsecond", "nanosecond", "epoch"};
        for (const char* x : so) if (n == x) return SO;
        for (const char* x : sl) if (n == x || n == std::string(x) + "_utc") return SL;
        return NONE;
    }
    case D_URI:  // HttpUriDissector.java:76-105
        if (n == "port") return SL;
        for (const char* x : {"protocol", "userinfo", "host", "path", "query", "ref"}) if (n == x) return SO;
        return NONE;
    case D_SETCOOKIE: return n == "expires" ? SL : SO;  // ResponseSetCookieDissector.java:63-72
    case D_UNIQUEID:  // ModUniqueIdDissector.java:76-100
        for (const char* x : {"epoch", "ip", "processid", "counter", "threadindex"}) if (n == x) return SL;
        return NONE;
    case D_CLF2NUM: case D_NUM2CLF: case D_SECMILLIS: case D_MS2US:  // TypeConvertBaseDissector.java:36-45
        return n.empty() ? SL : NONE;
    case D_BINIP: return n.empty() ? SL : NONE;  // NginxHttpdLogFormatDissector.java:151-160
    case D_UPSTREAM: {  // UpstreamModule.java:178-196 (same casts for .value and .redirected)
        const bool item = n.size() > 6 && (n.compare(n.size() - 6, 6, ".value") == 0 ||
                                           (n.size() > 11 && n.compare(n.size() - 11, 11, ".redirected") == 0));
        if (!item) return NONE;
        if (d.in_type == "UPSTREAM_BYTES_LIST") return SL;
        if (d.in_type == "UPSTREAM_SECOND_MILLIS_LIST") return SLD;
        return SO;
    }
    default:  // first line, protocol, query string, cookies, Set-Cookie lists, localized time: STRING_ONLY
        return SO;
    }
    (void)otype;
}

bool Plan::table_src(const std::string& path, TableSrc out[MAX_FMT], std::string& names, TableSrc* alt) const {
    const size_t colon = path.find(':');
    if (colon == std::string::npos || !device_ok_) return false;
    const std::string type = path.substr(0, colon), name = path.substr(colon + 1);
    for (int f = 0; f < MAX_FMT; ++f) out[f] = TableSrc{TC_NONE, 0, 0, 0};
    if (alt)
        for (int f = 0; f < MAX_FMT; ++f) alt[f] = TableSrc{TC_NONE, 0, 0, 0};
    for (int f = 0; f < prog_.n_fmt; ++f) {
        auto it = tsrc_[f].find(path);
        if (it != tsrc_[f].end()) {
            if (it->second.kind < 0) return false;
            out[f] = it->second;
            auto at = talt_[f].find(path);
            if (at != talt_[f].end()) {
                if (!alt) return false;
                alt[f] = at->second;
            }
            continue;
        }
        if (thost_exact_[f].count(path)) return false;
        // a query parameter: "STRING:<query string's name>.<parameter>" of the
        // longest such query string
        const std::string* best = nullptr;
        int q = -1;
        if (type == "STRING")
            for (const auto& kv : tqp_[f])
                if (name.size() > kv.first.size() + 1 && name.compare(0, kv.first.size(), kv.first) == 0 &&
                    name[kv.first.size()] == '.' && (!best || kv.first.size() > best->size())) {
                    best = &kv.first;
                    q = kv.second;
                }
        // a cookie / raw query parameter: "<TYPE>:<token path>.<name>" of a pair stage
        const std::string* pbest = nullptr;
        int ps = -1;
        for (const auto& kv : tpair_[f]) {
            const size_t c2 = kv.first.find(':');
            const std::string ktype = kv.first.substr(0, c2), kname = kv.first.substr(c2 + 1);
            if (ktype == type && name.size() > kname.size() + 1 && name.compare(0, kname.size(), kname) == 0 &&
                name[kname.size()] == '.' && (!pbest || kname.size() > pbest->size() - (c2 + 1))) {
                pbest = &kv.first;
                ps = kv.second;
            }
        }
        // ResponseSetCookieDissector outputs of a cookie of a Set-Cookie pair
        // stage: "STRING:<list>.<cookie>.value|expires|domain|comment|path",
        // "TIME.EPOCH:<list>.<cookie>.expires" (the cookie name may hold '.')
        if (!pbest && (type == "STRING" || type == "TIME.EPOCH")) {
            const size_t dot = name.rfind('.');
            if (dot != std::string::npos && dot > 0) {
                const std::string field = name.substr(dot + 1), stem = name.substr(0, dot);
                int sf = -1;
                if (type == "TIME.EPOCH") sf = field == "expires" ? SC_EXPIRES_MS : -1;
                else if (field == "value") sf = SC_VALUE;
                else if (field == "expires") sf = SC_EXPIRES_S;
                else if (field == "domain") sf = SC_DOMAIN;
                else if (field == "comment") sf = SC_COMMENT;
                else if (field == "path") sf = SC_PATH;
                const std::string* sbest = nullptr;
                int ss = -1;
                for (const auto& kv : tpair_[f]) {
                    if (kv.second >= 0 && prog_.pair[kv.second].kind != PK_SETC) continue;
                    const size_t c2 = kv.first.find(':');
                    const std::string kname = kv.first.substr(c2 + 1);
                    if (stem.size() > kname.size() + 1 && stem.compare(0, kname.size(), kname) == 0 &&
                        stem[kname.size()] == '.' && (!sbest || kname.size() > sbest->size() - (c2 + 1))) {
                        sbest = &kv.first;
                        ss = kv.second;
                    }
                }
                if (sbest && sf >= 0) {
                    if (ss < 0) return false;
                    const std::string cn = stem.substr(sbest->size() - sbest->find(':'));
                    if (names.size() + cn.size() > (size_t)TABLE_NAMES) return false;
                    out[f] = TableSrc{TC_SETC, ss | (sf << 8), (int32_t)names.size(), (int32_t)cn.size()};
                    names += cn;
                    continue;
                }
            }
        }
        if (pbest) {
            if (ps < 0) return false;
            const std::string pn = name.substr(pbest->size() - pbest->find(':'));
            if (names.size() + pn.size() > (size_t)TABLE_NAMES) return false;
            out[f] = TableSrc{TC_PAIR, ps, (int32_t)names.size(), (int32_t)pn.size()};
            names += pn;
            continue;
        }
        for (const auto& h : thost_prefix_[f])
            if ((name == h || (name.size() > h.size() && name.compare(0, h.size(), h) == 0 && name[h.size()] == '.')) &&
                (!best || h.size() > best->size()))
                return false;  // below a value only the replay dissects
        if (best) {
            if (q < 0) return false;
            const std::string pn = name.substr(best->size() + 1);
            if (names.size() + pn.size() > (size_t)TABLE_NAMES) return false;
            out[f] = TableSrc{TC_QP, q, (int32_t)names.size(), (int32_t)pn.size()};
            names += pn;
        }
    }
    return true;
}

int Plan::casts(const std::string& target) const {
    auto it = casts_.find(target);
    return it == casts_.end() ? -1 : it->second;
}

void Plan::find_useful(const std::set<std::string>& possible, const std::string& type, const std::string& name,
                       bool is_root) {
    std::string srid = type + ":" + name;
    if (located_.count(srid)) return;
    located_.insert(srid);
    for (const auto& dp : dis_) {
        const Dissector& d = *dp;
        if (d.in_type != type) continue;
        for (const auto& out : d.outs) {
            size_t colon = out.find(':');
            std::string otype = out.substr(0, colon), oname = out.substr(colon + 1);
            std::vector<std::string> checks;
            if (oname == "*") {
                std::string pre = name + ".";
                for (const auto& p : possible)
                    if (p.compare(0, pre.size(), pre) == 0) checks.push_back(p);
            } else if (is_root) checks.push_back(oname);
            else if (oname.empty()) checks.push_back(name);
            else checks.push_back(name + "." + oname);
            for (const auto& cf : checks) {
                if (!possible.count(cf) || compiled_.count(otype + ":" + cf)) continue;
                auto it = compiled_.find(srid);
                if (it == compiled_.end()) {
                    it = compiled_.emplace(srid, std::vector<Instance>{}).first;
                    useful_.insert(name);
                }
                Instance* in = nullptr;
                for (auto& x : it->second) if (x.cls == d.cls) in = &x;
                if (!in) {
                    it->second.push_back(Instance{d.cls, &d, {}});
                    in = &it->second.back();
                }
                in->requested.insert(extract_field_name(name, cf));
                casts_[otype + ":" + cf] = casts_of(d, otype, name, cf);
                if (d.cls == D_ROOT)
                    for (auto& f : formats_) f->requested.insert(cf);  // TokenFormatDissector.prepareForDissect
                find_useful(possible, otype, cf, false);
            }
        }
    }
    // the new types of a remapped name get their dissectors too (core/Parser.java:447-455)
    auto rm = remaps_.find(name);
    if (rm != remaps_.end())
        for (const auto& mt : rm->second)
            if (!compiled_.count(mt + ":" + name)) {
                casts_[mt + ":" + name] = CAST_S;  // "Retyped targets are ALWAYS String ONLY"
                find_useful(possible, mt, name, false);
            }
}

int Plan::build(const std::string& logformats, const std::vector<std::string>& fields, std::string& err,
                const std::vector<Remap>& remaps) {
    gen_ = g_plan_gen.fetch_add(1);
    int r = build_dissectors(logformats, err);
    if (r != LP_OK) return r;
    // Parser.addTypeRemapping (core/Parser.java:664-677): input trimmed and
    // lower-cased, type trimmed and upper-cased; the first casts given for a
    // pair are its castsOfTargets entry
    auto trim = [](const std::string& x) {  // String.trim: chars <= ' ' at both ends
        size_t a = 0, b = x.size();
        while (a < b && (uint8_t)x[a] <= ' ') ++a;
        while (b > a && (uint8_t)x[b - 1] <= ' ') --b;
        return x.substr(a, b - a);
    };
    for (const auto& m : remaps) {
        const std::string in = lower(trim(m.input)), ty = upper(trim(m.type));
        if (remaps_[in].insert(ty).second) casts_[ty + ":" + in] = m.casts;
    }
    for (const auto& f : fields) needed_.insert(cleanup_field(f));
    for (const auto& d : dis_)
        if (d->outs.empty()) {
            err = "InvalidDissectorException: Dissector cannot create any outputs: " + d->in_type;
            return LP_E_INVALID;
        }
    std::set<std::string> needed = needed_;
    needed.insert(root_type_ + ":");
    std::set<std::string> possible;
    for (const auto& n : needed) {
        std::string nm = n.substr(n.find(':') + 1);
        std::string sb;
        size_t s = 0;
        for (;;) {
            size_t dot = nm.find('.', s);
            std::string part = nm.substr(s, dot == std::string::npos ? std::string::npos : dot - s);
            if (sb.empty() || part.empty()) sb += part;
            else sb += "." + part;
            possible.insert(sb);
            if (dot == std::string::npos) break;
            s = dot + 1;
        }
    }
    find_useful(possible, root_type_, "", true);
    if (compiled_.empty()) {
        err = "MissingDissectorsException: There are no dissectors at all which makes this a completely useless parser.";
        return LP_E_MISSING;
    }
    if (formats_.empty()) {
        err = "InvalidDissectorException: Cannot run without logformats";
        return LP_E_INVALID;
    }
    for (const auto& t : needed_) {
        if (located_.count(t)) continue;
        if (!t.empty() && t.back() == '*') {
            if (t.size() >= 2 && t[t.size() - 2] == '.' && !located_.count(t.substr(0, t.size() - 2))) {
                err = "MissingDissectorsException: " + t;
                return LP_E_MISSING;
            }
        } else {
            err = "MissingDissectorsException: " + t;
            return LP_E_MISSING;
        }
    }
    compile_program();
    return device_ok_ ? LP_OK : LP_E_UNSUPPORTED;
}

int Plan::possible_paths(const std::string& logformats, int max_depth, std::vector<std::string>& out,
                         std::string& err, const std::vector<Remap>& remaps) {
    Plan p;
    p.build_dissectors(logformats, err);
    std::set<std::string> seen;
    std::function<void(const std::string&, const std::string&, int)> rec = [&](const std::string& base,
                                                                             const std::string& btype, int depth) {
        if (depth == 0) return;
        for (const auto& d : p.dis_) {
            if (d->in_type != btype) continue;
            for (const auto& o : d->outs) {
                size_t colon = o.find(':');
                std::string ctype = o.substr(0, colon), cname = o.substr(colon + 1);
                std::string cbase = base.empty() ? cname : cname.empty() ? base : base + "." + cname;
                std::string np = ctype + ":" + cbase;
                if (seen.insert(np).second) rec(cbase, ctype, depth - 1);
            }
        }
    };
    rec("", p.root_type_, max_depth);
    // each remapped path and what its new type's dissectors produce below it (core/Parser.java:954-962)
    for (const auto& m : remaps) {
        const std::string in = lower(m.input), ty = upper(m.type);
        seen.insert(ty + ":" + in);
        rec(in, ty, max_depth - 1);
    }
    out.assign(seen.begin(), seen.end());
    return LP_OK;
}

// ====================================================== device program
namespace {
// O_QPARAM: a query parameter's value (index: query stage * MAX_QNAMES + name index)
// O_SECMS: a SECOND_MILLIS stage's milliseconds (index: the stage); O_LITEM /
// O_LITEMMS: an upstream list item's value / its milliseconds (index:
// item << 3 | redirected << 2 | list stage, item_code below)
enum Origin { O_NONE, O_TOKEN, O_FL_URI, O_FL_PROTO, O_FL_METHOD, O_URI_QUERY, O_URI_PART, O_CONV, O_TIME, O_QPARAM,
              O_SECMS, O_LITEM, O_LITEMMS };
int item_code(int j, int k, int redirected) { return (k << 3) | (redirected << 2) | j; }
}

void Plan::compile_program() {
    Program& P = prog_;
    memset(&P, 0, sizeof P);
    if (!device_ok_) return;
    if ((int)formats_.size() > MAX_FMT) { device_ok_ = false; why_ = "too many LogFormats"; return; }
    P.n_fmt = (int)formats_.size();
    int lit_used = 0;
    auto add_lit = [&](const std::string& s) -> int {
        if (lit_used + (int)s.size() > MAX_LIT) return -1;
        memcpy(P.lit + lit_used, s.data(), s.size());
        int off = lit_used;
        lit_used += (int)s.size();
        return off;
    };
    // the elements of every LogFormat, one after the other (format f's
    // captured tokens take slots 0.. of that format)
    for (int fi = 0; fi < P.n_fmt; ++fi) {
        const Format& f = *formats_[fi];
        P.fmt_apache[fi] = f.kind == FMT_APACHE;
        P.fmt_elem0[fi] = (uint8_t)P.n_elems;
        std::set<std::string> seen_names;
        int n_tok = 0;
        for (int i = 0; i < (int)f.tokens.size(); ++i) {
            const Token& t = f.tokens[i];
            if (P.n_elems == MAX_ELEMS || P.n_elems - P.fmt_elem0[fi] == MAX_FMT_ELEMS) {
                device_ok_ = false;
                why_ = "too many LogFormat elements";
                return;
            }
            Elem& e = P.elems[P.n_elems++];
            memset(&e, 0, sizeof e);
            e.cap = -1;
            e.acls = -1;
            if (t.fixed) {
                e.kind = EK_LIT;
                int off = add_lit(t.regex);
                if (off < 0) { device_ok_ = false; why_ = "literal pool overflow"; return; }
                e.lit_off = (uint16_t)off;
                e.lit_len = (uint16_t)t.regex.size();
                for (int k = 0; k < 4 && k < (int)t.regex.size(); ++k) e.lit4 |= (uint32_t)(uint8_t)t.regex[k] << (8 * k);
                continue;
            }
            int k = elem_kind_of(t.regex);
            if (k < 0) { device_ok_ = false; why_ = "token regex not on the device: " + t.regex; return; }
            e.kind = (uint8_t)k;
            bool wanted = false;
            for (const auto& o : t.outs) if (f.requested.count(o.name)) wanted = true;
            if (wanted) {
                if (n_tok == MAX_TOK) { device_ok_ = false; why_ = "too many captured tokens"; return; }
                for (const auto& o : t.outs)
                    if (!seen_names.insert(o.type + ":" + o.name).second) {
                        device_ok_ = false;
                        why_ = "the same output is produced by two tokens";
                        return;
                    }
                tok_slot_[fi * 256 + i] = n_tok;
                e.cap = (int8_t)n_tok++;
            }
        }
        if (n_tok > P.n_tok) P.n_tok = n_tok;
    }
    P.fmt_elem0[P.n_fmt] = (uint8_t)P.n_elems;
    for (int fi = 0; fi < P.n_fmt; ++fi) {
        int q = 0;
        for (int i = P.fmt_elem0[fi]; i < P.fmt_elem0[fi + 1]; ++i)
            if (P.elems[i].kind == EK_LIT)
                for (int k = 0; k < P.elems[i].lit_len; ++k) q += P.lit[P.elems[i].lit_off + k] == '"';
        P.fmt_quotes[fi] = (uint8_t)(q > 255 ? 255 : q);
    }
    auto fmt_of_elem = [&](int i) {
        int fi = 0;
        while (i >= P.fmt_elem0[fi + 1]) ++fi;
        return fi;
    };
    // anchoring literal / determinism of each token element
    for (int i = 0; i < P.n_elems; ++i) {
        Elem& e = P.elems[i];
        if (e.kind == EK_LIT) continue;
        const int end = P.fmt_elem0[fmt_of_elem(i) + 1];
        e.last = i == end - 1;
        if (i + 1 < end && P.elems[i + 1].kind == EK_LIT) {
            e.nlit = 1;
            e.lit_off = P.elems[i + 1].lit_off;
            e.lit_len = P.elems[i + 1].lit_len;
        }
        uint8_t c0 = e.nlit ? P.lit[e.lit_off] : 0;
        if (e.nlit) e.lit4 = P.elems[i + 1].lit4;
        e.acls = (int8_t)(e.nlit ? bcls::class_of(c0) : -1);
        bool ws0 = c0 == ' ' || (c0 >= 9 && c0 <= 13);
        bool dig0 = c0 >= '0' && c0 <= '9';
        bool hex0 = dig0 || ((c0 | 32) >= 'a' && (c0 | 32) <= 'f');
        switch (e.kind) {
        case EK_NOSPACE: e.det = (e.nlit && ws0) || e.last; break;
        case EK_NUMBER: case EK_CLFNUMBER: case EK_NONZERO: e.det = (e.nlit && !dig0) || e.last; break;
        case EK_HEXNUMBER: case EK_CLFHEXNUMBER: e.det = (e.nlit && !hex0) || e.last; break;
        case EK_ANY_GREEDY: case EK_ANY_LAZY: e.det = e.last; break;
        case EK_TIME_US: case EK_ANYCHAR: case EK_MSEC: case EK_BINIP: case EK_UPLIST_NS: case EK_TIME_ISO:
        case EK_CACHE_STATUS:
            e.det = 1;
            break;
        case EK_DECIMAL: e.det = (e.nlit && !dig0) || e.last; break;
        case EK_NOSPACE3: e.det = (e.nlit && ws0) || e.last; break;
        default: e.det = 0; break;
        }
    }
    // greedy '.*' candidates are occurrences of the following literal; one
    // can only lead to a match if the rest of the line still holds every
    // later literal's copy of that literal's first byte (pruning, exact)
    for (int i = 0; i < P.n_elems; ++i) {
        Elem& e = P.elems[i];
        if (e.kind != EK_ANY_GREEDY || !e.nlit) continue;
        const uint8_t c0 = P.lit[e.lit_off];
        int need = 0;
        for (int j = i + 1; j < P.fmt_elem0[fmt_of_elem(i) + 1]; ++j)
            if (P.elems[j].kind == EK_LIT)
                for (int k = 0; k < P.elems[j].lit_len; ++k) need += P.lit[P.elems[j].lit_off + k] == c0;
        e.need = (uint8_t)(need > 255 ? 255 : need);
    }
    P.max_stack = 0;
    for (int fi = 0; fi < P.n_fmt; ++fi) {
        int depth = 0;
        for (int i = P.fmt_elem0[fi]; i < P.fmt_elem0[fi + 1]; ++i)
            if (P.elems[i].kind != EK_LIT && !P.elems[i].det) ++depth;
        if (depth > P.max_stack) P.max_stack = depth;
    }
    if (P.max_stack > MAX_STACK) { device_ok_ = false; why_ = "too many backtracking elements"; return; }
    int cur_fmt = 0;
    auto tk = [&](int oi) { return cur_fmt * 64 + oi; };  // (format, token slot) key of the stage maps
    // stages, walking the compiled tree from each captured token output.
    // remapped: this visit is a type remapping's second delivery of a value
    // (Parsable.addDissection with recursion, core/Parsable.java:160-176)
    std::set<std::string> remap_seen;  // remapped names whose values the walk reached
    // the requested fields of time stage t (TimeStampDissector outputs, the
    // replay's D_TIMESTAMP case)
    std::function<void(const Instance&, const std::string&, int)> treg_time;
    // device table sources (lp_table.h).  A path two sources deliver: a token
    // and a value derived from another token (e.g. NGINX $remote_addr and
    // $binary_remote_addr, both IP:connection.client.host) -- the root
    // dissector delivers every token before any derived value, so the
    // derived one is the later delivery (the value, when it has one) and the
    // token the earlier (alt); any other pair is left to the host table.
    auto treg = [&](const std::string& path, TableSrc ts) {
        auto& m = tsrc_[cur_fmt];
        auto& am = talt_[cur_fmt];
        auto it = m.find(path);
        if (it == m.end()) { m[path] = ts; return; }
        if (memcmp(&it->second, &ts, sizeof ts) == 0 || it->second.kind < 0) return;
        const TableSrc cur = it->second;
        if (!am.count(path) && (cur.kind == TC_TOKEN) != (ts.kind == TC_TOKEN)) {
            am[path] = cur.kind == TC_TOKEN ? cur : ts;
            it->second = cur.kind == TC_TOKEN ? ts : cur;
        } else {
            it->second.kind = -1;
        }
    };
    auto thost = [&](const std::string& name) { thost_prefix_[cur_fmt].insert(name); };
    treg_time = [&](const Instance& in, const std::string& complete, int t) {
        static const char* const fn[] = {"epoch", "day", "monthname", "month", "weekofweekyear", "weekyear", "year",
                                         "hour", "minute", "second", "millisecond", "microsecond", "nanosecond",
                                         "date", "time"};
        for (const auto& r : in.requested) {
            const bool utc = r.size() > 4 && r.compare(r.size() - 4, 4, "_utc") == 0;
            const std::string base = utc ? r.substr(0, r.size() - 4) : r;
            int tf = -1;
            for (int k = 0; k < 15; ++k) if (base == fn[k]) tf = k;
            if (tf < 0 || (utc && tf == TF_EPOCH)) continue;  // timezone: never delivered
            std::string type;
            for (const auto& o : in.d->outs)
                if (o.compare(o.find(':') + 1, std::string::npos, r) == 0) type = o.substr(0, o.find(':'));
            if (!type.empty()) treg(type + ":" + complete + "." + r, TableSrc{TC_TIME, t, tf, utc ? 1 : 0});
        }
    };
    // a pair stage (cookie header / raw query string) on token slot oi of the
    // current format; its pieces are "<key>.<name>" in the device table
    auto add_pair = [&](int oi, int kind, const std::string& key) {
        auto st = pair_of_tok_.find(tk(oi));
        if (st == pair_of_tok_.end()) {
            if (P.n_pair == MAX_PAIR) { device_ok_ = false; why_ = "too many cookie / query string tokens"; return false; }
            P.pair[P.n_pair] = PairStage{oi, cur_fmt, kind, 0};
            st = pair_of_tok_.emplace(tk(oi), P.n_pair++).first;
        }
        auto tp = tpair_[cur_fmt].emplace(key, st->second);  // two stages under one name: the host table decides
        if (!tp.second && tp.first->second != st->second) tp.first->second = -1;
        return true;
    };
    std::function<void(int, int, const std::string&, const std::string&, bool)> walk =
        [&](int ok, int oi, const std::string& type, const std::string& complete, bool remapped) {
            if (!device_ok_) return;
            if (!remapped) {
                auto rm = remaps_.find(complete);
                if (rm != remaps_.end()) {
                    remap_seen.insert(complete);
                    for (const auto& mt : rm->second) {
                        if (mt == type) {  // DissectionFailure for every line delivering the value
                            device_ok_ = false;
                            why_ = "type remapping to the value's own type";
                            return;
                        }
                        thost_exact_[cur_fmt].insert(mt + ":" + complete);  // the remapped delivery itself
                        walk(ok, oi, mt, complete, true);
                    }
                }
            }
            if (!useful_.count(complete)) return;
            auto it = compiled_.find(type + ":" + complete);
            if (it == compiled_.end()) return;
            for (const auto& in : it->second) {
                switch (in.cls) {
                case D_TIMESTAMP: case D_TIMESTAMP_ISO: {
                    if (ok != O_TOKEN) { device_ok_ = false; why_ = "timestamp from a derived value"; return; }
                    if (!time_of_tok_.count(tk(oi))) {
                        if (P.n_time == MAX_TIME) { device_ok_ = false; why_ = "too many timestamps"; return; }
                        P.time[P.n_time].tok = (int8_t)oi;
                        P.time[P.n_time].fmt = (int8_t)cur_fmt;
                        P.time[P.n_time].kind = in.cls == D_TIMESTAMP_ISO ? TK_ISO : TK_APACHE;
                        time_of_tok_[tk(oi)] = P.n_time++;
                    }
                    treg_time(in, complete, time_of_tok_[tk(oi)]);
                    break;
                }
                case D_STRFTIME: {
                    if (ok != O_TOKEN) { device_ok_ = false; why_ = "strftime from a derived value"; return; }
                    if (!time_of_tok_.count(tk(oi))) {
                        if (P.n_time == MAX_TIME) { device_ok_ = false; why_ = "too many timestamps"; return; }
                        const Token* tok = nullptr;
                        for (const auto& kv : tok_slot_)
                            if (kv.first / 256 == cur_fmt && kv.second == oi)
                                tok = &formats_[cur_fmt]->tokens[kv.first % 256];
                        TimeStage& T = P.time[P.n_time];
                        memset(&T, 0, sizeof T);
                        T.tok = (int8_t)oi;
                        T.fmt = (int8_t)cur_fmt;
                        T.kind = TK_STRF;
                        if (!tok || !tok->strftime || !strf_compile(tok->custom_param, T)) {
                            device_ok_ = false;
                            why_ = "strftime pattern outside the device subset";
                            return;
                        }
                        time_of_tok_[tk(oi)] = P.n_time++;
                    }
                    treg_time(in, complete, time_of_tok_[tk(oi)]);
                    break;
                }
                case D_LOCALIZED:
                    if (ok != O_TOKEN) { device_ok_ = false; why_ = "localized time from a derived value"; return; }
                    treg("TIME.LOCALIZEDSTRING:" + complete, TableSrc{TC_TOKEN, oi, 0, 0});
                    break;
                case D_SETCOOKIES: {
                    // ResponseSetCookieListDissector: split, joined and named by the
                    // URI kernel (a pair stage, PK_SETC); ResponseSetCookieDissector
                    // on a cookie string by the device table (TC_SETC, table_src) and
                    // the replay; the phase-1 guard proves HttpCookie.parse and
                    // parseExpire cannot throw (setcookie_ok)
                    if (ok != O_TOKEN) { device_ok_ = false; why_ = "Set-Cookie list from a derived value"; return; }
                    P.guard_setc[cur_fmt] |= 1 << oi;
                    if (!add_pair(oi, PK_SETC, "HTTP.SETCOOKIE:" + complete)) return;
                    const std::string pre = "HTTP.SETCOOKIE:" + complete + ".";
                    for (const auto& kv : compiled_)
                        if (kv.first.compare(0, pre.size(), pre) == 0) P.guard_setc_exp[cur_fmt] |= 1 << oi;
                    break;
                }
                case D_COOKIES: {
                    // RequestCookieListDissector: split, lower-cased and decoded by
                    // the URI kernel (a pair stage); the phase-1 guard proves the
                    // decode cannot fail (guard_pct)
                    if (ok != O_TOKEN) { device_ok_ = false; why_ = "cookies from a derived value"; return; }
                    P.guard_pct[cur_fmt] |= 1 << oi;
                    if (!add_pair(oi, PK_COOKIE, "HTTP.COOKIE:" + complete)) return;
                    break;
                }
                case D_FIRSTLINE: {
                    if (ok != O_TOKEN) { device_ok_ = false; why_ = "first line from a derived value"; return; }
                    int fidx;
                    if (!fl_of_tok_.count(tk(oi))) {
                        if (P.n_fl == MAX_FL) { device_ok_ = false; why_ = "too many first lines"; return; }
                        P.fl[P.n_fl].tok = (int8_t)oi;
                        P.fl[P.n_fl].fmt = (int8_t)cur_fmt;
                        fl_of_tok_[tk(oi)] = P.n_fl++;
                    }
                    fidx = fl_of_tok_[tk(oi)];
                    treg("HTTP.METHOD:" + complete + ".method", TableSrc{TC_FL, fidx, 0, 0});
                    treg("HTTP.URI:" + complete + ".uri", TableSrc{TC_FL, fidx, 1, 0});
                    treg("HTTP.PROTOCOL_VERSION:" + complete + ".protocol", TableSrc{TC_FL, fidx, 2, 0});
                    walk(O_FL_URI, fidx, "HTTP.URI", complete + ".uri", false);
                    walk(O_FL_PROTO, fidx, "HTTP.PROTOCOL_VERSION", complete + ".protocol", false);
                    walk(O_FL_METHOD, fidx, "HTTP.METHOD", complete + ".method", false);
                    break;
                }
                case D_PROTOCOL:
                    // the replay splits the value (first-line protocol, or a
                    // HTTP.PROTOCOL_VERSION token such as NGINX $server_protocol)
                    if (ok != O_FL_PROTO && ok != O_TOKEN) { device_ok_ = false; why_ = "protocol from a derived value"; return; }
                    if (ok == O_FL_PROTO) {
                        treg("HTTP.PROTOCOL:" + complete, TableSrc{TC_PROTO, oi, 0, 0});
                        treg("HTTP.PROTOCOL.VERSION:" + complete + ".version", TableSrc{TC_PROTO, oi, 1, 0});
                    } else {
                        thost_exact_[cur_fmt].insert("HTTP.PROTOCOL:" + complete);
                        thost(complete);
                    }
                    break;
                case D_URI: {
                    // a token, a first line's uri, or a remapped query parameter (derived stage)
                    std::map<int, int>& m = ok == O_TOKEN ? uri_of_tok_ : ok == O_QPARAM ? uri_of_qp_ : uri_of_fl_;
                    if (ok != O_TOKEN && ok != O_FL_URI && ok != O_QPARAM) { device_ok_ = false; why_ = "URI from a derived value"; return; }
                    const int key = ok == O_TOKEN ? tk(oi) : oi;  // first-line / query stages are already per format
                    if (!m.count(key)) {
                        if (P.n_uri == MAX_URI) { device_ok_ = false; why_ = "too many URIs"; return; }
                        UriStage& U = P.uri[P.n_uri];
                        memset(&U, 0, sizeof U);
                        U.src_tok = ok == O_TOKEN ? (int8_t)oi : -1;
                        U.src_fl = ok == O_FL_URI ? (int8_t)oi : -1;
                        U.src_q = ok == O_QPARAM ? oi / MAX_QNAMES : -1;
                        U.src_qname = ok == O_QPARAM ? oi % MAX_QNAMES : 0;
                        U.query_stage = -1;
                        U.fmt = (int8_t)cur_fmt;
                        m[key] = P.n_uri++;
                    }
                    int u = m[key];
                    UriStage& U = P.uri[u];
                    if (in.requested.count("query")) U.want_query = 1;
                    if (in.requested.count("path")) U.want_path = 1;
                    if (in.requested.count("ref")) U.want_ref = 1;
                    if (in.requested.count("userinfo")) U.want_userinfo = 1;
                    treg("HTTP.QUERYSTRING:" + complete + ".query", TableSrc{TC_URI, u, UP_QUERY, 0});
                    treg("HTTP.PATH:" + complete + ".path", TableSrc{TC_URI, u, UP_PATH, 0});
                    treg("HTTP.REF:" + complete + ".ref", TableSrc{TC_URI, u, UP_REF, 0});
                    treg("HTTP.PROTOCOL:" + complete + ".protocol", TableSrc{TC_URI, u, UP_PROTOCOL, 0});
                    treg("HTTP.HOST:" + complete + ".host", TableSrc{TC_URI, u, UP_HOST, 0});
                    treg("HTTP.PORT:" + complete + ".port", TableSrc{TC_URI, u, UP_PORT, 0});
                    treg("HTTP.USERINFO:" + complete + ".userinfo", TableSrc{TC_NULL, 0, 0, 0});
                    walk(O_URI_QUERY, u, "HTTP.QUERYSTRING", complete + ".query", false);
                    break;
                }
                case D_QUERY: {
                    if (ok == O_TOKEN) {
                        // a HTTP.QUERYSTRING token (%q, $args, $query_string):
                        // split, lower-cased and decoded by the URI kernel (a pair
                        // stage); the phase-1 guard proves the decode cannot fail
                        // (guard_pct, as for cookies)
                        P.guard_pct[cur_fmt] |= 1 << oi;
                        if (!add_pair(oi, PK_QUERY, "STRING:" + complete)) return;
                        break;
                    }
                    if (ok != O_URI_QUERY) { device_ok_ = false; why_ = "query string from a derived value"; return; }
                    UriStage& U = P.uri[oi];
                    U.want_query = 1;
                    if (U.query_stage < 0) {
                        if (P.n_query == MAX_QUERY) { device_ok_ = false; why_ = "too many query strings"; return; }
                        memset(&P.query[P.n_query], 0, sizeof(QueryStage));
                        P.query[P.n_query].uri = (int8_t)oi;
                        U.query_stage = (int8_t)P.n_query;
                        query_of_uri_[oi] = P.n_query++;
                    }
                    QueryStage& Q = P.query[U.query_stage];
                    {  // two query stages delivering under one name: the host table decides
                        auto tq = tqp_[cur_fmt].emplace(complete, U.query_stage);
                        if (!tq.second && tq.first->second != U.query_stage) tq.first->second = -1;
                    }
                    for (const auto& r : in.requested) {
                        if (r == "*") { Q.want_all = 1; continue; }
                        bool dup = false;
                        for (int k = 0; k < Q.n_names; ++k)
                            if (Q.name_len[k] == r.size() && !memcmp(P.lit + Q.name_off[k], r.data(), r.size())) dup = true;
                        if (dup) continue;
                        if (Q.n_names == MAX_QNAMES || r.size() > 255) { device_ok_ = false; why_ = "too many query names"; return; }
                        int off = add_lit(r);
                        if (off < 0) { device_ok_ = false; why_ = "literal pool overflow"; return; }
                        Q.name_off[Q.n_names] = (uint16_t)off;
                        Q.name_len[Q.n_names] = (uint8_t)r.size();
                        Q.n_names++;
                    }
                    // a remapped parameter: its value is dissected again under the new type
                    const int qsi = U.query_stage;
                    for (int k = 0; k < P.query[qsi].n_names; ++k) {
                        const std::string r((const char*)P.lit + P.query[qsi].name_off[k], P.query[qsi].name_len[k]);
                        const std::string pc = complete + "." + r;
                        if (!remaps_.count(pc)) continue;
                        qname_of_[std::to_string(qsi) + ":" + r] = k;
                        walk(O_QPARAM, qsi * MAX_QNAMES + k, "STRING", pc, false);
                        if (!device_ok_) return;
                    }
                    break;
                }
                case D_SECMILLIS:
                    // ConvertSecondsWithMillisStringDissector: phase 1 converts a
                    // token (a SECOND_MILLIS stage), the URI kernel every item of
                    // a SECOND_MILLIS upstream list (its table holds both)
                    if (ok == O_TOKEN) {
                        auto st = secms_of_tok_.find(tk(oi));
                        if (st == secms_of_tok_.end()) {
                            if (P.n_secms == MAX_SECMS) { device_ok_ = false; why_ = "too many SECOND_MILLIS values"; return; }
                            P.secms[P.n_secms] = SecmsStage{oi, cur_fmt};
                            st = secms_of_tok_.emplace(tk(oi), P.n_secms++).first;
                        }
                        treg(in.d->out_type + ":" + complete, TableSrc{TC_SECMS, st->second, 0, 0});
                        walk(O_SECMS, st->second, in.d->out_type, complete, false);
                    } else if (ok == O_LITEM) {
                        if (!P.list[oi & 3].secms) { device_ok_ = false; why_ = "SECOND_MILLIS of a non-time list"; return; }
                        treg(in.d->out_type + ":" + complete, TableSrc{TC_LIST_MS, oi & 3, oi >> 3, (oi >> 2) & 1});
                        walk(O_LITEMMS, oi, in.d->out_type, complete, false);
                    } else {
                        device_ok_ = false;
                        why_ = "SECOND_MILLIS converter on a derived value";
                        return;
                    }
                    break;
                case D_MS2US:
                    // ConvertMillisecondsIntoMicroseconds on a device millisecond value
                    if (ok == O_SECMS) treg(in.d->out_type + ":" + complete, TableSrc{TC_SECMS, oi, 1, 0});
                    else if (ok == O_LITEMMS) treg(in.d->out_type + ":" + complete, TableSrc{TC_LIST_MS, oi & 3, oi >> 3, ((oi >> 2) & 1) | 2});
                    else if (ok == O_TOKEN || ok == O_CONV) thost_exact_[cur_fmt].insert(in.d->out_type + ":" + complete);
                    else { device_ok_ = false; why_ = "converter on a derived value"; return; }
                    walk(O_CONV, oi, in.d->out_type, complete, false);
                    break;
                case D_BINIP:
                    if (ok == O_TOKEN) {
                        // BinaryIPDissector: phase 1 converts the token (a BinaryIP stage)
                        auto st = binip_of_tok_.find(tk(oi));
                        if (st == binip_of_tok_.end()) {
                            if (P.n_binip == MAX_BINIP) { device_ok_ = false; why_ = "too many binary IP values"; return; }
                            P.binip[P.n_binip] = BinipStage{oi, cur_fmt};
                            st = binip_of_tok_.emplace(tk(oi), P.n_binip++).first;
                        }
                        treg(in.d->out_type + ":" + complete, TableSrc{TC_BINIP, st->second, 0, 0});
                        walk(O_CONV, oi, in.d->out_type, complete, false);
                        break;
                    }
                    [[fallthrough]];
                case D_CLF2NUM: case D_NUM2CLF:
                    // value-level conversions, done in the replay from the token / list item
                    if (ok != O_TOKEN && ok != O_CONV && ok != O_LITEM) { device_ok_ = false; why_ = "converter on a derived value"; return; }
                    if (ok == O_TOKEN && (in.cls == D_CLF2NUM || in.cls == D_NUM2CLF))
                        treg(in.d->out_type + ":" + complete, TableSrc{in.cls == D_CLF2NUM ? TC_CLF2NUM : TC_NUM2CLF, oi, 0, 0});
                    else
                        thost_exact_[cur_fmt].insert(in.d->out_type + ":" + complete);
                    walk(O_CONV, oi, in.d->out_type, complete, false);
                    break;
                case D_UPSTREAM: {
                    // UpstreamListDissector: the URI kernel splits the list (the
                    // token's element kind, EK_UPLIST_*, proves it splits cleanly)
                    // into an item table in the line's region
                    if (ok != O_TOKEN) { device_ok_ = false; why_ = "upstream list from a derived value"; return; }
                    auto st = list_of_tok_.find(tk(oi));
                    if (st == list_of_tok_.end()) {
                        if (P.n_list == MAX_LIST) { device_ok_ = false; why_ = "too many upstream lists"; return; }
                        P.list[P.n_list] = ListStage{oi, cur_fmt, in.d->out_type == "SECOND_MILLIS" ? 1 : 0, 0};
                        st = list_of_tok_.emplace(tk(oi), P.n_list++).first;
                    }
                    const int j = st->second;
                    for (int k = 0; k < 32; ++k)
                        for (int vr = 0; vr < 2; ++vr) {
                            const std::string item = complete + "." + std::to_string(k) + (vr ? ".redirected" : ".value");
                            treg(in.d->out_type + ":" + item, TableSrc{TC_LIST, j, k, vr});
                            walk(O_LITEM, item_code(j, k, vr), in.d->out_type, item, false);
                        }
                    break;
                }
                default:
                    device_ok_ = false;
                    why_ = "dissector for input type " + in.d->in_type + " not on the device";
                    return;
                }
            }
        };
    for (cur_fmt = 0; cur_fmt < P.n_fmt; ++cur_fmt) {
        const Format& f = *formats_[cur_fmt];
        for (int i = 0; i < (int)f.tokens.size(); ++i) {
            auto it = tok_slot_.find(cur_fmt * 256 + i);
            if (it == tok_slot_.end()) continue;
            for (const auto& o : f.tokens[i].outs) {
                treg(o.type + ":" + o.name, TableSrc{TC_TOKEN, it->second, 0, 0});
                walk(O_TOKEN, it->second, o.type, o.name, false);
            }
        }
    }
    // a remapped name whose new type has dissectors but whose values the walk
    // never reached (e.g. a URI part): the replay could not follow it
    for (const auto& kv : remaps_)
        for (const auto& mt : kv.second)
            if (device_ok_ && compiled_.count(mt + ":" + kv.first) && !remap_seen.count(kv.first)) {
                device_ok_ = false;
                why_ = "type remapping of a value the device does not track: " + kv.first;
            }
    // histogram sources: the captured status token and the first first-line stage of each format
    for (int fi = 0; fi < P.n_fmt; ++fi) {
        P.hist_status[fi] = P.hist_fl[fi] = -1;
        int rank = 0;  // 2: request.status.last, 1: request.status
        const Format& f = *formats_[fi];
        for (int i = 0; i < (int)f.tokens.size(); ++i) {
            auto it = tok_slot_.find(fi * 256 + i);
            if (it == tok_slot_.end()) continue;
            for (const auto& o : f.tokens[i].outs) {
                const int r = o.name == "request.status.last" ? 2 : o.name == "request.status" ? 1 : 0;
                if (r > rank) { rank = r; P.hist_status[fi] = it->second; }
            }
        }
        for (int s = P.n_fl - 1; s >= 0; --s)
            if (P.fl[s].fmt == fi) P.hist_fl[fi] = s;
    }
}

std::string Plan::describe() const {
    std::string s;
    char b[256];
    snprintf(b, sizeof b, "device_ok=%d%s%s\n", (int)device_ok_, device_ok_ ? "" : " reason=", device_ok_ ? "" : why_.c_str());
    s += b;
    for (const auto& f : formats_) s += "format: " + f->cleaned + "\n";
    static const char* kn[] = {"LIT", "NOSPACE", "NUMBER", "CLFNUMBER", "HEXNUMBER", "CLFHEXNUMBER", "NONZERO",
                               "ANY_GREEDY", "ANY_LAZY", "TIME_US", "CLF_IP", "IP", "ANYCHAR", "DECIMAL", "MSEC",
                               "NOSPACE3", "UPLIST_DEC", "UPLIST_NUM", "UPLIST_NS", "BINIP", "TIME_ISO", "CACHE_STATUS"};
    constexpr int n_kn = (int)(sizeof kn / sizeof kn[0]);
    for (int i = 0; i < prog_.n_elems; ++i) {
        const Elem& e = prog_.elems[i];
        std::string lit = e.kind == EK_LIT ? std::string((const char*)prog_.lit + e.lit_off, e.lit_len) : "";
        snprintf(b, sizeof b, "  elem %2d %-12s cap=%2d det=%d last=%d nlit=%d %s\n", i, e.kind < n_kn ? kn[e.kind] : "?", e.cap, e.det,
                 e.last, e.nlit, e.kind == EK_LIT ? ("'" + lit + "'").c_str() : "");
        s += b;
    }
    snprintf(b, sizeof b, "  tokens=%d time=%d firstline=%d uri=%d query=%d\n", prog_.n_tok, prog_.n_time, prog_.n_fl,
             prog_.n_uri, prog_.n_query);
    s += b;
    return s;
}

// ================================================================ replay
struct Emission {
    std::string base, type, name;
    MVal v;
};
struct Plan::Ctx {
    const ResultView& R;
    int64_t i;
    const uint8_t* line;
    const uint8_t* arena;
    std::vector<std::pair<std::string, MVal>> rec;  // (TYPE:path, value) per setter call
    std::vector<Emission> em;                        // the delivering addDissection calls
    std::deque<std::string> pool;  // formatted date/time strings
};

namespace {
MVal mstr(const uint8_t* p, uint32_t len) {
    MVal v;
    v.p = p;
    v.len = len;
    return v;
}
MVal mnull() {
    MVal v;
    v.null = true;
    return v;
}
MVal mlong(int64_t l) {
    MVal v;
    v.is_long = true;
    v.l = l;
    return v;
}
const char* MONTH_FULL[] = {"January", "February", "March", "April", "May", "June", "July",
                            "August", "September", "October", "November", "December"};
}  // namespace

static thread_local int t_origin_kind = 0, t_origin_idx = 0, t_fmt = 0;  // t_fmt: the line's LogFormat

// Parsable.addDissection's decisions for one (type, base, name), memoized per
// thread and plan: the set / map lookups on strings dominated the replay
namespace {
struct EmitDec {
    std::string complete, needed;
    const std::vector<Instance>* ins = nullptr;  // further dissectors (useful intermediate)
    const std::set<std::string>* remap = nullptr;  // the name's type remappings
    bool exact = false, wild = false;
    bool remap_needed = false;  // a remapped delivery of the value is requested
};
struct EmitMemo {
    uint64_t gen = 0;
    std::unordered_map<std::string, EmitDec> m;
    std::string key;
};
thread_local EmitMemo t_memo;
}  // namespace

void Plan::emit(Ctx& c, const std::string& base, const std::string& type, const std::string& name, const MVal& v,
                const MVal* dv, bool recursion) const {
    EmitMemo& M = t_memo;
    if (M.gen != gen_) {
        M.m.clear();
        M.gen = gen_;
    }
    M.key.assign(type);
    M.key += '\x1f';
    M.key += base;
    M.key += '\x1f';
    M.key += name;
    auto it = M.m.find(M.key);
    if (it == M.m.end()) {
        EmitDec d;
        std::string wild;
        if (base.empty()) {
            d.complete = name;
            wild = type + ":*";
        } else {
            d.complete = name.empty() ? base : base + "." + name;
            wild = type + ":" + base + ".*";
        }
        d.needed = type + ":" + d.complete;
        if (useful_.count(d.complete)) {
            auto ci = compiled_.find(d.needed);
            if (ci != compiled_.end()) d.ins = &ci->second;
        }
        d.exact = needed_.count(d.needed) > 0;
        d.wild = needed_.count(wild) > 0;
        auto rm = remaps_.find(d.complete);
        if (rm != remaps_.end()) {
            d.remap = &rm->second;
            for (const auto& mt : rm->second)
                d.remap_needed = d.remap_needed || needed_.count(mt + ":" + d.complete) ||
                                 needed_.count(mt + (base.empty() ? ":*" : ":" + base + ".*"));
        }
        it = M.m.emplace(M.key, std::move(d)).first;
    }
    const EmitDec& d = it->second;  // node-based map: stays valid while the row inserts more
    if (d.remap && !recursion) {
        // the value again under each new type, first (core/Parsable.java:160-176;
        // a remapping to the value's own type left the whole plan to FALLBACK).
        // Not a dissector's addDissection call: the emission list holds the
        // original only (the caller's Parser.store replays the remapping).
        const int ok = t_origin_kind, oi = t_origin_idx;
        for (const auto& mt : *d.remap) {
            t_origin_kind = ok;
            t_origin_idx = oi;
            emit(c, base, mt, name, v, dv, true);
        }
        t_origin_kind = ok;
        t_origin_idx = oi;
    }
    if (d.ins) {
        const int ok = t_origin_kind, oi = t_origin_idx;
        for (const auto& in : *d.ins) {
            t_origin_kind = ok;
            t_origin_idx = oi;
            run_phase(c, in, d.complete, dv ? *dv : v);
        }
    }
    if (d.exact) c.rec.emplace_back(d.needed, v);
    if (d.wild) c.rec.emplace_back(d.needed, v);
    if ((d.exact || d.wild || d.remap_needed) && !recursion) c.em.push_back(Emission{base, type, name, v});
}

// The pieces of pair stage j for line c.i, in order, delivered under `type`
// (the requested names only, or all with "*").
void Plan::emit_pairs(Ctx& c, const Instance& in, const std::string& name, const char* type, int j) const {
    const ResultView& R = c.R;
    const uint32_t n = R.p_count[j][c.i];
    if (!n) return;
    const bool all = in.requested.count("*") > 0;
    const uint8_t* tab = c.arena + ref_off(R.p_tab[j][c.i]);
    auto at = [&](uint64_t r) { return mstr((ref_arena(r) ? c.arena : c.line) + ref_off(r), ref_len(r)); };
    t_origin_kind = O_NONE;
    t_origin_idx = 0;
    for (uint32_t k = 0; k < n; ++k) {
        uint64_t e[2];
        memcpy(e, tab + 16 * (size_t)k, 16);
        const MVal nm = at(e[0]);
        const std::string pn((const char*)nm.p, nm.len);
        if (!all && !in.requested.count(pn)) continue;
        emit(c, name, type, pn, at(e[1]));
    }
}

void Plan::run_phase(Ctx& c, const Instance& in, const std::string& name, const MVal& v) const {
    const ResultView& R = c.R;
    const int64_t i = c.i;
    const int ok = t_origin_kind, oi = t_origin_idx;
    auto has = [&](const char* n) { return in.requested.count(n) > 0; };
    auto set_origin = [](int k, int x) { t_origin_kind = k; t_origin_idx = x; };
    auto line_ref = [&](uint64_t r) {
        if (ref_amp(r)) {  // '&' + line / region bytes (rawQuery delivered without a copy)
            c.pool.emplace_back("&" + std::string((const char*)(ref_arena(r) ? c.arena : c.line) + ref_off(r), ref_len(r)));
            return mstr((const uint8_t*)c.pool.back().data(), (uint32_t)c.pool.back().size());
        }
        return mstr((ref_arena(r) ? c.arena : c.line) + ref_off(r), ref_len(r));
    };
    switch (in.cls) {
    case D_LOCALIZED:  // StrfTimeStampDissector.LocalizedTimeDissector (:117-120): the raw value
        if (has("")) emit(c, name, "TIME.LOCALIZEDSTRING", "", v);
        return;
    case D_TIMESTAMP: case D_TIMESTAMP_ISO: case D_STRFTIME: {
        if (v.null || v.len == 0) return;
        int t = time_of_tok_.at(t_fmt * 64 + oi);
        int64_t epoch = R.t_epoch[t][i];
        const int64_t nanos = in.cls == D_STRFTIME ? (int64_t)R.t_nano[t][i] : 0;
        if (has("epoch")) { set_origin(O_TIME, t); emit(c, name, "TIME.EPOCH", "epoch", mlong(epoch)); }
        for (int pass = 0; pass < 2; ++pass) {
            uint64_t w = pass == 0 ? R.t_local[t][i] : R.t_utc[t][i];
            const char* sfx = pass == 0 ? "" : "_utc";
            int64_t Y = w & 0xFFFF, MO = (w >> 16) & 15, D = (w >> 20) & 31, H = (w >> 25) & 31, MI = (w >> 30) & 63,
                    S = (w >> 36) & 63, WY = (w >> 42) & 0xFFFF, WK = (w >> 58) & 63;
            auto nm = [&](const char* b) { return std::string(b) + sfx; };
            set_origin(O_TIME, t);
            if (has(nm("day").c_str())) emit(c, name, "TIME.DAY", nm("day"), mlong(D));
            if (has(nm("monthname").c_str())) {
                const char* mn = MONTH_FULL[MO - 1];
                emit(c, name, "TIME.MONTHNAME", nm("monthname"), mstr((const uint8_t*)mn, (uint32_t)strlen(mn)));
            }
            if (has(nm("month").c_str())) emit(c, name, "TIME.MONTH", nm("month"), mlong(MO));
            if (has(nm("weekofweekyear").c_str())) emit(c, name, "TIME.WEEK", nm("weekofweekyear"), mlong(WK));
            if (has(nm("weekyear").c_str())) emit(c, name, "TIME.YEAR", nm("weekyear"), mlong(WY));
            if (has(nm("year").c_str())) emit(c, name, "TIME.YEAR", nm("year"), mlong(Y));
            if (has(nm("hour").c_str())) emit(c, name, "TIME.HOUR", nm("hour"), mlong(H));
            if (has(nm("minute").c_str())) emit(c, name, "TIME.MINUTE", nm("minute"), mlong(MI));
            if (has(nm("second").c_str())) emit(c, name, "TIME.SECOND", nm("second"), mlong(S));
            if (has(nm("millisecond").c_str())) emit(c, name, "TIME.MILLISECOND", nm("millisecond"), mlong(nanos / 1000000));
            if (has(nm("microsecond").c_str())) emit(c, name, "TIME.MICROSECOND", nm("microsecond"), mlong(nanos / 1000));
            if (has(nm("nanosecond").c_str())) emit(c, name, "TIME.NANOSECOND", nm("nanosecond"), mlong(nanos));
            if (has(nm("date").c_str())) {
                char b[32];
                snprintf(b, sizeof b, "%04lld-%02lld-%02lld", (long long)Y, (long long)MO, (long long)D);
                c.pool.emplace_back(b);
                emit(c, name, "TIME.DATE", nm("date"), mstr((const uint8_t*)c.pool.back().data(), (uint32_t)c.pool.back().size()));
            }
            if (has(nm("time").c_str())) {
                char b[32];
                snprintf(b, sizeof b, "%02lld:%02lld:%02lld", (long long)H, (long long)MI, (long long)S);
                c.pool.emplace_back(b);
                emit(c, name, "TIME.TIME", nm("time"), mstr((const uint8_t*)c.pool.back().data(), (uint32_t)c.pool.back().size()));
            }
        }
        return;
    }
    case D_FIRSTLINE: {
        int f = fl_of_tok_.at(t_fmt * 64 + oi);
        uint32_t kind = R.fl_kind[f][i];
        if (kind == FL_NONE) return;
        auto span = [&](uint32_t s) { return mstr(c.line + (s & 0xFFFF), (s >> 16) - (s & 0xFFFF)); };
        if (has("method")) { set_origin(O_FL_METHOD, f); emit(c, name, "HTTP.METHOD", "method", span(R.fl_method[f][i])); }
        if (has("uri")) { set_origin(O_FL_URI, f); emit(c, name, "HTTP.URI", "uri", span(R.fl_uri[f][i])); }
        if (kind == FL_FULL) {
            if (has("protocol")) { set_origin(O_FL_PROTO, f); emit(c, name, "HTTP.PROTOCOL_VERSION", "protocol", span(R.fl_proto[f][i])); }
        } else {
            set_origin(O_FL_PROTO, f);
            emit(c, name, "HTTP.PROTOCOL_VERSION", "protocol", mnull());
        }
        return;
    }
    case D_PROTOCOL: {
        if (v.null || v.len == 0 || (v.len == 1 && v.p[0] == '-')) return;
        // "HTTP/x.y".split("/", 2)
        uint32_t sl = 0;
        while (sl < v.len && v.p[sl] != '/') ++sl;
        set_origin(O_NONE, 0);
        if (sl < v.len) {
            if (has("")) emit(c, name, "HTTP.PROTOCOL", "", mstr(v.p, sl));
            if (has("version")) emit(c, name, "HTTP.PROTOCOL.VERSION", "version", mstr(v.p + sl + 1, v.len - sl - 1));
        } else {
            emit(c, name, "HTTP.PROTOCOL", "", mnull());
            emit(c, name, "HTTP.PROTOCOL.VERSION", "version", mnull());
        }
        return;
    }
    case D_URI: {
        if (v.null || v.len == 0) return;
        int u = ok == O_TOKEN ? uri_of_tok_.at(t_fmt * 64 + oi) : ok == O_QPARAM ? uri_of_qp_.at(oi) : uri_of_fl_.at(oi);
        uint32_t fl = R.u_flags[u][i];
        if (!(fl & UF_DONE)) return;
        if (has("query") || has("path") || has("ref")) {
            if (has("query")) {
                set_origin(O_URI_QUERY, u);
                emit(c, name, "HTTP.QUERYSTRING", "query", line_ref(R.u_query[u][i]));
            }
            set_origin(O_URI_PART, u);
            if (has("path")) emit(c, name, "HTTP.PATH", "path", line_ref(R.u_path[u][i]));
            if (has("ref")) emit(c, name, "HTTP.REF", "ref", (fl & UF_FRAG) ? line_ref(R.u_frag[u][i]) : mnull());
        }
        if (fl & UF_IS_URL) {
            set_origin(O_URI_PART, u);
            if (has("protocol")) emit(c, name, "HTTP.PROTOCOL", "protocol", (fl & UF_SCHEME) ? line_ref(R.u_scheme[u][i]) : mnull());
            if (has("userinfo")) emit(c, name, "HTTP.USERINFO", "userinfo", mnull());
            if (has("host")) emit(c, name, "HTTP.HOST", "host", (fl & UF_HOST) ? line_ref(R.u_host[u][i]) : mnull());
            if (has("port") && (fl & UF_PORT)) emit(c, name, "HTTP.PORT", "port", mlong(R.u_port[u][i]));
        }
        return;
    }
    case D_QUERY: {
        if (v.null || v.len == 0) return;
        if (ok == O_TOKEN) {
            // QueryStringFieldDissector.dissect (dissectors/QueryStringFieldDissector.java:75-104)
            // on a raw token: split("&") (trailing empty pieces dropped), names
            // lower-cased (not trimmed), values resilientUrlDecode'd -- the URI
            // kernel's piece table (lp_device.h pair_pieces / pair_fill)
            emit_pairs(c, in, name, "STRING", pair_of_tok_.at(t_fmt * 64 + oi));
            return;
        }
        int q = query_of_uri_.at(oi);
        uint32_t cnt = R.q_count[q][i];
        uint64_t tab = R.q_params[q][i];
        const uint64_t* t = (const uint64_t*)(c.arena + ref_off(tab));
        for (uint32_t k = 0; k < cnt; ++k) {
            if (t[2 * k] == REF_SKIP) continue;  // name not requested
            MVal nm = line_ref(t[2 * k]);
            MVal val = line_ref(t[2 * k + 1]);
            std::string pn((const char*)nm.p, nm.len);
            set_origin(O_NONE, 0);
            if (!qname_of_.empty()) {  // a remapped parameter: its derived URI stage follows it
                auto qn = qname_of_.find(std::to_string(q) + ":" + pn);
                if (qn != qname_of_.end()) set_origin(O_QPARAM, q * MAX_QNAMES + qn->second);
            }
            emit(c, name, "STRING", pn, val);
        }
        return;
    }
    case D_CLF2NUM: {
        // ConvertCLFIntoNumber: null or "-" -> 0L, else the same value
        bool dash = !v.null && !v.is_long && v.len == 1 && v.p[0] == '-';
        set_origin(O_CONV, oi);
        if (v.null || dash) emit(c, name, in.d->out_type, "", mlong(0));
        else emit(c, name, in.d->out_type, "", v);
        return;
    }
    case D_SECMILLIS: {
        // ConvertSecondsWithMillisStringDissector (translate/ConvertSecondsWithMillisStringDissector.java:33-40):
        // "S.F" -> S * 1000 + Long.parseLong(F), converted on the device: a
        // token by phase 1 (sm_ms), an upstream list item by the URI kernel
        // (its table entry)
        int64_t ms = 0;
        if (ok == O_TOKEN) {
            ms = R.sm_ms[secms_of_tok_.at(t_fmt * 64 + oi)][i];
        } else if (ok == O_LITEM) {
            const int j = oi & 3, k = oi >> 3, vr = (oi >> 2) & 1;
            const uint8_t* tab = c.arena + ref_off(R.l_tab[j][i]);
            memcpy(&ms, tab + (size_t)k * LIST_ENT_MS + 8 + 8 * vr, 8);
        } else {
            return;  // not reached: the planner keeps such programs off the device
        }
        set_origin(ok == O_TOKEN ? O_SECMS : O_LITEMMS, ok == O_TOKEN ? secms_of_tok_.at(t_fmt * 64 + oi) : oi);
        emit(c, name, in.d->out_type, "", mlong(ms));
        return;
    }
    case D_MS2US: {
        // ConvertMillisecondsIntoMicroseconds (translate/ConvertMillisecondsIntoMicroseconds.java:33-35)
        set_origin(O_CONV, oi);
        emit(c, name, in.d->out_type, "", mlong((int64_t)((uint64_t)v.l * 1000u)));
        return;
    }
    case D_UPSTREAM: {
        // UpstreamListDissector.dissect (nginxmodules/UpstreamListDissector.java:79-125):
        // servers = value.split(", "); parts = server.split(": "); outputs
        // parts[0].trim() and (parts.length == 1 ? parts[0] : parts[1]).trim(),
        // split on the device (lp_device.h uplist_items): the URI kernel's
        // item table in the line's region (value / redirected spans)
        if (v.null) return;
        const int j = list_of_tok_.at(t_fmt * 64 + oi);
        const uint32_t n = R.l_count[j][i];
        const uint32_t ent = prog_.list[j].secms ? LIST_ENT_MS : LIST_ENT;
        const uint8_t* tab = n ? c.arena + ref_off(R.l_tab[j][i]) : nullptr;
        for (uint32_t k = 0; k < n; ++k) {
            uint32_t sp[2];
            memcpy(sp, tab + (size_t)k * ent, 8);
            for (int vr = 0; vr < 2; ++vr) {
                set_origin(O_LITEM, item_code(j, (int)k, vr));
                emit(c, name, in.d->out_type, std::to_string(k) + (vr ? ".redirected" : ".value"),
                     mstr(c.line + (sp[vr] & 0xFFFFu), (sp[vr] >> 16) - (sp[vr] & 0xFFFFu)));
            }
        }
        return;
    }
    case D_COOKIES: {
        // RequestCookieListDissector.dissect (dissectors/RequestCookieListDissector.java:79-110):
        // Pattern("; ").split (trailing empty pieces dropped), name = the part
        // before the first '=' trimmed and lower-cased (just a name: value ""),
        // value = Utils.resilientUrlDecode of the trimmed rest -- the URI
        // kernel's piece table (lp_device.h pair_pieces / pair_fill)
        if (v.null || v.len == 0) return;
        emit_pairs(c, in, name, "HTTP.COOKIE", pair_of_tok_.at(t_fmt * 64 + oi));
        return;
    }
    case D_SETCOOKIES: {
        // ResponseSetCookieListDissector.dissect (dissectors/ResponseSetCookieListDissector.java:79-110):
        // the URI kernel's piece table (lp_device.h setc_pieces / pair_fill):
        // per cookie string in order its lower-cased name and the string itself
        if (v.null || v.len == 0) return;
        const bool all = has("*");
        const int j = pair_of_tok_.at(t_fmt * 64 + oi);
        const uint32_t n = R.p_count[j][i];
        const uint8_t* tab = n ? c.arena + ref_off(R.p_tab[j][i]) : nullptr;
        auto at = [&](uint64_t r) { return mstr((ref_arena(r) ? c.arena : c.line) + ref_off(r), ref_len(r)); };
        // (name, cookie string) in order; a name's further dissection reads
        // the Parsable's cache, which holds the LAST value added under that
        // name (core/Parsable.java:172-183, Parser.java:735-753)
        std::vector<std::pair<std::string, MVal>> got;
        for (uint32_t k = 0; k < n; ++k) {
            uint64_t e[2];
            memcpy(e, tab + 16 * (size_t)k, 16);
            const MVal nm = at(e[0]);
            std::string ns((const char*)nm.p, nm.len);
            if (all || has(ns.c_str())) got.emplace_back(std::move(ns), at(e[1]));
        }
        for (size_t k = 0; k < got.size(); ++k) {
            const MVal* last = &got[k].second;
            for (size_t q = k + 1; q < got.size(); ++q)
                if (got[q].first == got[k].first) last = &got[q].second;
            set_origin(O_NONE, 0);
            emit(c, name, "HTTP.SETCOOKIE", got[k].first, got[k].second, last);
        }
        return;
    }
    case D_SETCOOKIE: {
        // ResponseSetCookieDissector.dissect (dissectors/ResponseSetCookieDissector.java:78-135):
        // split(";"), each part trimmed and split("=", 2) with key and value
        // trimmed; part 0 is the "value", later parts "expires" (epoch seconds
        // as STRING, milliseconds as TIME.EPOCH; the device proved the date
        // matches "EEE, dd-MMM-yyyy HH:mm:ss GMT"), "domain", "comment", "path"
        if (v.null || v.len == 0) return;
        auto trim = [&](uint32_t& a, uint32_t& b) {
            while (a < b && v.p[a] <= ' ') ++a;
            while (b > a && v.p[b - 1] <= ' ') --b;
        };
        for (uint32_t ps = 0, part = 0; ps <= v.len; ++part) {
            uint32_t pe = ps;
            while (pe < v.len && v.p[pe] != ';') ++pe;
            uint32_t a = ps, b = pe;
            trim(a, b);
            uint32_t x = a;
            while (x < b && v.p[x] != '=') ++x;
            uint32_t ka = a, kb = x, va = x < b ? x + 1 : b, vb = b;
            trim(ka, kb);
            trim(va, vb);
            const std::string key((const char*)v.p + ka, kb - ka);
            set_origin(O_NONE, 0);
            if (pe == v.len && a == b && part > 0) break;  // a trailing empty part (split drops it)
            if (part == 0) {
                emit(c, name, "STRING", "value", mstr(v.p + va, vb - va));
            } else if (key == "expires") {
                const uint8_t* d = v.p + va;
                static const char mons[] = "JanFebMarAprMayJunJulAugSepOctNovDec";
                int mon = 1;
                for (int k = 0; k < 12; ++k)
                    if (d[8] == mons[3 * k] && d[9] == mons[3 * k + 1] && d[10] == mons[3 * k + 2]) mon = k + 1;
                auto d2 = [&](int i) { return (d[i] - '0') * 10 + (d[i + 1] - '0'); };
                const int64_t days = days_from_civil(d2(12) * 100 + d2(14), mon, d2(5));
                const int64_t ms = (days * 86400 + d2(17) * 3600 + d2(20) * 60 + d2(23)) * 1000;
                emit(c, name, "STRING", "expires", mlong(ms / 1000));
                set_origin(O_NONE, 0);
                emit(c, name, "TIME.EPOCH", "expires", mlong(ms));
            } else if (key == "domain" || key == "comment" || key == "path") {
                emit(c, name, "STRING", key, mstr(v.p + va, vb - va));
            }
            ps = pe + 1;
        }
        return;
    }
    case D_BINIP: {
        // NginxHttpdLogFormatDissector.BinaryIPDissector (:151-178): "\\xHH" x 4
        // -> the four bytes as Java (signed) bytes joined by '.'; the bytes
        // from phase 1 (a BinaryIP stage)
        if (v.null || v.len != 16 || ok != O_TOKEN) return;
        const uint32_t x = R.bip[binip_of_tok_.at(t_fmt * 64 + oi)][i];
        char ip[32];
        const int n = snprintf(ip, sizeof ip, "%d.%d.%d.%d", (int)(int8_t)(x & 0xFF), (int)(int8_t)((x >> 8) & 0xFF),
                               (int)(int8_t)((x >> 16) & 0xFF), (int)(int8_t)(x >> 24));
        set_origin(O_CONV, oi);
        c.pool.emplace_back(ip, (size_t)n);
        emit(c, name, in.d->out_type, "", mstr((const uint8_t*)c.pool.back().data(), (uint32_t)n));
        return;
    }
    case D_NUM2CLF: {
        // ConvertNumberIntoCLF: "0" -> null, else the same value
        bool zero = v.is_long ? v.l == 0 : (!v.null && v.len == 1 && v.p[0] == '0');
        set_origin(O_CONV, oi);
        if (zero) emit(c, name, in.d->out_type, "", mnull());
        else emit(c, name, in.d->out_type, "", v);
        return;
    }
    default:
        return;
    }
}

namespace {
void json_str(std::string& o, const uint8_t* p, uint32_t n) {
    o += '"';
    uint32_t run = 0;  // bytes [run, k) need no escape: appended in one go
    for (uint32_t k = 0; k < n; ++k) {
        const uint8_t ch = p[k];
        if (ch != '"' && ch != '\\' && ch >= 0x20) continue;
        o.append((const char*)p + run, k - run);
        run = k + 1;
        if (ch == '"') o += "\\\"";
        else if (ch == '\\') o += "\\\\";
        else {
            char b[8];
            snprintf(b, sizeof b, "\\u%04x", ch);
            o += b;
        }
    }
    o.append((const char*)p + run, n - run);
    o += '"';
}
void json_s(std::string& o, const std::string& s) { json_str(o, (const uint8_t*)s.data(), (uint32_t)s.size()); }
}  // namespace

// The token table in the canonical form tests/golden/extract_token_tables.py
// derives from the reference's Java sources: one entry per TokenParser in
// table order; "token" is the literal token or, for Named/Parameterized
// parsers, the Java regex they match the LogFormat with.
std::string token_table_json(bool nginx) {
    const TokenTable& T = nginx ? nginx_table() : apache_table();
    std::string o = "[";
    for (size_t k = 0; k < T.v.size(); ++k) {
        const TParser& t = T.v[k];
        std::string kind = "plain", tok = t.tok, custom;
        if (t.kind == TP_FIXED) kind = "fixed";
        if (t.kind == TP_NAMED) {
            kind = "named";
            tok = std::string("\\%\\{([a-z0-9\\-") + (t.underscore ? "_" : "") + "]*)\\}";
            for (char c : t.suffix) {
                if (c == '^') tok += '\\';
                tok += c;
            }
        }
        if (t.kind == TP_DOLLAR) kind = "named";
        if (t.kind == TP_PARAM) {
            kind = "param";
            tok = "\\%\\{" + t.pprefix + "([^\\}]*%[^\\}]*)\\}t";
        }
        if (t.strftime) custom = "StrfTimeStampDissector";
        o += k ? ",\n{" : "{";
        o += "\"kind\":";
        json_s(o, kind);
        o += ",\"token\":";
        json_s(o, tok);
        o += ",\"regex\":";
        json_s(o, t.regex);
        o += ",\"prio\":" + std::to_string(t.prio) + ",\"custom\":";
        if (custom.empty()) o += "null";
        else json_s(o, custom);
        o += ",\"outs\":[";
        for (size_t j = 0; j < t.outs.size(); ++j) {
            const TokOut& u = t.outs[j];
            o += j ? ",[" : "[";
            json_s(o, u.type);
            o += ',';
            json_s(o, u.name);
            o += ",[";
            bool first = true;
            for (auto [bit, nm] : {std::pair<int, const char*>{CAST_S, "STRING"}, {CAST_L, "LONG"}, {CAST_D, "DOUBLE"}})
                if (u.casts & bit) {
                    o += first ? "\"" : ",\"";
                    o += nm;
                    o += '"';
                    first = false;
                }
            o += "]]";
        }
        o += "]}";
    }
    return o + "]";
}

// Replays line c.i: every root token value through the dissector tree.
void Plan::replay(Ctx& c) const {
    const ResultView& R = c.R;
    const int64_t i = c.i;
    // memoized decisions: bounded (query / cookie names are open-ended);
    // cleared only between rows (emit keeps references into the map)
    if (t_memo.m.size() > (1u << 15)) t_memo.m.clear();
    c.rec.reserve(256);
    c.em.reserve(256);
    // the LogFormat the line was routed to (HttpdLogFormatDissector's active format)
    const int fi = prog_.n_fmt > 1 ? R.fmt_id[i] : 0;
    t_fmt = fi;
    const Format& f = *formats_[fi];
    for (const auto& kv : tok_slot_) {
        if (kv.first / 256 != fi) continue;
        int k = kv.second;
        uint32_t sp = R.tok_span[k][i];
        bool null = (R.tok_flags[i] >> k) & 1;
        MVal v = null ? mnull() : mstr(c.line + (sp & 0xFFFF), (sp >> 16) - (sp & 0xFFFF));
        for (const auto& o : f.tokens[kv.first % 256].outs) {
            t_origin_kind = O_TOKEN;
            t_origin_idx = k;
            emit(c, "", o.type, o.name, v);
        }
    }
}

int Plan::emit_row(const ResultView& R, int64_t i, EmitFn fn, void* ctx) const {
    Ctx c{R, i, R.input + R.line_off[i], R.region(i), {}, {}, {}};
    replay(c);
    for (const auto& e : c.em) {
        const int kind = e.v.is_long ? 2 : e.v.null ? 1 : 0;
        fn(ctx, e.base.c_str(), e.type.c_str(), e.name.c_str(), kind, e.v.p, e.v.len, e.v.l);
    }
    return (int)c.em.size();
}

int Plan::rec_row(const ResultView& R, int64_t i, RecFn fn, void* ctx) const {
    Ctx c{R, i, R.input + R.line_off[i], R.region(i), {}, {}, {}};
    replay(c);
    for (const auto& e : c.rec) fn(ctx, e.first, e.second);
    return (int)c.rec.size();
}

std::string Plan::record_json(const ResultView& R, int64_t i) const {
    Ctx c{R, i, R.input + R.line_off[i], R.region(i), {}, {}, {}};
    replay(c);
    std::stable_sort(c.rec.begin(), c.rec.end(),
                     [](const std::pair<std::string, MVal>& a, const std::pair<std::string, MVal>& b) {
                         return a.first < b.first;
                     });
    std::string o = "{";
    for (size_t a = 0; a < c.rec.size();) {
        if (a) o += ",";
        json_str(o, (const uint8_t*)c.rec[a].first.data(), (uint32_t)c.rec[a].first.size());
        o += ":[";
        size_t b = a;
        for (; b < c.rec.size() && c.rec[b].first == c.rec[a].first; ++b) {
            if (b > a) o += ",";
            const MVal& v = c.rec[b].second;
            char buf[64];
            if (v.is_long) {
                snprintf(buf, sizeof buf, "{\"l\":%lld}", (long long)v.l);
                o += buf;
            } else if (v.null) o += "null";
            else json_str(o, v.p, v.len);
        }
        o += "]";
        a = b;
    }
    o += "}";
    return o;
}

}  // namespace lp
