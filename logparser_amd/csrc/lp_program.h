// Compiled device program: the LogFormat turned into a flat element list
// (literal separators + field classes) plus the downstream dissector stages
// the requested paths need.  Plain-old-data; lives in __constant__ memory on
// the GPU.  Built on the host by lp_compile (plan.cpp).
//
// Reference: TokenFormatDissector.parseTokenLogFileDefinition / prepareForRun
// (hp/dissectors/tokenformat/TokenFormatDissector.java:179-213, 294-379)
// produce "^" + \Q..\E literals + (token regex) + "$"; here each token regex
// is mapped to an element kind with an exact leftmost-first candidate
// enumerator (lp_device.h).
#pragma once
#include <stdint.h>

#if !defined(__HIP__)
// host-only translation units (plan.cpp, the test-only tests/emu build)
#ifndef __host__
#define __host__
#endif
#ifndef __device__
#define __device__
#endif
#endif

#if defined(__HIP__)
#define LP_UNROLL _Pragma("unroll")
#define LP_INLINE __attribute__((always_inline)) inline
#else
#define LP_UNROLL
#define LP_INLINE inline
#endif

namespace lp {

// profiling build (-DLP_PROFILE, lp_device.h): per-wave timestamps of waves [PROF_W0, PROF_W0 + PROF_WAVES)
constexpr int PROF_WAVES = 16384, PROF_W0 = 1024, PROF_POINTS = 96;

constexpr int MAX_ELEMS = 96;
constexpr int MAX_FMT = 8;        // LogFormats of one HttpdLogFormatDissector (sticky routing)
constexpr int MAX_FMT_ELEMS = 64; // elements of one LogFormat (6-bit DFS stack index)
constexpr uint8_t FMT_UNKNOWN = 15; // routing state that depends on a line the device could not decide
constexpr int MAX_LIT = 2048;
constexpr int MAX_TOK = 16;      // captured tokens (bit k of the null/zero masks)
constexpr int MAX_TIME = 4;
constexpr int MAX_FL = 4;
constexpr int MAX_URI = 8;
constexpr int MAX_QUERY = 8;
constexpr int MAX_QNAMES = 32;   // explicitly requested query parameter names
constexpr int MAX_LINE = 8191;   // longer lines -> FALLBACK (13-bit offsets)
constexpr int MAX_STACK = 16;    // DFS choice points
constexpr int MAX_SECMS = 4;     // SECOND_MILLIS token conversions (ConvertSecondsWithMillisStringDissector)
constexpr int MAX_LIST = 4;      // NGINX upstream lists (UpstreamListDissector)
constexpr int MAX_BINIP = 2;     // NGINX $binary_remote_addr values (BinaryIPDissector)
constexpr int MAX_PAIR = 4;      // request cookie headers / raw-token query strings

// Element kinds = the token regexes of the Apache table
// (hp/dissectors/tokenformat/TokenParser.java:35-59).
enum ElemKind : uint8_t {
    EK_LIT = 0,
    EK_NOSPACE,      // [^\s]*
    EK_NUMBER,       // [0-9]+
    EK_CLFNUMBER,    // [0-9]+|-
    EK_HEXNUMBER,    // [0-9a-fA-F]+
    EK_CLFHEXNUMBER, // [0-9a-fA-F]+|-
    EK_NONZERO,      // [1-9][0-9]*
    EK_ANY_GREEDY,   // .*
    EK_ANY_LAZY,     // .*?
    EK_TIME_US,      // [0-3][0-9]/(?:[a-zA-Z]{3})/[1-9][0-9]{3}:[0-9]{2}:[0-9]{2}:[0-9]{2} [\+|\-][0-9]{4}
    EK_CLF_IP,       // IPv4|IPv6|-  (IPv4 dotted quad or '-' on device, else FALLBACK)
    EK_IP,           // IPv4|IPv6
    // NGINX token regexes (nginxmodules/CoreLogModule.java, UpstreamModule.java)
    EK_ANYCHAR,      // .                                  ($pipe)
    EK_DECIMAL,      // [0-9]+\.[0-9]+                      ($request_time, SECOND_MILLIS)
    EK_MSEC,         // [0-9]+\.[0-9][0-9][0-9]             ($msec)
    EK_NOSPACE3,     // [^\s]* [^\s]* [^\s]*                ($request)
    EK_UPLIST_DEC,   // X(?: *, *X(?: *: *X)?)*, X = [0-9]+\.[0-9]+   (upstream time lists)
    EK_UPLIST_NUM,   // X(?: *, *X(?: *: *X)?)*, X = [0-9]+            (upstream byte lists)
    EK_UPLIST_NS,    // X(?: *, *X(?: *: *X)?)*, X = [^\s]*           (upstream address / status lists)
    EK_BINIP,        // (\\x[0-9a-fA-F]{2}){4}                         ($binary_remote_addr)
    EK_TIME_ISO,     // [1-9][0-9]{3}-[0-1][0-9]-[0-3][0-9]T[0-9]{2}:[0-9]{2}:[0-9]{2}[\+|\-][0-9]{2}:[0-9]{2}
    EK_CACHE_STATUS, // (?:MISS|BYPASS|EXPIRED|STALE|UPDATING|REVALIDATED|HIT)  ($upstream_cache_status)
};

struct alignas(16) Elem {
    uint8_t kind;
    uint8_t det;       // only the first candidate can lead to an overall match
    int8_t cap;        // captured token slot, -1 = non-capturing (?:...)
    uint8_t last;      // last element (followed by '$')
    uint16_t lit_off;  // EK_LIT: own literal; tokens: following literal (if nlit)
    uint16_t lit_len;
    uint8_t nlit;      // token followed by a literal
    uint8_t need;      // ANY_GREEDY: occurrences of the literal's first byte in the literals from here to '$'
    int8_t acls;       // mask class (MC_*) holding the first byte of that literal, -1 none
    uint8_t pad;
    uint32_t lit4;     // first (up to) 4 bytes of that literal, little-endian
};

// An element in registers.  Device code reads an Elem as four dwords (one
// s_load_dwordx4 / ds_read_b128) and decodes the fields: a byte field read
// directly would be a per-lane global byte load with a full memory wait.
struct ElemV {
    int kind, det, cap, last, lit_off, lit_len, nlit, need, acls;
    uint32_t lit4;
};
template <typename P>
__host__ __device__ inline ElemV load_elem(P p) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(p);
    const uint32_t a = w[0], b = w[1], c = w[2];
    ElemV e;
    e.kind = (int)(a & 0xFFu);
    e.det = (int)((a >> 8) & 0xFFu);
    e.cap = (int)(int8_t)(uint8_t)(a >> 16);
    e.last = (int)(a >> 24);
    e.lit_off = (int)(b & 0xFFFFu);
    e.lit_len = (int)(b >> 16);
    e.nlit = (int)(c & 0xFFu);
    e.need = (int)((c >> 8) & 0xFFu);
    e.acls = (int)(int8_t)(uint8_t)(c >> 16);
    e.lit4 = w[3];
    return e;
}

// TimeStampDissector on a TIME.STAMP token (TK_APACHE: the fixed
// "dd/MMM/yyyy:HH:mm:ss ZZ" of hp/dissectors/TimeStampDissector.java:46), or
// StrfTimeStampDissector on a %{...}t token (TK_STRF,
// hp/dissectors/StrfTimeStampDissector.java:44-70): the DateTimeFormatter
// StrfTimeToDateTimeFormatter builds (:140-432) as a list of parser elements
// op[k] = SE_* | field << 8 | width << 16 | arg << 24, parsed left to right
// (lp_device.h parse_strf_time).
enum : uint8_t { TK_APACHE = 0, TK_STRF = 1, TK_ISO = 2 };  // TK_ISO: TIME.ISO8601 ($time_iso8601)
// java.time fields the conversions set (ChronoField unless noted)
enum : uint8_t {
    SF_YEAR, SF_MONTH, SF_DOM, SF_DOW, SF_ISODOW /* WeekFields.ISO.dayOfWeek() */, SF_DOY,
    SF_WBY /* WeekFields.of(en_US).weekBasedYear() */, SF_WOY /* WeekFields.ISO.weekOfYear() */, SF_HOD,
    SF_CHOD /* CLOCK_HOUR_OF_DAY */, SF_CHAP /* CLOCK_HOUR_OF_AMPM */, SF_AMPM, SF_MIN, SF_SEC, SF_MILLI, SF_MICRO,
    SF_OFFSET, SF_INSTANT, SF_NFIELDS
};
// parser elements: literal char (arg), fixed-width number, 1..19-digit
// number, padNext(2, ' ') + 1..19-digit number, 2-digit reduced value (base
// 2000), text table (arg: ST_*), offset "+HHMM", zone text
enum : uint8_t { SE_LIT, SE_NUM, SE_NUMV, SE_PAD2, SE_RED2, SE_TEXT, SE_OFF, SE_ZONE };
enum : uint8_t { ST_MON_SHORT, ST_MON_FULL, ST_DOW_SHORT, ST_DOW_FULL, ST_AMPM_UP, ST_AMPM_LOW };
constexpr int MAX_SF_OPS = 128;
// fields of a fixed-layout plan (TimeStage::fx_f): number, reduced number
// (base 2000), a text table (ST_MON_SHORT / ST_DOW_SHORT / AMPM), offset "+HHMM"
enum : uint8_t { FX_NUM, FX_RED2, FX_TEXT, FX_OFF };
constexpr int MAX_FX = 12;
// Stage structs hold 32-bit fields only: the kernels read them with scalar
// (dword) loads.
struct TimeStage {
    int32_t tok;
    int32_t fmt;     // the LogFormat whose token this is
    int32_t kind;    // TK_*
    int32_t zone;    // TK_STRF: the pattern has %z or %Z (else the formatter's zone is UTC)
    int32_t fixed_w; // TK_STRF: every op has a fixed width and they total fixed_w bytes (<= 32), else 0
    int32_t n_ops;
    uint32_t op[MAX_SF_OPS];
    // TK_STRF with fixed_w and no field parsed twice: the layout as byte
    // masks over the value's 32 bytes (strf_fixed); fx_n = 0: no such plan
    int32_t fx_n;                  // fields
    uint32_t fx_has;               // their SF_* bits
    uint32_t fx_lit[8], fx_litm[8]; // literal bytes (letters lower-case) and their positions
    uint32_t fx_fold[8];           // 0x20 at the literal letters (case-insensitive)
    uint32_t fx_dig[8];            // 0xFF at the bytes that must be ASCII digits
    uint32_t fx_f[MAX_FX];         // offset | width << 8 | field << 16 | FX_* code << 24
};

// HttpFirstLineDissector on an HTTP.FIRSTLINE token
// (hp/dissectors/HttpFirstLineDissector.java:56-134).
struct FlStage {
    int32_t tok;
    int32_t fmt;
};

// HttpUriDissector (hp/dissectors/HttpUriDissector.java:130-233) on either a
// token (e.g. request.referer), the uri of a first-line stage, or a query
// parameter that a type remapping (core/Parser.java:446-455, Parsable.java:
// 160-176) turned into an HTTP.URI (a "derived" stage: src_q >= 0; it runs
// in k_derived_lines, after the query pieces of its source are complete).
struct UriStage {
    int32_t src_tok;     // >= 0: token slot
    int32_t src_fl;      // >= 0: first-line stage (its uri)
    int32_t want_query;  // rawQuery needed (delivered or dissected further)
    int32_t want_path;
    int32_t want_ref;
    int32_t want_userinfo;
    int32_t query_stage; // QueryStringFieldDissector on its query, -1 none
    int32_t fmt;         // the LogFormat of its source token
    int32_t src_q;       // >= 0: query stage whose parameter src_qname (an index into its names) is the source
    int32_t src_qname;
};

// QueryStringFieldDissector (hp/dissectors/QueryStringFieldDissector.java:56-108)
struct QueryStage {
    int32_t uri;
    int32_t want_all;       // "*" requested
    int32_t n_names;        // explicitly requested (lower-case) names
    uint32_t name_off[MAX_QNAMES];  // into lit pool
    uint32_t name_len[MAX_QNAMES];
};

// ConvertSecondsWithMillisStringDissector on a captured token
// (translate/ConvertSecondsWithMillisStringDissector.java:33-40): "S.F" ->
// S * 1000 + F (the fraction read as an integer); phase 1 writes the int64.
struct SecmsStage {
    int32_t tok;
    int32_t fmt;
};

// UpstreamListDissector on a captured list token
// (nginxmodules/UpstreamListDissector.java:79-125): the items of
// split(", "), each server's split(": ") parts trimmed.  The URI kernel
// writes per line the item count and, in the line's arena region, one entry
// per item: the value and redirected spans (u32, line-relative), then for
// SECOND_MILLIS lists both as milliseconds (i64).
struct ListStage {
    int32_t tok;
    int32_t fmt;
    int32_t secms;  // the items are SECOND_MILLIS (their conversions are stored too)
    int32_t pad;
};
constexpr uint32_t LIST_ENT = 8, LIST_ENT_MS = 24;  // entry bytes without / with the milliseconds

// Name / value pieces of a captured token, split by the URI kernel into a
// table in the line's region, 16 bytes per piece: the name ref (lower-cased
// copy spilled when it has upper-case letters) and the value ref (decoded
// copy spilled when it has '%' / '+').
//   PK_COOKIE: RequestCookieListDissector (dissectors/RequestCookieListDissector.java:79-110)
//   PK_QUERY:  QueryStringFieldDissector on a raw token (%q, $args;
//              dissectors/QueryStringFieldDissector.java:76-108)
//   PK_SETC:   ResponseSetCookieListDissector (dissectors/ResponseSetCookieListDissector.java:86-110):
//              the cookie strings of a Set-Cookie list, named by HttpCookie.parse
//              (lower-cased), the value the cookie string itself (never decoded)
enum : int32_t { PK_COOKIE = 0, PK_QUERY = 1, PK_SETC = 2 };
struct PairStage {
    int32_t tok;
    int32_t fmt;
    int32_t kind;
    int32_t pad;
};

// NginxHttpdLogFormatDissector.BinaryIPDissector on a captured
// $binary_remote_addr token (hp/NginxHttpdLogFormatDissector.java:151-178):
// "\xHH" x 4 -> the four bytes; phase 1 writes them as one u32 (byte k of
// the address in bits 8k..8k+7), delivered as the bytes read as Java
// (signed) bytes joined by '.'.
struct BinipStage {
    int32_t tok;
    int32_t fmt;
};

// Stages (time / first line / URI) belong to one LogFormat: a line runs the
// stages of the format it was routed to.  Token slot k of a line is the k-th
// captured token of that line's format.
struct Program {
    int32_t n_elems;      // all formats
    int32_t n_tok;        // captured token slots (max over the formats)
    int32_t n_time, n_fl, n_uri, n_query;
    int32_t n_fmt;        // LogFormats; > 1: HttpdLogFormatDissector sticky routing
    int32_t max_stack;    // DFS depth bound = number of non-deterministic elements (<= MAX_STACK)
    int32_t fmt_elem0[MAX_FMT + 1];  // elements of format f: [fmt_elem0[f], fmt_elem0[f + 1])
    int32_t fmt_apache[MAX_FMT];     // 1 = Apache decodeExtractedValue rules, 0 = NGINX
    int32_t fmt_quotes[MAX_FMT];     // '"' bytes in format f's literals (a line needs at least as many)
    // run histograms (lp_histograms): format f's token slot of the response
    // status (request.status.last, else request.status), and its first-line
    // stage (the method); -1 none
    int32_t hist_status[MAX_FMT];
    int32_t hist_fl[MAX_FMT];
    // token slots of format f whose value the replay URL-decodes (request
    // cookies): bit k -> phase 1 sends the line to FALLBACK unless every '%'
    // is followed by two hex digits and the value is ASCII
    int32_t guard_pct[MAX_FMT];
    // token slots of format f holding a Set-Cookie header list the replay
    // splits into cookies (ResponseSetCookieListDissector): bit k -> phase 1
    // sends the line to FALLBACK unless the value is in the restated subset
    // where java.net.HttpCookie.parse cannot throw (setcookie_ok);
    // guard_setc_exp: the same slots whose cookies ResponseSetCookieDissector
    // dissects (every "expires" must then parse)
    int32_t guard_setc[MAX_FMT];
    int32_t guard_setc_exp[MAX_FMT];
    int32_t n_secms, n_list, n_binip, n_pair;
    SecmsStage secms[MAX_SECMS];
    ListStage list[MAX_LIST];
    BinipStage binip[MAX_BINIP];
    PairStage pair[MAX_PAIR];
    Elem elems[MAX_ELEMS];
    TimeStage time[MAX_TIME];
    FlStage fl[MAX_FL];
    UriStage uri[MAX_URI];
    QueryStage query[MAX_QUERY];
    alignas(4) uint8_t lit[MAX_LIT];
    // phase 2 runs (the URI kernel): URI stages or upstream list stages, whose
    // results live in the line's arena region
    __host__ __device__ LP_INLINE bool has_phase2() const { return n_uri > 0 || n_list > 0 || n_pair > 0; }
    // literal pool byte i, read as a dword (scalar load for a uniform index)
    __host__ __device__ uint32_t lit_byte(int i) const {
        return (reinterpret_cast<const uint32_t*>(lit)[i >> 2] >> (8 * (i & 3))) & 0xFFu;
    }
};

// Packed calendar fields (TimeStampDissector "as parsed" / "_utc" groups)
//   bits  0..15 year, 16..19 month, 20..24 day, 25..29 hour, 30..35 minute,
//   36..41 second, 42..57 week-based-year, 58..63 week-of-week-based-year
__host__ __device__ inline uint64_t pack_cal(uint32_t y, uint32_t mo, uint32_t d, uint32_t h, uint32_t mi,
                                             uint32_t s, uint32_t wy, uint32_t wk) {
    return (uint64_t)y | ((uint64_t)mo << 16) | ((uint64_t)d << 20) | ((uint64_t)h << 25) | ((uint64_t)mi << 30) |
           ((uint64_t)s << 36) | ((uint64_t)wy << 42) | ((uint64_t)wk << 58);
}

// A "ref" names a byte string: bits 0..31 offset, 32..61 length, bit 63 set
// when the bytes live in the line's arena region (else: relative to the
// line start).  Bit 62 (REF_AMP): the string is '&' followed by the bytes
// (line or region) -- the HttpUriDissector rawQuery of a query that needs no
// other rewriting, delivered without copying it.  A query table slot whose
// name was not requested holds REF_SKIP (~0) as its name ref.
constexpr uint64_t REF_ARENA = 1ull << 63;
constexpr uint64_t REF_AMP = 1ull << 62;
__host__ __device__ inline uint64_t mkref(uint32_t off, uint32_t len, bool arena) {
    return (uint64_t)off | ((uint64_t)len << 32) | (arena ? REF_ARENA : 0ull);
}
__host__ __device__ inline uint32_t ref_off(uint64_t r) { return (uint32_t)r; }
__host__ __device__ inline uint32_t ref_len(uint64_t r) { return (uint32_t)((r >> 32) & 0x3FFFFFFFu); }
__host__ __device__ inline bool ref_arena(uint64_t r) { return (r & REF_ARENA) != 0; }
__host__ __device__ inline bool ref_amp(uint64_t r) { return (r & REF_AMP) != 0; }

// Token span: start | end << 16 (line-relative)
__host__ __device__ inline uint32_t mkspan(uint32_t a, uint32_t b) { return a | (b << 16); }

// First-line stage info word
enum : uint32_t { FL_NONE = 0, FL_FULL = 1, FL_CHOPPED = 2 };

// URI stage flag bits
enum : uint32_t {
    UF_DONE = 1u << 0,       // dissected (input non-null, non-empty)
    UF_IS_URL = 1u << 1,     // not the dummy-protocol relative form
    UF_HOST = 1u << 2,       // host non-null
    UF_PORT = 1u << 3,       // port != -1
    UF_QUERY = 1u << 4,      // rawQuery non-null (else "")
    UF_FRAG = 1u << 5,       // fragment non-null
    UF_PATH = 1u << 6,       // path non-null
    UF_SCHEME = 1u << 7,     // scheme non-null
};

// Output column set of one batch (device pointers).
// Device pointers of the result columns and the arena are global-memory
// pointers on the device (global_load/global_store: a FLAT store would also
// count against lgkmcnt and stall the next LDS read of the same wave until
// the store is acknowledged).  Host code (and other translation units) sees
// plain pointers of the same size.
#if defined(__HIP_DEVICE_COMPILE__) && defined(LP_KERNEL_TU)
#define LP_G __attribute__((address_space(1)))
#else
#define LP_G
#endif

// Per-batch device bookkeeping (one block per handle, zeroed before each batch).
constexpr int ARENA_SHARDS = 64;  // arena bump pointers, each owning 1/64 of the arena
struct Meta {
    unsigned long long counters[8];  // lines, ok, bad, fallback, arena bytes written, URI source bytes read
    unsigned long long n_lines;      // lines of the batch (the line index's count)
    unsigned long long cap_ovf;      // 1: more lines than the columns hold (nothing parsed, retry)
    unsigned long long ovf_waves;    // waves queued for the direct (HBM) parse kernel
    unsigned long long arena_ovf;    // lines whose arena allocation did not fit its shard (retry)
    unsigned long long fmt_state;    // routed LogFormat after the batch's last line
    unsigned long long uri_ovf_waves;// waves whose URI bytes exceed the URI kernel's compact buffer (direct path)
    unsigned long long ovf_lines;    // lines the chunked parse kernel queued for the direct kernel
    unsigned long long deferred;     // chunks whose wave stopped waiting for its line number (second pass)
    // self-checks of the chunked kernels' own bookkeeping (line index, queued
    // lines): how many failed, and the first failure (kind, then four values;
    // see check_fail in parse.hip).  Non-zero fails the batch (LP_E_DEVICE).
    unsigned long long err;
    unsigned long long err_info[15];  // (5 used; the rest keeps shard_top on its own 128-B lines)
    unsigned long long shard_top[ARENA_SHARDS * 16];  // bump pointer of shard s at [16 s] (own 128-B line)
};

struct Columns {
    LP_G uint8_t* status;          // [n]
    const LP_G uint64_t* line_off; // [n+1]
    LP_G uint32_t* tok_span[MAX_TOK];
    LP_G uint32_t* tok_flags;      // bit k: value "-" (null); bit 16+k: value == "0"
    LP_G uint32_t* hist;           // run-histogram word of an OK line (lp_device.h hist_word)
    LP_G int64_t* t_epoch[MAX_TIME];
    LP_G uint64_t* t_local[MAX_TIME];
    LP_G uint64_t* t_utc[MAX_TIME];
    LP_G uint32_t* t_nano[MAX_TIME];   // nano-of-second (strftime msec_frac / usec_frac)
    LP_G uint32_t* fl_kind[MAX_FL];
    LP_G uint32_t* fl_method[MAX_FL];  // spans
    LP_G uint32_t* fl_uri[MAX_FL];
    LP_G uint32_t* fl_proto[MAX_FL];
    LP_G uint32_t* u_flags[MAX_URI];
    LP_G uint64_t* u_scheme[MAX_URI];
    LP_G uint64_t* u_host[MAX_URI];
    LP_G int32_t* u_port[MAX_URI];
    LP_G uint64_t* u_path[MAX_URI];
    LP_G uint64_t* u_query[MAX_URI];
    LP_G uint64_t* u_frag[MAX_URI];
    LP_G uint32_t* q_count[MAX_QUERY]; // params are (name ref, value ref) pairs in the arena
    LP_G uint64_t* q_params[MAX_QUERY];// ref to the param table in the arena
    LP_G int64_t* sm_ms[MAX_SECMS];    // SECOND_MILLIS stage s: the token as milliseconds
    LP_G uint32_t* l_count[MAX_LIST];  // upstream list stage j: items
    LP_G uint64_t* l_tab[MAX_LIST];    // ... region ref of its item table (ListStage)
    LP_G uint32_t* bip[MAX_BINIP];     // BinaryIP stage b: the address bytes
    LP_G uint32_t* p_count[MAX_PAIR];  // name / value pieces of pair stage j
    LP_G uint64_t* p_tab[MAX_PAIR];    // ... region ref of its piece table (PairStage)
    LP_G uint64_t* arena_base;         // [n]
    // sticky multi-format routing (Program::n_fmt > 1)
    LP_G uint16_t* fmt_match;          // [n] bit f: format f matches; bit 8+f: undecided on the device
    LP_G uint8_t* fmt_id;              // [n] the routed format, FMT_UNKNOWN
    LP_G uint64_t* fmt_chunk;          // per chunk of FMT_CHUNK lines: composed transition table, then entry state
    uint32_t fmt_init;                 // routing state before the first line (the handle's state)
    LP_G uint8_t* arena;
    uint64_t shard_cap;                  // arena bytes per shard (ARENA_SHARDS shards)
    LP_G Meta* meta;
    LP_G uint32_t* ovf_list;             // waves for the direct parse kernel
    LP_G uint32_t* uri_ovf_list;         // waves for the direct URI kernel
    LP_G uint32_t* wave_counts;          // [n_waves][WC_WORDS] lines ok bad fallback written (reduced after the launch)
    // chunked parse (one-format programs: the line index built inside the
    // parse kernel): per byte chunk the decoupled look-back word, its status
    // counts, and the lines queued for the direct kernel
    LP_G uint64_t* chunk_state;          // [n_chunks] aggregate / inclusive line counts
    LP_G uint32_t* chunk_counts;         // [n_chunks][WC_WORDS]
    LP_G uint32_t* ovf_lines;            // [cap_lines] line numbers
    LP_G uint32_t* deferred_chunks;      // [n_chunks] chunks left to the deferred pass (Meta::deferred of them)
    int64_t cap_lines;                   // lines the columns hold
};

}  // namespace lp
