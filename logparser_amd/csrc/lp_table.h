// Typed output columns built on the device (lp_result_table on a device
// view): for each requested "TYPE:path" the planner names the device column
// its value comes from (per LogFormat), and two kernels fill the caller's
// columns -- values and per-row string lengths, then (after a scan of the
// lengths) the string bytes -- in the Arrow layout of include/logparser_amd.h.
// The per-row choice mirrors Plan::replay exactly for the kinds below; a path
// the replay derives in any other way stays on the host table.
#pragma once
#include <stdint.h>

#include "lp_program.h"

namespace lp {

enum : int32_t {
    TC_NONE = 0,   // not delivered for this LogFormat
    TC_TOKEN,      // a = token slot: the value (null: "-")
    TC_CLF2NUM,    // a = token slot: ConvertCLFIntoNumber (null -> 0L, else the value)
    TC_NUM2CLF,    // a = token slot: ConvertNumberIntoCLF ("0" -> null, else the value)
    TC_TIME,       // a = time stage, b = TF_* field, c = 1: the _utc group
    TC_FL,         // a = first-line stage, b = 0 method / 1 uri / 2 protocol
    TC_PROTO,      // a = first-line stage, b = 0 protocol / 1 version (of its protocol)
    TC_URI,        // a = URI stage, b = UP_* part
    TC_QP,         // a = query stage, b / c = offset / length of the name in TableArgs::names (the last occurrence)
    TC_NULL,       // always null (HttpUriDissector's userinfo)
    TC_SECMS,      // a = SECOND_MILLIS stage: its milliseconds (b = 1: x 1000, MICROSECONDS)
    TC_LIST,       // a = upstream list stage, b = item, c = 0 value / 1 redirected
    TC_LIST_MS,    // a = SECOND_MILLIS list stage, b = item, c bit 0: redirected, bit 1: MICROSECONDS
    TC_BINIP,      // a = BinaryIP stage: its bytes as signed decimals joined by '.'
    TC_PAIR,       // a = pair stage (cookie / raw query), b / c = offset / length of the name in TableArgs::names (the last occurrence)
    TC_SETC,       // a = Set-Cookie pair stage | SC_* field << 8, b / c = the cookie name in TableArgs::names:
                   // ResponseSetCookieDissector on the name's last cookie string
};
// ResponseSetCookieDissector outputs (dissectors/ResponseSetCookieDissector.java:49-58)
enum : int32_t { SC_VALUE, SC_EXPIRES_S /* STRING:expires, seconds */, SC_EXPIRES_MS /* TIME.EPOCH:expires */,
                 SC_DOMAIN, SC_COMMENT, SC_PATH };
enum : int32_t { TF_EPOCH, TF_DAY, TF_MONTHNAME, TF_MONTH, TF_WEEK, TF_WEEKYEAR, TF_YEAR, TF_HOUR, TF_MINUTE,
                 TF_SECOND, TF_MILLI, TF_MICRO, TF_NANO, TF_DATE, TF_TIME };
enum : int32_t { UP_QUERY, UP_PATH, UP_REF, UP_PROTOCOL, UP_HOST, UP_PORT };

struct TableSrc {
    int32_t kind, a, b, c;
};

constexpr int MAX_TABLE_COLS = 32;
constexpr int TABLE_NAMES = 2048;

struct TableCol {
    int32_t kind;  // LP_CAST_STRING 1 / LONG 2 / DOUBLE 4
    int32_t pad;
    TableSrc src[MAX_FMT];
    // an earlier delivery of the same path (TC_NONE: none): the row's value
    // when src delivers none (ParsedRecord: a null is ignored, the last value
    // wins) -- a token that a converter of another token delivers again
    TableSrc alt[MAX_FMT];
    LP_G uint8_t* valid;
    LP_G int64_t* i64;   // STRING: offsets [count + 1]; LONG: values
    LP_G double* f64;
    LP_G uint8_t* chars;
};

// a STRING column's value of one row as k_table_values found it, for
// k_table_chars (TableArgs::srcw): tag in bits 63:62 -- SW_PTR the bytes'
// address (bit 61: a leading '&'), SW_LONG a long in bits 61:0 (two's
// complement), SW_SLOW anything else (a formatted date / time / month name /
// binary IP, or a long outside 62 bits): k_table_chars derives it again
constexpr uint64_t SW_AMP = 1ull << 61, SW_LONG = 1ull << 62, SW_SLOW = 2ull << 62;

struct TableArgs {
    int64_t first, count;
    int32_t n_cols, pad;
    LP_G uint64_t* srcw;  // [STRING column rank][count] value words (scratch)
    TableCol cols[MAX_TABLE_COLS];
    uint8_t names[TABLE_NAMES];
};

}  // namespace lp
