// Host-side setup of the logparser_amd engine: LogFormat -> tokens ->
// dissection tree for the requested paths -> device Program, plus the
// replay ("materializer") that turns one row of device results into the
// values the reference Parser would have delivered to the record.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "lp_program.h"

namespace lp {

constexpr int CAST_S = 1, CAST_L = 2, CAST_D = 4;

struct TokOut {
    std::string type, name;
    int casts = CAST_S;
};

struct Token {
    bool fixed = false;
    std::string regex;  // fixed: literal text
    int start = 0, len = 0, prio = 0;
    std::vector<TokOut> outs;
    bool strftime = false;
    std::string custom_type, custom_param;
};

enum FormatKind { FMT_APACHE = 1, FMT_NGINX = 2 };

struct Format {
    int kind = FMT_APACHE;
    std::string logformat, cleaned;
    std::vector<Token> tokens;
    std::vector<std::string> output_types;  // "TYPE:name", unique
    std::set<std::string> requested;        // TokenFormatDissector.requestedFields
};

enum DisClass {
    D_ROOT, D_TIMESTAMP, D_TIMESTAMP_ISO, D_FIRSTLINE, D_PROTOCOL, D_URI, D_QUERY, D_COOKIES, D_SETCOOKIES,
    D_SETCOOKIE, D_UNIQUEID, D_CLF2NUM, D_NUM2CLF, D_STRFTIME, D_LOCALIZED,
    D_BINIP, D_SECMILLIS, D_MS2US, D_UPSTREAM  // NGINX additional dissectors
};

struct Dissector {
    int cls;
    std::string in_type;
    std::vector<std::string> outs;  // "TYPE:name"
    std::string out_type;           // converters
};

struct Instance {
    int cls;
    const Dissector* d;
    std::set<std::string> requested;  // extractFieldName(input, output)
};

// one replay value
struct MVal {
    bool is_long = false;
    bool null = false;
    const uint8_t* p = nullptr;
    uint32_t len = 0;
    int64_t l = 0;
};

// Host copies of one batch's results (filled by capi.cpp)
struct HostResults {
    int64_t n = 0;
    std::vector<uint64_t> line_off;
    std::vector<uint8_t> status;
    std::vector<uint8_t> input;
    std::vector<uint8_t> arena;
    std::vector<uint64_t> arena_base;
    std::vector<std::vector<uint32_t>> tok_span;
    std::vector<uint32_t> tok_flags;
    std::vector<std::vector<int64_t>> t_epoch;
    std::vector<std::vector<uint64_t>> t_local, t_utc;
    std::vector<std::vector<uint32_t>> t_nano;
    std::vector<std::vector<uint32_t>> fl_kind, fl_method, fl_uri, fl_proto;
    std::vector<std::vector<uint32_t>> u_flags;
    std::vector<std::vector<uint64_t>> u_scheme, u_host, u_path, u_query, u_frag;
    std::vector<std::vector<int32_t>> u_port;
    std::vector<std::vector<uint32_t>> q_count;
    std::vector<std::vector<uint64_t>> q_params;
    std::vector<uint8_t> fmt_id;  // multi-format programs: the routed LogFormat per line
};

class Plan {
public:
    // returns LP_OK / LP_E_UNSUPPORTED / error; err filled on error
    int build(const std::string& logformats, const std::vector<std::string>& fields, std::string& err);
    static int possible_paths(const std::string& logformats, int max_depth, std::vector<std::string>& out,
                              std::string& err);

    const Program& program() const { return prog_; }
    bool device_ok() const { return device_ok_; }
    const std::string& unsupported_reason() const { return why_; }
    std::string describe() const;

    // canonical JSON record of line i (status OK)
    std::string record_json(const HostResults& R, int64_t i) const;

private:
    int build_dissectors(const std::string& logformats, std::string& err);
    void find_useful(const std::set<std::string>& possible, const std::string& type, const std::string& name,
                     bool is_root);
    void compile_program();

    // replay
    struct Ctx;
    void emit(Ctx& c, const std::string& base, const std::string& type, const std::string& name, const MVal& v) const;
    void run_phase(Ctx& c, const Instance& in, const std::string& name, const MVal& v) const;

    std::vector<std::unique_ptr<Format>> formats_;
    std::vector<std::unique_ptr<Dissector>> dis_;
    std::string root_type_ = "HTTPLOGLINE";
    std::set<std::string> needed_, useful_, located_;
    std::map<std::string, std::vector<Instance>> compiled_;
    Program prog_{};
    bool device_ok_ = true;
    std::string why_;
    // device stage bookkeeping for the replay
    std::map<int, int> tok_slot_;          // format * 256 + token index -> slot
    // stage maps keyed by format * 64 + slot (token stages) or stage index
    std::map<int, int> time_of_tok_, fl_of_tok_, uri_of_tok_;
    std::map<int, int> uri_of_fl_;
    std::map<int, int> query_of_uri_;
    // replay source tracking: emission id -> (kind, stage)
    std::map<std::string, std::pair<int, int>> src_;
};

}  // namespace lp
