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
#include "lp_table.h"

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

// Read-only view of one batch's results for the replay: the SoA columns,
// the line index, the input bytes and the side arena, all in host memory
// (a copy made by lp_result_copy, or the test-only emulation's vectors).
// Column k of a stage is indexed [k][line].
struct ResultView {
    int64_t n = 0;
    const uint64_t* line_off = nullptr;   // [n + 1]
    const uint8_t* status = nullptr;
    const uint8_t* input = nullptr;       // line i = input[line_off[i], line_off[i + 1] - 1) minus a "\r\n"'s '\r'
    const uint8_t* arena = nullptr;
    const uint64_t* arena_base = nullptr; // per line: arena offset of its region
    // arena offsets b are device offsets of ARENA_SHARDS shards of shard_cap
    // bytes; shard s starts at arena + shard_off[s] in this view
    uint64_t shard_cap = 0;
    uint64_t shard_off[ARENA_SHARDS] = {};
    const uint32_t* tok_span[MAX_TOK] = {};
    const uint32_t* tok_flags = nullptr;
    const int64_t* t_epoch[MAX_TIME] = {};
    const uint64_t* t_local[MAX_TIME] = {};
    const uint64_t* t_utc[MAX_TIME] = {};
    const uint32_t* t_nano[MAX_TIME] = {};
    const uint32_t* fl_kind[MAX_FL] = {};
    const uint32_t* fl_method[MAX_FL] = {};
    const uint32_t* fl_uri[MAX_FL] = {};
    const uint32_t* fl_proto[MAX_FL] = {};
    const uint32_t* u_flags[MAX_URI] = {};
    const uint64_t* u_scheme[MAX_URI] = {};
    const uint64_t* u_host[MAX_URI] = {};
    const uint64_t* u_path[MAX_URI] = {};
    const uint64_t* u_query[MAX_URI] = {};
    const uint64_t* u_frag[MAX_URI] = {};
    const int32_t* u_port[MAX_URI] = {};
    const uint32_t* q_count[MAX_QUERY] = {};
    const uint64_t* q_params[MAX_QUERY] = {};
    const int64_t* sm_ms[MAX_SECMS] = {};
    const uint32_t* l_count[MAX_LIST] = {};
    const uint64_t* l_tab[MAX_LIST] = {};
    const uint32_t* bip[MAX_BINIP] = {};
    const uint32_t* p_count[MAX_PAIR] = {};
    const uint64_t* p_tab[MAX_PAIR] = {};
    const uint8_t* fmt_id = nullptr;      // multi-format programs: the routed LogFormat per line
    // the bytes of line i's arena region
    const uint8_t* region(int64_t i) const {
        if (!arena) return nullptr;
        const uint64_t b = arena_base[i];
        if (!shard_cap) return arena + b;
        const uint64_t s = b / shard_cap;
        if (s >= (uint64_t)ARENA_SHARDS) return nullptr;  // no region (never for an OK line)
        return arena + shard_off[s] + (b - s * shard_cap);
    }
};

// the Apache or NGINX token table as canonical JSON (checked against the
// tables extracted from the reference's sources by the CPU tests)
std::string token_table_json(bool nginx);

// Parser.addTypeRemapping(input, newType, casts) (core/Parser.java:660-677)
struct Remap {
    std::string input, type;
    int casts = CAST_S;
};

class Plan {
public:
    // returns LP_OK / LP_E_UNSUPPORTED / error; err filled on error
    int build(const std::string& logformats, const std::vector<std::string>& fields, std::string& err,
              const std::vector<Remap>& remaps = {});
    static int possible_paths(const std::string& logformats, int max_depth, std::vector<std::string>& out,
                              std::string& err, const std::vector<Remap>& remaps = {});

    const Program& program() const { return prog_; }
    // Parser.getCasts(name) (core/Parser.java:127-129): CAST_* bits of a
    // "TYPE:path" the dissectors deliver for the requested paths, -1 unknown
    int casts(const std::string& target) const;
    bool device_ok() const { return device_ok_; }
    const std::string& unsupported_reason() const { return why_; }
    std::string describe() const;

    // canonical JSON record of line i (status OK)
    std::string record_json(const ResultView& R, int64_t i) const;
    // the reference's Parsable.addDissection(base, type, name, value) calls that
    // deliver line i's requested values (core/Parsable.java:142-193), in
    // emission order: kind 0 string (p, len), 1 null, 2 long (l)
    using EmitFn = void (*)(void* ctx, const char* base, const char* type, const char* name, int kind,
                            const uint8_t* p, uint32_t len, int64_t l);
    int emit_row(const ResultView& R, int64_t i, EmitFn fn, void* ctx) const;
    // the values Parser.store would hand the record's setters for line i:
    // (requested "TYPE:path", value) in delivery order (wildcard requests
    // by the value's full path)
    using RecFn = void (*)(void* ctx, const std::string& target, const MVal& v);
    int rec_row(const ResultView& R, int64_t i, RecFn fn, void* ctx) const;
    // where the device table finds a requested "TYPE:path" (lp_table.h), per
    // LogFormat; a query parameter's name is appended to `names` (its
    // offset / length in the source).  false: some LogFormat derives the
    // value in the host replay only
    // alt (optional): per LogFormat the earlier delivery used when out's
    // delivers no value (TC_NONE: none)
    bool table_src(const std::string& path, TableSrc out[MAX_FMT], std::string& names, TableSrc* alt = nullptr) const;

private:
    int build_dissectors(const std::string& logformats, std::string& err);
    void find_useful(const std::set<std::string>& possible, const std::string& type, const std::string& name,
                     bool is_root);
    void compile_program();
    int casts_of(const Dissector& d, const std::string& otype, const std::string& in_name, const std::string& cf) const;

    // replay
    struct Ctx;
    void replay(Ctx& c) const;
    // dv: the value further dissectors read (default v)
    void emit(Ctx& c, const std::string& base, const std::string& type, const std::string& name, const MVal& v,
              const MVal* dv = nullptr, bool recursion = false) const;
    void run_phase(Ctx& c, const Instance& in, const std::string& name, const MVal& v) const;
    void emit_pairs(Ctx& c, const Instance& in, const std::string& name, const char* type, int j) const;

    std::vector<std::unique_ptr<Format>> formats_;
    std::vector<std::unique_ptr<Dissector>> dis_;
    std::string root_type_ = "HTTPLOGLINE";
    std::set<std::string> needed_, useful_, located_;
    std::map<std::string, std::set<std::string>> remaps_;  // Parser.typeRemappings: input path -> new types
    std::map<std::string, int> casts_;  // castsOfTargets
    uint64_t gen_ = 0;                  // this build's id (the replay's per-thread memo)
    std::map<std::string, std::vector<Instance>> compiled_;
    Program prog_{};
    bool device_ok_ = true;
    std::string why_;
    // device stage bookkeeping for the replay
    std::map<int, int> tok_slot_;          // format * 256 + token index -> slot
    // stage maps keyed by format * 64 + slot (token stages) or stage index
    std::map<int, int> time_of_tok_, fl_of_tok_, uri_of_tok_;
    std::map<int, int> secms_of_tok_, list_of_tok_, binip_of_tok_;  // SECOND_MILLIS / upstream list / BinaryIP stages
    std::map<int, int> pair_of_tok_;       // cookie / raw query string stages
    std::map<std::string, int> tpair_[MAX_FMT];  // device table: "TYPE:<token path>" -> pair stage
    std::map<int, int> uri_of_fl_;
    std::map<int, int> query_of_uri_;
    std::map<int, int> uri_of_qp_;         // query stage * MAX_QNAMES + name index -> derived URI stage
    std::map<std::string, int> qname_of_;  // "query stage:name" -> name index (remapped parameters)
    // device table sources per LogFormat (compile_program): exact paths, the
    // query stages by the name of their query string, and what only the
    // replay derives (exact paths, and names below which it derives values)
    std::map<std::string, TableSrc> tsrc_[MAX_FMT];
    std::map<std::string, int> tqp_[MAX_FMT];
    std::map<std::string, TableSrc> talt_[MAX_FMT];  // the earlier delivery of a path two sources deliver
    std::set<std::string> thost_exact_[MAX_FMT], thost_prefix_[MAX_FMT];
    // replay source tracking: emission id -> (kind, stage)
    std::map<std::string, std::pair<int, int>> src_;
};

}  // namespace lp
