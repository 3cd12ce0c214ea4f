/*
 * ORACLE / TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's per-line hot path
 * (tool-recommender-bot/logparser, Java).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load liboracle.so; the product
 * (logparser_amd/, include/) never links it.
 *
 * It restates:
 *   HttpdLoglineParser.setupDissectors        HttpdLoglineParser.java:104-126
 *   Parser.assembleDissectors / parse / store core/Parser.java:237-458,716-876
 *   Parsable.addDissection (+ type remapping)  core/Parsable.java:142-193
 *   HttpdLogFormatDissector (multi-format)     HttpdLogFormatDissector.java:99-204
 *   TokenFormatDissector compile + dissect     tokenformat/TokenFormatDissector.java:127-379
 *   ApacheHttpdLogFormatDissector              ApacheHttpdLogFormatDissector.java:73-714
 *   TimeStampDissector (dd/MMM/yyyy:HH:mm:ss ZZ) dissectors/TimeStampDissector.java:404-564
 *   HttpFirstLine(Protocol)Dissector           dissectors/HttpFirstLine*.java
 *   HttpUriDissector                           dissectors/HttpUriDissector.java:130-233
 *   QueryStringFieldDissector + Utils          dissectors/QueryStringFieldDissector.java:76-108, Utils.java:38-65
 *   ConvertCLFIntoNumber / ConvertNumberIntoCLF translate/Convert*.java
 * Third-party algorithms restated from their published behaviour: JDK 8
 * java.util.regex (jregex.c), java.time SMART resolution for the pattern
 * above, java.net.URI (RFC 2396 parser), java.net.URLDecoder("UTF-16"),
 * commons-httpclient 3.1 URIUtil.encode, commons-lang3 3.8.1 unescapeHtml4
 * (basic + Latin-1 + numeric entities; other named entities -> UNSUPPORTED).
 *
 * Canonical per-line record (shared with the product's materializer):
 *   {"<TYPE:name>": [v, ...], ...}   keys sorted, values in emission order,
 *   v = "str" | null (String-valued) | {"l": n} | {"l": null} (Long-valued)
 */
#ifndef ORACLE_H
#define ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_OK = 0, ORC_BAD = 1, ORC_UNSUPPORTED = 2 };

typedef struct orc_parser orc_parser;

/* logformat: one or more formats separated by \n (HttpdLogFormatDissector
 * semantics).  fields: requested "TYPE:name" paths.  Returns NULL and fills
 * err if the setup fails (MissingDissectorsException, ...) or needs a
 * dissector this oracle does not restate ("unsupported: ..."). */
orc_parser *orc_new(const char *logformat, const char *const *fields, int nfields,
                    char *err, int errlen);
/* The same with Parser.addTypeRemapping(rm_in[k], rm_type[k]) for each k
 * (core/Parser.java:636-677, Parsable.java:160-176). */
orc_parser *orc_new_remapped(const char *logformat, const char *const *fields, int nfields,
                             const char *const *rm_in, const char *const *rm_type, int n_rm,
                             char *err, int errlen);
void orc_free(orc_parser *p);

/* Parse one line (no terminator).  Writes the canonical JSON record (NUL
 * terminated) into out when status is ORC_OK.  Returns ORC_OK / ORC_BAD
 * (DissectionFailure) / ORC_UNSUPPORTED (input outside the restated subset)
 * or -1 when out_cap is too small. */
int orc_parse(orc_parser *p, const char *line, int len, char *out, int out_cap);

/* Parser.getPossiblePaths(maxDepth) for a logformat; newline separated,
 * sorted.  Returns bytes written or -1. */
int orc_possible_paths(const char *logformat, int max_depth, char *out, int out_cap);

/* The regex TokenFormatDissector.prepareForRun would compile for format
 * index i (after orc_new).  Returns length or -1. */
int orc_format_regex(orc_parser *p, int i, char *out, int out_cap);

/* Bench helper: parse every '\n'-separated line of buf with nthreads
 * threads (one orc_parser clone per thread, as the reference requires one
 * Parser per thread).  Returns wall seconds; counts in out3[0..2] =
 * lines, ok, bad (+ unsupported in out3[3] if non-NULL array of 4). */
double orc_bench(const char *logformat, const char *const *fields, int nfields,
                 const char *buf, size_t nbytes, int nthreads, int64_t *out4);

/* Individual component restatements, exposed for unit tests. */
int orc_resilient_url_decode(const char *in, int len, char *out, int out_cap);

/* The Apache (nginx=0) or NGINX token table as canonical JSON (the form
 * tests/golden/extract_token_tables.py derives from the reference's Java
 * sources).  Returns bytes written or -1 when out_cap is too small. */
int orc_token_table(int nginx, char *out, int out_cap);

#ifdef __cplusplus
}
#endif
#endif
