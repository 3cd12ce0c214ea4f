/*
 * ORACLE / TEST INFRASTRUCTURE ONLY.  Never linked into the product
 * (logparser_amd/); only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.
 *
 * jregex: a small backtracking regular-expression engine that restates the
 * java.util.regex (JDK 8) semantics the reference relies on:
 *   - leftmost-first (priority) backtracking, greedy / lazy quantifiers,
 *     alternation tried left to right (java.util.regex.Pattern Branch/Curly);
 *   - '.' excludes \n \r U+0085 U+2028 U+2029 (Pattern.Dot);
 *   - '$' without MULTILINE also matches before a final line terminator
 *     (Pattern.Dollar);  '^' only at input start (Pattern.Begin);
 *   - \s = [ \t\n\x0B\f\r];  \Q..\E quoting (Pattern.quote output);
 *   - Java character-class parsing quirks ("[a-zA-Z-_]", "[\+|\-]").
 * Texts are arrays of Unicode code points.
 * A (pc,pos) visited bitmap makes the search polynomial without changing
 * which match is found (no back-references are supported).
 */
#ifndef ORACLE_JREGEX_H
#define ORACLE_JREGEX_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct jre jre;

/* pattern is UTF-8.  Returns NULL on syntax error (err filled). */
jre *jre_compile(const char *pattern, char *err, int errlen);
void jre_free(jre *re);
int jre_ngroups(const jre *re);

/* Matcher.find() starting the scan at 'from'.  caps must hold
 * 2*(ngroups+1) ints; unset groups are -1.  Returns 1 on match. */
int jre_find(const jre *re, const int *text, int n, int from, int *caps);

/* Matcher.matches(): whole input. */
int jre_matches(const jre *re, const int *text, int n, int *caps);

#ifdef __cplusplus
}
#endif
#endif
