/*
 * ORACLE / TEST INFRASTRUCTURE ONLY.
 * Java-String-like helpers for the oracle: strings are arrays of Unicode
 * code points allocated from a per-parse arena, with an explicit null flag
 * (java.lang.String null vs "").
 */
#ifndef ORACLE_OSTR_H
#define ORACLE_OSTR_H

#include <stddef.h>
#include <stdint.h>

#include "jregex.h"

typedef struct arena_blk { struct arena_blk *next; size_t used, cap; char data[]; } arena_blk;
typedef struct { arena_blk *head; } arena;

void *ar_alloc(arena *a, size_t n);
void ar_reset(arena *a);
void ar_free(arena *a);

typedef struct {
    const int *c;
    int n;
    int null; /* 1 = Java null */
} js;

js js_null(void);
js js_from_utf8(arena *a, const char *s, int len);
js js_lit(arena *a, const char *s);            /* from NUL-terminated UTF-8 */
js js_sub(js s, int from, int to);             /* substring (no copy) */
js js_cat(arena *a, js x, js y);
js js_cat3(arena *a, js x, js y, js z);
int js_eq(js x, js y);
int js_eq_lit(js x, const char *s);            /* ASCII literal compare */
int js_starts_lit(js x, const char *s);
int js_index_of_char(js s, int ch, int from);
int js_index_of(js s, js needle, int from);
js js_lower(arena *a, js s);                   /* toLowerCase() (ASCII + Latin-1 subset) */
js js_upper(arena *a, js s);
/* UTF-8 output into a malloc'd or arena buffer */
char *js_to_utf8(arena *a, js s, int *outlen);

/* regex helpers (Matcher.replaceAll / replaceFirst with $n references) */
js js_replace_all(arena *a, const jre *re, js s, const char *repl);
js js_replace_first(arena *a, const jre *re, js s, const char *repl);
/* String.replace(CharSequence, CharSequence) - literal */
js js_replace_lit(arena *a, js s, js from, js to);

/* String.split(regex) for a single literal char (Java fast path), with
 * trailing empty strings removed; limit 0.  Returns count, parts in *out. */
int js_split_char(arena *a, js s, int ch, js **out);
/* String.split(regex, limit) for a single literal char */
int js_split_char_limit(arena *a, js s, int ch, int limit, js **out);

#endif
