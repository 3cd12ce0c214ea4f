/*
 * ORACLE / TEST INFRASTRUCTURE ONLY -- see ostr.h.
 */
#include "ostr.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void *ar_alloc(arena *a, size_t n) {
    n = (n + 15) & ~(size_t)15;
    arena_blk *b = a->head;
    if (!b || b->used + n > b->cap) {
        size_t cap = n > (1u << 16) ? n : (1u << 16);
        arena_blk *nb = (arena_blk *)malloc(sizeof(arena_blk) + cap);
        if (!nb) { fprintf(stderr, "oracle arena: out of memory\n"); abort(); }
        nb->next = b;
        nb->used = 0;
        nb->cap = cap;
        a->head = nb;
        b = nb;
    }
    void *p = b->data + b->used;
    b->used += n;
    return p;
}

void ar_reset(arena *a) {
    /* keep the newest block, free the rest */
    arena_blk *b = a->head;
    if (!b) return;
    arena_blk *r = b->next;
    while (r) { arena_blk *nx = r->next; free(r); r = nx; }
    b->next = NULL;
    b->used = 0;
}

void ar_free(arena *a) {
    arena_blk *b = a->head;
    while (b) { arena_blk *nx = b->next; free(b); b = nx; }
    a->head = NULL;
}

js js_null(void) { js r = {NULL, 0, 1}; return r; }

js js_from_utf8(arena *a, const char *s, int len) {
    int *cp = (int *)ar_alloc(a, sizeof(int) * (size_t)(len + 1));
    int n = 0;
    const unsigned char *u = (const unsigned char *)s;
    for (int i = 0; i < len;) {
        unsigned c = u[i];
        if (c < 0x80) { cp[n++] = (int)c; i++; }
        else if ((c >> 5) == 6 && i + 1 < len && (u[i + 1] & 0xC0) == 0x80) {
            cp[n++] = (int)(((c & 0x1F) << 6) | (u[i + 1] & 0x3F)); i += 2;
        } else if ((c >> 4) == 14 && i + 2 < len && (u[i + 1] & 0xC0) == 0x80 && (u[i + 2] & 0xC0) == 0x80) {
            cp[n++] = (int)(((c & 0x0F) << 12) | ((u[i + 1] & 0x3F) << 6) | (u[i + 2] & 0x3F)); i += 3;
        } else if ((c >> 3) == 30 && i + 3 < len && (u[i + 1] & 0xC0) == 0x80 && (u[i + 2] & 0xC0) == 0x80 && (u[i + 3] & 0xC0) == 0x80) {
            cp[n++] = (int)(((c & 0x07) << 18) | ((u[i + 1] & 0x3F) << 12) | ((u[i + 2] & 0x3F) << 6) | (u[i + 3] & 0x3F)); i += 4;
        } else { cp[n++] = 0xFFFD; i++; }
    }
    js r = {cp, n, 0};
    return r;
}

js js_lit(arena *a, const char *s) { return js_from_utf8(a, s, (int)strlen(s)); }

js js_sub(js s, int from, int to) {
    js r = {s.c + from, to - from, 0};
    return r;
}

js js_cat(arena *a, js x, js y) {
    int *cp = (int *)ar_alloc(a, sizeof(int) * (size_t)(x.n + y.n + 1));
    if (x.n) memcpy(cp, x.c, sizeof(int) * (size_t)x.n);
    if (y.n) memcpy(cp + x.n, y.c, sizeof(int) * (size_t)y.n);
    js r = {cp, x.n + y.n, 0};
    return r;
}

js js_cat3(arena *a, js x, js y, js z) { return js_cat(a, js_cat(a, x, y), z); }

int js_eq(js x, js y) {
    if (x.null || y.null) return x.null && y.null;
    return x.n == y.n && (x.n == 0 || memcmp(x.c, y.c, sizeof(int) * (size_t)x.n) == 0);
}

int js_eq_lit(js x, const char *s) {
    if (x.null) return 0;
    int n = (int)strlen(s);
    if (n != x.n) return 0;
    for (int i = 0; i < n; i++) if (x.c[i] != (unsigned char)s[i]) return 0;
    return 1;
}

int js_starts_lit(js x, const char *s) {
    if (x.null) return 0;
    int n = (int)strlen(s);
    if (n > x.n) return 0;
    for (int i = 0; i < n; i++) if (x.c[i] != (unsigned char)s[i]) return 0;
    return 1;
}

int js_index_of_char(js s, int ch, int from) {
    for (int i = from < 0 ? 0 : from; i < s.n; i++) if (s.c[i] == ch) return i;
    return -1;
}

int js_index_of(js s, js nd, int from) {
    if (from < 0) from = 0;
    if (nd.n == 0) return from <= s.n ? from : -1;
    for (int i = from; i + nd.n <= s.n; i++)
        if (memcmp(s.c + i, nd.c, sizeof(int) * (size_t)nd.n) == 0) return i;
    return -1;
}

/* Character.toLowerCase for the code points that occur in log data; the
 * oracle restricts itself to Latin-1 (other code points unchanged, which is
 * also what the JDK does for most scripts without case). */
static int lc(int c) {
    if (c >= 'A' && c <= 'Z') return c + 32;
    if (c >= 0xC0 && c <= 0xDE && c != 0xD7) return c + 32;
    return c;
}
static int uc(int c) {
    if (c >= 'a' && c <= 'z') return c - 32;
    if (c >= 0xE0 && c <= 0xFE && c != 0xF7) return c - 32;
    return c;
}

js js_lower(arena *a, js s) {
    if (s.null) return s;
    int *cp = (int *)ar_alloc(a, sizeof(int) * (size_t)(s.n + 1));
    for (int i = 0; i < s.n; i++) cp[i] = lc(s.c[i]);
    js r = {cp, s.n, 0};
    return r;
}

js js_upper(arena *a, js s) {
    if (s.null) return s;
    int *cp = (int *)ar_alloc(a, sizeof(int) * (size_t)(s.n + 1));
    for (int i = 0; i < s.n; i++) cp[i] = uc(s.c[i]);
    js r = {cp, s.n, 0};
    return r;
}

char *js_to_utf8(arena *a, js s, int *outlen) {
    char *o = (char *)ar_alloc(a, (size_t)s.n * 4 + 1);
    int k = 0;
    for (int i = 0; i < s.n; i++) {
        unsigned c = (unsigned)s.c[i];
        if (c < 0x80) o[k++] = (char)c;
        else if (c < 0x800) { o[k++] = (char)(0xC0 | (c >> 6)); o[k++] = (char)(0x80 | (c & 0x3F)); }
        else if (c < 0x10000) { o[k++] = (char)(0xE0 | (c >> 12)); o[k++] = (char)(0x80 | ((c >> 6) & 0x3F)); o[k++] = (char)(0x80 | (c & 0x3F)); }
        else { o[k++] = (char)(0xF0 | (c >> 18)); o[k++] = (char)(0x80 | ((c >> 12) & 0x3F)); o[k++] = (char)(0x80 | ((c >> 6) & 0x3F)); o[k++] = (char)(0x80 | (c & 0x3F)); }
    }
    o[k] = 0;
    if (outlen) *outlen = k;
    return o;
}

/* ---- growable code point buffer */
typedef struct { int *c; int n, cap; } buf;
static void bput(buf *b, int ch) {
    if (b->n == b->cap) { b->cap = b->cap ? b->cap * 2 : 64; b->c = (int *)realloc(b->c, sizeof(int) * (size_t)b->cap); }
    b->c[b->n++] = ch;
}
static js bfinish(arena *a, buf *b) {
    int *cp = (int *)ar_alloc(a, sizeof(int) * (size_t)(b->n + 1));
    if (b->n) memcpy(cp, b->c, sizeof(int) * (size_t)b->n);
    js r = {cp, b->n, 0};
    free(b->c);
    return r;
}

/* Matcher.appendReplacement replacement-string processing: $n and \x */
static void append_repl(buf *b, const char *repl, const int *t, const int *caps, int ng) {
    const unsigned char *r = (const unsigned char *)repl;
    for (int i = 0; r[i];) {
        if (r[i] == '\\' && r[i + 1]) { bput(b, r[i + 1]); i += 2; continue; }
        if (r[i] == '$' && r[i + 1] >= '0' && r[i + 1] <= '9') {
            int g = r[i + 1] - '0';
            i += 2;
            /* Java takes more digits while the group number stays valid */
            while (r[i] >= '0' && r[i] <= '9' && g * 10 + (r[i] - '0') <= ng) { g = g * 10 + (r[i] - '0'); i++; }
            if (caps[2 * g] >= 0)
                for (int k = caps[2 * g]; k < caps[2 * g + 1]; k++) bput(b, t[k]);
            continue;
        }
        bput(b, r[i]);
        i++;
    }
}

static js replace_impl(arena *a, const jre *re, js s, const char *repl, int all) {
    int ng = jre_ngroups(re);
    int caps[2 * 64];
    buf b = {0};
    int from = 0, last = 0;
    int found = 0;
    while (from <= s.n && jre_find(re, s.c, s.n, from, caps)) {
        found = 1;
        for (int k = last; k < caps[0]; k++) bput(&b, s.c[k]);
        append_repl(&b, repl, s.c, caps, ng);
        last = caps[1];
        /* Matcher.find after an empty match advances by one */
        from = caps[1] == caps[0] ? caps[1] + 1 : caps[1];
        if (!all) break;
    }
    if (!found) { free(b.c); return s; }
    for (int k = last; k < s.n; k++) bput(&b, s.c[k]);
    return bfinish(a, &b);
}

js js_replace_all(arena *a, const jre *re, js s, const char *repl) { return replace_impl(a, re, s, repl, 1); }
js js_replace_first(arena *a, const jre *re, js s, const char *repl) { return replace_impl(a, re, s, repl, 0); }

js js_replace_lit(arena *a, js s, js from, js to) {
    buf b = {0};
    int i = 0, found = 0;
    if (from.n == 0) return s;
    while (i < s.n) {
        if (i + from.n <= s.n && memcmp(s.c + i, from.c, sizeof(int) * (size_t)from.n) == 0) {
            for (int k = 0; k < to.n; k++) bput(&b, to.c[k]);
            i += from.n;
            found = 1;
        } else bput(&b, s.c[i++]);
    }
    if (!found) { free(b.c); return s; }
    return bfinish(a, &b);
}

int js_split_char_limit(arena *a, js s, int ch, int limit, js **out) {
    /* String.split: limit > 0 -> at most limit parts, trailing kept;
     * limit == 0 -> trailing empty strings removed.  A zero-length input
     * gives [""] ; (Java 8: leading empty string kept). */
    int cnt = 1;
    for (int i = 0; i < s.n; i++) if (s.c[i] == ch) cnt++;
    js *parts = (js *)ar_alloc(a, sizeof(js) * (size_t)cnt);
    int np = 0, start = 0;
    for (int i = 0; i < s.n; i++) {
        if (s.c[i] == ch && (limit <= 0 || np < limit - 1)) {
            parts[np++] = js_sub(s, start, i);
            start = i + 1;
        }
    }
    if (np == 0) { parts[0] = s; *out = parts; return 1; }
    parts[np++] = js_sub(s, start, s.n);
    if (limit == 0) while (np > 0 && parts[np - 1].n == 0) np--;
    *out = parts;
    return np;
}

int js_split_char(arena *a, js s, int ch, js **out) { return js_split_char_limit(a, s, ch, 0, out); }
