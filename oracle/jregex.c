/*
 * ORACLE / TEST INFRASTRUCTURE ONLY -- see jregex.h.
 *
 * Restates the subset of java.util.regex.Pattern (JDK 8) used by the
 * reference: TokenFormatDissector.prepareForRun builds "^" + \Q..\E literals
 * + (token regex) groups + "$" (reference:
 * httpdlog/httpdlog-parser/src/main/java/nl/basjes/parse/httpdlog/dissectors/
 * tokenformat/TokenFormatDissector.java:179-213) and the dissectors use a
 * handful of fixed patterns (HttpFirstLineDissector.java:59-63,
 * HttpUriDissector.java:123-127, Utils.java:27-30, ...).
 *
 * Compilation: pattern -> AST -> backtracking VM program (SPLIT priority =
 * Java's try-first-alternative order).  Counted repetition is unrolled.
 */
#include "jregex.h"

#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>

/* ------------------------------------------------------------------ AST */
enum { N_LIT, N_ANY, N_CLASS, N_BOL, N_EOL, N_CAT, N_ALT, N_GROUP, N_REP };

typedef struct { int lo, hi; } rng;

typedef struct node {
    int kind;
    int c;                 /* N_LIT */
    int cls;               /* N_CLASS: index */
    int group;             /* N_GROUP: capture index, -1 = non capturing */
    int min, max, greedy;  /* N_REP (max -1 = inf) */
    struct node **kids;
    int nkids, capkids;
} node;

typedef struct {
    rng *r;
    int n, cap;
    int neg;
} cclass;

enum { I_CHAR, I_ANY, I_CLASS, I_SPLIT, I_JMP, I_SAVE, I_BOL, I_EOL, I_MATCH };
typedef struct { int op, a, b; } instr;

struct jre {
    instr *prog;
    int nprog, capprog;
    cclass *cls;
    int ncls, capcls;
    int ngroups;
};

typedef struct {
    const int *p;   /* pattern code points */
    int n, i;
    int ngroups;
    jre *re;
    char *err;
    int errlen;
    int failed;
} parser;

static void *xrealloc(void *p, size_t n) {
    void *q = realloc(p, n);
    if (!q) { fprintf(stderr, "jregex: out of memory\n"); abort(); }
    return q;
}

static node *mk(int kind) {
    node *n = (node *)calloc(1, sizeof(node));
    n->kind = kind;
    n->group = -1;
    return n;
}

static void addkid(node *p, node *k) {
    if (p->nkids == p->capkids) {
        p->capkids = p->capkids ? p->capkids * 2 : 4;
        p->kids = (node **)xrealloc(p->kids, sizeof(node *) * p->capkids);
    }
    p->kids[p->nkids++] = k;
}

static void freenode(node *n) {
    if (!n) return;
    for (int i = 0; i < n->nkids; i++) freenode(n->kids[i]);
    free(n->kids);
    free(n);
}

static void perr(parser *ps, const char *msg) {
    if (!ps->failed && ps->err && ps->errlen > 0)
        snprintf(ps->err, ps->errlen, "regex error at %d: %s", ps->i, msg);
    ps->failed = 1;
}

static int peek(parser *ps) { return ps->i < ps->n ? ps->p[ps->i] : -1; }
static int peekat(parser *ps, int k) { return ps->i + k < ps->n ? ps->p[ps->i + k] : -1; }

static int newclass(jre *re) {
    if (re->ncls == re->capcls) {
        re->capcls = re->capcls ? re->capcls * 2 : 8;
        re->cls = (cclass *)xrealloc(re->cls, sizeof(cclass) * re->capcls);
    }
    memset(&re->cls[re->ncls], 0, sizeof(cclass));
    return re->ncls++;
}

static void addrange(cclass *c, int lo, int hi) {
    if (c->n == c->cap) {
        c->cap = c->cap ? c->cap * 2 : 8;
        c->r = (rng *)xrealloc(c->r, sizeof(rng) * c->cap);
    }
    c->r[c->n].lo = lo;
    c->r[c->n].hi = hi;
    c->n++;
}

static void add_space(cclass *c) { /* \s = [ \t\n\x0B\f\r] */
    addrange(c, ' ', ' ');
    addrange(c, '\t', '\r'); /* 09 0A 0B 0C 0D */
}
static void add_digit(cclass *c) { addrange(c, '0', '9'); }
static void add_word(cclass *c) {
    addrange(c, 'a', 'z'); addrange(c, 'A', 'Z'); addrange(c, '0', '9'); addrange(c, '_', '_');
}

static int hexval(int c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

/* Parses an escape after '\'.  Returns a code point >= 0 for a single char,
 * or -2 when a predefined class was added into *cls (cls may be NULL
 * outside classes: then *clsidx receives a new class). */
static int parse_escape(parser *ps, cclass *into, int *newcls) {
    int c = peek(ps);
    if (c < 0) { perr(ps, "trailing backslash"); return -1; }
    ps->i++;
    int kind = 0; /* 1 space, 2 digit, 3 word ; negative = negated */
    switch (c) {
    case 's': kind = 1; break;
    case 'S': kind = -1; break;
    case 'd': kind = 2; break;
    case 'D': kind = -2; break;
    case 'w': kind = 3; break;
    case 'W': kind = -3; break;
    case 't': return '\t';
    case 'n': return '\n';
    case 'r': return '\r';
    case 'f': return '\f';
    case 'a': return 7;
    case 'e': return 27;
    case '0': { /* octal \0n, \0nn, \0mnn */
        int v = 0, k = 0;
        while (k < 3 && peek(ps) >= '0' && peek(ps) <= '7') { v = v * 8 + (peek(ps) - '0'); ps->i++; k++; }
        return v;
    }
    case 'x': {
        int h1 = hexval(peek(ps)), h2 = hexval(peekat(ps, 1));
        if (h1 < 0 || h2 < 0) { perr(ps, "bad \\x"); return -1; }
        ps->i += 2;
        return h1 * 16 + h2;
    }
    case 'u': {
        int v = 0;
        for (int k = 0; k < 4; k++) {
            int h = hexval(peek(ps));
            if (h < 0) { perr(ps, "bad \\u"); return -1; }
            v = v * 16 + h; ps->i++;
        }
        return v;
    }
    default:
        if ((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9')) {
            perr(ps, "unsupported escape");
            return -1;
        }
        return c; /* escaped non-alphanumeric is literal */
    }
    /* predefined class */
    cclass tmp; memset(&tmp, 0, sizeof tmp);
    cclass *dst = into;
    if (!into || kind < 0) dst = &tmp;
    int k = kind < 0 ? -kind : kind;
    if (k == 1) add_space(dst); else if (k == 2) add_digit(dst); else add_word(dst);
    if (into && kind > 0) return -2;
    if (into && kind < 0) {
        /* negated predefined class inside a class: add complement ranges */
        /* sort tmp ranges (small) */
        for (int a = 0; a < tmp.n; a++)
            for (int b = a + 1; b < tmp.n; b++)
                if (tmp.r[b].lo < tmp.r[a].lo) { rng t = tmp.r[a]; tmp.r[a] = tmp.r[b]; tmp.r[b] = t; }
        int lo = 0;
        for (int a = 0; a < tmp.n; a++) {
            if (tmp.r[a].lo > lo) addrange(into, lo, tmp.r[a].lo - 1);
            if (tmp.r[a].hi + 1 > lo) lo = tmp.r[a].hi + 1;
        }
        addrange(into, lo, 0x10FFFF);
        free(tmp.r);
        return -2;
    }
    /* outside a class */
    int ci = newclass(ps->re);
    cclass *c2 = &ps->re->cls[ci];
    for (int a = 0; a < tmp.n; a++) addrange(c2, tmp.r[a].lo, tmp.r[a].hi);
    c2->neg = kind < 0;
    free(tmp.r);
    *newcls = ci;
    return -2;
}

/* '[' already consumed */
static node *parse_class(parser *ps) {
    int ci = newclass(ps->re);
    if (peek(ps) == '^') { ps->re->cls[ci].neg = 1; ps->i++; }
    int items = 0;
    for (;;) {
        int c = peek(ps);
        if (c < 0) { perr(ps, "unclosed class"); return NULL; }
        if (c == ']' && items > 0) { ps->i++; break; }
        int lo;
        if (c == '\\') {
            ps->i++;
            lo = parse_escape(ps, &ps->re->cls[ci], NULL);
            if (ps->failed) return NULL;
            if (lo == -2) { items++; continue; }
        } else {
            if (c == '[') { perr(ps, "nested class unsupported"); return NULL; }
            if (c == '&' && peekat(ps, 1) == '&') { perr(ps, "class intersection unsupported"); return NULL; }
            lo = c;
            ps->i++;
        }
        /* possible range */
        if (peek(ps) == '-' && peekat(ps, 1) != ']' && peekat(ps, 1) != '[' && peekat(ps, 1) >= 0) {
            ps->i++; /* '-' */
            int hi;
            if (peek(ps) == '\\') {
                ps->i++;
                hi = parse_escape(ps, NULL, NULL);
                if (ps->failed) return NULL;
                if (hi < 0) { perr(ps, "bad range end"); return NULL; }
            } else {
                hi = peek(ps);
                ps->i++;
            }
            if (hi < lo) { perr(ps, "illegal range"); return NULL; }
            addrange(&ps->re->cls[ci], lo, hi);
        } else {
            addrange(&ps->re->cls[ci], lo, lo);
        }
        items++;
    }
    node *n = mk(N_CLASS);
    n->cls = ci;
    return n;
}

static node *parse_alt(parser *ps);

static int parse_int(parser *ps, int *out) {
    int v = 0, k = 0;
    while (peek(ps) >= '0' && peek(ps) <= '9') { v = v * 10 + (peek(ps) - '0'); ps->i++; k++; }
    *out = v;
    return k;
}

static node *parse_atom(parser *ps, node *cat) {
    int c = peek(ps);
    if (c == '(') {
        ps->i++;
        int grp = -1;
        if (peek(ps) == '?') {
            if (peekat(ps, 1) == ':') ps->i += 2;
            else { perr(ps, "unsupported group construct"); return NULL; }
        } else {
            grp = ++ps->ngroups;
        }
        node *inner = parse_alt(ps);
        if (ps->failed) { freenode(inner); return NULL; }
        if (peek(ps) != ')') { perr(ps, "missing )"); freenode(inner); return NULL; }
        ps->i++;
        node *g = mk(N_GROUP);
        g->group = grp;
        addkid(g, inner);
        return g;
    }
    if (c == '[') { ps->i++; return parse_class(ps); }
    if (c == '.') { ps->i++; return mk(N_ANY); }
    if (c == '^') { ps->i++; return mk(N_BOL); }
    if (c == '$') { ps->i++; return mk(N_EOL); }
    if (c == '\\') {
        if (peekat(ps, 1) == 'Q') {
            /* \Q ... \E : literal run appended directly to cat */
            ps->i += 2;
            node *last = NULL;
            while (ps->i < ps->n) {
                if (peek(ps) == '\\' && peekat(ps, 1) == 'E') { ps->i += 2; break; }
                node *l = mk(N_LIT);
                l->c = peek(ps);
                ps->i++;
                if (last) addkid(cat, last);
                last = l;
            }
            if (!last) return mk(N_CAT); /* empty */
            return last; /* quantifier (if any) binds to the last char, as in Java */
        }
        ps->i++;
        int ci = -1;
        int v = parse_escape(ps, NULL, &ci);
        if (ps->failed) return NULL;
        if (v == -2) { node *n = mk(N_CLASS); n->cls = ci; return n; }
        node *l = mk(N_LIT);
        l->c = v;
        return l;
    }
    if (c == '*' || c == '+' || c == '?') { perr(ps, "dangling quantifier"); return NULL; }
    if (c == '{') { perr(ps, "dangling {"); return NULL; }
    ps->i++;
    node *l = mk(N_LIT);
    l->c = c;
    return l;
}

static node *parse_concat(parser *ps) {
    node *cat = mk(N_CAT);
    for (;;) {
        int c = peek(ps);
        if (c < 0 || c == '|' || c == ')') break;
        node *a = parse_atom(ps, cat);
        if (ps->failed) { freenode(a); freenode(cat); return NULL; }
        /* quantifiers */
        for (;;) {
            int q = peek(ps);
            int mn, mx;
            if (q == '*') { mn = 0; mx = -1; ps->i++; }
            else if (q == '+') { mn = 1; mx = -1; ps->i++; }
            else if (q == '?') { mn = 0; mx = 1; ps->i++; }
            else if (q == '{' && peekat(ps, 1) >= '0' && peekat(ps, 1) <= '9') {
                ps->i++;
                parse_int(ps, &mn);
                if (peek(ps) == ',') {
                    ps->i++;
                    if (peek(ps) == '}') mx = -1;
                    else parse_int(ps, &mx);
                } else mx = mn;
                if (peek(ps) != '}') { perr(ps, "bad {n,m}"); freenode(a); freenode(cat); return NULL; }
                ps->i++;
            } else break;
            int greedy = 1;
            if (peek(ps) == '?') { greedy = 0; ps->i++; }
            else if (peek(ps) == '+') { perr(ps, "possessive unsupported"); freenode(a); freenode(cat); return NULL; }
            node *r = mk(N_REP);
            r->min = mn; r->max = mx; r->greedy = greedy;
            addkid(r, a);
            a = r;
        }
        addkid(cat, a);
    }
    return cat;
}

static node *parse_alt(parser *ps) {
    node *first = parse_concat(ps);
    if (ps->failed) return first;
    if (peek(ps) != '|') return first;
    node *alt = mk(N_ALT);
    addkid(alt, first);
    while (peek(ps) == '|') {
        ps->i++;
        node *n = parse_concat(ps);
        if (ps->failed) { freenode(n); return alt; }
        addkid(alt, n);
    }
    return alt;
}

/* --------------------------------------------------------------- codegen */
static int emit(jre *re, int op, int a, int b) {
    if (re->nprog == re->capprog) {
        re->capprog = re->capprog ? re->capprog * 2 : 64;
        re->prog = (instr *)xrealloc(re->prog, sizeof(instr) * re->capprog);
    }
    re->prog[re->nprog].op = op;
    re->prog[re->nprog].a = a;
    re->prog[re->nprog].b = b;
    return re->nprog++;
}

static void gen(jre *re, node *n) {
    switch (n->kind) {
    case N_LIT: emit(re, I_CHAR, n->c, 0); break;
    case N_ANY: emit(re, I_ANY, 0, 0); break;
    case N_CLASS: emit(re, I_CLASS, n->cls, 0); break;
    case N_BOL: emit(re, I_BOL, 0, 0); break;
    case N_EOL: emit(re, I_EOL, 0, 0); break;
    case N_CAT: for (int i = 0; i < n->nkids; i++) gen(re, n->kids[i]); break;
    case N_GROUP:
        if (n->group >= 0) emit(re, I_SAVE, 2 * n->group, 0);
        gen(re, n->kids[0]);
        if (n->group >= 0) emit(re, I_SAVE, 2 * n->group + 1, 0);
        break;
    case N_ALT: {
        int *jmps = (int *)malloc(sizeof(int) * n->nkids);
        for (int i = 0; i < n->nkids; i++) {
            if (i < n->nkids - 1) {
                int sp = emit(re, I_SPLIT, 0, 0);
                re->prog[sp].a = re->nprog;
                gen(re, n->kids[i]);
                jmps[i] = emit(re, I_JMP, 0, 0);
                re->prog[sp].b = re->nprog;
            } else {
                gen(re, n->kids[i]);
                jmps[i] = -1;
            }
        }
        for (int i = 0; i < n->nkids; i++)
            if (jmps[i] >= 0) re->prog[jmps[i]].a = re->nprog;
        free(jmps);
        break;
    }
    case N_REP: {
        node *k = n->kids[0];
        for (int i = 0; i < n->min; i++) gen(re, k);
        if (n->max < 0) {
            int loop = emit(re, I_SPLIT, 0, 0);
            int body = re->nprog;
            gen(re, k);
            emit(re, I_JMP, loop, 0);
            int out = re->nprog;
            if (n->greedy) { re->prog[loop].a = body; re->prog[loop].b = out; }
            else { re->prog[loop].a = out; re->prog[loop].b = body; }
        } else {
            int opt = n->max - n->min;
            int *splits = (int *)malloc(sizeof(int) * (opt > 0 ? opt : 1));
            for (int i = 0; i < opt; i++) {
                splits[i] = emit(re, I_SPLIT, 0, 0);
                int body = re->nprog;
                gen(re, k);
                if (n->greedy) re->prog[splits[i]].a = body;
                else re->prog[splits[i]].b = body;
            }
            int out = re->nprog;
            for (int i = 0; i < opt; i++) {
                if (n->greedy) re->prog[splits[i]].b = out;
                else re->prog[splits[i]].a = out;
            }
            free(splits);
        }
        break;
    }
    }
}

/* UTF-8 -> code points */
static int *utf8_to_cp(const char *s, int *outn) {
    int len = (int)strlen(s);
    int *cp = (int *)malloc(sizeof(int) * (len + 1));
    int n = 0;
    const unsigned char *u = (const unsigned char *)s;
    for (int i = 0; i < len;) {
        unsigned c = u[i];
        if (c < 0x80) { cp[n++] = c; i++; }
        else if ((c >> 5) == 6 && i + 1 < len) { cp[n++] = ((c & 0x1F) << 6) | (u[i + 1] & 0x3F); i += 2; }
        else if ((c >> 4) == 14 && i + 2 < len) { cp[n++] = ((c & 0x0F) << 12) | ((u[i + 1] & 0x3F) << 6) | (u[i + 2] & 0x3F); i += 3; }
        else if ((c >> 3) == 30 && i + 3 < len) { cp[n++] = ((c & 0x07) << 18) | ((u[i + 1] & 0x3F) << 12) | ((u[i + 2] & 0x3F) << 6) | (u[i + 3] & 0x3F); i += 4; }
        else { cp[n++] = 0xFFFD; i++; }
    }
    *outn = n;
    return cp;
}

jre *jre_compile(const char *pattern, char *err, int errlen) {
    jre *re = (jre *)calloc(1, sizeof(jre));
    parser ps;
    memset(&ps, 0, sizeof ps);
    ps.p = utf8_to_cp(pattern, &ps.n);
    ps.re = re;
    ps.err = err;
    ps.errlen = errlen;
    node *root = parse_alt(&ps);
    if (!ps.failed && ps.i != ps.n) perr(&ps, "unbalanced )");
    if (ps.failed) {
        freenode(root);
        free((void *)ps.p);
        jre_free(re);
        return NULL;
    }
    re->ngroups = ps.ngroups;
    emit(re, I_SAVE, 0, 0);
    gen(re, root);
    emit(re, I_SAVE, 1, 0);
    emit(re, I_MATCH, 0, 0);
    freenode(root);
    free((void *)ps.p);
    return re;
}

void jre_free(jre *re) {
    if (!re) return;
    for (int i = 0; i < re->ncls; i++) free(re->cls[i].r);
    free(re->cls);
    free(re->prog);
    free(re);
}

int jre_ngroups(const jre *re) { return re->ngroups; }

/* -------------------------------------------------------------- execute */
static int class_match(const cclass *c, int ch) {
    int in = 0;
    for (int i = 0; i < c->n; i++)
        if (ch >= c->r[i].lo && ch <= c->r[i].hi) { in = 1; break; }
    return c->neg ? !in : in;
}

static int is_dot(int ch) { /* Pattern.Dot */
    return ch != '\n' && ch != '\r' && (ch | 1) != 0x2029 && ch != 0x85;
}

static int eol_match(const int *t, int n, int i) { /* Pattern.Dollar, !multiline */
    if (i < n - 2) return 0;
    if (i == n - 2) return t[i] == '\r' && t[i + 1] == '\n';
    if (i < n) {
        int ch = t[i];
        if (ch == '\n') { if (i > 0 && t[i - 1] == '\r') return 0; }
        else if (ch == '\r' || ch == 0x85 || (ch | 1) == 0x2029) {}
        else return 0;
    }
    return 1;
}

typedef struct { int kind, pc, pos; } frame; /* kind 0 branch, 1 restore cap (pc=index,pos=old) */

typedef struct {
    uint64_t *visited;
    size_t vwords;
    frame *stk;
    int cap;
} scratch;

static __thread scratch tls;

static int run(const jre *re, const int *t, int n, int start, int *caps, int full) {
    int ncap = 2 * (re->ngroups + 1);
    int sp = 0;
#define PUSH(k_, a_, b_) do { \
        if (sp == tls.cap) { tls.cap = tls.cap ? tls.cap * 2 : 1024; tls.stk = (frame *)xrealloc(tls.stk, sizeof(frame) * tls.cap); } \
        tls.stk[sp].kind = (k_); tls.stk[sp].pc = (a_); tls.stk[sp].pos = (b_); sp++; } while (0)
    PUSH(0, 0, start);
    const size_t stride = (size_t)n + 1;
    while (sp > 0) {
        frame f = tls.stk[--sp];
        if (f.kind == 1) { caps[f.pc] = f.pos; continue; }
        int pc = f.pc, pos = f.pos;
        for (;;) {
            size_t bit = (size_t)pc * stride + (size_t)pos;
            uint64_t m = 1ull << (bit & 63);
            if (tls.visited[bit >> 6] & m) break;
            tls.visited[bit >> 6] |= m;
            const instr *in = &re->prog[pc];
            int ok = 1;
            switch (in->op) {
            case I_CHAR: if (pos < n && t[pos] == in->a) { pc++; pos++; } else ok = 0; break;
            case I_ANY: if (pos < n && is_dot(t[pos])) { pc++; pos++; } else ok = 0; break;
            case I_CLASS: if (pos < n && class_match(&re->cls[in->a], t[pos])) { pc++; pos++; } else ok = 0; break;
            case I_BOL: if (pos == 0) pc++; else ok = 0; break;
            case I_EOL: if (eol_match(t, n, pos)) pc++; else ok = 0; break;
            case I_JMP: pc = in->a; break;
            case I_SPLIT: PUSH(0, in->b, pos); pc = in->a; break;
            case I_SAVE: PUSH(1, in->a, caps[in->a]); caps[in->a] = pos; pc++; break;
            case I_MATCH: (void)ncap; if (!full || pos == n) return 1; ok = 0; break;
            }
            if (!ok) break;
        }
    }
#undef PUSH
    return 0;
}

static void prep(const jre *re, int n) {
    size_t bits = (size_t)re->nprog * ((size_t)n + 1);
    size_t words = (bits + 63) / 64;
    if (words > tls.vwords) {
        free(tls.visited);
        tls.visited = (uint64_t *)malloc(words * 8);
        tls.vwords = words;
    }
    memset(tls.visited, 0, words * 8);
}

int jre_find(const jre *re, const int *text, int n, int from, int *caps) {
    int ncap = 2 * (re->ngroups + 1);
    prep(re, n);
    for (int s = from; s <= n; s++) {
        for (int i = 0; i < ncap; i++) caps[i] = -1;
        if (run(re, text, n, s, caps, 0)) return 1;
    }
    for (int i = 0; i < ncap; i++) caps[i] = -1;
    return 0;
}

int jre_matches(const jre *re, const int *text, int n, int *caps) {
    /* Matcher.matches(): like find at 0 but the match must end at n
     * (java.util.regex.Pattern.LastNode with ENDANCHOR). */
    int ncap = 2 * (re->ngroups + 1);
    prep(re, n);
    for (int i = 0; i < ncap; i++) caps[i] = -1;
    if (run(re, text, n, 0, caps, 1)) return 1;
    for (int i = 0; i < ncap; i++) caps[i] = -1;
    return 0;
}
