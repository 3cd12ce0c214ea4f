/*
 * ORACLE / TEST INFRASTRUCTURE ONLY.
 *
 * Per-line record digests for whole-batch parity at headline scale
 * (tests/test_gpu_parity.py test_headline_parity_gpu): every line of a
 * multi-million-line batch is parsed by the oracle and replayed from the
 * engine's results, and both sides reduce each line to (status, 64-bit
 * FNV-1a of the canonical JSON record), so that the comparison needs no
 * per-line Python work.  The engine side is reached only through a function
 * pointer the test passes in (lp_result_record_json of the product's C ABI):
 * this library never links the product.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static uint64_t fnv1a(const char *s, size_t n) {
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; i++) {
        h ^= (uint8_t)s[i];
        h *= 1099511628211ull;
    }
    return h;
}

/* ---------------------------------------------------------------- oracle */
typedef struct {
    const char *logformat;
    const char *const *fields;
    int nfields;
    const char *buf;
    const int64_t *starts; /* line k = [starts[k], starts[k + 1] - 1) */
    int64_t from, to;
    int64_t warm_from; /* lines [warm_from, from) parsed first, results dropped */
    uint8_t *status;
    uint64_t *hash;
    int err;
} orc_job;

static void *orc_thread(void *arg) {
    orc_job *j = (orc_job *)arg;
    char e[256];
    orc_parser *p = orc_new(j->logformat, j->fields, j->nfields, e, sizeof e);
    if (!p) { j->err = 1; return NULL; }
    const int cap = 1 << 20;
    char *out = (char *)malloc((size_t)cap);
    /* several LogFormats: the parser's sticky active format
     * (HttpdLogFormatDissector.java:173-204) at line `from` is the one a
     * single parser over the whole buffer would hold when the warm-up lines
     * hold a line that exactly one format matches (the state after such a
     * line does not depend on the state before it) -- with mutually
     * exclusive formats, any OK line */
    int warm_ok = j->warm_from == j->from;
    for (int64_t k = j->warm_from; k < j->from; k++) {
        const int64_t a = j->starts[k], b = j->starts[k + 1] - 1;
        const int st = orc_parse(p, j->buf + a, (int)(b - a), out, cap);
        if (st < 0) { j->err = 2; break; }
        if (st == ORC_OK) warm_ok = 1;
    }
    if (!warm_ok) j->err = 4;
    for (int64_t k = j->from; k < j->to && !j->err; k++) {
        const int64_t a = j->starts[k], b = j->starts[k + 1] - 1;
        const int st = orc_parse(p, j->buf + a, (int)(b - a), out, cap);
        if (st < 0) { j->err = 2; break; }
        j->status[k] = (uint8_t)st;
        j->hash[k] = st == ORC_OK ? fnv1a(out, strlen(out)) : 0;
    }
    free(out);
    orc_free(p);
    return NULL;
}

/* Every '\n'-terminated line of buf: status (ORC_*) and the record digest
 * per line.  One LogFormat: one fresh parser per thread is the reference's
 * own per-thread Parser (warmup 0).  Several LogFormats (sticky active
 * format): each thread's parser first runs over the `warmup` lines before
 * its range, which must hold an OK line (see orc_thread; formats that are
 * mutually exclusive).  Returns the line count, -1 when more than
 * max_lines, -2 on a parser error, -4 when a warm-up held no OK line. */
int64_t orc_digest_lines_w(const char *logformat, const char *const *fields, int nfields, const char *buf,
                           size_t nbytes, int nthreads, int64_t max_lines, int64_t warmup, uint8_t *status,
                           uint64_t *hash) {
    int64_t n = 0;
    for (const char *q = buf; (q = (const char *)memchr(q, '\n', nbytes - (size_t)(q - buf))) != NULL; q++) n++;
    if (n > max_lines) return -1;
    int64_t *starts = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n + 1));
    int64_t k = 0;
    starts[0] = 0;
    for (size_t i = 0; i < nbytes; i++)
        if (buf[i] == '\n') starts[++k] = (int64_t)i + 1;
    if (nthreads < 1) nthreads = 1;
    orc_job *jobs = (orc_job *)calloc((size_t)nthreads, sizeof(orc_job));
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)nthreads);
    for (int t = 0; t < nthreads; t++) {
        const int64_t from = n * t / nthreads;
        jobs[t] = (orc_job){logformat, fields, nfields, buf, starts, from, n * (t + 1) / nthreads,
                            from > warmup ? from - warmup : 0, status, hash, 0};
        pthread_create(&th[t], NULL, orc_thread, &jobs[t]);
    }
    int err = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        err |= jobs[t].err;
    }
    free(jobs);
    free(th);
    free(starts);
    return err ? (err & 4 ? -4 : -2) : n;
}

int64_t orc_digest_lines(const char *logformat, const char *const *fields, int nfields, const char *buf,
                         size_t nbytes, int nthreads, int64_t max_lines, uint8_t *status, uint64_t *hash) {
    return orc_digest_lines_w(logformat, fields, nfields, buf, nbytes, nthreads, max_lines, 0, status, hash);
}

/* ---------------------------------------------------------------- engine */
/* int64_t lp_result_record_json(lp_handle*, const lp_result*, int64_t, char*, size_t) */
typedef int64_t (*record_json_fn)(void *h, const void *r, int64_t i, char *out, size_t cap);

typedef struct {
    record_json_fn fn;
    void *h;
    const void *r;
    const uint8_t *status;
    int64_t from, to;
    uint64_t *hash;
    int err;
} eng_job;

static void *eng_thread(void *arg) {
    eng_job *j = (eng_job *)arg;
    size_t cap = 1 << 20;
    char *out = (char *)malloc(cap);
    for (int64_t k = j->from; k < j->to; k++) {
        j->hash[k] = 0;
        if (j->status[k] != 0) continue;
        const int64_t n = j->fn(j->h, j->r, k, out, cap);
        if (n < 0) { j->err = 1; break; }
        j->hash[k] = fnv1a(out, (size_t)n);
    }
    free(out);
    return NULL;
}

/* The engine's records of lines [0, n) of a host result (lp_result_copy),
 * digested on nthreads threads; lines whose status is not OK get 0.
 * Returns 0, or -1 when a record could not be built. */
int dg_engine(record_json_fn fn, void *h, const void *r, const uint8_t *status, int64_t n, int nthreads,
              uint64_t *hash) {
    if (nthreads < 1) nthreads = 1;
    eng_job *jobs = (eng_job *)calloc((size_t)nthreads, sizeof(eng_job));
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)nthreads);
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (eng_job){fn, h, r, status, n * t / nthreads, n * (t + 1) / nthreads, hash, 0};
        pthread_create(&th[t], NULL, eng_thread, &jobs[t]);
    }
    int err = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        err |= jobs[t].err;
    }
    free(jobs);
    free(th);
    return err ? -1 : 0;
}
