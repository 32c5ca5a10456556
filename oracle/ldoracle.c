/* ldoracle.c -- C restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Used by tests/ (parity at sizes the Python oracle is too slow for) and by
 * bench.py's cpu_baseline leg (kind "port").  Never linked into libldgpu.so.
 *
 * Follows, rule by rule (same rules as oracle/ldoracle.py):
 *   ldo_score  -- LanguageDetectorModel.detect(Array[Byte], ...)
 *                 LanguageDetectorModel.scala:131-156: for n in gramLengths (order,
 *                 duplicates repeat), for every window of the Scala sliding(n)
 *                 (partial rule: 0<len<n -> one window = whole text), a map hit does
 *                 s[l] = s[l] + row[l] (F2J daxpy, a = 1.0), then breeze argmax
 *                 (first max, strict >).
 *   ldo_count  -- computeGrams + reduceGrams, LanguageDetector.scala:25-66: per doc,
 *                 per n, every window counted; summed per (lang, gram).  Raw int64
 *                 sums are exported; the JVM Int wrap is applied by the caller.
 *
 * Keys are arbitrary-length byte strings compared with memcmp: deliberately a
 * different representation from the device's packed u64 keys.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ hashing */
static uint64_t hbytes(const uint8_t* p, int64_t n) {
    uint64_t h = 1469598103934665603ull; /* FNV-1a 64 */
    for (int64_t i = 0; i < n; ++i) { h ^= p[i]; h *= 1099511628211ull; }
    h ^= h >> 29; h *= 0xbf58476d1ce4e5b9ull; h ^= h >> 32;
    return h;
}

typedef struct { uint64_t h; const uint8_t* p; int64_t len; int64_t idx; } entry;

typedef struct {
    entry* e; int64_t cap; int64_t n;
} hmap;

static void hm_init(hmap* m, int64_t want) {
    int64_t cap = 16;
    while (cap < 2 * want) cap <<= 1;
    m->e = (entry*)calloc((size_t)cap, sizeof(entry));
    m->cap = cap; m->n = 0;
    for (int64_t i = 0; i < cap; ++i) m->e[i].idx = -1;
}

static int64_t hm_find(const hmap* m, const uint8_t* p, int64_t len, uint64_t h) {
    int64_t mask = m->cap - 1, s = (int64_t)(h & (uint64_t)mask);
    for (;;) {
        const entry* e = &m->e[s];
        if (e->idx < 0) return -1;
        if (e->h == h && e->len == len && memcmp(e->p, p, (size_t)len) == 0) return e->idx;
        s = (s + 1) & mask;
    }
}

static void hm_grow(hmap* m);

/* insert if absent; returns the entry's idx (new idx = next_idx when inserted) */
static int64_t hm_upsert(hmap* m, const uint8_t* p, int64_t len, uint64_t h, int64_t next_idx, int* inserted) {
    if (2 * (m->n + 1) > m->cap) hm_grow(m);
    int64_t mask = m->cap - 1, s = (int64_t)(h & (uint64_t)mask);
    for (;;) {
        entry* e = &m->e[s];
        if (e->idx < 0) {
            e->h = h; e->p = p; e->len = len; e->idx = next_idx; m->n++;
            *inserted = 1; return next_idx;
        }
        if (e->h == h && e->len == len && memcmp(e->p, p, (size_t)len) == 0) { *inserted = 0; return e->idx; }
        s = (s + 1) & mask;
    }
}

static void hm_grow(hmap* m) {
    hmap n2; hm_init(&n2, m->cap);
    for (int64_t i = 0; i < m->cap; ++i) {
        if (m->e[i].idx < 0) continue;
        int64_t mask = n2.cap - 1, s = (int64_t)(m->e[i].h & (uint64_t)mask);
        while (n2.e[s].idx >= 0) s = (s + 1) & mask;
        n2.e[s] = m->e[i]; n2.n++;
    }
    free(m->e); *m = n2;
}

/* -------------------------------------------------------------------- score */
typedef struct {
    hmap m; int32_t L; const double* rows; uint8_t* blob;
    const uint64_t* masks; const double* vals; /* mask form: row i = vals[i] at the set bits, 0.0 elsewhere */
} ldo_table;

static void index_keys(ldo_table* t, int64_t n_rows, const int64_t* key_offsets) {
    hm_init(&t->m, n_rows);
    for (int64_t i = 0; i < n_rows; ++i) {
        const uint8_t* p = t->blob + (key_offsets[i] - key_offsets[0]);
        int64_t len = key_offsets[i + 1] - key_offsets[i];
        uint64_t h = hbytes(p, len);
        int ins;
        int64_t idx = hm_upsert(&t->m, p, len, h, i, &ins);
        if (!ins) { /* Scala toMap: a later duplicate key overwrites */
            int64_t mask = t->m.cap - 1, s = (int64_t)(h & (uint64_t)mask);
            while (t->m.e[s].idx != idx) s = (s + 1) & mask;
            t->m.e[s].idx = i; t->m.e[s].p = p;
        }
    }
}

ldo_table* ldo_table_create(int64_t n_rows, const uint8_t* key_bytes, const int64_t* key_offsets,
                            const double* rows, int32_t L) {
    ldo_table* t = (ldo_table*)calloc(1, sizeof(ldo_table));
    int64_t nb = key_offsets[n_rows] - key_offsets[0];
    t->blob = (uint8_t*)malloc((size_t)(nb > 0 ? nb : 1));
    memcpy(t->blob, key_bytes + key_offsets[0], (size_t)nb);
    double* r = (double*)malloc(sizeof(double) * (size_t)(n_rows * L > 0 ? n_rows * L : 1));
    memcpy(r, rows, sizeof(double) * (size_t)(n_rows * L));
    t->rows = r; t->L = L;
    index_keys(t, n_rows, key_offsets);
    return t;
}

/* The same map given in mask form (rows too large to expand: 10M x 200):
 * row i is vals[i] at the languages set in masks[i][0 .. ceil(L/64)), 0.0
 * elsewhere -- scored as exactly that dense row. */
ldo_table* ldo_table_create_masks(int64_t n_rows, const uint8_t* key_bytes, const int64_t* key_offsets,
                                  const uint64_t* masks, const double* vals, int32_t L) {
    ldo_table* t = (ldo_table*)calloc(1, sizeof(ldo_table));
    int64_t nb = key_offsets[n_rows] - key_offsets[0];
    const int64_t S = (L + 63) / 64;
    t->blob = (uint8_t*)malloc((size_t)(nb > 0 ? nb : 1));
    memcpy(t->blob, key_bytes + key_offsets[0], (size_t)nb);
    uint64_t* m = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(n_rows * S > 0 ? n_rows * S : 1));
    double* v = (double*)malloc(sizeof(double) * (size_t)(n_rows > 0 ? n_rows : 1));
    memcpy(m, masks, sizeof(uint64_t) * (size_t)(n_rows * S));
    memcpy(v, vals, sizeof(double) * (size_t)n_rows);
    t->masks = m; t->vals = v; t->L = L;
    index_keys(t, n_rows, key_offsets);
    return t;
}

void ldo_table_destroy(ldo_table* t) {
    if (!t) return;
    free(t->m.e); free((void*)t->rows); free((void*)t->masks); free((void*)t->vals); free(t->blob); free(t);
}

static int32_t score_one(const ldo_table* t, const int32_t* G, int32_t nG, const uint8_t* d, int64_t len,
                         double* s) {
    const int32_t L = t->L;
    for (int32_t l = 0; l < L; ++l) s[l] = 0.0;
    for (int32_t gi = 0; gi < nG; ++gi) {
        int64_t n = G[gi];
        int64_t nw = len == 0 ? 0 : (len < n ? 1 : len - n + 1);
        int64_t wl = len < n ? len : n;
        for (int64_t p = 0; p < nw; ++p) {
            int64_t r = hm_find(&t->m, d + p, wl, hbytes(d + p, wl));
            if (r < 0) continue;
            if (t->masks) {
                const uint64_t* mk = t->masks + r * ((L + 63) / 64);
                const double v = t->vals[r];
                for (int32_t l = 0; l < L; ++l) s[l] = s[l] + 1.0 * (((mk[l / 64] >> (l % 64)) & 1u) ? v : 0.0);
                continue;
            }
            const double* row = t->rows + r * L;
            for (int32_t l = 0; l < L; ++l) s[l] = s[l] + 1.0 * row[l];
        }
    }
    int32_t bi = 0; double best = s[0];
    for (int32_t l = 1; l < L; ++l) if (s[l] > best) { best = s[l]; bi = l; }
    return bi;
}

typedef struct {
    const ldo_table* t; const int32_t* G; int32_t nG; const uint8_t* bytes; const int64_t* off;
    int64_t d0, d1; int32_t* labels; double* scores;
} score_job;

static void* score_worker(void* arg) {
    score_job* j = (score_job*)arg;
    const int32_t L = j->t->L;
    double* tmp = (double*)malloc(sizeof(double) * (size_t)L);
    for (int64_t d = j->d0; d < j->d1; ++d) {
        double* s = j->scores ? j->scores + d * L : tmp;
        j->labels[d] = score_one(j->t, j->G, j->nG, j->bytes + j->off[d], j->off[d + 1] - j->off[d], s);
    }
    free(tmp);
    return NULL;
}

/* labels[n_docs]; scores nullable [n_docs][L]; nthreads >= 1 */
int ldo_score(const ldo_table* t, const int32_t* G, int32_t nG, const uint8_t* bytes, const int64_t* offsets,
              int64_t n_docs, int32_t* labels, double* scores, int32_t nthreads) {
    if (t->L < 1) return 1;
    for (int32_t i = 0; i < nG; ++i) if (G[i] <= 0) return 1;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256]; score_job jobs[256];
    for (int32_t i = 0; i < nthreads; ++i) {
        jobs[i] = (score_job){t, G, nG, bytes, offsets, n_docs * i / nthreads, n_docs * (i + 1) / nthreads, labels, scores};
        if (nthreads == 1) score_worker(&jobs[i]);
        else pthread_create(&th[i], NULL, score_worker, &jobs[i]);
    }
    if (nthreads > 1) for (int32_t i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
    return 0;
}

/* table hits (windows whose key is in the table) of the documents, summed
 * (the reference's loop of score_one, LanguageDetectorModel.scala:139-149,
 * without the adds): bench.py's bytes model of a table beyond the caches */
int64_t ldo_hits(const ldo_table* t, const int32_t* G, int32_t nG, const uint8_t* bytes, const int64_t* offsets,
                 int64_t n_docs) {
    int64_t hits = 0;
    for (int64_t d = 0; d < n_docs; ++d) {
        const uint8_t* p = bytes + offsets[d];
        const int64_t len = offsets[d + 1] - offsets[d];
        for (int32_t gi = 0; gi < nG; ++gi) {
            const int64_t n = G[gi];
            const int64_t nw = len == 0 ? 0 : (len < n ? 1 : len - n + 1), wl = len < n ? len : n;
            for (int64_t q = 0; q < nw; ++q) hits += hm_find(&t->m, p + q, wl, hbytes(p + q, wl)) >= 0;
        }
    }
    return hits;
}

/* -------------------------------------------------------------------- count */
/* reduceGrams keys its sums by (language, gram) (LanguageDetector.scala:57-65):
 * so does this table -- one slot per distinct (gram, language) pair holding
 * its count; the gram rows of an export are assembled from the sorted pairs. */
typedef struct { uint64_t h; const uint8_t* p; int64_t len; int32_t lang; int64_t cnt; } pentry;

typedef struct {
    pentry* e; int64_t cap; int64_t n; int32_t L;
    const pentry** sorted; int64_t n_grams, key_bytes; /* export view (built on demand) */
} ldo_counts;

static uint64_t pair_hash(uint64_t h, int32_t lang) {
    uint64_t x = h ^ ((uint64_t)(uint32_t)lang * 0x9e3779b97f4a7c15ull);
    x ^= x >> 31; x *= 0xd6e8feb86659fd93ull; x ^= x >> 32;
    return x;
}

static ldo_counts* counts_new(int32_t L, int64_t want) {
    ldo_counts* c = (ldo_counts*)calloc(1, sizeof(ldo_counts));
    int64_t cap = 1024;
    while (cap < 2 * want) cap <<= 1;
    c->L = L; c->cap = cap;
    c->e = (pentry*)calloc((size_t)cap, sizeof(pentry));
    return c;
}

static void pm_add(ldo_counts* c, const uint8_t* p, int64_t len, uint64_t h, int32_t lang, int64_t cnt);

static void pm_grow(ldo_counts* c) {
    pentry* old = c->e;
    const int64_t oc = c->cap;
    c->cap *= 2; c->n = 0;
    c->e = (pentry*)calloc((size_t)c->cap, sizeof(pentry));
    for (int64_t i = 0; i < oc; ++i) if (old[i].p) pm_add(c, old[i].p, old[i].len, old[i].h, old[i].lang, old[i].cnt);
    free(old);
}

/* count of (gram p[0..len), lang) += cnt; h = hbytes of the gram */
static void pm_add(ldo_counts* c, const uint8_t* p, int64_t len, uint64_t h, int32_t lang, int64_t cnt) {
    if (2 * (c->n + 1) > c->cap) pm_grow(c);
    const int64_t mask = c->cap - 1;
    int64_t s = (int64_t)(pair_hash(h, lang) & (uint64_t)mask);
    for (;;) {
        pentry* e = &c->e[s];
        if (!e->p) { *e = (pentry){h, p, len, lang, cnt}; c->n++; return; }
        if (e->h == h && e->lang == lang && e->len == len && memcmp(e->p, p, (size_t)len) == 0) { e->cnt += cnt; return; }
        s = (s + 1) & mask;
    }
}

ldo_counts* ldo_count(const uint8_t* bytes, const int64_t* offsets, const int32_t* doc_lang, int64_t n_docs,
                      int32_t L, const int32_t* G, int32_t nG) {
    ldo_counts* c = counts_new(L, 1024);
    for (int64_t d = 0; d < n_docs; ++d) {
        const uint8_t* p = bytes + offsets[d];
        int64_t len = offsets[d + 1] - offsets[d];
        int32_t lang = doc_lang[d];
        if (lang < 0 || lang >= L) continue;
        for (int32_t gi = 0; gi < nG; ++gi) {
            int64_t n = G[gi];
            int64_t nw = len == 0 ? 0 : (len < n ? 1 : len - n + 1);
            int64_t wl = len < n ? len : n;
            for (int64_t i = 0; i < nw; ++i) pm_add(c, p + i, wl, hbytes(p + i, wl), lang, 1);
        }
    }
    return c;
}

/* Multithreaded ldo_count (the CPU baseline of bench.py's FIT line, SURVEY
 * §8d: N host threads): computeGrams per thread over a contiguous range of
 * documents (balanced by bytes) into a private table -- Spark's map side --
 * then reduceGrams: thread p sums every private table's pairs of hash
 * partition p (the shuffle), and the partitions (disjoint pairs) are
 * concatenated into one table.  Same counts as ldo_count. */
typedef struct {
    const uint8_t* bytes; const int64_t* off; const int32_t* lang; int64_t d0, d1; int32_t L; const int32_t* G;
    int32_t nG; ldo_counts* local; ldo_counts** locals; int32_t nthreads, part; ldo_counts* out;
} count_job;

static void* count_map_worker(void* arg) {
    count_job* j = (count_job*)arg;
    j->local = ldo_count(j->bytes, j->off + j->d0, j->lang + j->d0, j->d1 - j->d0, j->L, j->G, j->nG);
    return NULL;
}

static int32_t part_of(const pentry* e, int32_t nthreads) {
    return (int32_t)((pair_hash(e->h, e->lang) >> 40) % (uint64_t)nthreads);
}

static void* count_reduce_worker(void* arg) {
    count_job* j = (count_job*)arg;
    int64_t want = 0;
    for (int32_t t = 0; t < j->nthreads; ++t) want += j->locals[t]->n / j->nthreads;
    j->out = counts_new(j->L, want);
    for (int32_t t = 0; t < j->nthreads; ++t) {
        const ldo_counts* c = j->locals[t];
        for (int64_t i = 0; i < c->cap; ++i) {
            const pentry* e = &c->e[i];
            if (e->p && part_of(e, j->nthreads) == j->part) pm_add(j->out, e->p, e->len, e->h, e->lang, e->cnt);
        }
    }
    return NULL;
}

static void counts_free(ldo_counts* c) {
    if (!c) return;
    free(c->e); free(c->sorted); free(c);
}

ldo_counts* ldo_count_mt(const uint8_t* bytes, const int64_t* offsets, const int32_t* doc_lang, int64_t n_docs,
                         int32_t L, const int32_t* G, int32_t nG, int32_t nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    if (nthreads == 1 || n_docs < 2 * nthreads) return ldo_count(bytes, offsets, doc_lang, n_docs, L, G, nG);
    pthread_t th[256]; count_job jobs[256]; ldo_counts* locals[256];
    const int64_t b0 = offsets[0], nb = offsets[n_docs] - b0;
    int64_t d = 0;
    for (int32_t t = 0; t < nthreads; ++t) {
        const int64_t goal = b0 + nb * (t + 1) / nthreads;
        int64_t d1 = d;
        while (d1 < n_docs && (offsets[d1] < goal || t + 1 == nthreads)) ++d1;
        jobs[t] = (count_job){bytes, offsets, doc_lang, d, d1, L, G, nG, NULL, locals, nthreads, t, NULL};
        d = d1;
        pthread_create(&th[t], NULL, count_map_worker, &jobs[t]);
    }
    for (int32_t t = 0; t < nthreads; ++t) { pthread_join(th[t], NULL); locals[t] = jobs[t].local; }
    for (int32_t t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, count_reduce_worker, &jobs[t]);
    for (int32_t t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    for (int32_t t = 0; t < nthreads; ++t) counts_free(locals[t]);
    int64_t total = 0;
    for (int32_t t = 0; t < nthreads; ++t) total += jobs[t].out->n;
    ldo_counts* c = counts_new(L, total);
    for (int32_t t = 0; t < nthreads; ++t) {
        const ldo_counts* o = jobs[t].out;
        for (int64_t i = 0; i < o->cap; ++i) {
            const pentry* e = &o->e[i];
            if (e->p) pm_add(c, e->p, e->len, e->h, e->lang, e->cnt);
        }
        counts_free(jobs[t].out);
    }
    return c;
}

static int cmp_pentry(const void* a, const void* b) {
    const pentry* x = *(const pentry* const*)a; const pentry* y = *(const pentry* const*)b;
    if (x->len != y->len) return x->len < y->len ? -1 : 1;
    const int m = memcmp(x->p, y->p, (size_t)x->len);
    if (m) return m;
    return x->lang < y->lang ? -1 : (x->lang > y->lang);
}

/* the pairs sorted by (gram length, unsigned bytes, language); distinct grams */
static void sorted_view(ldo_counts* c) {
    if (c->sorted) return;
    c->sorted = (const pentry**)malloc(sizeof(pentry*) * (size_t)(c->n > 0 ? c->n : 1));
    int64_t k = 0;
    for (int64_t i = 0; i < c->cap; ++i) if (c->e[i].p) c->sorted[k++] = &c->e[i];
    qsort(c->sorted, (size_t)k, sizeof(pentry*), cmp_pentry);
    c->n_grams = c->key_bytes = 0;
    for (int64_t i = 0; i < k; ++i) {
        const pentry* e = c->sorted[i];
        if (i && e->len == c->sorted[i - 1]->len && memcmp(e->p, c->sorted[i - 1]->p, (size_t)e->len) == 0) continue;
        c->n_grams++;
        c->key_bytes += e->len;
    }
}

int64_t ldo_counts_size(ldo_counts* c) { sorted_view(c); return c->n_grams; }
int64_t ldo_counts_key_bytes(ldo_counts* c) { sorted_view(c); return c->key_bytes; }
int64_t ldo_counts_pairs(const ldo_counts* c) { return c->n; }

/* export sorted by (length, unsigned bytes); sparse: key_bytes, key_offsets
 * [n+1], pair_offsets [n+1], the pairs' languages (ascending per gram) and
 * counts; dense (ldo_counts_export): counts[n][L] */
void ldo_counts_export_sparse(ldo_counts* c, uint8_t* key_bytes, int64_t* key_offsets, int64_t* pair_offsets,
                              int32_t* langs, int64_t* counts) {
    sorted_view(c);
    int64_t o = 0, g = -1;
    key_offsets[0] = 0;
    pair_offsets[0] = 0;
    for (int64_t i = 0; i < c->n; ++i) {
        const pentry* e = c->sorted[i];
        if (!(i && e->len == c->sorted[i - 1]->len && memcmp(e->p, c->sorted[i - 1]->p, (size_t)e->len) == 0)) {
            ++g;
            memcpy(key_bytes + o, e->p, (size_t)e->len);
            o += e->len;
            key_offsets[g + 1] = o;
        }
        pair_offsets[g + 1] = i + 1;
        langs[i] = e->lang;
        counts[i] = e->cnt;
    }
}

void ldo_counts_export(ldo_counts* c, uint8_t* key_bytes, int64_t* key_offsets, int64_t* counts) {
    sorted_view(c);
    int64_t o = 0, g = -1;
    key_offsets[0] = 0;
    memset(counts, 0, sizeof(int64_t) * (size_t)(c->n_grams * c->L));
    for (int64_t i = 0; i < c->n; ++i) {
        const pentry* e = c->sorted[i];
        if (!(i && e->len == c->sorted[i - 1]->len && memcmp(e->p, c->sorted[i - 1]->p, (size_t)e->len) == 0)) {
            ++g;
            memcpy(key_bytes + o, e->p, (size_t)e->len);
            o += e->len;
            key_offsets[g + 1] = o;
        }
        counts[g * c->L + e->lang] = e->cnt;
    }
}

void ldo_counts_destroy(ldo_counts* c) { counts_free(c); }
