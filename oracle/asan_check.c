/* asan_check.c -- the C restatement (ldoracle.c) under AddressSanitizer and
 * UBSan (make -C oracle asan; SURVEY §5 "race detection / sanitizers").  TEST
 * INFRASTRUCTURE ONLY.  Exercises every entry point on random corpora with the
 * edge cases of the reference's rules (empty documents, documents shorter than
 * n, keys up to 15 bytes, duplicate gram lengths, unsupported labels, many
 * threads) and checks what the rules fix without a second restatement: every
 * window counted once, labels in range, dense and mask forms scoring alike.
 * Exit status 0 = clean (the sanitizers abort on any error they find). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct ldo_table ldo_table;
typedef struct ldo_counts ldo_counts;
ldo_table* ldo_table_create(int64_t, const uint8_t*, const int64_t*, const double*, int32_t);
ldo_table* ldo_table_create_masks(int64_t, const uint8_t*, const int64_t*, const uint64_t*, const double*, int32_t);
void ldo_table_destroy(ldo_table*);
int ldo_score(const ldo_table*, const int32_t*, int32_t, const uint8_t*, const int64_t*, int64_t, int32_t*, double*,
              int32_t);
ldo_counts* ldo_count(const uint8_t*, const int64_t*, const int32_t*, int64_t, int32_t, const int32_t*, int32_t);
int64_t ldo_counts_size(const ldo_counts*);
int64_t ldo_counts_key_bytes(const ldo_counts*);
void ldo_counts_export(const ldo_counts*, uint8_t*, int64_t*, int64_t*);
void ldo_counts_destroy(ldo_counts*);

static uint64_t rs = 88172645463325252ull;
static uint32_t rnd(uint32_t n) {
    rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17;
    return (uint32_t)(rs % n);
}

#define CHECK(c)                                                   \
    do {                                                           \
        if (!(c)) {                                                \
            fprintf(stderr, "asan_check: %s failed (line %d)\n", #c, __LINE__); \
            return 1;                                              \
        }                                                          \
    } while (0)

static int64_t windows(int64_t len, int n) { return len == 0 ? 0 : (len < n ? 1 : len - n + 1); }

static int run(int L, const int32_t* G, int nG, int n_docs, int max_len, const char* alphabet) {
    const int na = (int)strlen(alphabet);
    int64_t* off = malloc(sizeof(int64_t) * (n_docs + 1));
    int32_t* lang = malloc(sizeof(int32_t) * n_docs);
    off[0] = 0;
    for (int d = 0; d < n_docs; ++d) {
        const int len = d < 8 ? d : (int)rnd((uint32_t)max_len + 1);  /* 0..7 first: partial windows */
        off[d + 1] = off[d] + len;
        lang[d] = d % 17 == 5 ? -1 : (int32_t)rnd((uint32_t)L);       /* -1: an unsupported label */
    }
    /* exactly off[n] bytes: a read past the corpus is an ASan error */
    uint8_t* bytes = malloc((size_t)(off[n_docs] > 0 ? off[n_docs] : 1));
    for (int64_t i = 0; i < off[n_docs]; ++i) bytes[i] = (uint8_t)alphabet[rnd((uint32_t)na)];

    ldo_counts* c = ldo_count(bytes, off, lang, n_docs, L, G, nG);
    const int64_t n = ldo_counts_size(c), nb = ldo_counts_key_bytes(c);
    uint8_t* kb = malloc((size_t)(nb > 0 ? nb : 1));
    int64_t* ko = malloc(sizeof(int64_t) * (n + 1));
    int64_t* cnt = malloc(sizeof(int64_t) * (size_t)(n * L > 0 ? n * L : 1));
    ldo_counts_export(c, kb, ko, cnt);
    int64_t total = 0, expect = 0;
    for (int64_t i = 0; i < n * L; ++i) total += cnt[i];
    for (int d = 0; d < n_docs; ++d)
        if (lang[d] >= 0)
            for (int g = 0; g < nG; ++g) expect += windows(off[d + 1] - off[d], G[g]);
    CHECK(total == expect);
    for (int64_t i = 0; i < n; ++i) CHECK(ko[i + 1] > ko[i] && ko[i + 1] - ko[i] <= 15);

    /* a table of every counted gram: dense rows and the same rows in mask form */
    const int S = (L + 63) / 64;
    double* rows = calloc((size_t)(n * L > 0 ? n * L : 1), sizeof(double));
    uint64_t* masks = calloc((size_t)(n * S > 0 ? n * S : 1), sizeof(uint64_t));
    double* vals = malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    for (int64_t i = 0; i < n; ++i) {
        vals[i] = 0.25 + (double)(i % 7);
        for (int l = 0; l < L; ++l)
            if (cnt[i * L + l]) {
                rows[i * L + l] = vals[i];
                masks[i * S + l / 64] |= 1ull << (l % 64);
            }
    }
    ldo_table* td = ldo_table_create(n, kb, ko, rows, L);
    ldo_table* tm = ldo_table_create_masks(n, kb, ko, masks, vals, L);
    int32_t* la = malloc(sizeof(int32_t) * n_docs);
    int32_t* lb = malloc(sizeof(int32_t) * n_docs);
    double* sa = malloc(sizeof(double) * (size_t)n_docs * L);
    double* sb = malloc(sizeof(double) * (size_t)n_docs * L);
    CHECK(ldo_score(td, G, nG, bytes, off, n_docs, la, sa, 7) == 0);
    CHECK(ldo_score(tm, G, nG, bytes, off, n_docs, lb, sb, 3) == 0);
    CHECK(memcmp(la, lb, sizeof(int32_t) * n_docs) == 0);
    CHECK(memcmp(sa, sb, sizeof(double) * (size_t)n_docs * L) == 0);
    for (int d = 0; d < n_docs; ++d) CHECK(la[d] >= 0 && la[d] < L);
    CHECK(ldo_score(td, G, nG, bytes, off, n_docs, lb, NULL, 1) == 0);  /* labels only */
    CHECK(memcmp(la, lb, sizeof(int32_t) * n_docs) == 0);
    ldo_table_destroy(td);
    ldo_table_destroy(tm);
    ldo_counts_destroy(c);
    free(la); free(lb); free(sa); free(sb); free(rows); free(masks); free(vals);
    free(kb); free(ko); free(cnt); free(bytes); free(off); free(lang);
    return 0;
}

int main(void) {
    const int32_t g1[] = {1, 2, 3, 4, 5}, g2[] = {3, 1, 3}, g3[] = {8, 2, 15, 9}, g4[] = {7};
    int rc = 0;
    rc |= run(20, g1, 5, 600, 400, "abcdefghij ");
    rc |= run(3, g2, 3, 400, 100, "ab");
    rc |= run(70, g3, 4, 300, 60, "abcd ");
    rc |= run(130, g4, 1, 200, 300, "abcdefghijklmnopqrstuvwxyz");
    if (!rc) puts("asan_check: clean");
    return rc;
}
