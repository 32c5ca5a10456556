/* asan_driver.c -- libldgpu.so's host code under AddressSanitizer:
 * links lib/libldgpu_asan.so (make -C spark-languagedetector_amd asan: host
 * code instrumented, device code the product's) and the C restatement
 * (oracle/ldoracle.c, the checker), and drives the C ABI on a GPU -- count,
 * export (dense and sparse ranges), add, fit table, model from masks, host
 * scoring, error paths -- checking counts and labels/scores against the
 * restatement.  Build: tools/build_asan.sh; run on a GPU box.  Exit 0 = clean. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/ldgpu.h"

typedef struct ldo_table ldo_table;
typedef struct ldo_counts ldo_counts;
ldo_table* ldo_table_create_masks(int64_t, const uint8_t*, const int64_t*, const uint64_t*, const double*, int32_t);
void ldo_table_destroy(ldo_table*);
int ldo_score(const ldo_table*, const int32_t*, int32_t, const uint8_t*, const int64_t*, int64_t, int32_t*, double*,
              int32_t);
ldo_counts* ldo_count(const uint8_t*, const int64_t*, const int32_t*, int64_t, int32_t, const int32_t*, int32_t);
int64_t ldo_counts_size(const ldo_counts*);
int64_t ldo_counts_key_bytes(const ldo_counts*);
void ldo_counts_export(const ldo_counts*, uint8_t*, int64_t*, int64_t*);
void ldo_counts_destroy(ldo_counts*);

static uint64_t rs = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(uint32_t n) {
    rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17;
    return (uint32_t)(rs % n);
}

#define OK(x)                                                                                   \
    do {                                                                                        \
        int rc_ = (x);                                                                          \
        if (rc_) {                                                                              \
            fprintf(stderr, "asan_driver: %s -> %d (%s), line %d\n", #x, rc_, ldgpu_last_error(), __LINE__); \
            return 1;                                                                           \
        }                                                                                       \
    } while (0)
#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            fprintf(stderr, "asan_driver: %s failed, line %d\n", #c, __LINE__); \
            return 1;                                                         \
        }                                                                     \
    } while (0)

static int run(ldgpu_ctx* ctx, int L, const int32_t* G, int nG, int n_docs, int max_len, const char* alphabet) {
    const int na = (int)strlen(alphabet);
    int64_t* off = malloc(sizeof(int64_t) * (n_docs + 1));
    int32_t* lang = malloc(sizeof(int32_t) * n_docs);
    off[0] = 0;
    for (int d = 0; d < n_docs; ++d) {
        off[d + 1] = off[d] + (d < 8 ? d : (int)rnd((uint32_t)max_len + 1));
        lang[d] = d % 13 == 3 ? -1 : (int32_t)rnd((uint32_t)L);
    }
    const int64_t nbytes = off[n_docs];
    uint8_t* bytes = malloc((size_t)(nbytes > 0 ? nbytes : 1));  /* exactly the corpus: no slack */
    for (int64_t i = 0; i < nbytes; ++i) bytes[i] = (uint8_t)alphabet[rnd((uint32_t)na)];

    /* FIT: device counts vs the restatement (two calls accumulate) */
    ldgpu_counts* c = NULL;
    OK(ldgpu_counts_create(ctx, L, G, nG, 16, &c));
    OK(ldgpu_count(c, bytes, off, lang, n_docs));
    OK(ldgpu_count(c, bytes, off, lang, n_docs / 3));
    int64_t n = 0, nb = 0;
    OK(ldgpu_counts_size(c, &n, &nb));
    uint8_t* kb = malloc((size_t)(nb > 0 ? nb : 1));
    int64_t* ko = malloc(sizeof(int64_t) * (n + 1));
    int64_t* cnt = malloc(sizeof(int64_t) * (size_t)(n * L > 0 ? n * L : 1));
    OK(ldgpu_counts_export(c, kb, ko, cnt));
    ldo_counts* oc = ldo_count(bytes, off, lang, n_docs, L, G, nG);
    ldo_counts* oc3 = ldo_count(bytes, off, lang, n_docs / 3, L, G, nG);
    CHECK(ldo_counts_size(oc) == n && ldo_counts_key_bytes(oc) == nb);
    uint8_t* okb = malloc((size_t)(nb > 0 ? nb : 1));
    int64_t* oko = malloc(sizeof(int64_t) * (n + 1));
    int64_t* ocnt = malloc(sizeof(int64_t) * (size_t)(n * L > 0 ? n * L : 1));
    ldo_counts_export(oc, okb, oko, ocnt);
    CHECK(memcmp(kb, okb, (size_t)nb) == 0 && memcmp(ko, oko, sizeof(int64_t) * (n + 1)) == 0);
    {   /* the second call's documents counted twice */
        const int64_t n3 = ldo_counts_size(oc3), nb3 = ldo_counts_key_bytes(oc3);
        uint8_t* kb3 = malloc((size_t)(nb3 > 0 ? nb3 : 1));
        int64_t* ko3 = malloc(sizeof(int64_t) * (n3 + 1));
        int64_t* c3 = malloc(sizeof(int64_t) * (size_t)(n3 * L > 0 ? n3 * L : 1));
        ldo_counts_export(oc3, kb3, ko3, c3);
        int64_t j = 0;
        for (int64_t i = 0; i < n && j < n3; ++i) {
            const int64_t li = ko[i + 1] - ko[i], lj = ko3[j + 1] - ko3[j];
            if (li == lj && memcmp(kb + ko[i], kb3 + ko3[j], (size_t)li) == 0) {
                for (int l = 0; l < L; ++l) ocnt[i * L + l] += c3[j * L + l];
                ++j;
            }
        }
        CHECK(j == n3);
        free(kb3); free(ko3); free(c3);
    }
    CHECK(memcmp(cnt, ocnt, sizeof(int64_t) * (size_t)(n * L)) == 0);
    /* sparse export in ranges, added into a fresh table: the same counts */
    ldgpu_counts* c2 = NULL;
    OK(ldgpu_counts_create(ctx, L, G, nG, 0, &c2));
    for (int64_t first = 0; first < n;) {
        const int64_t m = first + 1000 < n ? 1000 : n - first;
        int64_t skb = 0, sp = 0;
        OK(ldgpu_counts_sparse_size(c, first, m, &skb, &sp));
        uint8_t* sk = malloc((size_t)(skb > 0 ? skb : 1));
        int64_t* sko = malloc(sizeof(int64_t) * (m + 1));
        int64_t* spo = malloc(sizeof(int64_t) * (m + 1));
        int32_t* spl = malloc(sizeof(int32_t) * (size_t)(sp > 0 ? sp : 1));
        int64_t* spc = malloc(sizeof(int64_t) * (size_t)(sp > 0 ? sp : 1));
        OK(ldgpu_counts_export_sparse(c, first, m, sk, sko, spo, spl, spc));
        OK(ldgpu_counts_add_sparse(c2, m, sk, sko, spo, spl, spc));
        free(sk); free(sko); free(spo); free(spl); free(spc);
        first += m;
    }
    int64_t* cnt2 = malloc(sizeof(int64_t) * (size_t)(n * L > 0 ? n * L : 1));
    OK(ldgpu_counts_export(c2, kb, ko, cnt2));
    CHECK(memcmp(cnt, cnt2, sizeof(int64_t) * (size_t)(n * L)) == 0);
    /* error paths */
    CHECK(ldgpu_counts_export_sparse(c, n, 1, kb, ko, ko, NULL, NULL) == LDGPU_EINVAL);
    CHECK(ldgpu_count(c, bytes, NULL, lang, 3) == LDGPU_EINVAL);

    /* the fit table in mask form -> a model; host scoring vs the restatement */
    int64_t rows = 0, rkb = 0;
    OK(ldgpu_fit_table_size(c, 40, &rows, &rkb));
    const int S = (L + 63) / 64;
    uint8_t* tkb = malloc((size_t)(rkb > 0 ? rkb : 1));
    int64_t* tko = malloc(sizeof(int64_t) * (rows + 1));
    uint64_t* tm = malloc(sizeof(uint64_t) * (size_t)(rows * S > 0 ? rows * S : 1));
    double* tv = malloc(sizeof(double) * (size_t)(rows > 0 ? rows : 1));
    OK(ldgpu_fit_table_export_masks(c, tkb, tko, tm, tv));
    ldgpu_model* m = NULL;
    OK(ldgpu_model_create_masks(ctx, rows, tkb, tko, tm, tv, L, G, nG, &m));
    int32_t* lab = malloc(sizeof(int32_t) * n_docs);
    int32_t* olab = malloc(sizeof(int32_t) * n_docs);
    double* sc = malloc(sizeof(double) * (size_t)n_docs * L);
    double* osc = malloc(sizeof(double) * (size_t)n_docs * L);
    OK(ldgpu_score(m, bytes, off, n_docs, lab, sc));
    ldo_table* ot = ldo_table_create_masks(rows, tkb, tko, tm, tv, L);
    CHECK(ldo_score(ot, G, nG, bytes, off, n_docs, olab, osc, 4) == 0);
    CHECK(memcmp(lab, olab, sizeof(int32_t) * n_docs) == 0);
    CHECK(memcmp(sc, osc, sizeof(double) * (size_t)n_docs * L) == 0);
    OK(ldgpu_score(m, bytes, off, n_docs, lab, NULL));
    CHECK(memcmp(lab, olab, sizeof(int32_t) * n_docs) == 0);
    int32_t flags = 0;
    OK(ldgpu_model_layout(m, &flags));
    OK(ldgpu_model_destroy(m));
    ldo_table_destroy(ot);
    OK(ldgpu_counts_destroy(c));
    OK(ldgpu_counts_destroy(c2));
    ldo_counts_destroy(oc);
    ldo_counts_destroy(oc3);
    free(lab); free(olab); free(sc); free(osc); free(tkb); free(tko); free(tm); free(tv);
    free(kb); free(ko); free(cnt); free(cnt2); free(okb); free(oko); free(ocnt);
    free(bytes); free(off); free(lang);
    return 0;
}

int main(void) {
    ldgpu_ctx* ctx = NULL;
    OK(ldgpu_ctx_create(0, &ctx));
    const int32_t g1[] = {1, 2, 3, 4, 5}, g2[] = {3, 1, 3}, g3[] = {8, 2, 12}, g4[] = {1, 2, 3, 4, 5, 6, 7};
    int rc = 0;
    rc |= run(ctx, 20, g1, 5, 3000, 600, "abcdefghijklmnop ");
    rc |= run(ctx, 3, g2, 3, 1000, 200, "ab ");
    rc |= run(ctx, 7, g3, 3, 800, 80, "abcd ");
    rc |= run(ctx, 200, g4, 7, 600, 300, "abcdefghijklmnopqrstuvwxyz");
    OK(ldgpu_ctx_destroy(ctx));
    if (!rc) puts("asan_driver: clean");
    return rc;
}
