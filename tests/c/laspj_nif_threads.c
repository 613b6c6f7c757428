/*
 * The NIF-level entry points (include/laspj.h "NIF entry points") driven the way a NIF
 * drives them: several BEAM schedulers, one context each, calling merge / value / equal /
 * inflation on term_to_binary images at the same time.  Uses nothing but laspj.h.
 *
 * argv[1]: a case file written by tests/test_gpu_nif.py (the oracle's answers):
 *   u32 ncases, then per case: u32 op, i32 verdict, i32 result, u64 la + bytes, u64 lb +
 *   bytes, u64 lexp + bytes (the expected image).  op: lasp_orset images 0 merge, 1 value,
 *   2 equal, 3 inflation, 4 strict inflation; lasp_gset images 5..9 likewise; 10 / 11 an
 *   OR-Set / G-Set resident variable (write a, bind b: result = the bind status, exp = the
 *   value read back); 20 + k (OR-Set) / 120 + k (G-Set) a list body from images, k = 0
 *   union, 1 intersection, 2 product, 3 map, 4 filter, 5 fold (b = the fun's results), 6
 *   value, 7 bind (a = Value0, b = Value, result = status, exp = the written value).
 * argv[2]: threads (default 4).  Every thread creates its own context, runs every case
 * three times in its own rotation and compares verdicts, booleans and images byte for
 * byte.  Prints "laspj NIF threads OK" and the summed counters.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "laspj.h"

typedef struct {
    uint32_t op;
    int32_t verdict, result;
    uint8_t *a, *b, *exp;
    uint64_t la, lb, lexp;
} nif_case;

static nif_case* cases;
static uint32_t ncases;

typedef struct {
    int tid, fails;
    uint64_t stats[LASPJ_NIF_STATS];
    char msg[256];
} worker;

static int rd(FILE* f, void* p, size_t n) { return fread(p, 1, n, f) == n ? 0 : -1; }

static uint8_t* rd_blob(FILE* f, uint64_t* n) {
    if (rd(f, n, 8)) return NULL;
    uint8_t* p = malloc(*n ? *n : 1);
    if (p && *n && rd(f, p, *n)) {
        free(p);
        return NULL;
    }
    return p;
}

static int load(const char* path) {
    FILE* f = fopen(path, "rb");
    if (!f) return -1;
    if (rd(f, &ncases, 4)) return -1;
    cases = calloc(ncases, sizeof *cases);
    for (uint32_t i = 0; i < ncases; ++i) {
        nif_case* c = &cases[i];
        if (rd(f, &c->op, 4) || rd(f, &c->verdict, 4) || rd(f, &c->result, 4)) return -1;
        if (!(c->a = rd_blob(f, &c->la)) || !(c->b = rd_blob(f, &c->lb)) ||
            !(c->exp = rd_blob(f, &c->lexp)))
            return -1;
    }
    fclose(f);
    return 0;
}

static void* run(void* arg) {
    worker* w = arg;
    laspj_ctx* ctx = NULL;
    if (laspj_ctx_create(0, &ctx) != LASPJ_OK) {
        snprintf(w->msg, sizeof w->msg, "thread %d: ctx_create failed", w->tid);
        w->fails++;
        return NULL;
    }
    for (int round = 0; round < 3 && !w->fails; ++round) {
        for (uint32_t k = 0; k < ncases && !w->fails; ++k) {
            const uint32_t i = (k + 13u * (uint32_t)w->tid + 5u * (uint32_t)round) % ncases;
            const nif_case* c = &cases[i];
            const uint8_t* out = NULL;
            uint64_t olen = 0;
            int32_t verdict = -1, result = -1;
            int st;
            int image = 0;                  /* the answer is an image (else a boolean) */
            const uint32_t op = c->op;
            if (op <= 9) {
                const int g = op >= 5;
                const uint32_t o = g ? op - 5 : op;
                image = o <= 1;
                if (o == 0)
                    st = g ? laspj_gset_etf_merge(ctx, c->a, c->la, c->b, c->lb, &out, &olen, &verdict)
                           : laspj_orset_etf_merge(ctx, c->a, c->la, c->b, c->lb, &out, &olen, &verdict);
                else if (o == 1)
                    st = g ? laspj_gset_etf_value(ctx, c->a, c->la, &out, &olen, &verdict)
                           : laspj_orset_etf_value(ctx, c->a, c->la, &out, &olen, &verdict);
                else if (o == 2)
                    st = g ? laspj_gset_etf_equal(ctx, c->a, c->la, c->b, c->lb, &result, &verdict)
                           : laspj_orset_etf_equal(ctx, c->a, c->la, c->b, c->lb, &result, &verdict);
                else
                    st = g ? laspj_gset_etf_inflation(ctx, c->a, c->la, c->b, c->lb, o == 4,
                                                      &result, &verdict)
                           : laspj_orset_etf_inflation(ctx, c->a, c->la, c->b, c->lb, o == 4,
                                                       &result, &verdict);
            } else if (op == 10 || op == 11) {
                laspj_var* v = NULL;
                int32_t wv = -1, rv = -1;
                st = laspj_var_create(ctx, op == 10 ? LASPJ_KIND_ORSET : LASPJ_KIND_GSET, &v);
                if (st == LASPJ_OK) st = laspj_var_etf_write(v, c->a, c->la, &wv);
                if (st == LASPJ_OK) st = laspj_var_etf_bind(v, c->b, c->lb, &result, &verdict);
                if (st == LASPJ_OK) st = laspj_var_etf_read(v, &out, &olen, &rv);
                if (st == LASPJ_OK && (wv != LASPJ_NIF_OK || rv != LASPJ_NIF_OK)) verdict = -2;
                image = 2;                  /* both: the status and the value */
                if (v) laspj_var_destroy(v);
            } else {
                const int32_t kind = op >= 120 ? LASPJ_KIND_GSET : LASPJ_KIND_ORSET;
                const uint32_t k = op >= 120 ? op - 120 : op - 20;
                image = 1;
                switch (k) {
                case 0: st = laspj_list_etf_union(ctx, kind, c->a, c->la, c->b, c->lb, &out, &olen, &verdict); break;
                case 1: st = laspj_list_etf_intersection(ctx, kind, c->a, c->la, c->b, c->lb, &out, &olen, &verdict); break;
                case 2: st = laspj_list_etf_product(ctx, kind, c->a, c->la, c->b, c->lb, &out, &olen, &verdict); break;
                case 3: st = laspj_list_etf_map(ctx, kind, c->a, c->la, c->b, c->lb, &out, &olen, &verdict); break;
                case 4: st = laspj_list_etf_filter(ctx, kind, c->a, c->la, c->b, c->lb, &out, &olen, &verdict); break;
                case 5: st = laspj_list_etf_fold(ctx, kind, c->a, c->la, c->b, c->lb, &out, &olen, &verdict); break;
                case 6: st = laspj_list_etf_value(ctx, kind, c->a, c->la, &out, &olen, &verdict); break;
                default:
                    st = laspj_list_etf_bind(ctx, kind, c->a, c->la, c->b, c->lb, &out, &olen, &result, &verdict);
                    image = result == 1 ? 2 : 3;     /* status, and the image when written */
                }
            }
            if (st != LASPJ_OK) {
                snprintf(w->msg, sizeof w->msg, "thread %d case %u: status %d (%s)", w->tid, i, st,
                         laspj_ctx_last_error(ctx));
                w->fails++;
            } else if (verdict != c->verdict) {
                snprintf(w->msg, sizeof w->msg, "thread %d case %u: verdict %d, want %d", w->tid,
                         i, verdict, c->verdict);
                w->fails++;
            } else if (verdict == LASPJ_NIF_OK && (image == 1 || image == 2) &&
                       (olen != c->lexp || memcmp(out, c->exp, olen) != 0)) {
                snprintf(w->msg, sizeof w->msg, "thread %d case %u (op %u): image differs (%llu vs %llu B)",
                         w->tid, i, c->op, (unsigned long long)olen, (unsigned long long)c->lexp);
                w->fails++;
            } else if (verdict == LASPJ_NIF_OK && image != 1 && result != c->result) {
                snprintf(w->msg, sizeof w->msg, "thread %d case %u: result %d, want %d", w->tid,
                         i, result, c->result);
                w->fails++;
            }
        }
    }
    laspj_nif_stats(ctx, w->stats, LASPJ_NIF_STATS);
    laspj_ctx_destroy(ctx);
    return NULL;
}

int main(int argc, char** argv) {
    if (argc < 2 || load(argv[1])) {
        fprintf(stderr, "usage: %s CASES [THREADS]\n", argv[0]);
        return 2;
    }
    const int nt = argc > 2 ? atoi(argv[2]) : 4;
    pthread_t th[64];
    worker ws[64];
    memset(ws, 0, sizeof ws);
    for (int t = 0; t < nt && t < 64; ++t) {
        ws[t].tid = t;
        pthread_create(&th[t], NULL, run, &ws[t]);
    }
    int fails = 0;
    uint64_t sum[LASPJ_NIF_STATS] = {0};
    for (int t = 0; t < nt && t < 64; ++t) {
        pthread_join(th[t], NULL);
        if (ws[t].fails) {
            fprintf(stderr, "%s\n", ws[t].msg);
            fails++;
        }
        for (int k = 0; k < LASPJ_NIF_STATS; ++k) sum[k] += ws[t].stats[k];
    }
    if (fails) return 1;
    printf("stats calls=%llu passes=%llu registrations=%llu resets=%llu rebuilds=%llu "
           "host_encoded=%llu fallbacks=%llu\n",
           (unsigned long long)sum[0], (unsigned long long)sum[1], (unsigned long long)sum[2],
           (unsigned long long)sum[3], (unsigned long long)sum[4], (unsigned long long)sum[5],
           (unsigned long long)sum[6]);
    printf("laspj NIF threads OK (%d threads x %u cases x 3)\n", nt, ncases);
    return 0;
}
