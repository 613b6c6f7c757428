/*
 * The NIF-level entry points (include/laspj.h "NIF entry points") driven the way a NIF
 * drives them: several BEAM schedulers, one context each, calling merge / value / equal /
 * inflation on term_to_binary images at the same time.  Uses nothing but laspj.h.
 *
 * argv[1]: a case file written by tests/test_gpu_nif.py (the oracle's answers):
 *   u32 ncases, then per case: u32 op (0 merge, 1 value, 2 equal, 3 inflation,
 *   4 strict inflation), i32 verdict, i32 result, u64 la + bytes, u64 lb + bytes,
 *   u64 lexp + bytes (the expected image for merge / value).
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
            switch (c->op) {
            case 0: st = laspj_orset_etf_merge(ctx, c->a, c->la, c->b, c->lb, &out, &olen, &verdict); break;
            case 1: st = laspj_orset_etf_value(ctx, c->a, c->la, &out, &olen, &verdict); break;
            case 2: st = laspj_orset_etf_equal(ctx, c->a, c->la, c->b, c->lb, &result, &verdict); break;
            default:
                st = laspj_orset_etf_inflation(ctx, c->a, c->la, c->b, c->lb, c->op == 4,
                                               &result, &verdict);
            }
            if (st != LASPJ_OK) {
                snprintf(w->msg, sizeof w->msg, "thread %d case %u: status %d (%s)", w->tid, i, st,
                         laspj_ctx_last_error(ctx));
                w->fails++;
            } else if (verdict != c->verdict) {
                snprintf(w->msg, sizeof w->msg, "thread %d case %u: verdict %d, want %d", w->tid,
                         i, verdict, c->verdict);
                w->fails++;
            } else if (verdict == LASPJ_NIF_OK && c->op <= 1 &&
                       (olen != c->lexp || memcmp(out, c->exp, olen) != 0)) {
                snprintf(w->msg, sizeof w->msg, "thread %d case %u: image differs (%llu vs %llu B)",
                         w->tid, i, (unsigned long long)olen, (unsigned long long)c->lexp);
                w->fails++;
            } else if (verdict == LASPJ_NIF_OK && c->op >= 2 && result != c->result) {
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
