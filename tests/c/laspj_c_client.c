/*
 * A C caller of liblaspj.so that uses nothing but include/laspj.h — what an Erlang NIF
 *  does on the drop-in boundary: create a context, batches of
 * replicas, merge/2, value/1, stats/1, is_inflation/3, update/3 through apply_ops,
 * and the error convention (negative status + laspj_ctx_last_error, no exceptions).
 * Checks every result on the host and prints "laspj C client OK".
 *   build: gcc -std=c11 -O2 -Iinclude tests/c/laspj_c_client.c -Llasp_amd -llaspj \
 *              -Wl,-rpath,<abs>/lasp_amd -o laspj_c_client
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "laspj.h"

#define CHECK(call)                                                                    \
    do {                                                                               \
        int st_ = (call);                                                              \
        if (st_ != LASPJ_OK) {                                                         \
            fprintf(stderr, "%s:%d: %s -> %d (%s): %s\n", __FILE__, __LINE__, #call,   \
                    st_, laspj_strerror(st_), ctx ? laspj_ctx_last_error(ctx) : "");   \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

#define EXPECT(cond)                                                                   \
    do {                                                                               \
        if (!(cond)) {                                                                 \
            fprintf(stderr, "%s:%d: expected %s\n", __FILE__, __LINE__, #cond);        \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

static int popc(uint64_t x) { return __builtin_popcountll(x); }

int main(void) {
    laspj_ctx* ctx = NULL;
    EXPECT(laspj_abi_version() == LASPJ_ABI_VERSION);
    int ndev = 0;
    CHECK(laspj_device_count(&ndev));
    EXPECT(ndev >= 1);
    CHECK(laspj_ctx_create(0, &ctx));

    enum { R = 8, E = 256, W = E / 64 };
    laspj_batch *a, *b, *c;
    CHECK(laspj_orset_batch_create(ctx, R, E, &a));
    CHECK(laspj_orset_batch_create(ctx, R, E, &b));
    CHECK(laspj_orset_batch_create(ctx, R, E, &c));
    CHECK(laspj_batch_fill_synthetic(ctx, a, 2, 0));
    CHECK(laspj_batch_fill_synthetic(ctx, b, 3, 0));

    /* merge/2 (lasp_orset.erl:128-134): p|p', r|r' */
    CHECK(laspj_orset_join(ctx, c, a, b));
    static uint64_t ha[R * E * 2], hb[R * E * 2], hc[R * E * 2];
    CHECK(laspj_batch_download(ctx, a, 0, R, ha));
    CHECK(laspj_batch_download(ctx, b, 0, R, hb));
    CHECK(laspj_batch_download(ctx, c, 0, R, hc));
    for (int i = 0; i < R * E * 2; ++i) EXPECT(hc[i] == (ha[i] | hb[i]));

    /* value/1, stats/1, is_inflation/3 of the merge over its inputs */
    laspj_buf *bits, *counts, *flags;
    CHECK(laspj_buf_create(ctx, (uint64_t)R * W * 8, &bits));
    CHECK(laspj_buf_create(ctx, (uint64_t)R * 24, &counts));
    CHECK(laspj_buf_create(ctx, R, &flags));
    CHECK(laspj_orset_value(ctx, c, bits));
    CHECK(laspj_orset_stats(ctx, c, counts));
    static uint64_t hbits[R * W], hcounts[R * 3];
    uint8_t hflags[R];
    CHECK(laspj_buf_download(ctx, bits, 0, hbits, sizeof hbits));
    CHECK(laspj_buf_download(ctx, counts, 0, hcounts, sizeof hcounts));
    for (int i = 0; i < R; ++i) {
        uint64_t elems = 0, adds = 0, rems = 0;
        for (int e = 0; e < E; ++e) {
            uint64_t p = hc[(i * E + e) * 2], r = hc[(i * E + e) * 2 + 1];
            int live = (p & ~r) != 0;
            EXPECT((int)((hbits[i * W + e / 64] >> (e % 64)) & 1u) == live);
            elems += p != 0;
            adds += popc(p & ~r);
            rems += popc(r);
        }
        EXPECT(hcounts[i * 3] == elems && hcounts[i * 3 + 1] == adds &&
               hcounts[i * 3 + 2] == rems);
    }
    CHECK(laspj_orset_inflation(ctx, a, c, 0, flags));
    CHECK(laspj_buf_download(ctx, flags, 0, hflags, R));
    for (int i = 0; i < R; ++i) EXPECT(hflags[i] == 1);

    /* update/3 (lasp_orset.erl:99-117): add slot 0 of element 5, then remove element 5
     * and element 6 (not present -> {error, {precondition, {not_present, 6}}}) */
    laspj_batch* s;
    CHECK(laspj_orset_batch_create(ctx, 1, E, &s));
    laspj_op ops[3];
    memset(ops, 0, sizeof ops);
    ops[0].replica = 0, ops[0].element = 5, ops[0].kind = LASPJ_OP_ADD, ops[0].slot = 0;
    ops[0].flags = LASPJ_OP_FLAG_NEW_CALL;
    ops[1].replica = 0, ops[1].element = 5, ops[1].kind = LASPJ_OP_REMOVE;
    ops[1].flags = LASPJ_OP_FLAG_NEW_CALL;
    ops[2].replica = 0, ops[2].element = 6, ops[2].kind = LASPJ_OP_REMOVE;
    ops[2].flags = LASPJ_OP_FLAG_NEW_CALL;
    int32_t status[3];
    CHECK(laspj_orset_apply_ops(ctx, s, ops, 3, status));
    EXPECT(status[0] == LASPJ_OPST_APPLIED && status[1] == LASPJ_OPST_APPLIED &&
           status[2] == LASPJ_OPST_NOT_PRESENT);
    static uint64_t hs[E * 2];
    CHECK(laspj_batch_download(ctx, s, 0, 1, hs));
    EXPECT(hs[5 * 2] == 1 && hs[5 * 2 + 1] == 1);

    /* the error convention: shapes that disagree are a status, not a crash */
    laspj_batch* odd;
    CHECK(laspj_orset_batch_create(ctx, R, E + 1, &odd));
    int st = laspj_orset_join(ctx, c, a, odd);
    EXPECT(st == LASPJ_E_SHAPE);
    EXPECT(strlen(laspj_ctx_last_error(ctx)) > 0);

    CHECK(laspj_ctx_synchronize(ctx));
    laspj_batch_destroy(odd);
    laspj_batch_destroy(s);
    laspj_buf_destroy(flags);
    laspj_buf_destroy(counts);
    laspj_buf_destroy(bits);
    laspj_batch_destroy(c);
    laspj_batch_destroy(b);
    laspj_batch_destroy(a);
    CHECK(laspj_ctx_destroy(ctx));
    printf("laspj C client OK\n");
    return 0;
}
