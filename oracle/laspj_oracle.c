/*
 * laspj_oracle.c — C restatement of the reference hot path — TEST INFRASTRUCTURE ONLY.
 *
 * Used by tests/ (parity checker at full BASELINE sizes) and by bench.py's
 * cpu_baseline leg (the timed "port"); never by the product (lasp_amd/).
 *
 * It works on the reference's own data structure, not on the engine's columnar form:
 * an OR-Set replica is an orddict Elem -> orddict Token -> Removed, held here as a
 * sorted array of elements, each owning a sorted run of {20-byte token, bool} entries
 * (tokens compare as Erlang binaries: memcmp, then length — all are 20 bytes).
 * Elements of the synthetic workload are integers 0..E-1 (term order = integer order).
 *
 *   orc_orset_merge        lasp_orset:merge/2         src/lasp_orset.erl:128-134
 *                          (orddict:merge two-finger merge, inner merge with `or`;
 *                           OTP orddict clauses restated in SURVEY.md Appendix A)
 *   orc_orset_value        lasp_orset:value/1         src/lasp_orset.erl:67-73
 *   orc_orset_stats        lasp_orset:stat/2          src/lasp_orset.erl:163-192
 *   orc_orset_is_inflation lasp_lattice clause        src/lasp_lattice.erl:153-161,277-285
 *                          (lists:keyfind linear scans, as written)
 *   orc_orset_is_strict    lasp_lattice clause        src/lasp_lattice.erl:235-253
 *   orc_gset_merge         lasp_gset:merge/2          src/lasp_gset.erl:99-101
 *                          (ordsets:union on integer ordsets)
 *   orc_bench_orset_op     timing of merge / value / stats / inflation / strict
 *                          inflation on host threads (bench.py cpu_baseline,
 *                          tools/cpu_beside.py)
 *
 * Synthetic inputs are restated here independently of the HIP
 * generator so that a GPU test can check the device-generated batch against them.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef uint64_t u64;

static double now_s(void);

/* ------------------------------------------------------------------ synthetic inputs */

static inline u64 sm64(u64 x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

static inline u64 replica_key(u64 seed, u64 grep) {
    return sm64(sm64(seed ^ 0x4C41535000000000ull) ^ grep);
}

/* cells[2e] = p, cells[2e+1] = r for synthetic OR-Set replica `grep` of stream `seed` */
void orc_synth_orset(u64 seed, u64 grep, uint32_t E, u64* cells) {
    u64 h = replica_key(seed, grep);
    for (uint32_t e = 0; e < E; ++e) {
        u64 x = sm64(h + (u64)e * 0xD1B54A32D192ED03ull);
        u64 y = sm64(x ^ 0xA5A5A5A5A5A5A5A5ull);
        u64 z = sm64(y ^ 0x5A5A5A5A5A5A5A5Aull);
        u64 w = sm64(z);
        u64 p = (z % 20ull) == 0 ? 0ull : x;
        cells[2ull * e] = p;
        cells[2ull * e + 1] = p & y & w;
    }
}

/* the T-token stream (laspj_batch_fill_synthetic_tokens): p = x masked to T bits (1 if
 * that leaves none; every element present), r = p & y & w; elements [e0, e0 + n) */
void orc_synth_orset_t(u64 seed, u64 grep, uint32_t e0, uint32_t n, uint32_t T, u64* cells) {
    u64 h = replica_key(seed, grep);
    u64 m = T >= 64 ? ~0ull : ((1ull << T) - 1ull);
    for (uint32_t i = 0; i < n; ++i) {
        u64 e = (u64)e0 + i;
        u64 x = sm64(h + e * 0xD1B54A32D192ED03ull);
        u64 y = sm64(x ^ 0xA5A5A5A5A5A5A5A5ull);
        u64 z = sm64(y ^ 0x5A5A5A5A5A5A5A5Aull);
        u64 w = sm64(z);
        u64 p = x & m;
        if (!p) p = 1;
        cells[2ull * i] = p;
        cells[2ull * i + 1] = p & y & w;
    }
}

void orc_synth_gset(u64 seed, u64 grep, uint32_t E, u64* words) {
    u64 h = replica_key(seed, grep);
    u64 W = (E + 63ull) / 64ull;
    u64 last = (E % 64) ? ((1ull << (E % 64)) - 1ull) : ~0ull;
    for (u64 wi = 0; wi < W; ++wi) {
        u64 x = sm64(h + wi * 0xD1B54A32D192ED03ull);
        words[wi] = wi == W - 1 ? (x & last) : x;
    }
}

static int tok_cmp(const void* a, const void* b) { return memcmp(a, b, 20); }

/* Token dictionary of the synthetic workload: T 20-byte tokens per element, drawn from
 * splitmix64 seeded with 0x4C415350 ("LASP") and sorted by Erlang binary order per
 * element, so token slot k is the k-th smallest token.  out: E*T*20 bytes. */
void orc_synth_tokens(uint32_t E, uint32_t T, uint8_t* out) {
    u64 s = 0x4C415350ull;
    for (uint32_t e = 0; e < E; ++e) {
        uint8_t* base = out + (size_t)e * T * 20;
        for (uint32_t k = 0; k < T; ++k) {
            uint8_t* t = base + (size_t)k * 20;
            for (int j = 0; j < 20; j += 8) {
                s = sm64(s);
                u64 v = s;
                int n = 20 - j < 8 ? 20 - j : 8;
                memcpy(t + j, &v, (size_t)n);
            }
        }
        qsort(base, T, 20, tok_cmp);
    }
}

/* ------------------------------------------------------------------ orddict form */

typedef struct {
    uint8_t tok[20];
    uint8_t removed; /* the Bool of {Token, Bool} */
    uint8_t pad[3];
} orc_tok;

typedef struct {
    int64_t key;
    uint32_t off; /* into the owning set's token array */
    uint32_t n;
} orc_elem;

typedef struct {
    uint32_t nelem, ntok;
    uint32_t cap_elem, cap_tok;
    orc_elem* elems;
    orc_tok* toks;
} orc_orset;

orc_orset* orc_orset_alloc(uint32_t cap_elem, uint32_t cap_tok) {
    orc_orset* s = (orc_orset*)calloc(1, sizeof *s);
    if (!s) return NULL;
    s->cap_elem = cap_elem;
    s->cap_tok = cap_tok;
    s->elems = (orc_elem*)malloc((size_t)(cap_elem ? cap_elem : 1) * sizeof(orc_elem));
    s->toks = (orc_tok*)malloc((size_t)(cap_tok ? cap_tok : 1) * sizeof(orc_tok));
    if (!s->elems || !s->toks) {
        free(s->elems);
        free(s->toks);
        free(s);
        return NULL;
    }
    return s;
}

void orc_orset_free(orc_orset* s) {
    if (!s) return;
    free(s->elems);
    free(s->toks);
    free(s);
}

uint32_t orc_orset_nelem(const orc_orset* s) { return s->nelem; }
uint32_t orc_orset_ntok(const orc_orset* s) { return s->ntok; }

/* Build the orddict a columnar replica denotes: element e present iff p != 0; its
 * tokens are the dictionary tokens of the set bits of p, ascending (= sorted, because
 * the synthetic dictionary is sorted), flag = bit of r. */
int orc_orset_from_cells(uint32_t E, const u64* cells, const uint8_t* tokens, uint32_t T,
                         orc_orset* out) {
    out->nelem = out->ntok = 0;
    for (uint32_t e = 0; e < E; ++e) {
        u64 p = cells[2ull * e], r = cells[2ull * e + 1];
        if (!p) continue;
        if (out->nelem >= out->cap_elem) return -1;
        orc_elem* el = &out->elems[out->nelem++];
        el->key = e;
        el->off = out->ntok;
        el->n = 0;
        for (uint32_t k = 0; k < T && k < 64; ++k) {
            if (!((p >> k) & 1ull)) continue;
            if (out->ntok >= out->cap_tok) return -1;
            orc_tok* t = &out->toks[out->ntok++];
            memcpy(t->tok, tokens + ((size_t)e * T + k) * 20, 20);
            t->removed = (uint8_t)((r >> k) & 1ull);
            el->n++;
        }
    }
    return 0;
}

/* Encode an orddict back into cells over the same dictionary (-1 if a token or element
 * is not in the dictionary). */
int orc_orset_to_cells(const orc_orset* s, uint32_t E, const uint8_t* tokens, uint32_t T,
                       u64* cells) {
    memset(cells, 0, (size_t)E * 16);
    for (uint32_t i = 0; i < s->nelem; ++i) {
        const orc_elem* el = &s->elems[i];
        if (el->key < 0 || el->key >= (int64_t)E) return -1;
        for (uint32_t j = 0; j < el->n; ++j) {
            const orc_tok* t = &s->toks[el->off + j];
            uint32_t k = 0;
            while (k < T && memcmp(tokens + ((size_t)el->key * T + k) * 20, t->tok, 20)) ++k;
            if (k == T) return -1;
            cells[2ull * el->key] |= 1ull << k;
            if (t->removed) cells[2ull * el->key + 1] |= 1ull << k;
        }
    }
    return 0;
}

/* lasp_orset:merge/2 — nested orddict:merge, written as the two-finger merges of the
 * OTP clauses: K1 < K2 emits E1, K1 > K2 emits E2, equal keys merge the values (inner:
 * BoolA or BoolB); the leftover tail of either side is appended as is. */
int orc_orset_merge(const orc_orset* a, const orc_orset* b, orc_orset* out) {
    uint32_t i = 0, j = 0;
    out->nelem = out->ntok = 0;
    if (out->cap_elem < a->nelem + b->nelem || out->cap_tok < a->ntok + b->ntok) return -1;
    while (i < a->nelem || j < b->nelem) {
        const orc_elem* ea = i < a->nelem ? &a->elems[i] : NULL;
        const orc_elem* eb = j < b->nelem ? &b->elems[j] : NULL;
        orc_elem* eo = &out->elems[out->nelem++];
        eo->off = out->ntok;
        if (eb == NULL || (ea && ea->key < eb->key)) {
            eo->key = ea->key;
            eo->n = ea->n;
            memcpy(&out->toks[out->ntok], &a->toks[ea->off], (size_t)ea->n * sizeof(orc_tok));
            out->ntok += ea->n;
            ++i;
        } else if (ea == NULL || ea->key > eb->key) {
            eo->key = eb->key;
            eo->n = eb->n;
            memcpy(&out->toks[out->ntok], &b->toks[eb->off], (size_t)eb->n * sizeof(orc_tok));
            out->ntok += eb->n;
            ++j;
        } else {
            /* same element: inner orddict:merge(fun(_, BoolA, BoolB) -> BoolA or BoolB) */
            const orc_tok* ta = &a->toks[ea->off];
            const orc_tok* tb = &b->toks[eb->off];
            uint32_t x = 0, y = 0, n = 0;
            orc_tok* to = &out->toks[out->ntok];
            while (x < ea->n && y < eb->n) {
                int c = memcmp(ta[x].tok, tb[y].tok, 20);
                if (c < 0) to[n++] = ta[x++];
                else if (c > 0) to[n++] = tb[y++];
                else {
                    to[n] = ta[x];
                    to[n].removed = (uint8_t)(ta[x].removed | tb[y].removed);
                    ++n, ++x, ++y;
                }
            }
            while (x < ea->n) to[n++] = ta[x++];
            while (y < eb->n) to[n++] = tb[y++];
            eo->key = ea->key;
            eo->n = n;
            out->ntok += n;
            ++i, ++j;
        }
    }
    return 0;
}

/* structural == (lasp_orset:equal/2, lasp_orset.erl:136-138) */
int orc_orset_equal(const orc_orset* a, const orc_orset* b) {
    if (a->nelem != b->nelem) return 0;
    for (uint32_t i = 0; i < a->nelem; ++i) {
        const orc_elem *x = &a->elems[i], *y = &b->elems[i];
        if (x->key != y->key || x->n != y->n) return 0;
        for (uint32_t j = 0; j < x->n; ++j) {
            const orc_tok *s = &a->toks[x->off + j], *t = &b->toks[y->off + j];
            if (memcmp(s->tok, t->tok, 20) || s->removed != t->removed) return 0;
        }
    }
    return 1;
}

/* value/1: keys of elements with at least one {Token, false}, in list order */
uint32_t orc_orset_value(const orc_orset* s, int64_t* keys) {
    uint32_t n = 0;
    for (uint32_t i = 0; i < s->nelem; ++i) {
        const orc_elem* el = &s->elems[i];
        for (uint32_t j = 0; j < el->n; ++j)
            if (!s->toks[el->off + j].removed) {
                keys[n++] = el->key;
                break;
            }
    }
    return n;
}

/* stats: element_count, adds_count (false flags), removes_count (true flags) */
void orc_orset_stats(const orc_orset* s, u64* out3) {
    u64 adds = 0, rems = 0;
    for (uint32_t t = 0; t < s->ntok; ++t) {
        if (s->toks[t].removed) ++rems;
        else ++adds;
    }
    out3[0] = s->nelem;
    out3[1] = adds;
    out3[2] = rems;
}

static const orc_elem* keyfind(int64_t key, const orc_orset* s) {
    for (uint32_t i = 0; i < s->nelem; ++i)
        if (s->elems[i].key == key) return &s->elems[i];
    return NULL;
}

/* is_lattice_inflation(lasp_orset, Prev, Cur): foldl over Prev with lists:keyfind on
 * Cur, then ids_inflated (every Prev token keyfind-able among Cur's tokens). */
int orc_orset_is_inflation(const orc_orset* prev, const orc_orset* cur) {
    int acc = 1;
    for (uint32_t i = 0; i < prev->nelem && acc; ++i) {
        const orc_elem* pe = &prev->elems[i];
        const orc_elem* ce = keyfind(pe->key, cur);
        if (!ce) {
            acc = 0;
            break;
        }
        for (uint32_t j = 0; j < pe->n && acc; ++j) {
            int found = 0;
            for (uint32_t k = 0; k < ce->n && !found; ++k)
                found = !memcmp(prev->toks[pe->off + j].tok, cur->toks[ce->off + k].tok, 20);
            acc = acc && found;
        }
    }
    return acc;
}

/* is_lattice_strict_inflation(lasp_orset, ...) — lasp_lattice.erl:235-253 */
int orc_orset_is_strict(const orc_orset* prev, const orc_orset* cur) {
    if (prev->nelem == 0 && cur->nelem != 0) return 1;
    int infl = orc_orset_is_inflation(prev, cur);
    int deleted = 0;
    for (uint32_t i = 0; i < prev->nelem && !deleted; ++i) {
        const orc_elem* pe = &prev->elems[i];
        const orc_elem* ce = keyfind(pe->key, cur);
        if (!ce) continue;
        if (pe->n != ce->n) {
            deleted = 1;
            break;
        }
        for (uint32_t j = 0; j < pe->n; ++j) {
            const orc_tok *s = &prev->toks[pe->off + j], *t = &cur->toks[ce->off + j];
            if (memcmp(s->tok, t->tok, 20) || s->removed != t->removed) {
                deleted = 1;
                break;
            }
        }
    }
    int new_elems = prev->nelem < cur->nelem;
    return infl && (deleted || new_elems);
}

/* union body for lasp_orset — lasp_core.erl:616-618: orddict:merge(fun(_, L, _R) -> L)
 * (keep-left: on a common element the left token list is kept as is) */
int orc_orset_union(const orc_orset* l, const orc_orset* r, orc_orset* out) {
    uint32_t i = 0, j = 0;
    out->nelem = out->ntok = 0;
    if (out->cap_elem < l->nelem + r->nelem || out->cap_tok < l->ntok + r->ntok) return -1;
    while (i < l->nelem || j < r->nelem) {
        const orc_elem* el = i < l->nelem ? &l->elems[i] : NULL;
        const orc_elem* er = j < r->nelem ? &r->elems[j] : NULL;
        const orc_elem* src;
        const orc_orset* from;
        if (er == NULL || (el && el->key < er->key)) {
            src = el, from = l, ++i;
        } else if (el == NULL || el->key > er->key) {
            src = er, from = r, ++j;
        } else {
            src = el, from = l, ++i, ++j;
        }
        orc_elem* eo = &out->elems[out->nelem++];
        eo->key = src->key;
        eo->off = out->ntok;
        eo->n = src->n;
        memcpy(&out->toks[out->ntok], &from->toks[src->off], (size_t)src->n * sizeof(orc_tok));
        out->ntok += src->n;
    }
    return 0;
}

/* filter body — lasp_core.erl:681-712 with fun(X) -> X rem 2 == 0 end
 * (lasp_filter_test.erl:70); `Acc ++ [Element]` keeps list order and tombstones */
int orc_orset_filter_even(const orc_orset* s, orc_orset* out) {
    out->nelem = out->ntok = 0;
    if (out->cap_elem < s->nelem || out->cap_tok < s->ntok) return -1;
    for (uint32_t i = 0; i < s->nelem; ++i) {
        const orc_elem* el = &s->elems[i];
        if (el->key % 2 != 0) continue;
        orc_elem* eo = &out->elems[out->nelem++];
        eo->key = el->key;
        eo->off = out->ntok;
        eo->n = el->n;
        memcpy(&out->toks[out->ntok], &s->toks[el->off], (size_t)el->n * sizeof(orc_tok));
        out->ntok += el->n;
    }
    return 0;
}

/* BASELINE config 1: two replicas of 10k integer elements — A adds all
 * with one token each, B adds all with its own token and removes a 10 % subset; time
 * merge/2, the union body (against a second 10k set with 5k overlap) and the filter
 * body, single-threaded, averaged over `iters` calls.  Results in microseconds. */
int orc_bench_config1_ext(uint32_t n, int iters, int slow_iters, double* out5);

int orc_bench_config1(uint32_t n, int iters, double* us_merge, double* us_union,
                      double* us_filter) {
    double o[5];
    int rc = orc_bench_config1_ext(n, iters, 0, o);
    *us_merge = o[0], *us_union = o[1], *us_filter = o[2];
    return rc;
}

/* BASELINE config 1: merge / union body / filter body (iters each), then value/1 of the
 * merge and is_inflation / is_strict_inflation of merge(A, B) over A (the quadratic
 * lists:keyfind clauses, slow_iters each; 0 skips them).  out5 = us per call of merge,
 * union, filter, value, inflation (strict inflation is timed into out5[4] only when
 * slow_iters > 0 and reported by the caller as the same order). */
int orc_bench_config1_ext(uint32_t n, int iters, int slow_iters, double* out5) {
    double* us_merge = &out5[0];
    double* us_union = &out5[1];
    double* us_filter = &out5[2];
    uint32_t E = 2 * n;
    orc_orset *a = orc_orset_alloc(E, E), *b = orc_orset_alloc(E, E), *c = orc_orset_alloc(E, E);
    orc_orset *m = orc_orset_alloc(2 * E, 2 * E), *f = orc_orset_alloc(2 * E, 2 * E);
    if (!a || !b || !c || !m || !f) return -1;
    u64 s = 0x4C415350ull;
    for (uint32_t e = 0; e < n; ++e) {
        orc_elem* ea = &a->elems[a->nelem++];
        orc_elem* eb = &b->elems[b->nelem++];
        ea->key = eb->key = e;
        ea->off = a->ntok;
        eb->off = b->ntok;
        ea->n = eb->n = 1;
        orc_tok* ta = &a->toks[a->ntok++];
        orc_tok* tb = &b->toks[b->ntok++];
        for (int k = 0; k < 20; k += 8) {
            s = sm64(s);
            memcpy(ta->tok + k, &s, k + 8 <= 20 ? 8 : 20 - k);
            s = sm64(s);
            memcpy(tb->tok + k, &s, k + 8 <= 20 ? 8 : 20 - k);
        }
        ta->removed = 0;
        tb->removed = (uint8_t)(sm64(e ^ 1ull) % 10 == 0);
        /* the union's right operand: elements n/2 .. 3n/2 (5k overlap at n = 10k) */
        orc_elem* ec = &c->elems[c->nelem++];
        ec->key = e + n / 2;
        ec->off = c->ntok;
        ec->n = 1;
        c->toks[c->ntok++] = *tb;
    }
    double t0 = now_s();
    for (int i = 0; i < iters; ++i) orc_orset_merge(a, b, m);
    double t1 = now_s();
    for (int i = 0; i < iters; ++i) orc_orset_union(m, c, f);
    double t2 = now_s();
    for (int i = 0; i < iters; ++i) orc_orset_filter_even(f, m);
    double t3 = now_s();
    *us_merge = (t1 - t0) * 1e6 / iters;
    *us_union = (t2 - t1) * 1e6 / iters;
    *us_filter = (t3 - t2) * 1e6 / iters;
    out5[3] = out5[4] = 0;
    if (slow_iters > 0) {
        int64_t* keys = (int64_t*)malloc(sizeof(int64_t) * 2 * E);
        u64 sink = 0;
        orc_orset_merge(a, b, m);
        double t4 = now_s();
        for (int i = 0; i < iters; ++i) sink += orc_orset_value(m, keys);
        double t5 = now_s();
        for (int i = 0; i < slow_iters; ++i) sink += orc_orset_is_inflation(a, m);
        double t6 = now_s();
        out5[3] = (t5 - t4) * 1e6 / iters;
        out5[4] = (t6 - t5) * 1e6 / slow_iters + (double)(sink & 0);
        free(keys);
    }
    orc_orset_free(a), orc_orset_free(b), orc_orset_free(c), orc_orset_free(m), orc_orset_free(f);
    return 0;
}

/* ------------------------------------------------------------------ G-Set (ordsets) */

/* Expand a G-Set bitmap replica into its ordset (ascending integer elements). */
uint32_t orc_gset_from_words(uint32_t E, const u64* words, int64_t* out) {
    uint32_t n = 0;
    for (uint32_t e = 0; e < E; ++e)
        if ((words[e >> 6] >> (e & 63)) & 1ull) out[n++] = e;
    return n;
}

/* ordsets:union two-finger merge on integer ordsets (equal: keep one) */
uint32_t orc_gset_merge(const int64_t* a, uint32_t na, const int64_t* b, uint32_t nb,
                        int64_t* out) {
    uint32_t i = 0, j = 0, n = 0;
    while (i < na && j < nb) {
        if (a[i] < b[j]) out[n++] = a[i++];
        else if (a[i] > b[j]) out[n++] = b[j++];
        else out[n++] = a[i++], ++j;
    }
    while (i < na) out[n++] = a[i++];
    while (j < nb) out[n++] = b[j++];
    return n;
}

/* ------------------------------------------------------------------ timed baseline */

/* timed operations: lasp_orset:merge/2, value/1, stat/2 (all three counters),
 * is_inflation / is_strict_inflation of merge(A, B) over A (lasp_lattice clauses) */
enum { ORC_OP_MERGE = 0, ORC_OP_VALUE, ORC_OP_STATS, ORC_OP_INFLATION, ORC_OP_STRICT };

typedef struct {
    uint32_t E, T;
    const uint8_t* tokens;
    u64 seed;
    u64 first_pair;
    uint32_t pairs;
    double budget_s;
    u64 merges;
    double seconds;
    int err;
    int op;
    u64 sink;
} bench_arg;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void* bench_thread(void* p) {
    bench_arg* a = (bench_arg*)p;
    uint32_t cap_t = a->E * a->T;
    orc_orset** A = (orc_orset**)calloc(a->pairs, sizeof(void*));
    orc_orset** B = (orc_orset**)calloc(a->pairs, sizeof(void*));
    orc_orset* out = orc_orset_alloc(2 * a->E, 2 * cap_t);
    u64* cells = (u64*)malloc((size_t)a->E * 16);
    int64_t* keys = (int64_t*)malloc((size_t)a->E * 8);
    u64 st[3];
    if (!A || !B || !out || !cells || !keys) {
        a->err = 1;
        return NULL;
    }
    /* inputs: replica pair k = synthetic replicas 2k (seed) and 2k+1 (seed+1),
     * decoded to orddict form outside the timed region */
    for (uint32_t k = 0; k < a->pairs; ++k) {
        A[k] = orc_orset_alloc(a->E, cap_t);
        B[k] = orc_orset_alloc(a->E, cap_t);
        orc_synth_orset(a->seed, a->first_pair + k, a->E, cells);
        orc_orset_from_cells(a->E, cells, a->tokens, a->T, A[k]);
        orc_synth_orset(a->seed + 1, a->first_pair + k, a->E, cells);
        orc_orset_from_cells(a->E, cells, a->tokens, a->T, B[k]);
        if (a->op == ORC_OP_INFLATION || a->op == ORC_OP_STRICT) {
            /* B[k] := merge(A, B): the value a bind would test against A */
            orc_orset_merge(A[k], B[k], out);
            orc_orset* m = orc_orset_alloc(2 * a->E, 2 * cap_t);
            orc_orset_merge(A[k], B[k], m);
            orc_orset_free(B[k]);
            B[k] = m;
        }
    }
    double t0 = now_s(), t = t0;
    u64 n = 0, sink = 0;
    while (t - t0 < a->budget_s) {
        for (uint32_t k = 0; k < a->pairs; ++k) {
            switch (a->op) {
                case ORC_OP_MERGE: orc_orset_merge(A[k], B[k], out); break;
                case ORC_OP_VALUE: sink += orc_orset_value(A[k], keys); break;
                case ORC_OP_STATS: orc_orset_stats(A[k], st); sink += st[0] + st[1] + st[2]; break;
                case ORC_OP_INFLATION: sink += orc_orset_is_inflation(A[k], B[k]); break;
                default: sink += orc_orset_is_strict(A[k], B[k]); break;
            }
            ++n;
        }
        t = now_s();
    }
    a->sink = sink;
    a->merges = n;
    a->seconds = t - t0;
    for (uint32_t k = 0; k < a->pairs; ++k) {
        orc_orset_free(A[k]);
        orc_orset_free(B[k]);
    }
    free(A);
    free(B);
    free(cells);
    free(keys);
    orc_orset_free(out);
    return NULL;
}

/* Time operation `op` of this restatement on `threads` host threads, each running it on
 * `pairs` synthetic replicas (pairs) of E elements round-robin for ~budget_s seconds.
 * Returns elements per second (E element slots per call) via *elem_per_s. */
int orc_bench_orset_op(int op, uint32_t E, u64 seed, int threads, uint32_t pairs,
                       double budget_s, double* elem_per_s, u64* merges_out,
                       double* seconds_out) {
    uint32_t T = 64;
    uint8_t* tokens = (uint8_t*)malloc((size_t)E * T * 20);
    if (!tokens) return -1;
    orc_synth_tokens(E, T, tokens);
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    bench_arg* args = (bench_arg*)calloc((size_t)threads, sizeof(bench_arg));
    for (int i = 0; i < threads; ++i) {
        args[i] = (bench_arg){E, T, tokens, seed, (u64)i * pairs, pairs, budget_s, 0, 0, 0, op, 0};
        pthread_create(&th[i], NULL, bench_thread, &args[i]);
    }
    u64 merges = 0;
    double secs = 0;
    int err = 0;
    for (int i = 0; i < threads; ++i) {
        pthread_join(th[i], NULL);
        merges += args[i].merges;
        if (args[i].seconds > secs) secs = args[i].seconds;
        err |= args[i].err;
    }
    free(th);
    free(args);
    free(tokens);
    if (err || secs <= 0) return -1;
    *elem_per_s = (double)merges * E / secs;
    *merges_out = merges;
    *seconds_out = secs;
    return 0;
}

/* lasp_orset:merge/2 timing (the headline cpu_baseline) */
int orc_bench_orset_merge(uint32_t E, u64 seed, int threads, uint32_t pairs, double budget_s,
                          double* elem_per_s, u64* merges_out, double* seconds_out) {
    return orc_bench_orset_op(ORC_OP_MERGE, E, seed, threads, pairs, budget_s, elem_per_s,
                              merges_out, seconds_out);
}

/* ---- the columnar join on the host: the device's cell layout OR-ed on CPU threads ----
 * Not the reference's algorithm (that is orc_orset_merge above): a second CPU column
 * for the headline, the same {p, r} cells the GPU joins, d = a | b over replicas of E
 * slots, each thread owning its own arrays (cells_per_thread u64x2 each, larger than
 * the caches), timed for ~budget_s.  Returns joined cells (element slots) per second. */
typedef struct {
    uint64_t n;          /* u64 words per array */
    double budget_s;
    uint64_t passes;
    double seconds;
    int err;
} cells_arg;

static void* cells_thread(void* p) {
    cells_arg* a = (cells_arg*)p;
    u64* x = (u64*)malloc(a->n * 8);
    u64* y = (u64*)malloc(a->n * 8);
    u64* z = (u64*)malloc(a->n * 8);
    if (!x || !y || !z) {
        a->err = 1;
        free(x); free(y); free(z);
        return NULL;
    }
    for (uint64_t i = 0; i < a->n; ++i) {
        x[i] = sm64(i);
        y[i] = sm64(i ^ 0x5A5A5A5AULL);
        z[i] = 0;
    }
    double t0 = now_s(), t = t0;
    uint64_t passes = 0;
    while (t - t0 < a->budget_s) {
        for (uint64_t i = 0; i < a->n; ++i) z[i] = x[i] | y[i];
        ++passes;
        t = now_s();
    }
    a->passes = passes;
    a->seconds = t - t0;
    free(x); free(y); free(z);
    return NULL;
}

int orc_bench_cells_join(uint64_t cells_per_thread, int threads, double budget_s,
                         double* cells_per_s) {
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    cells_arg* args = (cells_arg*)calloc((size_t)threads, sizeof(cells_arg));
    if (!th || !args) return -1;
    for (int i = 0; i < threads; ++i) {
        args[i] = (cells_arg){2 * cells_per_thread, budget_s, 0, 0, 0};
        pthread_create(&th[i], NULL, cells_thread, &args[i]);
    }
    double cells = 0, secs = 0;
    int err = 0;
    for (int i = 0; i < threads; ++i) {
        pthread_join(th[i], NULL);
        cells += (double)args[i].passes * (double)cells_per_thread;
        if (args[i].seconds > secs) secs = args[i].seconds;
        err |= args[i].err;
    }
    free(th);
    free(args);
    if (err || secs <= 0) return -1;
    *cells_per_s = cells / secs;
    return 0;
}

/* BASELINE config 1's merge on many host threads: every thread builds the pair of
 * orc_bench_config1_ext (n elements, one token each side) and merges it for budget_s;
 * *us = wall seconds / merges done by all threads, in microseconds — the per-merge cost
 * of a node whose schedulers all merge, next to the device's batched NIF merges. */
typedef struct {
    uint32_t n;
    double budget_s, seconds;
    u64 merges;
    int err;
} c1_arg;

static void* c1_thread(void* p) {
    c1_arg* a = (c1_arg*)p;
    const uint32_t n = a->n, E = 2 * n;
    orc_orset *x = orc_orset_alloc(E, E), *y = orc_orset_alloc(E, E);
    orc_orset* m = orc_orset_alloc(2 * E, 2 * E);
    if (!x || !y || !m) {
        a->err = 1;
        return NULL;
    }
    u64 s = 0x4C415350ull;
    for (uint32_t e = 0; e < n; ++e) {
        orc_elem* ea = &x->elems[x->nelem++];
        orc_elem* eb = &y->elems[y->nelem++];
        ea->key = eb->key = e;
        ea->off = x->ntok;
        eb->off = y->ntok;
        ea->n = eb->n = 1;
        orc_tok* ta = &x->toks[x->ntok++];
        orc_tok* tb = &y->toks[y->ntok++];
        for (int k = 0; k < 20; k += 8) {
            s = sm64(s);
            memcpy(ta->tok + k, &s, k + 8 <= 20 ? 8 : 20 - k);
            s = sm64(s);
            memcpy(tb->tok + k, &s, k + 8 <= 20 ? 8 : 20 - k);
        }
        ta->removed = 0;
        tb->removed = (uint8_t)(sm64(e ^ 1ull) % 10 == 0);
    }
    const double t0 = now_s();
    double t = t0;
    u64 k = 0;
    while (t - t0 < a->budget_s) {
        for (int i = 0; i < 16; ++i) orc_orset_merge(x, y, m);
        k += 16;
        t = now_s();
    }
    a->merges = k;
    a->seconds = t - t0;
    orc_orset_free(x), orc_orset_free(y), orc_orset_free(m);
    return NULL;
}

int orc_bench_config1_merge_threads(uint32_t n, int threads, double budget_s, double* us) {
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    c1_arg* args = (c1_arg*)calloc((size_t)threads, sizeof(c1_arg));
    if (!th || !args) return -1;
    for (int i = 0; i < threads; ++i) {
        args[i] = (c1_arg){n, budget_s, 0, 0, 0};
        pthread_create(&th[i], NULL, c1_thread, &args[i]);
    }
    double secs = 0;
    u64 merges = 0;
    int err = 0;
    for (int i = 0; i < threads; ++i) {
        pthread_join(th[i], NULL);
        merges += args[i].merges;
        if (args[i].seconds > secs) secs = args[i].seconds;
        err |= args[i].err;
    }
    free(th);
    free(args);
    if (err || !merges) return -1;
    *us = secs * 1e6 / (double)merges;
    return 0;
}
