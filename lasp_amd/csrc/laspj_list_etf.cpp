// The combinator bodies and bind/3 on list values, from term_to_binary images
// (include/laspj.h "list bodies from images").  lasp_core's bodies (lasp_core.erl:460-712)
// bind lists that are not orddicts — intersection entries `{X, Cx ++ Cy}`, product pairs
// with reversed token pairs, reordered / repeated map and fold keys, the G-Set `L ++ R` —
// and every later re-run merges them with Type:merge run as written.  A NIF that keeps
// those values as Erlang terms calls these with their images: the image is walked into
// list items over a dictionary of this call's terms (laspj_host.cpp list_walk), the
// device's list kernels (laspj_lists.hip) run the body or the bind, and the answer's items
// are written back into an image (list_write), which the NIF hands to binary_to_term.
//
// A fun (map / filter / fold) is the caller's to evaluate: laspj_list_etf_args gives the
// distinct arguments the body would pass it, in first-appearance order, as the image of a
// list; the NIF maps the fun over that list in Erlang and passes the image of the results
// in the same order.  Each call is self-contained: the dictionary holds only its own terms
// (dense term-order ranks over them), so no state survives between calls but scratch.
// FALLBACK: a value that is not a proper list of {Key, [{Token, true|false}]} (OR-Set) /
// of terms (G-Set), a key with more than 64 distinct tokens, two `==`-equal terms under
// different images, a G-Set body over 2-tuple elements the reference runs its OR-Set
// branch on with a non-list causality (intersection, product) — the NIF then runs the
// reference's own body.

#include <algorithm>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "laspj_internal.h"

namespace laspj {

struct ListEtfState {
    std::mutex mu;
    std::string out;          // the last answer image (valid until the context's next call)
    uint64_t calls = 0;
};

namespace {

enum class LOp { ARGS, MAP, FILTER, FOLD, UNION, INTERSECTION, PRODUCT, BIND, VALUE };

ListEtfState* lstate(laspj_ctx* ctx) {
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (!ctx->listetf) ctx->listetf = new (std::nothrow) ListEtfState;
    return ctx->listetf;
}

int32_t list_kind(int32_t kind) {
    return kind == LASPJ_KIND_GSET ? LASPJ_KIND_GSET_LIST : LASPJ_KIND_ORSET_LIST;
}

// RAII owners of the ABI objects a call creates
struct Batch {
    laspj_batch* b = nullptr;
    ~Batch() {
        if (b) laspj_batch_destroy(b);
    }
};
struct Buf {
    laspj_buf* b = nullptr;
    ~Buf() {
        if (b) laspj_buf_destroy(b);
    }
};
struct Dict {
    laspj_dict* d = nullptr;
    ~Dict() {
        if (d) laspj_dict_destroy(d);
    }
};

int upload_list(laspj_ctx* ctx, int32_t kind, const ListItems& it, Batch* out) {
    const uint32_t n = (uint32_t)it.keys.size(), nt = (uint32_t)it.toks.size();
    if (int s = laspj_list_batch_create(ctx, list_kind(kind), 1, std::max(n, 1u),
                                        std::max(nt, 1u), &out->b))
        return s;
    return laspj_list_upload(ctx, out->b, 0, n, it.keys.data(), it.toff.data(),
                             nt ? it.toks.data() : nullptr);
}

int download_list(laspj_ctx* ctx, laspj_batch* b, ListItems* it) {
    uint32_t cnt[2] = {0, 0};
    if (int s = laspj_list_counts(ctx, b, cnt)) return s;
    it->keys.assign(std::max(cnt[0], 1u), 0);
    it->toff.assign(cnt[0] + 1ull, 0);
    it->toks.assign(std::max(cnt[1], 1u), 0);
    if (int s = laspj_list_download(ctx, b, 0, it->keys.data(), it->toff.data(), it->toks.data()))
        return s;
    it->keys.resize(cnt[0]);
    it->toks.resize(cnt[1]);
    return LASPJ_OK;
}

// the rank tables of the call's dictionary on the device
struct Order {
    Buf kr, gr;
    laspj_list_order o{};
};

int make_order(laspj_ctx* ctx, laspj_dict* dict, Order* ord) {
    std::vector<uint32_t> kr, gr;
    if (int s = list_ranks(dict, &kr, &gr)) return s;
    const uint32_t K = (uint32_t)std::max<size_t>(kr.size(), 1);
    kr.resize(K, 0);
    gr.resize(64ull * K, 0);
    if (int s = laspj_buf_create(ctx, 4ull * K, &ord->kr.b)) return s;
    if (int s = laspj_buf_create(ctx, 4ull * gr.size(), &ord->gr.b)) return s;
    if (int s = laspj_buf_upload(ctx, ord->kr.b, 0, kr.data(), 4ull * K)) return s;
    if (int s = laspj_buf_upload(ctx, ord->gr.b, 0, gr.data(), 4ull * gr.size())) return s;
    ord->o.krank = ord->kr.b;
    ord->o.nkeys = K;
    ord->o.grank = ord->gr.b;
    ord->o.ntokens = (uint32_t)gr.size();
    return LASPJ_OK;
}

int upload_table(laspj_ctx* ctx, const void* p, uint64_t bytes, Buf* out) {
    if (int s = laspj_buf_create(ctx, std::max<uint64_t>(bytes, 8), &out->b)) return s;
    return bytes ? laspj_buf_upload(ctx, out->b, 0, p, bytes) : LASPJ_OK;
}

// the distinct arguments in first-appearance order, and per element slot its index there
void distinct_args(const std::vector<uint32_t>& args, std::vector<uint32_t>* order,
                   std::vector<int64_t>* pos, uint32_t nslots) {
    pos->assign(nslots, -1);
    order->clear();
    for (uint32_t a : args)
        if ((*pos)[a] < 0) {
            (*pos)[a] = (int64_t)order->size();
            order->push_back(a);
        }
}

// the elements of a proper list image (131 + list) as term images (a STRING_EXT byte as
// the SMALL_INTEGER_EXT image it stands for)
bool list_terms(const uint8_t* p, uint64_t n, std::vector<std::string>* out) {
    out->clear();
    if (n < 2 || p[0] != 131 || list_term_len(p + 1, n - 1) != n - 1) return false;
    const uint8_t* t = p + 1;
    const size_t tn = n - 1;
    if (t[0] == 106) return true;
    if (t[0] == 107) {
        const uint32_t cnt = ((uint32_t)t[1] << 8) | t[2];
        for (uint32_t i = 0; i < cnt; ++i) out->push_back(std::string{(char)97, (char)t[3 + i]});
        return true;
    }
    if (t[0] != 108) return false;
    const uint32_t cnt = ((uint32_t)t[1] << 24) | ((uint32_t)t[2] << 16) | ((uint32_t)t[3] << 8) | t[4];
    size_t off = 5;
    for (uint32_t i = 0; i < cnt; ++i) {
        const size_t l = list_term_len(t + off, tn - off);
        if (!l) return false;
        out->emplace_back((const char*)t + off, l);
        off += l;
    }
    return off < tn && t[off] == 106;                    // a proper list
}

// `F(V) =:= true` on the result's image (any of the four atom encodings)
bool is_true(const std::string& v) {
    const uint8_t* p = (const uint8_t*)v.data();
    if (v.size() == 7 && (p[0] == 100 || p[0] == 118) && p[1] == 0 && p[2] == 4)
        return std::memcmp(p + 3, "true", 4) == 0;
    if (v.size() == 6 && (p[0] == 115 || p[0] == 119) && p[1] == 4)
        return std::memcmp(p + 2, "true", 4) == 0;
    return false;
}

// a 2-tuple element's parts {A, B}: A's image length (0: not a 2-tuple)
size_t pair_first(std::string_view img) {
    if (img.size() < 3 || (uint8_t)img[0] != 104 || (uint8_t)img[1] != 2) return 0;
    return list_term_len((const uint8_t*)img.data() + 2, img.size() - 2);
}

struct Args {
    const uint8_t* a = nullptr;
    uint64_t na = 0;
    const uint8_t* b = nullptr;         // second operand (union, ...) or the fun results
    uint64_t nb = 0;
};

// one call; *verdict OK / FALLBACK, st->out the answer image, *status for BIND
int body(laspj_ctx* ctx, ListEtfState* S, LOp op, int32_t kind, const Args& in, int32_t* status,
         int32_t* verdict) {
    Dict dict;
    if (laspj_dict_create(&dict.d) != LASPJ_OK) return LASPJ_E_NOMEM;
    *verdict = LASPJ_NIF_FALLBACK;
    const bool gset = kind == LASPJ_KIND_GSET;
    const bool fun = op == LOp::ARGS || op == LOp::MAP || op == LOp::FILTER || op == LOp::FOLD;
    ListItems x, y, z;
    std::vector<uint32_t> args;
    int st = list_walk(dict.d, kind, in.a, in.na, &x, fun ? &args : nullptr);
    if (st == LASPJ_E_NOMEM) return st;
    if (st != LASPJ_DEC_OK) return LASPJ_OK;
    const bool two = op == LOp::UNION || op == LOp::INTERSECTION || op == LOp::PRODUCT ||
                     op == LOp::BIND;
    if (two) {
        st = list_walk(dict.d, kind, in.b, in.nb, &y, nullptr);
        if (st == LASPJ_E_NOMEM) return st;
        if (st != LASPJ_DEC_OK) return LASPJ_OK;
    }
    // G-Set 2-tuple elements go down the bodies' OR-Set branch with a causality that is not
    // a token list: intersection (keyfind + ++) and product are the reference's to run
    if (gset && (op == LOp::INTERSECTION || op == LOp::PRODUCT))
        for (const ListItems* it : {&x, &y})
            for (uint64_t k : it->keys)
                if (pair_first(list_elem_image(dict.d, (uint32_t)k))) return LASPJ_OK;
    Batch bx, by, bz;
    if (op != LOp::ARGS) {
        if (int s = upload_list(ctx, kind, x, &bx)) return s;
        if (two)
            if (int s = upload_list(ctx, kind, y, &by)) return s;
        if (int s = laspj_list_batch_create(ctx, list_kind(kind), 1, 1, 1, &bz.b)) return s;
    }
    Order ord;
    const uint32_t K0 = list_dict_elements(dict.d);
    std::vector<uint32_t> dorder;
    std::vector<int64_t> pos;
    if (fun) distinct_args(args, &dorder, &pos, K0);
    std::vector<std::string> res;
    if ((op == LOp::MAP || op == LOp::FILTER || op == LOp::FOLD) &&
        (!list_terms(in.b, in.nb, &res) || res.size() != dorder.size()))
        return fail(ctx, LASPJ_E_INVAL, "list_etf: %zu fun results for %zu arguments",
                    res.size(), dorder.size());
    // per element slot of an entry: the argument's position and (G-Set 2-tuple) its tail
    auto tail_of = [&](uint32_t e) -> std::string_view {
        std::string_view img = list_elem_image(dict.d, e);
        const size_t l0 = gset ? pair_first(img) : 0;
        return l0 ? img.substr(2 + l0) : std::string_view();
    };
    auto out_key = [&](const std::string& v, std::string_view tail, uint64_t* key) -> int {
        std::string t = v;
        if (!tail.empty()) {
            std::string u{(char)104, (char)2};
            u += t;
            u.append(tail.data(), tail.size());
            t.swap(u);
        }
        uint32_t slot = 0;
        const int s = list_register(dict.d, (const uint8_t*)t.data(), t.size(), &slot);
        *key = slot;
        return s;
    };
    switch (op) {
    case LOp::ARGS: {
        // the distinct arguments as a list image
        x.keys.assign(dorder.begin(), dorder.end());
        x.toff.assign(x.keys.size() + 1, 0);
        x.toks.clear();
        if (int s = list_write(dict.d, LASPJ_KIND_GSET, x, &S->out)) return s;
        *verdict = LASPJ_NIF_OK;
        return LASPJ_OK;
    }
    case LOp::MAP:
    case LOp::FILTER:
    case LOp::FOLD: {
        // tables per element slot of the input's entries (per_entry = 0)
        Buf t1, t2;
        const uint32_t nidx = K0;
        std::vector<uint64_t> keys(nidx, 0);
        std::vector<uint8_t> keep(nidx, 0);
        std::vector<uint32_t> off(nidx + 1ull, 0);
        std::vector<uint64_t> fk;
        std::vector<char> seen(nidx, 0);
        // per slot, the position of its argument's result (the fold below reads it)
        std::vector<int64_t> argpos(nidx, -1);
        for (size_t i = 0; i < x.keys.size(); ++i) {
            const uint32_t e = (uint32_t)x.keys[i];
            if (seen[e]) continue;
            seen[e] = 1;
            const int64_t p = pos[args[i]];
            argpos[e] = p;
            std::string_view tail = tail_of(e);
            if (op == LOp::FILTER) {
                keep[e] = is_true(res[(size_t)p]) ? 1 : 0;
            } else if (op == LOp::MAP) {
                if (int s = out_key(res[(size_t)p], tail, &keys[e])) {
                    if (s == LASPJ_E_NOMEM) return s;
                    return LASPJ_OK;                      // FALLBACK
                }
            }
        }
        if (op == LOp::FOLD) {
            // keys of slot e: off[e] .. off[e + 1]
            for (uint32_t e = 0; e < nidx; ++e) {
                off[e] = (uint32_t)fk.size();
                if (!seen[e]) continue;
                const int64_t p = argpos[e];
                const std::string img = std::string(1, (char)131) + res[(size_t)p];
                std::vector<std::string> vs;
                if (!list_terms((const uint8_t*)img.data(), img.size(), &vs))
                    return fail(ctx, LASPJ_E_INVAL, "list_etf_fold: a result is not a list");
                std::string_view tail = tail_of(e);
                for (const std::string& v : vs) {
                    uint64_t k = 0;
                    if (int s = out_key(v, tail, &k)) {
                        if (s == LASPJ_E_NOMEM) return s;
                        return LASPJ_OK;
                    }
                    fk.push_back(k);
                }
            }
            off[nidx] = (uint32_t)fk.size();
        }
        int s = LASPJ_OK;
        if (op == LOp::MAP) {
            if ((s = upload_table(ctx, keys.data(), 8ull * nidx, &t1))) return s;
            s = laspj_list_map(ctx, bz.b, bx.b, t1.b, nidx, 0);
        } else if (op == LOp::FILTER) {
            if ((s = upload_table(ctx, keep.data(), nidx, &t1))) return s;
            s = laspj_list_filter(ctx, bz.b, bx.b, t1.b, nidx, 0);
        } else {
            if ((s = upload_table(ctx, off.data(), 4ull * (nidx + 1), &t1))) return s;
            if ((s = upload_table(ctx, fk.data(), 8ull * fk.size(), &t2))) return s;
            s = laspj_list_fold(ctx, bz.b, bx.b, t1.b, t2.b, nidx, 0);
        }
        if (s) return s;
        break;
    }
    case LOp::UNION:
        if (int s = make_order(ctx, dict.d, &ord)) return s;
        if (int s = laspj_list_union(ctx, bz.b, bx.b, by.b, &ord.o)) return s;
        break;
    case LOp::INTERSECTION:
        if (int s = make_order(ctx, dict.d, &ord)) return s;
        if (int s = laspj_list_intersection(ctx, bz.b, bx.b, by.b, &ord.o)) return s;
        break;
    case LOp::PRODUCT:
        if (int s = laspj_list_product(ctx, bz.b, bx.b, by.b)) return s;
        break;
    case LOp::VALUE:
        if (gset) {
            S->out.assign((const char*)in.a, in.na);      // ordsets:to_list: the identity
            *verdict = LASPJ_NIF_OK;
            return LASPJ_OK;
        }
        {
            Batch bv;                                      // value/1 is a G-Set list
            if (int s = laspj_list_batch_create(ctx, LASPJ_KIND_GSET_LIST, 1, 1, 1, &bv.b)) return s;
            if (int s = laspj_list_value(ctx, bv.b, bx.b)) return s;
            if (int s = download_list(ctx, bv.b, &z)) return s;
        }
        if (int s = list_write(dict.d, LASPJ_KIND_GSET, z, &S->out)) return s;
        *verdict = LASPJ_NIF_OK;
        return LASPJ_OK;
    case LOp::BIND: {
        if (int s = make_order(ctx, dict.d, &ord)) return s;
        uint8_t stb = 0;
        if (int s = laspj_list_bind(ctx, bz.b, bx.b, by.b, &ord.o, &stb)) return s;
        *status = stb;
        if (stb != 1) {
            S->out.clear();
            *verdict = LASPJ_NIF_OK;
            return LASPJ_OK;
        }
        break;
    }
    }
    if (int s = download_list(ctx, bz.b, &z)) return s;
    if (int s = list_write(dict.d, kind, z, &S->out)) return s;
    *verdict = LASPJ_NIF_OK;
    return LASPJ_OK;
}

int entry(laspj_ctx* ctx, LOp op, int32_t kind, const Args& in, const uint8_t** out,
          uint64_t* out_len, int32_t* status, int32_t* verdict) {
    if (!ctx) return LASPJ_E_INVAL;
    if (kind != LASPJ_KIND_ORSET && kind != LASPJ_KIND_GSET)
        return fail(ctx, LASPJ_E_KIND, "list_etf: OR-Set or G-Set lists");
    if (!verdict || !out || !out_len || (op == LOp::BIND && !status) || (!in.a && in.na) ||
        (!in.b && in.nb))
        return fail(ctx, LASPJ_E_INVAL, "list_etf: null argument");
    ListEtfState* S = lstate(ctx);
    if (!S) return fail(ctx, LASPJ_E_NOMEM, "list_etf: state allocation");
    std::lock_guard<std::mutex> lk(S->mu);
    ++S->calls;
    int32_t stv = 0;
    int s;
    try {
        s = body(ctx, S, op, kind, in, &stv, verdict);
    } catch (const std::bad_alloc&) {
        s = fail(ctx, LASPJ_E_NOMEM, "list_etf: host allocation");
    }
    if (s) return s;
    if (status) *status = stv;
    const bool answer = *verdict == LASPJ_NIF_OK && !(op == LOp::BIND && stv != 1);
    *out = answer ? reinterpret_cast<const uint8_t*>(S->out.data()) : nullptr;
    *out_len = answer ? S->out.size() : 0;
    return LASPJ_OK;
}

}  // namespace

void list_etf_destroy(laspj_ctx* ctx) {
    delete ctx->listetf;
    ctx->listetf = nullptr;
}

}  // namespace laspj

using laspj::Args;
using laspj::LOp;

extern "C" {

int laspj_list_etf_args(laspj_ctx* ctx, int32_t kind, const uint8_t* v, uint64_t nv,
                        const uint8_t** out, uint64_t* out_len, int32_t* verdict) {
    return laspj::entry(ctx, LOp::ARGS, kind, Args{v, nv, nullptr, 0}, out, out_len, nullptr,
                        verdict);
}

int laspj_list_etf_map(laspj_ctx* ctx, int32_t kind, const uint8_t* v, uint64_t nv,
                       const uint8_t* results, uint64_t nr, const uint8_t** out,
                       uint64_t* out_len, int32_t* verdict) {
    return laspj::entry(ctx, LOp::MAP, kind, Args{v, nv, results, nr}, out, out_len, nullptr,
                        verdict);
}

int laspj_list_etf_filter(laspj_ctx* ctx, int32_t kind, const uint8_t* v, uint64_t nv,
                          const uint8_t* results, uint64_t nr, const uint8_t** out,
                          uint64_t* out_len, int32_t* verdict) {
    return laspj::entry(ctx, LOp::FILTER, kind, Args{v, nv, results, nr}, out, out_len, nullptr,
                        verdict);
}

int laspj_list_etf_fold(laspj_ctx* ctx, int32_t kind, const uint8_t* v, uint64_t nv,
                        const uint8_t* results, uint64_t nr, const uint8_t** out,
                        uint64_t* out_len, int32_t* verdict) {
    return laspj::entry(ctx, LOp::FOLD, kind, Args{v, nv, results, nr}, out, out_len, nullptr,
                        verdict);
}

int laspj_list_etf_union(laspj_ctx* ctx, int32_t kind, const uint8_t* l, uint64_t nl,
                         const uint8_t* r, uint64_t nr, const uint8_t** out, uint64_t* out_len,
                         int32_t* verdict) {
    return laspj::entry(ctx, LOp::UNION, kind, Args{l, nl, r, nr}, out, out_len, nullptr,
                        verdict);
}

int laspj_list_etf_intersection(laspj_ctx* ctx, int32_t kind, const uint8_t* l, uint64_t nl,
                                const uint8_t* r, uint64_t nr, const uint8_t** out,
                                uint64_t* out_len, int32_t* verdict) {
    return laspj::entry(ctx, LOp::INTERSECTION, kind, Args{l, nl, r, nr}, out, out_len, nullptr,
                        verdict);
}

int laspj_list_etf_product(laspj_ctx* ctx, int32_t kind, const uint8_t* l, uint64_t nl,
                           const uint8_t* r, uint64_t nr, const uint8_t** out, uint64_t* out_len,
                           int32_t* verdict) {
    return laspj::entry(ctx, LOp::PRODUCT, kind, Args{l, nl, r, nr}, out, out_len, nullptr,
                        verdict);
}

int laspj_list_etf_value(laspj_ctx* ctx, int32_t kind, const uint8_t* v, uint64_t nv,
                         const uint8_t** out, uint64_t* out_len, int32_t* verdict) {
    return laspj::entry(ctx, LOp::VALUE, kind, Args{v, nv, nullptr, 0}, out, out_len, nullptr,
                        verdict);
}

int laspj_list_etf_bind(laspj_ctx* ctx, int32_t kind, const uint8_t* value0, uint64_t n0,
                        const uint8_t* value, uint64_t n, const uint8_t** out, uint64_t* out_len,
                        int32_t* status, int32_t* verdict) {
    return laspj::entry(ctx, LOp::BIND, kind, Args{value0, n0, value, n}, out, out_len, status,
                        verdict);
}

}  // extern "C"
