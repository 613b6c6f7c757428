// Wire codec: `to_binary/1` payloads of every replica of a batch, written on the device
// (lasp_orset.erl:198-200, lasp_gset.erl:111-113).
//
// A payload is <<Tag, Vers>> (optional) ++ term_to_binary(State): the external term
// format image of the replica's orddict [{Elem, [{Token, Bool}]}] (or G-Set ordset).
// Each dictionary term's own image comes from the host once per distinct term; the
// device assembles replicas from cells:
//
//   element   104 2  <elem image>  108 <n:32>  {104 2 <token image> <atom>}*n  106
//   atom      true = 100 0 4 "true" (7 B), false = 100 0 5 "false" (8 B)   (ATOM_EXT)
//   OR-Set    131 108 <n:32> element* 106    |  131 106 when empty
//   G-Set     131 107 <n:16> byte*  (every element a 0..255 integer, n < 65536: STRING_EXT)
//             131 108 <n:32> <elem image>* 106  |  131 106 when empty
//
// Two launches: k_*_etf_size (one wave per replica: payload size, dictionary check)
// feeding a device exclusive scan (hipcub) into the caller's offsets, then
// k_*_etf_write (one 256-thread block per replica: elements in term order, a block
// scan of their sizes gives every thread its output position).  The path is
// write-bound: a payload is ~15-70x the bytes of its cells.

#include <hipcub/hipcub.hpp>

#include <new>
#include <vector>

#include "laspj_internal.h"

struct laspj_etf_dict {
    laspj_ctx* ctx = nullptr;
    uint32_t elements = 0;
    bool has_tokens = false;
    uint32_t tok_uniform = 0;     // every used token image has this length (0: mixed)
    void* block = nullptr;        // one device allocation holding the arrays below
    const uint8_t* elem_blob = nullptr;
    const uint32_t* elem_off = nullptr;    // E + 1
    const uint32_t* elem_order = nullptr;  // E
    const uint8_t* elem_byte = nullptr;    // E: 1 = image is SMALL_INTEGER_EXT (97, v)
    const uint8_t* tok_blob = nullptr;
    const uint32_t* tok_off = nullptr;     // 64E + 1
    const uint8_t* tok_order = nullptr;    // 64E
    const uint64_t* tok_mask = nullptr;    // E: token slots with an image
};

namespace laspj {
namespace {

typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

constexpr int kBlock = 256;

struct DictView {
    const uint8_t* elem_blob;
    const uint32_t* elem_off;
    const uint32_t* elem_order;
    const uint8_t* elem_byte;
    const uint8_t* tok_blob;
    const uint32_t* tok_off;
    const uint8_t* tok_order;
    const uint64_t* tok_mask;
    uint32_t tok_uniform;
};

DictView view(const laspj_etf_dict* d) {
    return {d->elem_blob, d->elem_off, d->elem_order, d->elem_byte, d->tok_blob,
            d->tok_off, d->tok_order, d->tok_mask, d->tok_uniform};
}

__device__ __forceinline__ u64 wave_sum(u64 v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// bytes of one present OR-Set element: 104 2 <elem> 108 <n:32> tokens 106
__device__ __forceinline__ uint32_t orset_elem_size(const DictView& d, uint32_t e, u64 p,
                                                    u64 r) {
    uint32_t el = d.elem_off[e + 1] - d.elem_off[e];
    uint32_t tl;
    if (d.tok_uniform) {
        tl = (uint32_t)__popcll(p) * d.tok_uniform;
    } else {
        tl = 0;
        for (u64 m = p; m; m &= m - 1) {
            uint32_t k = 64u * e + (uint32_t)__ffsll((long long)m) - 1u;
            tl += d.tok_off[k + 1] - d.tok_off[k];
        }
    }
    // per token: 104 2 (2) + atom (8 for false, 7 for true) + image
    return 2u + el + 5u + 1u + 10u * (uint32_t)__popcll(p) - (uint32_t)__popcll(r & p) + tl;
}

__global__ __launch_bounds__(kBlock) void k_orset_etf_size(const u64x2* cells, uint64_t R,
                                                           uint32_t E, DictView d, uint32_t hdr,
                                                           u64* sizes, uint32_t* flag) {
    const int lane = threadIdx.x & 63;
    const uint64_t waves = (uint64_t)gridDim.x * (kBlock / 64);
    for (uint64_t rep = (uint64_t)blockIdx.x * (kBlock / 64) + threadIdx.x / 64; rep < R;
         rep += waves) {
        const u64x2* c = cells + rep * E;
        u64 sum = 0, n = 0;
        bool bad = false;
        for (uint32_t e = lane; e < E; e += 64) {
            u64x2 v = c[e];
            if (!v.x) continue;
            ++n;
            bad |= d.elem_off[e + 1] == d.elem_off[e] || (v.x & ~d.tok_mask[e]) != 0;
            if (!bad) sum += orset_elem_size(d, e, v.x, v.y);
        }
        sum = wave_sum(sum);
        n = wave_sum(n);
        bool any_bad = __ballot(bad) != 0;
        if (lane == 0) {
            sizes[rep] = hdr + 1u + (n ? 5u + sum + 1u : 1u);
            if (any_bad) atomicOr(flag, 1u);
        }
    }
}

// block-wide exclusive scan of one value per thread (256 threads = 4 waves)
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* lds4,
                                                    uint32_t* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    if (lane == 63) lds4[w] = x;
    __syncthreads();
    uint32_t before = 0, all = 0;
#pragma unroll
    for (int i = 0; i < kBlock / 64; ++i) {
        uint32_t s = lds4[i];
        if (i < w) before += s;
        all += s;
    }
    __syncthreads();
    *total = all;
    return before + x - v;
}

__device__ __forceinline__ uint8_t* put_bytes(uint8_t* o, const uint8_t* src, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i) o[i] = src[i];
    return o + n;
}

__device__ __forceinline__ uint8_t* put_be32(uint8_t* o, uint32_t v) {
    o[0] = (uint8_t)(v >> 24);
    o[1] = (uint8_t)(v >> 16);
    o[2] = (uint8_t)(v >> 8);
    o[3] = (uint8_t)v;
    return o + 4;
}

__device__ __forceinline__ uint8_t* put_atom_bool(uint8_t* o, bool t) {
    o[0] = 100;
    o[1] = 0;
    if (t) {
        o[2] = 4; o[3] = 't'; o[4] = 'r'; o[5] = 'u'; o[6] = 'e';
        return o + 7;
    }
    o[2] = 5; o[3] = 'f'; o[4] = 'a'; o[5] = 'l'; o[6] = 's'; o[7] = 'e';
    return o + 8;
}

__device__ void orset_elem_write(const DictView& d, uint32_t e, u64 p, u64 r, uint8_t* o) {
    o[0] = 104;
    o[1] = 2;
    o = put_bytes(o + 2, d.elem_blob + d.elem_off[e], d.elem_off[e + 1] - d.elem_off[e]);
    o[0] = 108;
    o = put_be32(o + 1, (uint32_t)__popcll(p));
    const uint8_t* ord = d.tok_order + 64u * e;
    for (int j = 0; j < 64; ++j) {
        uint32_t k = ord[j];
        if (k >= 64) break;
        if (!((p >> k) & 1ull)) continue;
        o[0] = 104;
        o[1] = 2;
        uint32_t t = 64u * e + k;
        o = put_bytes(o + 2, d.tok_blob + d.tok_off[t], d.tok_off[t + 1] - d.tok_off[t]);
        o = put_atom_bool(o, (r >> k) & 1ull);
    }
    o[0] = 106;
}

__global__ __launch_bounds__(kBlock) void k_orset_etf_write(const u64x2* cells, uint64_t R,
                                                            uint32_t E, DictView d, int tag,
                                                            int vers, const u64* offs,
                                                            uint8_t* out) {
    __shared__ uint32_t lds4[kBlock / 64];
    const uint32_t hdr = tag >= 0 ? 2u : 0u;
    for (uint64_t rep = blockIdx.x; rep < R; rep += gridDim.x) {
        const u64x2* c = cells + rep * E;
        const u64 base = offs[rep], end = offs[rep + 1];
        u64 cursor = base + hdr + 6u;
        uint32_t n = 0;
        for (uint32_t c0 = 0; c0 < E; c0 += kBlock) {
            uint32_t i = c0 + threadIdx.x;
            uint32_t e = i < E ? d.elem_order[i] : 0u;
            u64x2 v = i < E ? c[e] : u64x2{0, 0};
            uint32_t sz = v.x ? orset_elem_size(d, e, v.x, v.y) : 0u;
            uint32_t tot, cnt;
            uint32_t pos = block_excl_scan(sz, lds4, &tot);
            block_excl_scan(v.x ? 1u : 0u, lds4, &cnt);
            if (v.x && cursor + pos + sz <= end) orset_elem_write(d, e, v.x, v.y, out + cursor + pos);
            cursor += tot;
            n += cnt;
        }
        if (threadIdx.x == 0) {
            uint8_t* o = out + base;
            if (hdr) {
                o[0] = (uint8_t)tag;
                o[1] = (uint8_t)vers;
            }
            o[hdr] = 131;
            if (n) {
                o[hdr + 1] = 108;
                put_be32(o + hdr + 2, n);
                if (cursor < end) out[cursor] = 106;
            } else {
                o[hdr + 1] = 106;
            }
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(kBlock) void k_gset_etf_size(const u64* words, uint64_t R,
                                                          uint32_t E, uint32_t W, DictView d,
                                                          uint32_t hdr, u64* sizes,
                                                          uint32_t* flag) {
    const int lane = threadIdx.x & 63;
    const uint64_t waves = (uint64_t)gridDim.x * (kBlock / 64);
    for (uint64_t rep = (uint64_t)blockIdx.x * (kBlock / 64) + threadIdx.x / 64; rep < R;
         rep += waves) {
        const u64* w = words + rep * W;
        u64 sum = 0, n = 0;
        bool bad = false, allbyte = true;
        for (uint32_t wi = lane; wi < W; wi += 64) {
            for (u64 m = w[wi]; m; m &= m - 1) {
                uint32_t e = 64u * wi + (uint32_t)__ffsll((long long)m) - 1u;
                if (e >= E) { bad = true; break; }
                uint32_t el = d.elem_off[e + 1] - d.elem_off[e];
                bad |= el == 0;
                allbyte &= d.elem_byte[e] != 0;
                sum += el;
                ++n;
            }
        }
        sum = wave_sum(sum);
        n = wave_sum(n);
        bool any_bad = __ballot(bad) != 0, every_byte = __ballot(!allbyte) == 0;
        if (lane == 0) {
            u64 body = n == 0 ? 1u : (every_byte && n < 65536u) ? 3u + n : 5u + sum + 1u;
            sizes[rep] = hdr + 1u + body;
            if (any_bad) atomicOr(flag, 1u);
        }
    }
}

__global__ __launch_bounds__(kBlock) void k_gset_etf_write(const u64* words, uint64_t R,
                                                           uint32_t E, uint32_t W, DictView d,
                                                           int tag, int vers, const u64* offs,
                                                           uint8_t* out) {
    __shared__ uint32_t lds4[kBlock / 64];
    const uint32_t hdr = tag >= 0 ? 2u : 0u;
    for (uint64_t rep = blockIdx.x; rep < R; rep += gridDim.x) {
        const u64* w = words + rep * W;
        const u64 base = offs[rep], end = offs[rep + 1];
        // pass 1: element count and whether STRING_EXT applies
        uint32_t n_part = 0, nonbyte_part = 0;
        for (uint32_t wi = threadIdx.x; wi < W; wi += kBlock) {
            for (u64 m = w[wi]; m; m &= m - 1) {
                uint32_t e = 64u * wi + (uint32_t)__ffsll((long long)m) - 1u;
                ++n_part;
                nonbyte_part += e >= E || d.elem_byte[e] == 0;
            }
        }
        uint32_t n, nonbyte;
        block_excl_scan(n_part, lds4, &n);
        block_excl_scan(nonbyte_part, lds4, &nonbyte);
        const bool str = n > 0 && nonbyte == 0 && n < 65536u;
        u64 cursor = base + hdr + 1u + (str ? 3u : 5u);
        for (uint32_t c0 = 0; c0 < E && n; c0 += kBlock) {
            uint32_t i = c0 + threadIdx.x;
            uint32_t e = i < E ? d.elem_order[i] : 0u;
            bool here = i < E && ((w[e >> 6] >> (e & 63u)) & 1ull);
            uint32_t el = d.elem_off[e + 1] - d.elem_off[e];
            uint32_t sz = here ? (str ? 1u : el) : 0u;
            uint32_t tot;
            uint32_t pos = block_excl_scan(sz, lds4, &tot);
            if (here && cursor + pos + sz <= end) {
                const uint8_t* src = d.elem_blob + d.elem_off[e];
                if (str) out[cursor + pos] = src[1];
                else put_bytes(out + cursor + pos, src, el);
            }
            cursor += tot;
        }
        if (threadIdx.x == 0) {
            uint8_t* o = out + base;
            if (hdr) {
                o[0] = (uint8_t)tag;
                o[1] = (uint8_t)vers;
            }
            o[hdr] = 131;
            if (n == 0) {
                o[hdr + 1] = 106;
            } else if (str) {
                o[hdr + 1] = 107;
                o[hdr + 2] = (uint8_t)(n >> 8);
                o[hdr + 3] = (uint8_t)n;
            } else {
                o[hdr + 1] = 108;
                put_be32(o + hdr + 2, n);
                if (cursor < end) out[cursor] = 106;
            }
        }
        __syncthreads();
    }
}

struct Guard {
    std::lock_guard<std::mutex> lk;
    explicit Guard(laspj_ctx* c) : lk(c->mu) { hipSetDevice(c->device); }
};

int reserve_scratch(laspj_ctx* ctx, uint64_t need) {
    if (ctx->scratch_bytes >= need) return LASPJ_OK;
    if (ctx->scratch) {
        LJ_HIP(ctx, hipStreamSynchronize(ctx->stream));
        hipFree(ctx->scratch);
        ctx->scratch = nullptr;
        ctx->scratch_bytes = 0;
    }
    if (hipMalloc(&ctx->scratch, need) != hipSuccess) {
        hipGetLastError();
        return fail(ctx, LASPJ_E_NOMEM, "etf: scratch allocation of %llu bytes",
                    (unsigned long long)need);
    }
    ctx->scratch_bytes = need;
    return LASPJ_OK;
}

int check_args(laspj_ctx* ctx, const laspj_batch* b, const laspj_etf_dict* d, int32_t kind,
               const char* what) {
    if (!ctx || !b || b->ctx != ctx || !d || d->ctx != ctx)
        return fail(ctx, LASPJ_E_INVAL, "%s: null handle or handle of another context", what);
    if (b->kind != kind) return fail(ctx, LASPJ_E_KIND, "%s: wrong batch kind %d", what, b->kind);
    if (d->elements != b->elements)
        return fail(ctx, LASPJ_E_SHAPE, "%s: dictionary has %u element slots, batch %u", what,
                    d->elements, b->elements);
    if (kind == LASPJ_KIND_ORSET && !d->has_tokens)
        return fail(ctx, LASPJ_E_INVAL, "%s: dictionary has no token images", what);
    return LASPJ_OK;
}

int etf_size(laspj_ctx* ctx, const laspj_batch* b, const laspj_etf_dict* d, int tag,
             laspj_buf* offsets, uint64_t* total, int32_t kind, const char* what) {
    if (int s = check_args(ctx, b, d, kind, what)) return s;
    if (!offsets || offsets->ctx != ctx || offsets->bytes < 8ull * (b->replicas + 1) || !total)
        return fail(ctx, LASPJ_E_RANGE, "%s: offsets must hold replicas + 1 uint64", what);
    Guard g(ctx);
    const uint64_t R = b->replicas, n = R + 1;
    size_t temp = 0;
    LJ_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(nullptr, temp, (const u64*)nullptr,
                                                 (u64*)nullptr, n, ctx->stream));
    const uint64_t sizes_bytes = (8ull * n + 255ull) & ~255ull;
    if (int s = reserve_scratch(ctx, sizes_bytes + temp)) return s;
    u64* sizes = static_cast<u64*>(ctx->scratch);
    void* tmp = static_cast<char*>(ctx->scratch) + sizes_bytes;
    LJ_HIP(ctx, hipMemsetAsync(ctx->flag, 0, 4, ctx->stream));
    LJ_HIP(ctx, hipMemsetAsync(sizes + R, 0, 8, ctx->stream));
    const uint32_t hdr = tag >= 0 ? 2u : 0u;
    uint64_t blocks = (R + 3) / 4, cap = (uint64_t)ctx->cus * 16;
    int grid = (int)(blocks < cap ? blocks : cap);
    if (kind == LASPJ_KIND_ORSET)
        hipLaunchKernelGGL(k_orset_etf_size, dim3(grid), dim3(kBlock), 0, ctx->stream,
                           reinterpret_cast<const u64x2*>(b->dev), R, b->elements, view(d), hdr,
                           sizes, ctx->flag);
    else
        hipLaunchKernelGGL(k_gset_etf_size, dim3(grid), dim3(kBlock), 0, ctx->stream,
                           (const u64*)b->dev, R, b->elements,
                           (uint32_t)b->words_per_replica, view(d), hdr, sizes, ctx->flag);
    LJ_LAUNCHED(ctx);
    LJ_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(tmp, temp, sizes, static_cast<u64*>(offsets->dev),
                                                 n, ctx->stream));
    uint32_t flag = 0;
    LJ_HIP(ctx, hipMemcpyAsync(&flag, ctx->flag, 4, hipMemcpyDeviceToHost, ctx->stream));
    LJ_HIP(ctx, hipMemcpyAsync(total, static_cast<u64*>(offsets->dev) + R, 8,
                               hipMemcpyDeviceToHost, ctx->stream));
    LJ_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (flag)
        return fail(ctx, LASPJ_E_RANGE, "%s: a present element or token slot has no image in "
                    "the dictionary", what);
    return LASPJ_OK;
}

int etf_write(laspj_ctx* ctx, const laspj_batch* b, const laspj_etf_dict* d, int tag, int vers,
              const laspj_buf* offsets, laspj_buf* out, int32_t kind, const char* what) {
    if (int s = check_args(ctx, b, d, kind, what)) return s;
    if (!offsets || offsets->ctx != ctx || offsets->bytes < 8ull * (b->replicas + 1))
        return fail(ctx, LASPJ_E_RANGE, "%s: offsets must hold replicas + 1 uint64", what);
    if (!out || out->ctx != ctx) return fail(ctx, LASPJ_E_INVAL, "%s: bad output buffer", what);
    if (tag > 255 || vers < 0 || vers > 255)
        return fail(ctx, LASPJ_E_INVAL, "%s: tag and version are bytes", what);
    Guard g(ctx);
    const uint64_t R = b->replicas;
    uint64_t total = 0;
    LJ_HIP(ctx, hipMemcpyAsync(&total, static_cast<u64*>(offsets->dev) + R, 8,
                               hipMemcpyDeviceToHost, ctx->stream));
    LJ_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (out->bytes < total)
        return fail(ctx, LASPJ_E_RANGE, "%s: output holds %llu bytes, payloads need %llu", what,
                    (unsigned long long)out->bytes, (unsigned long long)total);
    uint64_t cap = (uint64_t)ctx->cus * 8;
    int grid = (int)(R < cap ? R : cap);
    if (kind == LASPJ_KIND_ORSET)
        hipLaunchKernelGGL(k_orset_etf_write, dim3(grid), dim3(kBlock), 0, ctx->stream,
                           reinterpret_cast<const u64x2*>(b->dev), R, b->elements, view(d), tag,
                           vers, static_cast<const u64*>(offsets->dev),
                           static_cast<uint8_t*>(out->dev));
    else
        hipLaunchKernelGGL(k_gset_etf_write, dim3(grid), dim3(kBlock), 0, ctx->stream,
                           (const u64*)b->dev, R, b->elements, (uint32_t)b->words_per_replica,
                           view(d), tag, vers, static_cast<const u64*>(offsets->dev),
                           static_cast<uint8_t*>(out->dev));
    LJ_LAUNCHED(ctx);
    return LASPJ_OK;
}

}  // namespace
}  // namespace laspj

using laspj::fail;

extern "C" {

int laspj_etf_dict_create(laspj_ctx* ctx, uint32_t E, const uint8_t* elem_blob,
                          const uint32_t* elem_off, const uint32_t* elem_order,
                          const uint8_t* tok_blob, const uint32_t* tok_off,
                          const uint8_t* tok_order, laspj_etf_dict** out) {
    if (!ctx || !out || !elem_off || !elem_order || (!elem_blob && elem_off[E]))
        return fail(ctx, LASPJ_E_INVAL, "etf_dict_create: null argument");
    *out = nullptr;
    if (E == 0) return fail(ctx, LASPJ_E_SHAPE, "etf_dict_create: no element slots");
    const bool toks = tok_off != nullptr;
    if (toks && (!tok_order || (!tok_blob && tok_off[64ull * E])))
        return fail(ctx, LASPJ_E_INVAL, "etf_dict_create: token arrays incomplete");
    // host-side validation and derived arrays
    std::vector<uint8_t> ebyte(E, 0);
    std::vector<uint64_t> tmask(E, 0);
    for (uint32_t e = 0; e < E; ++e) {
        if (elem_off[e + 1] < elem_off[e] || elem_order[e] >= E)
            return fail(ctx, LASPJ_E_RANGE, "etf_dict_create: element offsets / order invalid");
        ebyte[e] = elem_off[e + 1] - elem_off[e] == 2 && elem_blob[elem_off[e]] == 97;
    }
    uint32_t uniform = 0;
    bool mixed = false;
    if (toks) {
        for (uint64_t t = 0; t < 64ull * E; ++t) {
            if (tok_off[t + 1] < tok_off[t])
                return fail(ctx, LASPJ_E_RANGE, "etf_dict_create: token offsets decrease");
            uint32_t len = tok_off[t + 1] - tok_off[t];
            if (!len) continue;
            tmask[t / 64] |= 1ull << (t % 64);
            if (!uniform) uniform = len;
            else if (uniform != len) mixed = true;
        }
        for (uint32_t e = 0; e < E; ++e) {
            uint64_t seen = 0;
            for (int j = 0; j < 64; ++j) {
                uint8_t k = tok_order[64ull * e + j];
                if (k >= 64) break;
                if (!((tmask[e] >> k) & 1ull) || ((seen >> k) & 1ull))
                    return fail(ctx, LASPJ_E_RANGE,
                                "etf_dict_create: token order of element %u names slot %u "
                                "twice or without an image", e, k);
                seen |= 1ull << k;
            }
            if (seen != tmask[e])
                return fail(ctx, LASPJ_E_RANGE,
                            "etf_dict_create: token order of element %u misses a slot", e);
        }
    }
    const uint64_t eblob = elem_off[E], tblob = toks ? tok_off[64ull * E] : 0;
    auto al = [](uint64_t x) { return (x + 255ull) & ~255ull; };
    const uint64_t o_eoff = 0, o_eord = o_eoff + al(4ull * (E + 1)), o_eb = o_eord + al(4ull * E),
                   o_mask = o_eb + al(E), o_toff = o_mask + al(8ull * E),
                   o_tord = o_toff + (toks ? al(4ull * (64ull * E + 1)) : 0),
                   o_eblob = o_tord + (toks ? al(64ull * E) : 0), o_tblob = o_eblob + al(eblob + 1),
                   bytes = o_tblob + al(tblob + 1);
    auto* d = new (std::nothrow) laspj_etf_dict;
    if (!d) return fail(ctx, LASPJ_E_NOMEM, "etf_dict_create: host allocation");
    std::lock_guard<std::mutex> lk(ctx->mu);
    hipSetDevice(ctx->device);
    if (hipMalloc(&d->block, bytes) != hipSuccess) {
        hipGetLastError();
        delete d;
        return fail(ctx, LASPJ_E_NOMEM, "etf_dict_create: hipMalloc(%llu)", (unsigned long long)bytes);
    }
    char* base = static_cast<char*>(d->block);
    auto up = [&](uint64_t off, const void* src, uint64_t n) {
        return n ? hipMemcpy(base + off, src, n, hipMemcpyHostToDevice) : hipSuccess;
    };
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = up(o_eoff, elem_off, 4ull * (E + 1));
    if (e == hipSuccess) e = up(o_eord, elem_order, 4ull * E);
    if (e == hipSuccess) e = up(o_eb, ebyte.data(), E);
    if (e == hipSuccess) e = up(o_mask, tmask.data(), 8ull * E);
    if (e == hipSuccess && toks) e = up(o_toff, tok_off, 4ull * (64ull * E + 1));
    if (e == hipSuccess && toks) e = up(o_tord, tok_order, 64ull * E);
    if (e == hipSuccess) e = up(o_eblob, elem_blob, eblob);
    if (e == hipSuccess && toks) e = up(o_tblob, tok_blob, tblob);
    if (e != hipSuccess) {
        hipFree(d->block);
        delete d;
        return fail(ctx, LASPJ_E_DEVICE, "etf_dict_create: upload: %s", hipGetErrorString(e));
    }
    d->ctx = ctx;
    d->elements = E;
    d->has_tokens = toks;
    d->tok_uniform = mixed ? 0u : uniform;
    d->elem_off = reinterpret_cast<const uint32_t*>(base + o_eoff);
    d->elem_order = reinterpret_cast<const uint32_t*>(base + o_eord);
    d->elem_byte = reinterpret_cast<const uint8_t*>(base + o_eb);
    d->tok_mask = reinterpret_cast<const uint64_t*>(base + o_mask);
    d->tok_off = toks ? reinterpret_cast<const uint32_t*>(base + o_toff) : nullptr;
    d->tok_order = toks ? reinterpret_cast<const uint8_t*>(base + o_tord) : nullptr;
    d->elem_blob = reinterpret_cast<const uint8_t*>(base + o_eblob);
    d->tok_blob = toks ? reinterpret_cast<const uint8_t*>(base + o_tblob) : nullptr;
    *out = d;
    return LASPJ_OK;
}

int laspj_etf_dict_destroy(laspj_etf_dict* d) {
    if (!d) return LASPJ_E_INVAL;
    {
        std::lock_guard<std::mutex> lk(d->ctx->mu);
        hipSetDevice(d->ctx->device);
        hipStreamSynchronize(d->ctx->stream);
        hipFree(d->block);
    }
    delete d;
    return LASPJ_OK;
}

int laspj_orset_etf_size(laspj_ctx* ctx, const laspj_batch* b, const laspj_etf_dict* d, int tag,
                         laspj_buf* offsets, uint64_t* total) {
    return laspj::etf_size(ctx, b, d, tag, offsets, total, LASPJ_KIND_ORSET, "orset_etf_size");
}

int laspj_orset_etf_write(laspj_ctx* ctx, const laspj_batch* b, const laspj_etf_dict* d, int tag,
                          int vers, const laspj_buf* offsets, laspj_buf* out) {
    return laspj::etf_write(ctx, b, d, tag, vers, offsets, out, LASPJ_KIND_ORSET,
                            "orset_etf_write");
}

int laspj_gset_etf_size(laspj_ctx* ctx, const laspj_batch* b, const laspj_etf_dict* d, int tag,
                        laspj_buf* offsets, uint64_t* total) {
    return laspj::etf_size(ctx, b, d, tag, offsets, total, LASPJ_KIND_GSET, "gset_etf_size");
}

int laspj_gset_etf_write(laspj_ctx* ctx, const laspj_batch* b, const laspj_etf_dict* d, int tag,
                         int vers, const laspj_buf* offsets, laspj_buf* out) {
    return laspj::etf_write(ctx, b, d, tag, vers, offsets, out, LASPJ_KIND_GSET,
                            "gset_etf_write");
}

}  // extern "C"
