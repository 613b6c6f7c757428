// OR-Sets with more than 64 token slots per element (LASPJ_KIND_ORSET_WIDE).
//
// add_elem mints a fresh token per add and never collects tombstones
// (lasp_orset.erl:222-241, 261-262): an element re-added ~22 times on N = 3 replicas
// outgrows the 64-bit {p, r} cell.  A wide batch gives every (replica, element slot) k
// {p, r} pairs (T = 64 k token slots, token slot t in pair t / 64, bit t % 64), so such an
// element stays on the join path.  The layout is the narrow one with k times the words:
// pair j of cell (i, e) at ((i E + e) k + j) 16 bytes, so the join / reduce / equality /
// bind entry points run unchanged over the words (merge is still the OR of everything),
// and the per-element predicates below fold an element's k pairs:
//   value/1   (lasp_orset.erl:67-73):  any(p & ~r) over the pairs
//   removed   (:90-95):                any(r)
//   stats/1   (:156-192):              element present = any(p), popcounts summed
//   is_inflation (lasp_lattice.erl:153-161, 277-285): every Prev token in Cur
//   is_strict_inflation (:235-253):    inflation and some pair differs (on canonical
//                                      values that is "a token dict of a common element
//                                      =/= or length(Prev) < length(Cur)")
//   update/3  (:99-117):               ADD sets bit t % 64 of pair t / 64, REMOVE sets
//                                      r = p in every pair
// Every kernel streams the batch once; the predicates reduce per replica with one wave per
// (replica, segment of elements) and per-replica atomics in a zeroed record.

#include <algorithm>

#include "laspj_internal.h"

namespace laspj {
namespace {

typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

constexpr int kB = 256;
constexpr uint32_t kWSeg = 1024;      // elements per (replica, segment) item

__device__ __forceinline__ u64x2 ld2(const u64x2* p) { return __builtin_nontemporal_load(p); }

__device__ __forceinline__ u64 wsum(u64 v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// value / removed: one lane per element, a wave per 64 elements -> one bit word
template <bool REMOVED>
__global__ __launch_bounds__(kB) void k_wide_value(const u64x2* cells, u64* out, uint64_t R,
                                                   uint32_t E, uint32_t k) {
    const uint32_t W = (E + 63u) / 64u;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nw = (uint64_t)gridDim.x * (kB / 64);
    for (uint64_t it = ((uint64_t)blockIdx.x * kB + threadIdx.x) >> 6; it < R * W; it += nw) {
        const uint64_t rep = it / W;
        const uint32_t e = (uint32_t)(it - rep * W) * 64u + lane;
        bool vis = false;
        if (e < E) {
            const u64x2* c = cells + (rep * E + e) * k;
            for (uint32_t j = 0; j < k; ++j) {
                const u64x2 v = ld2(c + j);
                vis |= REMOVED ? v.y != 0 : (v.x & ~v.y) != 0;
            }
        }
        const u64 m = __ballot(vis);
        if (lane == 0) out[rep * W + (it - rep * W)] = m;
    }
}

// stats: {element_count, adds, removes} summed into rec (3 words per replica, zeroed)
__global__ __launch_bounds__(kB) void k_wide_stats(const u64x2* cells, u64* rec, uint64_t R,
                                                   uint32_t E, uint32_t k, uint32_t nseg) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nw = (uint64_t)gridDim.x * (kB / 64);
    for (uint64_t it = ((uint64_t)blockIdx.x * kB + threadIdx.x) >> 6; it < R * nseg; it += nw) {
        const uint64_t rep = it / nseg;
        const uint32_t e0 = (uint32_t)(it - rep * nseg) * kWSeg, e1 = min(E, e0 + kWSeg);
        u64 elems = 0, adds = 0, rems = 0;
        for (uint32_t e = e0 + lane; e < e1; e += 64) {
            const u64x2* c = cells + (rep * E + e) * k;
            bool pres = false;
            for (uint32_t j = 0; j < k; ++j) {
                const u64x2 v = ld2(c + j);
                pres |= v.x != 0;
                adds += __popcll(v.x & ~v.y);
                rems += __popcll(v.y);
            }
            elems += pres;
        }
        elems = wsum(elems);
        adds = wsum(adds);
        rems = wsum(rems);
        if (lane == 0) {
            if (elems) atomicAdd(rec + 3 * rep, elems);
            if (adds) atomicAdd(rec + 3 * rep + 1, adds);
            if (rems) atomicAdd(rec + 3 * rep + 2, rems);
        }
    }
}

// inflation flags per cur replica in flags[rep] (zeroed): bit 0 a Prev token missing from
// Cur, bit 1 some pair differs
__global__ __launch_bounds__(kB) void k_wide_inflation(const u64x2* prev, const u64x2* cur,
                                                       uint32_t* flags, uint64_t R, uint32_t E,
                                                       uint32_t k, uint32_t nseg, bool bcast) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nw = (uint64_t)gridDim.x * (kB / 64);
    const uint64_t pairs = (uint64_t)E * k;
    for (uint64_t it = ((uint64_t)blockIdx.x * kB + threadIdx.x) >> 6; it < R * nseg; it += nw) {
        const uint64_t rep = it / nseg;
        const uint64_t q0 = (it - rep * nseg) * (uint64_t)kWSeg * k;
        const uint64_t q1 = min(pairs, q0 + (uint64_t)kWSeg * k);
        const u64x2* p = prev + (bcast ? 0 : rep) * pairs;
        const u64x2* c = cur + rep * pairs;
        bool viol = false, diff = false;
        for (uint64_t q = q0 + lane; q < q1; q += 64) {
            const u64x2 a = ld2(p + q), b = ld2(c + q);
            viol |= (a.x & ~b.x) != 0;
            diff |= (a.x != b.x) | (a.y != b.y);
        }
        const uint32_t f = (__ballot(viol) ? 1u : 0u) | (__ballot(diff) ? 2u : 0u);
        if (lane == 0 && f) atomicOr(flags + rep, f);
    }
}

__global__ void k_wide_finish(uint32_t* flags, uint8_t* out, uint64_t R, bool strict) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < R;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t f = flags[i];
        const bool infl = !(f & 1u);
        out[i] = (strict ? infl && (f & 2u) : infl) ? 1 : 0;
        flags[i] = 0;
    }
}

__global__ void k_wide_stats_out(u64* rec, u64* out, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        out[i] = rec[i];
        rec[i] = 0;
    }
}

// update/3 on wide cells: as k_apply_ops (one thread per replica's run of ops, one
// update/3 call at a time, rolled back whole when a remove finds its element absent or an
// INSERT its token present); token slot = slot | pad << 8
__global__ __launch_bounds__(kB) void k_wide_apply(u64* state, uint64_t E, uint32_t k,
                                                   const laspj_op* ops, uint64_t nops,
                                                   int32_t* status) {
    const uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x;
    if (i >= nops) return;
    const uint64_t rep = ops[i].replica;
    if (i > 0 && ops[i - 1].replica == rep) return;
    uint64_t end = i + 1;
    while (end < nops && ops[end].replica == rep) ++end;
    u64* s = state + rep * E * 2ull * k;
    auto tok = [&](const laspj_op& o) { return (uint32_t)o.slot | ((uint32_t)o.pad << 8); };
    auto present = [&](uint32_t e) {
        for (uint32_t j = 0; j < k; ++j)
            if (s[(e * (uint64_t)k + j) * 2]) return true;
        return false;
    };
    uint64_t c0 = i;
    while (c0 < end) {
        uint64_t c1 = c0 + 1;
        while (c1 < end && !(ops[c1].flags & LASPJ_OP_FLAG_NEW_CALL)) ++c1;
        uint64_t bad = ~0ull;
        int32_t why = LASPJ_OPST_NOT_PRESENT;
        for (uint64_t q = c0; q < c1 && bad == ~0ull; ++q) {
            const uint32_t e = ops[q].element;
            if (ops[q].kind == LASPJ_OP_REMOVE) {
                bool pres = present(e);
                for (uint64_t j = c0; j < q && !pres; ++j)
                    pres = ops[j].kind != LASPJ_OP_REMOVE && ops[j].element == e;
                if (!pres) bad = q;
            } else if (ops[q].kind == LASPJ_OP_INSERT) {
                const uint32_t t = tok(ops[q]);
                bool ex = (s[(e * (uint64_t)k + t / 64u) * 2] >> (t % 64u)) & 1ull;
                for (uint64_t j = c0; j < q && !ex; ++j)
                    ex = ops[j].kind != LASPJ_OP_REMOVE && ops[j].element == e && tok(ops[j]) == t;
                if (ex) {
                    bad = q;
                    why = LASPJ_OPST_KEY_EXISTS;
                }
            }
        }
        if (bad != ~0ull) {
            for (uint64_t q = c0; q < c1; ++q) status[q] = q == bad ? why : LASPJ_OPST_ROLLED_BACK;
        } else {
            for (uint64_t q = c0; q < c1; ++q) {
                const laspj_op& o = ops[q];
                u64* cell = s + (uint64_t)o.element * k * 2ull;
                if (o.kind != LASPJ_OP_REMOVE) {
                    const uint32_t t = tok(o);
                    cell[2 * (t / 64u)] |= 1ull << (t % 64u);           // {Token, false}
                    cell[2 * (t / 64u) + 1] &= ~(1ull << (t % 64u));
                } else {
                    for (uint32_t j = 0; j < k; ++j) cell[2 * j + 1] = cell[2 * j];
                }
                status[q] = LASPJ_OPST_APPLIED;
            }
        }
        c0 = c1;
    }
}

// dst pair j of cell c = src pair j (j < k1) else {0, 0}: one lane per dst pair
__global__ __launch_bounds__(kB) void k_wide_widen(u64x2* dst, const u64x2* src, uint64_t cells,
                                                   uint32_t k1, uint32_t k2) {
    const uint64_t n = cells * k2;
    for (uint64_t q = (uint64_t)blockIdx.x * kB + threadIdx.x; q < n;
         q += (uint64_t)gridDim.x * kB) {
        const uint64_t c = q / k2;
        const uint32_t j = (uint32_t)(q - c * k2);
        dst[q] = j < k1 ? ld2(src + c * k1 + j) : u64x2{0, 0};
    }
}

int grid_for(const laspj_ctx* ctx, uint64_t waves) {
    const uint64_t blocks = (waves + 3) / 4, cap = (uint64_t)ctx->cus * 16;
    return (int)std::max<uint64_t>(1, std::min(blocks, cap));
}

// a zeroed device record of `bytes` in ctx->partials (grown; kept zeroed between calls)
hipError_t wide_record(laspj_ctx* ctx, uint64_t bytes, void** out) {
    if (ctx->partials_bytes < bytes) {
        if (ctx->partials) {
            hipStreamSynchronize(ctx->stream);
            hipFree(ctx->partials);
            ctx->partials = nullptr;
            ctx->partials_bytes = 0;
        }
        const uint64_t want = std::max<uint64_t>(bytes, 1 << 16);
        if (hipError_t e = dev_malloc(ctx, &ctx->partials, want)) return e;
        if (hipError_t e = hipMemsetAsync(ctx->partials, 0, want, ctx->stream)) return e;
        ctx->partials_bytes = want;
    }
    *out = ctx->partials;
    return hipSuccess;
}

}  // namespace

hipError_t launch_wide_value(laspj_ctx* ctx, const laspj_batch* b, uint64_t* out, bool removed) {
    const uint32_t k = b->tok_words, W = (b->elements + 63u) / 64u;
    const int grid = grid_for(ctx, b->replicas * W);
    auto* c = reinterpret_cast<const u64x2*>(b->dev);
    if (removed)
        hipLaunchKernelGGL(k_wide_value<true>, dim3(grid), dim3(kB), 0, ctx->stream, c,
                           (u64*)out, b->replicas, b->elements, k);
    else
        hipLaunchKernelGGL(k_wide_value<false>, dim3(grid), dim3(kB), 0, ctx->stream, c,
                           (u64*)out, b->replicas, b->elements, k);
    return hipGetLastError();
}

hipError_t launch_wide_stats(laspj_ctx* ctx, const laspj_batch* b, uint64_t* out) {
    void* rec = nullptr;
    if (hipError_t e = wide_record(ctx, 24ull * b->replicas, &rec)) return e;
    const uint32_t nseg = (b->elements + kWSeg - 1) / kWSeg;
    hipLaunchKernelGGL(k_wide_stats, dim3(grid_for(ctx, b->replicas * nseg)), dim3(kB), 0,
                       ctx->stream, reinterpret_cast<const u64x2*>(b->dev), (u64*)rec,
                       b->replicas, b->elements, b->tok_words, nseg);
    const uint64_t n = 3ull * b->replicas;
    hipLaunchKernelGGL(k_wide_stats_out, dim3((unsigned)std::min<uint64_t>((n + 255) / 256, 4096)),
                       dim3(256), 0, ctx->stream, (u64*)rec, (u64*)out, n);
    return hipGetLastError();
}

hipError_t launch_wide_inflation(laspj_ctx* ctx, const laspj_batch* prev, const laspj_batch* cur,
                                 bool strict, uint8_t* out) {
    void* rec = nullptr;
    if (hipError_t e = wide_record(ctx, 4ull * cur->replicas, &rec)) return e;
    const uint32_t nseg = (cur->elements + kWSeg - 1) / kWSeg;
    hipLaunchKernelGGL(k_wide_inflation, dim3(grid_for(ctx, cur->replicas * nseg)), dim3(kB), 0,
                       ctx->stream, reinterpret_cast<const u64x2*>(prev->dev),
                       reinterpret_cast<const u64x2*>(cur->dev), (uint32_t*)rec, cur->replicas,
                       cur->elements, cur->tok_words, nseg, prev->replicas != cur->replicas);
    hipLaunchKernelGGL(k_wide_finish,
                       dim3((unsigned)std::min<uint64_t>((cur->replicas + 255) / 256, 4096)),
                       dim3(256), 0, ctx->stream, (uint32_t*)rec, out, cur->replicas, strict);
    return hipGetLastError();
}

hipError_t launch_wide_widen(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src) {
    const uint64_t cells = dst->replicas * (uint64_t)dst->elements;
    const uint64_t n = cells * dst->tok_words;
    hipLaunchKernelGGL(k_wide_widen, dim3(grid_for(ctx, (n + 63) / 64)), dim3(kB), 0, ctx->stream,
                       reinterpret_cast<u64x2*>(dst->dev), reinterpret_cast<const u64x2*>(src->dev),
                       cells, src->tok_words, dst->tok_words);
    return hipGetLastError();
}

hipError_t launch_wide_apply(laspj_ctx* ctx, laspj_batch* b, const laspj_op* ops, uint64_t nops,
                             int32_t* status) {
    const uint64_t grid = (nops + kB - 1) / kB;
    hipLaunchKernelGGL(k_wide_apply, dim3((unsigned)grid), dim3(kB), 0, ctx->stream,
                       (u64*)b->dev, (uint64_t)b->elements, b->tok_words, ops, nops, status);
    return hipGetLastError();
}

}  // namespace laspj
