// Many variables in one launch: the bind path and the process loop of a store whose
// variables are separate batches (one per #dv, lasp_core.erl:291-312; the {strict, V}
// re-checks of lasp_process.erl:61-95).  The caller hands arrays of batch handles; the
// runtime uploads one descriptor per variable, and one kernel walks every variable's
// words in 2048-word segments (one wave per (variable, segment)), so a vnode's worth of
// binds or re-checks costs one launch and one status download instead of one
// synchronous round trip per variable.
//
//   bind_many:      status[i] = 0 when cur[i] =:= val[i] (bind is a no-op,
//                   lasp_core.erl:294-296), else dst[i] := cur[i] ⊔ val[i] (OR for set
//                   bitmaps, per-actor max for G-Counters) and status[i] = 1 — for
//                   canonical values the merge always inflates cur, and the reference
//                   writes whenever it does (:301-303), even when nothing changed.
//   inflation_many: out[i] = is_inflation / is_strict_inflation of prev[i] -> cur[i]
//                   (lasp_lattice.erl:137-161, 169-179, 212-253, 273-275), per kind.

#include <new>
#include <algorithm>
#include <vector>

#include <cstring>

#include "laspj_internal.h"

namespace laspj {
namespace {

typedef unsigned long long u64;

constexpr uint64_t kMSeg = 2048;          // words per (variable, segment) item

struct MItem {
    u64* dst;
    const u64* a;        // cur / prev
    const u64* b;        // val / cur
    uint64_t words;
    uint64_t seg0;       // first segment index of this variable
    int32_t kind;
    uint32_t pad;
};

__device__ __forceinline__ u64 wsum(u64 v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// the variable owning global segment `s` (binary search over seg0)
__device__ __forceinline__ uint32_t owner(const MItem* it, uint32_t n, uint64_t s) {
    uint32_t lo = 0, hi = n;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (it[mid].seg0 <= s) lo = mid;
        else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(256) void k_bind_many(const MItem* items, uint32_t n,
                                                   uint64_t nseg, uint32_t* status) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nw = (uint64_t)gridDim.x * 4;
    for (uint64_t s = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6; s < nseg; s += nw) {
        const uint32_t i = owner(items, n, s);
        const MItem it = items[i];
        const uint64_t lo = (s - it.seg0) * kMSeg;
        const uint64_t hi = min(it.words, lo + kMSeg);
        const bool mx = it.kind == LASPJ_KIND_GCOUNTER;
        bool diff = false;
        for (uint64_t w = lo + lane; w < hi; w += 64) {
            const u64 x = it.a[w], y = it.b[w];
            diff |= x != y;
            it.dst[w] = mx ? (x > y ? x : y) : (x | y);
        }
        if (__ballot(diff) != 0 && lane == 0) atomicOr(status + i, 1u);
    }
}

// per-variable record {flags, np, nc, -}: flags bit 0 = violation, bit 1 = a common
// element's cell changed (OR-Set) / a Cur bit outside Prev (G-Set)
__global__ __launch_bounds__(256) void k_inflation_many(const MItem* items, uint32_t n,
                                                        uint64_t nseg, int strict,
                                                        u64* rec) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nw = (uint64_t)gridDim.x * 4;
    for (uint64_t s = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6; s < nseg; s += nw) {
        const uint32_t i = owner(items, n, s);
        const MItem it = items[i];
        const uint64_t lo = (s - it.seg0) * kMSeg;
        const uint64_t hi = min(it.words, lo + kMSeg);
        bool viol = false, changed = false;
        u64 np = 0, nc = 0;
        if (it.kind == LASPJ_KIND_ORSET) {
            // words alternate p, r; a lane takes whole cells
            for (uint64_t w = lo + 2 * lane; w + 1 < hi; w += 128) {
                const u64 pp = it.a[w], pr = it.a[w + 1], cp = it.b[w], cr = it.b[w + 1];
                viol |= (pp & ~cp) != 0;
                changed |= (pp != 0) & (cp != 0) & ((pp != cp) | (pr != cr));
                np += pp != 0;
                nc += cp != 0;
            }
        } else if (it.kind == LASPJ_KIND_ORSET_WIDE) {
            // {p, r} pairs, k per element: inflation = every Prev token in Cur; strict =
            // and some pair differs (a common element's tokens or an element new in Cur)
            for (uint64_t w = lo + 2 * lane; w + 1 < hi; w += 128) {
                const u64 pp = it.a[w], pr = it.a[w + 1], cp = it.b[w], cr = it.b[w + 1];
                viol |= (pp & ~cp) != 0;
                changed |= (pp != cp) | (pr != cr);
            }
        } else if (it.kind == LASPJ_KIND_GSET) {
            for (uint64_t w = lo + lane; w < hi; w += 64) {
                const u64 p = it.a[w], c = it.b[w];
                viol |= (p & ~c) != 0;
                changed |= (c & ~p) != 0;
            }
        } else {                                      // G-Counter
            for (uint64_t w = lo + lane; w < hi; w += 64) {
                const u64 p = it.a[w], c = it.b[w];
                viol |= p > c;
                np += p;
                nc += c;
            }
        }
        u64 f = (__ballot(viol) != 0 ? 1ull : 0ull) | (__ballot(changed) != 0 ? 2ull : 0ull);
        np = wsum(np);
        nc = wsum(nc);
        if (lane == 0) {
            u64* r = rec + 4ull * i;
            if (f) atomicOr(r, f);
            if (np) atomicAdd(r + 1, np);
            if (nc) atomicAdd(r + 2, nc);
        }
    }
}

__global__ void k_many_status(const uint32_t* st, uint8_t* out, uint32_t n) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        out[i] = st[i] ? 1 : 0;
}

__global__ void k_inflation_many_finish(const MItem* items, uint32_t n, int strict,
                                        const u64* rec, uint8_t* out) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const u64 f = rec[4ull * i], np = rec[4ull * i + 1], nc = rec[4ull * i + 2];
        const bool infl = !(f & 1);
        bool res = infl;
        if (strict) {
            const int32_t k = items[i].kind;
            if (k == LASPJ_KIND_ORSET) res = infl && ((f & 2) || np < nc);   // [] case: np < nc
            else if (k == LASPJ_KIND_GSET || k == LASPJ_KIND_ORSET_WIDE) res = infl && (f & 2);
            else res = np < nc;                                              // value(P) < value(C)
        }
        out[i] = res ? 1 : 0;
    }
}

}  // namespace
}  // namespace laspj

using laspj::fail;
using namespace laspj;

namespace {

struct MGuard {
    std::lock_guard<std::mutex> lk;
    explicit MGuard(laspj_ctx* c) : lk(c->mu) { hipSetDevice(c->device); }
};

bool many_kind(int32_t k) {
    return k == LASPJ_KIND_ORSET || k == LASPJ_KIND_GSET || k == LASPJ_KIND_GCOUNTER ||
           k == LASPJ_KIND_ORSET_WIDE;
}

// validate the triples / pairs and build the descriptors; returns the segment count
int describe(laspj_ctx* ctx, uint32_t n, laspj_batch* const* dst, const laspj_batch* const* a,
             const laspj_batch* const* b, std::vector<MItem>* items, uint64_t* nseg,
             const char* what) {
    items->resize(n);
    uint64_t seg = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const laspj_batch* x = a[i];
        const laspj_batch* y = b[i];
        laspj_batch* d = dst ? dst[i] : nullptr;
        if (!x || !y || x->ctx != ctx || y->ctx != ctx || (dst && (!d || d->ctx != ctx)))
            return fail(ctx, LASPJ_E_INVAL, "%s: item %u: null batch or other context", what, i);
        if (!many_kind(x->kind) || x->kind != y->kind || (d && d->kind != x->kind))
            return fail(ctx, LASPJ_E_KIND, "%s: item %u: kinds", what, i);
        if (x->replicas != 1 || y->replicas != 1 || (d && d->replicas != 1) ||
            x->words_per_replica != y->words_per_replica ||
            (d && d->words_per_replica != x->words_per_replica) || x->elements != y->elements)
            return fail(ctx, LASPJ_E_SHAPE, "%s: item %u: one replica of one shape each", what, i);
        MItem& m = (*items)[i];
        m.dst = d ? reinterpret_cast<u64*>(d->dev) : nullptr;
        m.a = reinterpret_cast<const u64*>(x->dev);
        m.b = reinterpret_cast<const u64*>(y->dev);
        m.words = x->words_per_replica;
        m.seg0 = seg;
        m.kind = x->kind;
        m.pad = 0;
        seg += (m.words + kMSeg - 1) / kMSeg;
    }
    *nseg = seg;
    if (!dst) return LASPJ_OK;
    // every dst is written while every cur / val is read by other waves: a dst may
    // overlap nothing but its own cur exactly (the in-place bind), and no other dst
    struct Iv {
        uintptr_t lo, hi;
        uint32_t item;
    };
    std::vector<Iv> ds(n);
    for (uint32_t i = 0; i < n; ++i) {
        const uintptr_t lo = (uintptr_t)dst[i]->dev;
        ds[i] = {lo, lo + 8 * (uintptr_t)dst[i]->words_per_replica, i};
    }
    std::sort(ds.begin(), ds.end(), [](const Iv& x, const Iv& y) { return x.lo < y.lo; });
    for (uint32_t k = 1; k < n; ++k)
        if (ds[k].lo < ds[k - 1].hi)
            return fail(ctx, LASPJ_E_INVAL, "%s: items %u and %u: dst ranges overlap", what,
                        ds[k - 1].item, ds[k].item);
    for (uint32_t i = 0; i < n; ++i) {
        for (int side = 0; side < 2; ++side) {
            const laspj_batch* r = side ? b[i] : a[i];
            const uintptr_t lo = (uintptr_t)r->dev, hi = lo + 8 * (uintptr_t)r->words_per_replica;
            // dst ranges starting below hi, walked down while they still reach past lo
            auto it = std::lower_bound(ds.begin(), ds.end(), hi,
                                       [](const Iv& x, uintptr_t v) { return x.lo < v; });
            while (it != ds.begin()) {
                --it;
                if (it->hi <= lo) break;
                const bool own_cur = side == 0 && it->item == i && it->lo == lo && it->hi == hi;
                if (!own_cur)
                    return fail(ctx, LASPJ_E_INVAL, "%s: item %u's dst overlaps item %u's %s",
                                what, it->item, i, side ? "val" : "cur");
            }
        }
    }
    return LASPJ_OK;
}

int grid_of(const laspj_ctx* ctx, uint64_t nseg) {
    uint64_t g = (nseg + 3) / 4, cap = (uint64_t)ctx->cus * 16;
    return (int)(g < cap ? (g ? g : 1) : cap);
}

// descriptors + per-item words in one scratch allocation (ctx->lscratch is shared with
// the list kernels; these calls synchronise before returning, so reuse is safe)
void* mscratch(laspj_ctx* ctx, uint64_t bytes) {
    if (ctx->lscratch_bytes < bytes) {
        if (ctx->lscratch) {
            hipStreamSynchronize(ctx->stream);
            hipFree(ctx->lscratch);
            ctx->lscratch = nullptr;
            ctx->lscratch_bytes = 0;
        }
        if (laspj::dev_malloc(ctx, &ctx->lscratch, bytes) != hipSuccess) {
            hipGetLastError();
            return nullptr;
        }
        ctx->lscratch_bytes = bytes;
    }
    return ctx->lscratch;
}

}  // namespace

extern "C" {

// bind_many into a device buffer (status) or, host, into host memory through the
// context's mapped answer block (one synchronisation, no separate download)
static int bind_many_impl(laspj_ctx* ctx, uint32_t n, laspj_batch* const* dst,
                          const laspj_batch* const* cur, const laspj_batch* const* val,
                          laspj_buf* status, uint8_t* host) {
    if (!ctx || (n && (!dst || !cur || !val)))
        return fail(ctx, LASPJ_E_INVAL, "bind_many: null argument");
    if (!host && (!status || status->ctx != ctx || status->bytes < n))
        return fail(ctx, LASPJ_E_RANGE, "bind_many: status buffer (n bytes)");
    if (!n) return LASPJ_OK;
    std::vector<MItem> items;
    uint64_t nseg = 0;
    if (int s = describe(ctx, n, dst, cur, val, &items, &nseg, "bind_many")) return s;
    MGuard g(ctx);
    if (host && ctx->many_h_bytes < n) {
        if (ctx->many_h) {
            hipStreamSynchronize(ctx->stream);
            hipHostFree(ctx->many_h);
            ctx->many_h = nullptr;
            ctx->many_h_bytes = 0;
        }
        const uint64_t want = std::max<uint64_t>(n, 4096);
        if (hipHostMalloc(&ctx->many_h, want, hipHostMallocCoherent) != hipSuccess) {
            hipGetLastError();
            ctx->many_h = nullptr;
            return fail(ctx, LASPJ_E_NOMEM, "bind_many: pinned statuses");
        }
        ctx->many_h_bytes = want;
        LJ_HIP(ctx, hipHostGetDevicePointer(&ctx->many_hd, ctx->many_h, 0));
    }
    const uint64_t db = sizeof(MItem) * n, sb = 4ull * n;
    char* base = static_cast<char*>(mscratch(ctx, db + sb));
    if (!base) return fail(ctx, LASPJ_E_NOMEM, "bind_many: scratch");
    auto* dev_items = reinterpret_cast<MItem*>(base);
    auto* st = reinterpret_cast<uint32_t*>(base + db);
    // the descriptors staged in the pinned ring when they are few: then nothing here has to
    // wait — every later use of the batches and of the status buffer is on the context's
    // stream — unless a buffer's device address was handed out (other streams may read it)
    const void* staged = laspj::stage_small(ctx, items.data(), db);
    LJ_HIP(ctx, hipMemcpyAsync(dev_items, staged ? staged : items.data(), db,
                               hipMemcpyHostToDevice, ctx->stream));
    LJ_HIP(ctx, hipMemsetAsync(st, 0, sb, ctx->stream));
    hipLaunchKernelGGL(k_bind_many, dim3(grid_of(ctx, nseg)), dim3(256), 0, ctx->stream,
                       dev_items, n, nseg, st);
    LJ_LAUNCHED(ctx);
    const unsigned fg = (unsigned)((n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024);
    hipLaunchKernelGGL(k_many_status, dim3(fg), dim3(256), 0, ctx->stream, st,
                       static_cast<uint8_t*>(host ? ctx->many_hd : status->dev), n);
    LJ_LAUNCHED(ctx);
    if (host) {
        LJ_HIP(ctx, hipStreamSynchronize(ctx->stream));
        std::memcpy(host, ctx->many_h, n);
        return LASPJ_OK;
    }
    bool exported = !staged || status->exported;
    for (uint32_t i = 0; i < n && !exported; ++i)
        exported = dst[i]->exported || cur[i]->exported || val[i]->exported;
    if (exported) LJ_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return LASPJ_OK;
}

int laspj_batch_bind_many(laspj_ctx* ctx, uint32_t n, laspj_batch* const* dst,
                          const laspj_batch* const* cur, const laspj_batch* const* val,
                          laspj_buf* status) {
    return bind_many_impl(ctx, n, dst, cur, val, status, nullptr);
}

int laspj_batch_bind_many_host(laspj_ctx* ctx, uint32_t n, laspj_batch* const* dst,
                               const laspj_batch* const* cur, const laspj_batch* const* val,
                               uint8_t* status) {
    if (n && !status) return fail(ctx, LASPJ_E_INVAL, "bind_many_host: null status");
    return bind_many_impl(ctx, n, dst, cur, val, nullptr, status);
}

int laspj_batch_inflation_many(laspj_ctx* ctx, uint32_t n, const laspj_batch* const* prev,
                               const laspj_batch* const* cur, int strict, laspj_buf* out) {
    if (!ctx || (n && (!prev || !cur)))
        return fail(ctx, LASPJ_E_INVAL, "inflation_many: null argument");
    if (!out || out->ctx != ctx || out->bytes < n)
        return fail(ctx, LASPJ_E_RANGE, "inflation_many: output buffer (n bytes)");
    if (!n) return LASPJ_OK;
    std::vector<MItem> items;
    uint64_t nseg = 0;
    if (int s = describe(ctx, n, nullptr, prev, cur, &items, &nseg, "inflation_many")) return s;
    MGuard g(ctx);
    const uint64_t db = sizeof(MItem) * n, rb = 32ull * n;
    char* base = static_cast<char*>(mscratch(ctx, db + rb));
    if (!base) return fail(ctx, LASPJ_E_NOMEM, "inflation_many: scratch");
    auto* dev_items = reinterpret_cast<MItem*>(base);
    auto* rec = reinterpret_cast<u64*>(base + db);
    LJ_HIP(ctx, hipMemcpyAsync(dev_items, items.data(), db, hipMemcpyHostToDevice, ctx->stream));
    LJ_HIP(ctx, hipMemsetAsync(rec, 0, rb, ctx->stream));
    hipLaunchKernelGGL(k_inflation_many, dim3(grid_of(ctx, nseg)), dim3(256), 0, ctx->stream,
                       dev_items, n, nseg, strict, rec);
    LJ_LAUNCHED(ctx);
    const unsigned fg = (unsigned)((n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024);
    hipLaunchKernelGGL(k_inflation_many_finish, dim3(fg), dim3(256), 0, ctx->stream, dev_items,
                       n, strict, rec, static_cast<uint8_t*>(out->dev));
    LJ_LAUNCHED(ctx);
    LJ_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return LASPJ_OK;
}

}  // extern "C"
