// liblaspj runtime: contexts, device buffers, batches, events and the C-ABI entry
// points (include/laspj.h).  Kernels live in laspj_kernels.hip.
//
// Every entry point validates handles and shapes on the host before anything is
// launched, locks the context mutex (the NIF calls one context from many BEAM
// schedulers, SURVEY.md §8b "Threading"), and reports failures through an int status
// plus ctx->err.  No C++ exception escapes: allocation failures surface as
// LASPJ_E_NOMEM via the nothrow paths below.

#include <cstdarg>
#include <cstring>
#include <new>
#include <vector>

#include "laspj_internal.h"

namespace laspj {

int fail(laspj_ctx* ctx, int code, const char* fmt, ...) {
    if (ctx) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        ctx->err = buf;
    }
    return code;
}

}  // namespace laspj

using laspj::fail;

namespace {

struct Guard {
    laspj_ctx* ctx;
    std::lock_guard<std::mutex> lk;
    explicit Guard(laspj_ctx* c) : ctx(c), lk(c->mu) { hipSetDevice(c->device); }
};

bool same_ctx(const laspj_ctx* ctx, const laspj_batch* b) { return b && b->ctx == ctx; }

int check_pair(laspj_ctx* ctx, const laspj_batch* x, const laspj_batch* y, int32_t kind,
               const char* what) {
    if (!same_ctx(ctx, x) || !same_ctx(ctx, y))
        return fail(ctx, LASPJ_E_INVAL, "%s: null batch or batch of another context", what);
    if (x->kind != kind || y->kind != kind)
        return fail(ctx, LASPJ_E_KIND, "%s: wrong batch kind (%d, %d; want %d)", what, x->kind,
                    y->kind, kind);
    if (x->elements != y->elements || x->replicas != y->replicas ||
        x->words_per_replica != y->words_per_replica)
        return fail(ctx, LASPJ_E_SHAPE, "%s: shapes differ (%llu x %u vs %llu x %u)", what,
                    (unsigned long long)x->replicas, x->elements,
                    (unsigned long long)y->replicas, y->elements);
    return LASPJ_OK;
}

int check_buf(laspj_ctx* ctx, const laspj_buf* buf, uint64_t need, const char* what) {
    if (!buf || buf->ctx != ctx)
        return fail(ctx, LASPJ_E_INVAL, "%s: null output buffer or buffer of another context",
                    what);
    if (buf->bytes < need)
        return fail(ctx, LASPJ_E_RANGE, "%s: output buffer holds %llu bytes, needs %llu", what,
                    (unsigned long long)buf->bytes, (unsigned long long)need);
    return LASPJ_OK;
}

uint64_t words_per(int32_t kind, uint32_t elements, uint32_t er) {
    switch (kind) {
        case LASPJ_KIND_ORSET: return 2ull * elements;
        case LASPJ_KIND_GSET: return (elements + 63ull) / 64ull;
        case LASPJ_KIND_ORSET_CONCAT: return 4ull * elements;
        case LASPJ_KIND_ORSET_PRODUCT: return ((uint64_t)elements * er + 1ull) / 2ull;
        case LASPJ_KIND_GSET_PRODUCT: return (uint64_t)elements * ((er + 63ull) / 64ull);
        case LASPJ_KIND_GCOUNTER: return elements;
        case LASPJ_KIND_ORSET_PRODUCT_WIDE: return 4ull * elements * er;
        case LASPJ_KIND_ORSET_WIDE: return 2ull * elements * er;        // er: token words
    }
    return 0;
}

bool is_product(int32_t kind) {
    return kind == LASPJ_KIND_ORSET_PRODUCT || kind == LASPJ_KIND_GSET_PRODUCT ||
           kind == LASPJ_KIND_ORSET_PRODUCT_WIDE;
}

int batch_create(laspj_ctx* ctx, int32_t kind, uint64_t replicas, uint32_t elements,
                 laspj_batch** out, uint32_t er = 0) {
    if (!ctx || !out) return fail(ctx, LASPJ_E_INVAL, "batch_create: null argument");
    *out = nullptr;
    if (replicas == 0 || elements == 0 || (is_product(kind) && er == 0))
        return fail(ctx, LASPJ_E_SHAPE, "batch_create: replicas and elements must be > 0");
    Guard g(ctx);
    auto* b = new (std::nothrow) laspj_batch;
    if (!b) return fail(ctx, LASPJ_E_NOMEM, "batch_create: host allocation");
    b->ctx = ctx;
    b->kind = kind;
    b->elements = elements;
    b->elements_r = is_product(kind) ? er : 0;
    b->tok_words = kind == LASPJ_KIND_ORSET_WIDE ? er : 1;
    b->cells = is_product(kind) ? (uint64_t)elements * er : elements;
    b->replicas = replicas;
    b->words_per_replica = words_per(kind, elements, er);
    uint64_t bytes = laspj::bytes_of(b);
    if (replicas > (~0ull / 8ull) / b->words_per_replica) {
        delete b;
        return fail(ctx, LASPJ_E_SHAPE, "batch_create: size overflow");
    }
    void* mem = nullptr;
    hipError_t e = laspj::dev_alloc(ctx, bytes, &mem);
    if (e != hipSuccess) {
        delete b;
        hipGetLastError();
        return fail(ctx, LASPJ_E_NOMEM, "batch_create: hipMalloc(%llu) failed: %s",
                    (unsigned long long)bytes, hipGetErrorString(e));
    }
    b->dev = static_cast<uint64_t*>(mem);
    e = hipMemsetAsync(b->dev, 0, bytes, ctx->stream);  // new/0 for every replica
    if (e != hipSuccess) {
        laspj::dev_release(ctx, b->dev, bytes);
        delete b;
        return fail(ctx, LASPJ_E_DEVICE, "batch_create: memset: %s", hipGetErrorString(e));
    }
    *out = b;
    return LASPJ_OK;
}

}  // namespace

namespace laspj {

// size classes: powers of two up to 4 MiB, then eighths of the next power of two (a
// block just past a power of two no longer takes twice its size)
static uint64_t cache_class(uint64_t bytes) {
    uint64_t c = 256;
    while (c < bytes) c <<= 1;
    if (c <= (4ull << 20)) return c;
    const uint64_t step = c >> 4;                       // c / 2 < bytes <= c
    return (bytes + step - 1) / step * step;
}

hipError_t dev_malloc(laspj_ctx* ctx, void** out, uint64_t bytes) {
    hipError_t e = hipMalloc(out, bytes);
    if (e != hipSuccess && !ctx->cache.empty()) {      // give the cached blocks back, retry
        hipGetLastError();
        dev_cache_clear(ctx);
        e = hipMalloc(out, bytes);
    }
    return e;
}

hipError_t dev_alloc(laspj_ctx* ctx, uint64_t bytes, void** out) {
    if (bytes <= kCacheMax) {
        const uint64_t c = cache_class(bytes);
        auto it = ctx->cache.find(c);
        if (it != ctx->cache.end() && !it->second.empty()) {
            *out = it->second.back();
            it->second.pop_back();
            ctx->cached_bytes -= c;
            return hipSuccess;
        }
        bytes = c;
    }
    return dev_malloc(ctx, out, bytes);
}

void dev_release(laspj_ctx* ctx, void* p, uint64_t bytes) {
    if (!p) return;
    if (bytes <= kCacheMax) {
        const uint64_t c = cache_class(bytes);
        if (ctx->cached_bytes + c <= kCacheCap) {
            ctx->cache[c].push_back(p);
            ctx->cached_bytes += c;
            return;
        }
    }
    hipStreamSynchronize(ctx->stream);
    hipFree(p);
}

void dev_cache_clear(laspj_ctx* ctx) {
    if (ctx->cache.empty()) return;
    hipStreamSynchronize(ctx->stream);
    for (auto& kv : ctx->cache)
        for (void* p : kv.second) hipFree(p);
    ctx->cache.clear();
    ctx->cached_bytes = 0;
}

hipError_t readback(laspj_ctx* ctx, const ReadPiece* pieces, int n) {
    uint64_t total = 0;
    for (int i = 0; i < n; ++i) total += (pieces[i].bytes + 15) & ~15ull;
    const bool stage = ctx->pinned && total <= laspj_ctx::kPinned;
    uint64_t at = 0;
    for (int i = 0; i < n; ++i) {
        if (!pieces[i].bytes) continue;
        void* to = stage ? static_cast<char*>(ctx->pinned) + at : pieces[i].host;
        hipError_t e = hipMemcpyAsync(to, pieces[i].dev, pieces[i].bytes, hipMemcpyDeviceToHost,
                                      ctx->stream);
        if (e != hipSuccess) return e;
        at += (pieces[i].bytes + 15) & ~15ull;
    }
    hipError_t e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess || !stage) return e;
    at = 0;
    for (int i = 0; i < n; ++i) {
        if (pieces[i].bytes)
            memcpy(pieces[i].host, static_cast<const char*>(ctx->pinned) + at, pieces[i].bytes);
        at += (pieces[i].bytes + 15) & ~15ull;
    }
    return hipSuccess;
}

}  // namespace laspj

extern "C" {

int laspj_abi_version(void) { return LASPJ_ABI_VERSION; }

const char* laspj_strerror(int s) {
    switch (s) {
        case LASPJ_OK: return "ok";
        case LASPJ_E_INVAL: return "invalid argument";
        case LASPJ_E_NOMEM: return "out of memory";
        case LASPJ_E_DEVICE: return "device error";
        case LASPJ_E_SHAPE: return "shape mismatch";
        case LASPJ_E_KIND: return "wrong batch kind";
        case LASPJ_E_RANGE: return "out of range";
        case LASPJ_E_COMM: return "communicator error";
        case LASPJ_E_UNSUPPORTED: return "unsupported";
        case LASPJ_E_FUN: return "fun failed";
        default: return "unknown status";
    }
}

int laspj_device_count(int* n) {
    if (!n) return LASPJ_E_INVAL;
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) {
        hipGetLastError();
        c = 0;
    }
    *n = c;
    return LASPJ_OK;
}

int laspj_ctx_create(int device, laspj_ctx** out) {
    if (!out) return LASPJ_E_INVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) {
        hipGetLastError();
        return LASPJ_E_DEVICE;
    }
    auto* ctx = new (std::nothrow) laspj_ctx;
    if (!ctx) return LASPJ_E_NOMEM;
    ctx->device = device;
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return LASPJ_E_DEVICE;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
        ctx->cus = prop.multiProcessorCount;
    if (hipMalloc(reinterpret_cast<void**>(&ctx->flag), 256) != hipSuccess) {
        hipStreamDestroy(ctx->stream);
        delete ctx;
        return LASPJ_E_NOMEM;
    }
    if (hipHostMalloc(&ctx->pinned, laspj_ctx::kPinned, hipHostMallocDefault) != hipSuccess) {
        hipGetLastError();
        ctx->pinned = nullptr;            // readbacks then go to pageable memory directly
    }
    *out = ctx;
    return LASPJ_OK;
}

int laspj_ctx_destroy(laspj_ctx* ctx) {
    if (!ctx) return LASPJ_E_INVAL;
    laspj::nif_destroy(ctx);
    laspj::list_etf_destroy(ctx);
    {
        Guard g(ctx);
        hipStreamSynchronize(ctx->stream);
        if (ctx->scratch) hipFree(ctx->scratch);
        if (ctx->flag) hipFree(ctx->flag);
        if (ctx->partials) hipFree(ctx->partials);
        if (ctx->lscratch) hipFree(ctx->lscratch);
        if (ctx->ltab) hipFree(ctx->ltab);
        if (ctx->lbind) hipFree(ctx->lbind);
        if (ctx->lbind_h) hipHostFree(ctx->lbind_h);
        if (ctx->lfz) hipFree(ctx->lfz);
        if (ctx->lfi) hipFree(ctx->lfi);
        if (ctx->lspec) hipFree(ctx->lspec);
        if (ctx->many_h) hipHostFree(ctx->many_h);
        laspj::dev_cache_clear(ctx);
        if (ctx->pinned) hipHostFree(ctx->pinned);
        if (ctx->dstage) hipHostFree(ctx->dstage);
        if (ctx->upring) hipHostFree(ctx->upring);
        hipStreamDestroy(ctx->stream);
    }
    delete ctx;
    return LASPJ_OK;
}

const char* laspj_ctx_last_error(const laspj_ctx* ctx) { return ctx ? ctx->err.c_str() : ""; }

int laspj_ctx_synchronize(laspj_ctx* ctx) {
    if (!ctx) return LASPJ_E_INVAL;
    Guard g(ctx);
    LJ_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return LASPJ_OK;
}

int laspj_ctx_set_tuning(laspj_ctx* ctx, int knob, int64_t value) {
    if (!ctx) return LASPJ_E_INVAL;
    Guard g(ctx);
    switch (knob) {
        case LASPJ_TUNE_STREAM_GRID:
            if (value < 0 || value > (1 << 20))
                return fail(ctx, LASPJ_E_INVAL, "tuning: grid out of range");
            ctx->tune_grid = value;
            return LASPJ_OK;
        case LASPJ_TUNE_STREAM_UNROLL:
            if (!(value == 0 || value == 1 || value == 2 || value == 4 || value == 8))
                return fail(ctx, LASPJ_E_INVAL, "tuning: unroll must be 0,1,2,4,8");
            ctx->tune_unroll = value;
            return LASPJ_OK;
        case LASPJ_TUNE_STREAM_NT:
            ctx->tune_nt = value;
            return LASPJ_OK;
        case LASPJ_TUNE_PRODUCT_ROWS:
            if (!(value == 0 || value == 32 || value == 64 || value == 128 || value == 256))
                return fail(ctx, LASPJ_E_INVAL, "tuning: product rows must be 0,32,64,128,256");
            ctx->tune_product_rows = value;
            return LASPJ_OK;
        case LASPJ_TUNE_PRODUCT_COLS:
            if (!(value == 0 || value == 1024 || value == 2048 || value == 4096))
                return fail(ctx, LASPJ_E_INVAL, "tuning: product cols must be 0,1024,2048,4096");
            ctx->tune_product_cols = value;
            return LASPJ_OK;
        case LASPJ_TUNE_REDUCE_KERNEL:
            if (value < 0 || value > 4)
                return fail(ctx, LASPJ_E_INVAL, "tuning: reduce kernel must be 0..4");
            ctx->tune_reduce = value;
            return LASPJ_OK;
        case LASPJ_TUNE_ETF_KERNEL:
            if (value < 0 || value > 6)
                return fail(ctx, LASPJ_E_INVAL, "tuning: etf kernel must be 0..6");
            ctx->tune_etf = value;
            return LASPJ_OK;
        case LASPJ_TUNE_ETF_READ:
            if (value < 0 || value > 15 || value == 9)
                return fail(ctx, LASPJ_E_INVAL, "tuning: etf read must be 0..8 or 10..15");
            ctx->tune_etf_read = value;
            return LASPJ_OK;
        case LASPJ_TUNE_ETF_SEG:
            if (value < 0 || value > (1ll << 30) || (value % 256) != 0)
                return fail(ctx, LASPJ_E_INVAL, "tuning: etf segment bytes must be 0 or a "
                            "multiple of 256");
            ctx->tune_etf_seg = value;
            return LASPJ_OK;
        case LASPJ_TUNE_LIST_WALK:
            if (value < 0 || value > 3) return fail(ctx, LASPJ_E_INVAL, "tuning: list walk 0 .. 3");
            ctx->tune_list_walk = value;
            return LASPJ_OK;
        case LASPJ_TUNE_NIF_PASSES:
            if (value < 0 || value > 16) return fail(ctx, LASPJ_E_INVAL, "tuning: NIF passes 0..16");
            ctx->tune_nif_passes = value;
            return LASPJ_OK;
        case LASPJ_TUNE_LIST_CHUNK:
            if (value != 0 && (value < 64 || value >= (1 << 20)))
                return fail(ctx, LASPJ_E_INVAL, "tuning: list chunk 0 or 64 .. 2^20");
            ctx->tune_list_chunk = value;
            return LASPJ_OK;

        default:
            return fail(ctx, LASPJ_E_INVAL, "tuning: unknown knob %d", knob);
    }
}

// ------------------------------------------------------------------------- buffers

int laspj_buf_create(laspj_ctx* ctx, uint64_t bytes, laspj_buf** out) {
    if (!ctx || !out) return fail(ctx, LASPJ_E_INVAL, "buf_create: null argument");
    *out = nullptr;
    Guard g(ctx);
    auto* b = new (std::nothrow) laspj_buf;
    if (!b) return fail(ctx, LASPJ_E_NOMEM, "buf_create: host allocation");
    b->ctx = ctx;
    b->bytes = bytes;
    if (bytes) {
        hipError_t e = laspj::dev_alloc(ctx, bytes, &b->dev);
        if (e != hipSuccess) {
            delete b;
            hipGetLastError();
            return fail(ctx, LASPJ_E_NOMEM, "buf_create: hipMalloc(%llu): %s",
                        (unsigned long long)bytes, hipGetErrorString(e));
        }
        e = hipMemsetAsync(b->dev, 0, bytes, ctx->stream);
        if (e != hipSuccess) {
            laspj::dev_release(ctx, b->dev, bytes);
            delete b;
            return fail(ctx, LASPJ_E_DEVICE, "buf_create: memset: %s", hipGetErrorString(e));
        }
    }
    *out = b;
    return LASPJ_OK;
}

int laspj_buf_destroy(laspj_buf* b) {
    if (!b) return LASPJ_E_INVAL;
    {
        Guard g(b->ctx);
        // an exported block may still be in use on another stream (a collective, a torch
        // kernel): wait for the device before the block cache can hand it out again
        if (b->exported) hipDeviceSynchronize();
        laspj::dev_release(b->ctx, b->dev, b->bytes);
    }
    delete b;
    return LASPJ_OK;
}

uint64_t laspj_buf_bytes(const laspj_buf* b) { return b ? b->bytes : 0; }

int laspj_buf_device_ptr(const laspj_buf* b, void** out) {
    if (!b || !out) return LASPJ_E_INVAL;
    b->exported = true;
    *out = b->dev;
    return LASPJ_OK;
}

}  // extern "C"

namespace laspj {
// a copy of src[0, bytes) in the context's pinned ring, to be copied to the device on its
// stream; null when it does not fit (bytes > kUpSmall) or the ring cannot be allocated.
// Call with ctx->mu held.
const void* stage_small(laspj_ctx* ctx, const void* src, uint64_t bytes) {
    if (bytes > laspj_ctx::kUpSmall) return nullptr;
    if (!ctx->upring) {
        if (hipHostMalloc(&ctx->upring, laspj_ctx::kUpRing, hipHostMallocDefault) != hipSuccess) {
            hipGetLastError();
            ctx->upring = nullptr;
            return nullptr;
        }
        void* dp = nullptr;
        if (hipHostGetDevicePointer(&dp, ctx->upring, 0) != hipSuccess) {
            hipGetLastError();
            dp = nullptr;
        }
        ctx->upring_dev = static_cast<const uint8_t*>(dp);
    }
    const uint64_t need = (bytes + 255) & ~255ull;
    if (ctx->upring_at + need > laspj_ctx::kUpRing) {
        // the ring's earlier copies must be done before its bytes are rewritten
        if (hipStreamSynchronize(ctx->stream) != hipSuccess) return nullptr;
        ctx->upring_at = 0;
    }
    char* slot = static_cast<char*>(ctx->upring) + ctx->upring_at;
    std::memcpy(slot, src, bytes);
    ctx->upring_at += need;
    return slot;
}

const void* staged_dev(const laspj_ctx* ctx, const void* slot) {
    if (!ctx->upring_dev || !slot) return nullptr;
    return ctx->upring_dev + (static_cast<const char*>(slot) - static_cast<const char*>(ctx->upring));
}
}  // namespace laspj

extern "C" {

int laspj_buf_upload(laspj_ctx* ctx, laspj_buf* b, uint64_t off, const void* src,
                     uint64_t bytes) {
    if (!ctx || !b || b->ctx != ctx || (!src && bytes))
        return fail(ctx, LASPJ_E_INVAL, "buf_upload: bad argument");
    if (off > b->bytes || bytes > b->bytes - off)
        return fail(ctx, LASPJ_E_RANGE, "buf_upload: range out of bounds");
    Guard g(ctx);
    if (!bytes) return LASPJ_OK;
    if (bytes <= laspj_ctx::kUpSmall && !b->exported) {
        // small and used on the context's stream only: staged in the pinned ring, the copy
        // enqueued, no wait (every later kernel, copy or readback of the buffer is on the
        // same stream, after it)
        if (const void* slot = laspj::stage_small(ctx, src, bytes)) {
            LJ_HIP(ctx, hipMemcpyAsync(static_cast<char*>(b->dev) + off, slot, bytes,
                                       hipMemcpyHostToDevice, ctx->stream));
            return LASPJ_OK;
        }
    }
    LJ_HIP(ctx, hipMemcpyAsync(static_cast<char*>(b->dev) + off, src, bytes,
                               hipMemcpyHostToDevice, ctx->stream));
    LJ_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return LASPJ_OK;
}

int laspj_buf_download(laspj_ctx* ctx, const laspj_buf* b, uint64_t off, void* dst,
                       uint64_t bytes) {
    if (!ctx || !b || b->ctx != ctx || (!dst && bytes))
        return fail(ctx, LASPJ_E_INVAL, "buf_download: bad argument");
    if (off > b->bytes || bytes > b->bytes - off)
        return fail(ctx, LASPJ_E_RANGE, "buf_download: range out of bounds");
    Guard g(ctx);
    if (!bytes) return LASPJ_OK;
    LJ_HIP(ctx, laspj::readback(ctx, dst, static_cast<const char*>(b->dev) + off, bytes));
    return LASPJ_OK;
}

// ------------------------------------------------------------------------- batches

int laspj_orset_batch_create(laspj_ctx* ctx, uint64_t replicas, uint32_t elements,
                             laspj_batch** out) {
    return batch_create(ctx, LASPJ_KIND_ORSET, replicas, elements, out);
}

int laspj_orset_wide_batch_create(laspj_ctx* ctx, uint64_t replicas, uint32_t elements,
                                  uint32_t token_words, laspj_batch** out) {
    if (token_words < 1 || token_words > 16)
        return fail(ctx, LASPJ_E_INVAL, "orset_wide_batch_create: token words must be 1..16");
    return batch_create(ctx, LASPJ_KIND_ORSET_WIDE, replicas, elements, out, token_words);
}

int laspj_orset_widen(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src) {
    if (!same_ctx(ctx, dst) || !same_ctx(ctx, src))
        return fail(ctx, LASPJ_E_INVAL, "orset_widen: bad batch");
    if (dst->kind != LASPJ_KIND_ORSET_WIDE ||
        (src->kind != LASPJ_KIND_ORSET && src->kind != LASPJ_KIND_ORSET_WIDE))
        return fail(ctx, LASPJ_E_KIND, "orset_widen: OR-Set source, wide destination");
    if (dst->replicas != src->replicas || dst->elements != src->elements ||
        src->tok_words > dst->tok_words)
        return fail(ctx, LASPJ_E_SHAPE, "orset_widen: shapes differ or the source is wider");
    if (dst->dev == src->dev) return fail(ctx, LASPJ_E_INVAL, "orset_widen: dst aliases src");
    Guard g(ctx);
    LJ_HIP(ctx, laspj::launch_wide_widen(ctx, dst, src));
    return LASPJ_OK;
}

int laspj_gset_batch_create(laspj_ctx* ctx, uint64_t replicas, uint32_t elements,
                            laspj_batch** out) {
    return batch_create(ctx, LASPJ_KIND_GSET, replicas, elements, out);
}

int laspj_batch_destroy(laspj_batch* b) {
    if (!b) return LASPJ_E_INVAL;
    {
        Guard g(b->ctx);
        if (b->owns && b->exported) hipDeviceSynchronize();        // as laspj_buf_destroy
        if (b->owns) laspj::dev_release(b->ctx, b->dev, laspj::bytes_of(b));
    }
    delete b;
    return LASPJ_OK;
}

int laspj_batch_wrap(laspj_ctx* ctx, int32_t kind, void* dev, uint64_t bytes,
                     uint64_t replicas, uint32_t elements, laspj_batch** out) {
    if (!ctx || !out || !dev) return fail(ctx, LASPJ_E_INVAL, "batch_wrap: null argument");
    *out = nullptr;
    if (kind != LASPJ_KIND_ORSET && kind != LASPJ_KIND_GSET && kind != LASPJ_KIND_GCOUNTER)
        return fail(ctx, LASPJ_E_KIND, "batch_wrap: OR-Set, G-Set or G-Counter only");
    if (replicas == 0 || elements == 0)
        return fail(ctx, LASPJ_E_SHAPE, "batch_wrap: empty shape");
    uint64_t wpr = words_per(kind, elements, 0);
    if (replicas > (~0ull / 8ull) / wpr || replicas * wpr * 8ull != bytes)
        return fail(ctx, LASPJ_E_SHAPE, "batch_wrap: %llu bytes do not hold %llu x %u",
                    (unsigned long long)bytes, (unsigned long long)replicas, elements);
    if (reinterpret_cast<uintptr_t>(dev) % 16)
        return fail(ctx, LASPJ_E_INVAL, "batch_wrap: device pointer not 16-byte aligned");
    auto* b = new (std::nothrow) laspj_batch;
    if (!b) return fail(ctx, LASPJ_E_NOMEM, "batch_wrap: host allocation");
    b->ctx = ctx;
    b->kind = kind;
    b->elements = elements;
    b->cells = elements;
    b->replicas = replicas;
    b->words_per_replica = wpr;
    b->dev = static_cast<uint64_t*>(dev);
    b->owns = false;
    *out = b;
    return LASPJ_OK;
}

int laspj_batch_reduce_chunks(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                              uint32_t nchunks) {
    if (!same_ctx(ctx, dst) || !same_ctx(ctx, src))
        return fail(ctx, LASPJ_E_INVAL, "reduce_chunks: bad batch");
    if (dst->kind != src->kind || laspj_is_list(dst->kind))
        return fail(ctx, LASPJ_E_KIND, "reduce_chunks: kinds differ or list batch");
    if (nchunks == 0 || dst->words_per_replica != src->words_per_replica ||
        dst->elements != src->elements || dst->replicas * (uint64_t)nchunks != src->replicas)
        return fail(ctx, LASPJ_E_SHAPE, "reduce_chunks: need src replicas = nchunks x dst");
    if (dst->dev == src->dev) return fail(ctx, LASPJ_E_INVAL, "reduce_chunks: dst aliases src");
    Guard g(ctx);
    // the join of the batch's lattice: OR for bitmaps, per-actor max for G-Counters
    LJ_HIP(ctx, laspj::launch_reduce_chunks(ctx, dst->dev, src->dev,
                                            dst->replicas * dst->words_per_replica, nchunks,
                                            dst->kind == LASPJ_KIND_GCOUNTER));
    return LASPJ_OK;
}

int laspj_batch_join_n(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* const* srcs,
                       uint32_t n) {
    if (!same_ctx(ctx, dst) || !srcs || n < 1 || n > 8)
        return fail(ctx, LASPJ_E_INVAL, "join_n: bad batch or n not in 1..8");
    if (laspj_is_list(dst->kind)) return fail(ctx, LASPJ_E_KIND, "join_n: list batch");
    const uint64_t* p[8];
    for (uint32_t j = 0; j < n; ++j) {
        const laspj_batch* s = srcs[j];
        if (!same_ctx(ctx, s)) return fail(ctx, LASPJ_E_INVAL, "join_n: bad source %u", j);
        if (s->kind != dst->kind) return fail(ctx, LASPJ_E_KIND, "join_n: kinds differ");
        if (s->replicas != dst->replicas || s->elements != dst->elements ||
            s->words_per_replica != dst->words_per_replica)
            return fail(ctx, LASPJ_E_SHAPE, "join_n: shapes differ");
        p[j] = s->dev;
    }
    Guard g(ctx);
    LJ_HIP(ctx, laspj::launch_reduce_ptrs(ctx, dst->dev, p, n,
                                          dst->replicas * dst->words_per_replica,
                                          dst->kind == LASPJ_KIND_GCOUNTER));
    return LASPJ_OK;
}

int laspj_batch_info_get(const laspj_batch* b, laspj_batch_info* out) {
    if (!b || !out) return LASPJ_E_INVAL;
    out->kind = b->kind;
    out->elements = b->elements;
    out->replicas = b->replicas;
    out->bytes_per_replica = b->words_per_replica * 8ull;
    out->bytes = laspj::bytes_of(b);
    out->elements_r = b->elements_r;
    out->token_words = b->tok_words;
    out->cells_per_replica = b->cells;
    return LASPJ_OK;
}

int laspj_batch_device_ptr(const laspj_batch* b, void** out) {
    if (!b || !out) return LASPJ_E_INVAL;
    if (laspj_is_list(b->kind)) return LASPJ_E_KIND;
    b->exported = true;
    *out = b->dev;
    return LASPJ_OK;
}

int laspj_batch_download_range(laspj_ctx* ctx, const laspj_batch* b, uint64_t offset,
                               uint64_t bytes, void* host) {
    if (!same_ctx(ctx, b) || (!host && bytes))
        return fail(ctx, LASPJ_E_INVAL, "batch_download_range: bad argument");
    if (laspj_is_list(b->kind))
        return fail(ctx, LASPJ_E_KIND, "batch_download_range: list batches use laspj_list_download");
    const uint64_t total = laspj::bytes_of(b);
    if (offset > total || bytes > total - offset)
        return fail(ctx, LASPJ_E_RANGE, "batch_download_range: range out of bounds");
    Guard g(ctx);
    if (!bytes) return LASPJ_OK;
    LJ_HIP(ctx, laspj::readback(ctx, host, reinterpret_cast<const char*>(b->dev) + offset, bytes));
    return LASPJ_OK;
}

int laspj_batch_upload(laspj_ctx* ctx, laspj_batch* b, uint64_t first, uint64_t count,
                       const void* host) {
    if (!same_ctx(ctx, b) || (!host && count))
        return fail(ctx, LASPJ_E_INVAL, "batch_upload: bad argument");
    if (laspj_is_list(b->kind))
        return fail(ctx, LASPJ_E_KIND, "batch_upload: list batches use laspj_list_upload");
    if (first > b->replicas || count > b->replicas - first)
        return fail(ctx, LASPJ_E_RANGE, "batch_upload: replicas [%llu, +%llu) out of %llu",
                    (unsigned long long)first, (unsigned long long)count,
                    (unsigned long long)b->replicas);
    Guard g(ctx);
    uint64_t rb = b->words_per_replica * 8ull;
    LJ_HIP(ctx, hipMemcpyAsync(reinterpret_cast<char*>(b->dev) + first * rb, host, count * rb,
                               hipMemcpyHostToDevice, ctx->stream));
    LJ_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return LASPJ_OK;
}

int laspj_batch_download(laspj_ctx* ctx, const laspj_batch* b, uint64_t first,
                         uint64_t count, void* host) {
    if (!same_ctx(ctx, b) || (!host && count))
        return fail(ctx, LASPJ_E_INVAL, "batch_download: bad argument");
    if (laspj_is_list(b->kind))
        return fail(ctx, LASPJ_E_KIND, "batch_download: list batches use laspj_list_download");
    if (first > b->replicas || count > b->replicas - first)
        return fail(ctx, LASPJ_E_RANGE, "batch_download: replicas out of range");
    Guard g(ctx);
    uint64_t rb = b->words_per_replica * 8ull;
    LJ_HIP(ctx, laspj::readback(ctx, host, reinterpret_cast<const char*>(b->dev) + first * rb, count * rb));
    return LASPJ_OK;
}

int laspj_batch_clear(laspj_ctx* ctx, laspj_batch* b) {
    if (!same_ctx(ctx, b)) return fail(ctx, LASPJ_E_INVAL, "batch_clear: bad argument");
    Guard g(ctx);
    LJ_HIP(ctx, hipMemsetAsync(b->dev, 0, laspj::bytes_of(b), ctx->stream));
    return LASPJ_OK;
}

int laspj_batch_fill_synthetic_tokens(laspj_ctx* ctx, laspj_batch* b, uint64_t seed,
                                      uint64_t replica_base, uint32_t token_slots) {
    if (!same_ctx(ctx, b)) return fail(ctx, LASPJ_E_INVAL, "fill_synthetic: bad argument");
    if (b->kind != LASPJ_KIND_ORSET)
        return fail(ctx, LASPJ_E_KIND, "fill_synthetic_tokens: OR-Set batches only");
    if (token_slots < 1 || token_slots > 64)
        return fail(ctx, LASPJ_E_INVAL, "fill_synthetic_tokens: token slots must be 1..64");
    Guard g(ctx);
    const uint64_t mask = token_slots == 64 ? ~0ull : ((1ull << token_slots) - 1ull);
    LJ_HIP(ctx, laspj::launch_fill_synthetic(ctx, b, seed, replica_base, mask));
    return LASPJ_OK;
}

int laspj_batch_fill_synthetic(laspj_ctx* ctx, laspj_batch* b, uint64_t seed,
                               uint64_t replica_base) {
    if (!same_ctx(ctx, b)) return fail(ctx, LASPJ_E_INVAL, "fill_synthetic: bad argument");
    if (b->kind != LASPJ_KIND_ORSET && b->kind != LASPJ_KIND_GSET &&
        b->kind != LASPJ_KIND_GCOUNTER && b->kind != LASPJ_KIND_ORSET_WIDE)
        return fail(ctx, LASPJ_E_KIND, "fill_synthetic: OR-Set, G-Set or G-Counter batches only");
    Guard g(ctx);
    if (b->kind == LASPJ_KIND_ORSET_WIDE) {
        // pair j of element e = the narrow stream's cell e k + j (bench data)
        laspj_batch v = *b;
        v.kind = LASPJ_KIND_ORSET;
        v.elements = b->elements * b->tok_words;
        v.cells = v.elements;
        v.tok_words = 1;
        v.owns = false;
        LJ_HIP(ctx, laspj::launch_fill_synthetic(ctx, &v, seed, replica_base));
        return LASPJ_OK;
    }
    LJ_HIP(ctx, laspj::launch_fill_synthetic(ctx, b, seed, replica_base));
    return LASPJ_OK;
}

// the OR-Set entry points take wide batches too (the same words, k pairs per cell)
static int32_t orset_kind(const laspj_batch* a, int32_t kind) {
    return kind == LASPJ_KIND_ORSET && a && a->kind == LASPJ_KIND_ORSET_WIDE
               ? LASPJ_KIND_ORSET_WIDE : kind;
}

int laspj_orset_fragment(laspj_ctx* ctx, const laspj_batch* b, uint32_t element,
                         laspj_buf* out) {
    if (!same_ctx(ctx, b)) return fail(ctx, LASPJ_E_INVAL, "orset_fragment: bad batch");
    if (b->kind != LASPJ_KIND_ORSET && b->kind != LASPJ_KIND_ORSET_WIDE)
        return fail(ctx, LASPJ_E_KIND, "orset_fragment: kind");
    if (element >= b->elements) return fail(ctx, LASPJ_E_RANGE, "orset_fragment: element slot");
    if (int s = check_buf(ctx, out, 16ull * b->replicas * b->tok_words, "orset_fragment")) return s;
    Guard g(ctx);
    LJ_HIP(ctx, laspj::launch_orset_fragment(ctx, b, element, out->dev));
    return LASPJ_OK;
}

int laspj_orset_precondition_context(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src) {
    if (int s = check_pair(ctx, dst, src, orset_kind(src, LASPJ_KIND_ORSET),
                           "orset_precondition_context"))
        return s;
    Guard g(ctx);
    LJ_HIP(ctx, laspj::launch_orset_context(ctx, dst, src));
    return LASPJ_OK;
}

static int gather_inflation_impl(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                                 const laspj_buf* index, const laspj_buf* head,
                                 const laspj_buf* next, const laspj_batch* prev, int strict,
                                 laspj_buf* out, const char* what) {
    if (!same_ctx(ctx, dst) || !same_ctx(ctx, src) || !same_ctx(ctx, prev))
        return fail(ctx, LASPJ_E_INVAL, "%s: bad batch", what);
    if (dst->kind != LASPJ_KIND_ORSET || src->kind != LASPJ_KIND_ORSET ||
        prev->kind != LASPJ_KIND_ORSET)
        return fail(ctx, LASPJ_E_KIND, "%s: OR-Set batches only", what);
    if (dst->replicas != src->replicas || prev->elements != dst->elements ||
        (prev->replicas != dst->replicas && prev->replicas != 1))
        return fail(ctx, LASPJ_E_SHAPE, "%s: shapes", what);
    if (dst->dev == src->dev || dst->dev == prev->dev)
        return fail(ctx, LASPJ_E_INVAL, "%s: dst aliases an input", what);
    if (int s = check_buf(ctx, index, 4ull * dst->elements, what)) return s;
    if (head || next) {
        if (!head || !next) return fail(ctx, LASPJ_E_INVAL, "%s: head and next go together", what);
        if (int s = check_buf(ctx, head, 4ull * dst->elements, what)) return s;
        if (int s = check_buf(ctx, next, 4ull * dst->elements, what)) return s;
    }
    if (int s = check_buf(ctx, out, dst->replicas, what)) return s;
    Guard g(ctx);
    LJ_HIP(ctx, laspj::launch_gather_inflation(
                    ctx, dst, src, static_cast<const uint32_t*>(index->dev),
                    head ? static_cast<const uint32_t*>(head->dev) : nullptr,
                    next ? static_cast<const uint32_t*>(next->dev) : nullptr, prev, strict != 0,
                    static_cast<uint8_t*>(out->dev)));
    return LASPJ_OK;
}

int laspj_orset_gather_inflation(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                                 const laspj_buf* index, const laspj_batch* prev, int strict,
                                 laspj_buf* out) {
    return gather_inflation_impl(ctx, dst, src, index, nullptr, nullptr, prev, strict, out,
                                 "gather_inflation");
}

int laspj_orset_gather_inflation_keyed(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                                       const laspj_buf* index, const laspj_buf* head,
                                       const laspj_buf* next, const laspj_batch* prev, int strict,
                                       laspj_buf* out) {
    if (!head || !next) return fail(ctx, LASPJ_E_INVAL, "gather_inflation_keyed: head / next");
    return gather_inflation_impl(ctx, dst, src, index, head, next, prev, strict, out,
                                 "gather_inflation_keyed");
}

// ------------------------------------------------------------------------- joins

static int join_impl(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* a,
                     const laspj_batch* b, int32_t kind, const char* what) {
    kind = orset_kind(a, kind);
    if (int s = check_pair(ctx, a, b, kind, what)) return s;
    if (int s = check_pair(ctx, dst, a, kind, what)) return s;
    Guard g(ctx);
    LJ_HIP(ctx, laspj::launch_or(ctx, dst->dev, a->dev, b->dev,
                                 a->replicas * a->words_per_replica));
    return LASPJ_OK;
}

int laspj_batch_join(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* a,
                     const laspj_batch* b) {
    if (!same_ctx(ctx, dst) || !same_ctx(ctx, a) || !same_ctx(ctx, b))
        return fail(ctx, LASPJ_E_INVAL, "batch_join: bad batch");
    if (a->kind != b->kind || dst->kind != a->kind)
        return fail(ctx, LASPJ_E_KIND, "batch_join: kinds differ");
    if (laspj_is_list(a->kind))
        return fail(ctx, LASPJ_E_KIND, "batch_join: list batches join with laspj_list_merge");
    if (a->replicas != b->replicas || dst->replicas != a->replicas ||
        a->words_per_replica != b->words_per_replica ||
        dst->words_per_replica != a->words_per_replica || a->elements != b->elements ||
        a->elements_r != b->elements_r)
        return fail(ctx, LASPJ_E_SHAPE, "batch_join: shapes differ");
    Guard g(ctx);
    const uint64_t words = a->replicas * a->words_per_replica;
    if (a->kind == LASPJ_KIND_GCOUNTER)     // riak_dt_gcounter merge: per-actor max
        LJ_HIP(ctx, laspj::launch_max(ctx, dst->dev, a->dev, b->dev, words));
    else
        LJ_HIP(ctx, laspj::launch_or(ctx, dst->dev, a->dev, b->dev, words));
    return LASPJ_OK;
}

int laspj_orset_join(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* a,
                     const laspj_batch* b) {
    return join_impl(ctx, dst, a, b, LASPJ_KIND_ORSET, "orset_join");
}

int laspj_gset_join(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* a,
                    const laspj_batch* b) {
    return join_impl(ctx, dst, a, b, LASPJ_KIND_GSET, "gset_join");
}

static int reduce_impl(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                       uint32_t group, int32_t kind, const char* what) {
    if (!same_ctx(ctx, dst) || !same_ctx(ctx, src))
        return fail(ctx, LASPJ_E_INVAL, "%s: bad batch", what);
    kind = orset_kind(src, kind);
    if (dst->kind != kind || src->kind != kind)
        return fail(ctx, LASPJ_E_KIND, "%s: wrong batch kind", what);
    if (group == 0 || dst->elements != src->elements ||
        dst->words_per_replica != src->words_per_replica ||
        dst->replicas * (uint64_t)group != src->replicas)
        return fail(ctx, LASPJ_E_SHAPE, "%s: need src replicas = dst replicas * group", what);
    if (dst->dev == src->dev) return fail(ctx, LASPJ_E_INVAL, "%s: dst aliases src", what);
    Guard g(ctx);
    LJ_HIP(ctx, laspj::launch_reduce_or(ctx, dst->dev, src->dev, dst->replicas, group,
                                        src->words_per_replica));
    return LASPJ_OK;
}

int laspj_orset_reduce(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                       uint32_t group) {
    return reduce_impl(ctx, dst, src, group, LASPJ_KIND_ORSET, "orset_reduce");
}

int laspj_gset_reduce(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                      uint32_t group) {
    return reduce_impl(ctx, dst, src, group, LASPJ_KIND_GSET, "gset_reduce");
}

// ------------------------------------------------------------------------- predicates

static int value_impl(laspj_ctx* ctx, const laspj_batch* b, laspj_buf* out, bool removed) {
    const char* what = removed ? "orset_removed" : "orset_value";
    if (!same_ctx(ctx, b)) return fail(ctx, LASPJ_E_INVAL, "%s: bad batch", what);
    bool ok_kind = b->kind == LASPJ_KIND_ORSET || b->kind == LASPJ_KIND_ORSET_WIDE ||
                   (!removed && (b->kind == LASPJ_KIND_ORSET_CONCAT ||
                                 b->kind == LASPJ_KIND_ORSET_PRODUCT ||
                                 b->kind == LASPJ_KIND_ORSET_PRODUCT_WIDE));
    if (!ok_kind) return fail(ctx, LASPJ_E_KIND, "%s: not an OR-Set batch", what);
    uint64_t need = b->replicas * ((b->cells + 63ull) / 64ull) * 8ull;
    if (int s = check_buf(ctx, out, need, what)) return s;
    Guard g(ctx);
    if (b->kind == LASPJ_KIND_ORSET_WIDE)
        LJ_HIP(ctx, laspj::launch_wide_value(ctx, b, static_cast<uint64_t*>(out->dev), removed));
    else
        LJ_HIP(ctx, laspj::launch_orset_value(ctx, b, static_cast<uint64_t*>(out->dev), removed));
    return LASPJ_OK;
}

int laspj_orset_value(laspj_ctx* ctx, const laspj_batch* b, laspj_buf* out) {
    return value_impl(ctx, b, out, false);
}

int laspj_orset_removed(laspj_ctx* ctx, const laspj_batch* b, laspj_buf* out) {
    return value_impl(ctx, b, out, true);
}

int laspj_orset_stats(laspj_ctx* ctx, const laspj_batch* b, laspj_buf* out) {
    if (!same_ctx(ctx, b)) return fail(ctx, LASPJ_E_INVAL, "orset_stats: bad batch");
    if (b->kind != LASPJ_KIND_ORSET && b->kind != LASPJ_KIND_ORSET_WIDE)
        return fail(ctx, LASPJ_E_KIND, "orset_stats: not an OR-Set");
    if (int s = check_buf(ctx, out, b->replicas * 24ull, "orset_stats")) return s;
    Guard g(ctx);
    if (b->kind == LASPJ_KIND_ORSET_WIDE)
        LJ_HIP(ctx, laspj::launch_wide_stats(ctx, b, static_cast<uint64_t*>(out->dev)));
    else
        LJ_HIP(ctx, laspj::launch_orset_stats(ctx, b, static_cast<uint64_t*>(out->dev)));
    return LASPJ_OK;
}

int laspj_gset_stats(laspj_ctx* ctx, const laspj_batch* b, laspj_buf* out) {
    if (!same_ctx(ctx, b)) return fail(ctx, LASPJ_E_INVAL, "gset_stats: bad batch");
    if (b->kind != LASPJ_KIND_GSET) return fail(ctx, LASPJ_E_KIND, "gset_stats: not a G-Set");
    if (int s = check_buf(ctx, out, b->replicas * 8ull, "gset_stats")) return s;
    Guard g(ctx);
    LJ_HIP(ctx, laspj::launch_gset_stats(ctx, b, static_cast<uint64_t*>(out->dev)));
    return LASPJ_OK;
}

static int equal_impl(laspj_ctx* ctx, const laspj_batch* a, const laspj_batch* b,
                      laspj_buf* out, int32_t kind, const char* what) {
    kind = orset_kind(a, kind);
    if (int s = check_pair(ctx, a, b, kind, what)) return s;
    if (int s = check_buf(ctx, out, a->replicas, what)) return s;
    Guard g(ctx);
    LJ_HIP(ctx, laspj::launch_equal(ctx, a, b, static_cast<uint8_t*>(out->dev)));
    return LASPJ_OK;
}

int laspj_orset_equal(laspj_ctx* ctx, const laspj_batch* a, const laspj_batch* b,
                      laspj_buf* out) {
    return equal_impl(ctx, a, b, out, LASPJ_KIND_ORSET, "orset_equal");
}

int laspj_gset_equal(laspj_ctx* ctx, const laspj_batch* a, const laspj_batch* b,
                     laspj_buf* out) {
    return equal_impl(ctx, a, b, out, LASPJ_KIND_GSET, "gset_equal");
}

static int inflation_impl(laspj_ctx* ctx, const laspj_batch* prev, const laspj_batch* cur,
                          int strict, laspj_buf* out, int32_t kind, const char* what) {
    if (!same_ctx(ctx, prev) || !same_ctx(ctx, cur))
        return fail(ctx, LASPJ_E_INVAL, "%s: bad batch", what);
    kind = orset_kind(cur, kind);
    if (prev->kind != kind || cur->kind != kind)
        return fail(ctx, LASPJ_E_KIND, "%s: wrong batch kind", what);
    if (prev->elements != cur->elements || prev->tok_words != cur->tok_words ||
        !(prev->replicas == cur->replicas || prev->replicas == 1))
        return fail(ctx, LASPJ_E_SHAPE, "%s: prev must have cur's replicas or 1", what);
    if (int s = check_buf(ctx, out, cur->replicas, what)) return s;
    Guard g(ctx);
    if (kind == LASPJ_KIND_ORSET_WIDE)
        LJ_HIP(ctx, laspj::launch_wide_inflation(ctx, prev, cur, strict != 0,
                                                 static_cast<uint8_t*>(out->dev)));
    else if (kind == LASPJ_KIND_ORSET)
        LJ_HIP(ctx, laspj::launch_orset_inflation(ctx, prev, cur, strict != 0,
                                                  static_cast<uint8_t*>(out->dev)));
    else
        LJ_HIP(ctx, laspj::launch_gset_inflation(ctx, prev, cur, strict != 0,
                                                 static_cast<uint8_t*>(out->dev)));
    return LASPJ_OK;
}

int laspj_orset_inflation(laspj_ctx* ctx, const laspj_batch* prev, const laspj_batch* cur,
                          int strict, laspj_buf* out) {
    return inflation_impl(ctx, prev, cur, strict, out, LASPJ_KIND_ORSET, "orset_inflation");
}

int laspj_gset_inflation(laspj_ctx* ctx, const laspj_batch* prev, const laspj_batch* cur,
                         int strict, laspj_buf* out) {
    return inflation_impl(ctx, prev, cur, strict, out, LASPJ_KIND_GSET, "gset_inflation");
}

// ------------------------------------------------------------------------- updates

static int apply_ops_impl(laspj_ctx* ctx, laspj_batch* b, const laspj_op* ops, uint64_t nops,
                          int32_t* status, int32_t kind, const char* what) {
    if (!same_ctx(ctx, b) || (!ops && nops))
        return fail(ctx, LASPJ_E_INVAL, "%s: bad argument", what);
    kind = orset_kind(b, kind);
    if (b->kind != kind) return fail(ctx, LASPJ_E_KIND, "%s: wrong batch kind", what);
    const uint32_t tslots = 64u * b->tok_words;
    // Host-side validation: every op addresses a real cell and the list is grouped by
    // replica, which is what the one-thread-per-replica-run kernel relies on.
    for (uint64_t i = 0; i < nops; ++i) {
        const laspj_op& o = ops[i];
        if (o.replica >= b->replicas || o.element >= b->elements)
            return fail(ctx, LASPJ_E_RANGE, "%s: op %llu addresses (%llu, %u) outside %llu x %u",
                        what, (unsigned long long)i, (unsigned long long)o.replica, o.element,
                        (unsigned long long)b->replicas, b->elements);
        const uint32_t tslot = kind == LASPJ_KIND_ORSET_WIDE ? (uint32_t)o.slot | ((uint32_t)o.pad << 8)
                                                              : o.slot;
        if (tslot >= tslots || (kind != LASPJ_KIND_ORSET_WIDE && o.pad))
            return fail(ctx, LASPJ_E_RANGE, "%s: op %llu token slot %u >= %u", what,
                        (unsigned long long)i, tslot, tslots);
        bool ok_kind = kind == LASPJ_KIND_ORSET || kind == LASPJ_KIND_ORSET_WIDE
                           ? (o.kind == LASPJ_OP_ADD || o.kind == LASPJ_OP_REMOVE ||
                              o.kind == LASPJ_OP_INSERT)
                           : o.kind == LASPJ_OP_ADD;
        if (!ok_kind) return fail(ctx, LASPJ_E_INVAL, "%s: op %llu has kind %u", what,
                                  (unsigned long long)i, o.kind);
        if (i && ops[i - 1].replica > o.replica)
            return fail(ctx, LASPJ_E_INVAL, "%s: ops not sorted by replica at %llu", what,
                        (unsigned long long)i);
        // no status array: only for ADDs, whose precondition cannot fail (every status
        // would be APPLIED), so nothing is read back and nothing waits for the device
        if (!status && o.kind != LASPJ_OP_ADD)
            return fail(ctx, LASPJ_E_INVAL, "%s: a null status needs every op to be an ADD",
                        what);
    }
    if (!nops) return LASPJ_OK;
    Guard g(ctx);
    uint64_t need = nops * (sizeof(laspj_op) + sizeof(int32_t));
    if (ctx->scratch_bytes < need) {
        if (ctx->scratch) {
            LJ_HIP(ctx, hipStreamSynchronize(ctx->stream));
            hipFree(ctx->scratch);
            ctx->scratch = nullptr;
            ctx->scratch_bytes = 0;
        }
        if (laspj::dev_malloc(ctx, &ctx->scratch, need) != hipSuccess) {
            hipGetLastError();
            return fail(ctx, LASPJ_E_NOMEM, "%s: scratch allocation", what);
        }
        ctx->scratch_bytes = need;
    }
    auto* dops = static_cast<laspj_op*>(ctx->scratch);
    auto* dst = reinterpret_cast<int32_t*>(dops + nops);
    LJ_HIP(ctx, hipMemcpyAsync(dops, ops, nops * sizeof(laspj_op), hipMemcpyHostToDevice,
                               ctx->stream));
    if (kind == LASPJ_KIND_ORSET_WIDE)
        LJ_HIP(ctx, laspj::launch_wide_apply(ctx, b, dops, nops, dst));
    else
        LJ_HIP(ctx, laspj::launch_apply_ops(ctx, b, dops, nops, dst));
    if (status) LJ_HIP(ctx, laspj::readback(ctx, status, dst, nops * sizeof(int32_t)));
    return LASPJ_OK;
}

int laspj_orset_apply_ops(laspj_ctx* ctx, laspj_batch* b, const laspj_op* ops, uint64_t nops,
                          int32_t* status) {
    return apply_ops_impl(ctx, b, ops, nops, status, LASPJ_KIND_ORSET, "orset_apply_ops");
}

int laspj_gset_apply_ops(laspj_ctx* ctx, laspj_batch* b, const laspj_op* ops, uint64_t nops,
                         int32_t* status) {
    return apply_ops_impl(ctx, b, ops, nops, status, LASPJ_KIND_GSET, "gset_apply_ops");
}

// ------------------------------------------------------------------------- combinators

int laspj_orset_union(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                      const laspj_batch* r) {
    if (int s = check_pair(ctx, l, r, LASPJ_KIND_ORSET, "orset_union")) return s;
    if (int s = check_pair(ctx, dst, l, LASPJ_KIND_ORSET, "orset_union")) return s;
    Guard g(ctx);
    LJ_HIP(ctx, laspj::launch_orset_union(ctx, dst, l, r));
    return LASPJ_OK;
}

int laspj_orset_filter(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                       const laspj_buf* keep) {
    if (int s = check_pair(ctx, dst, src, LASPJ_KIND_ORSET, "orset_filter")) return s;
    if (int s = check_buf(ctx, keep, (src->elements + 63ull) / 64ull * 8ull, "orset_filter"))
        return s;
    Guard g(ctx);
    LJ_HIP(ctx, laspj::launch_orset_filter(ctx, dst, src, static_cast<const uint64_t*>(keep->dev)));
    return LASPJ_OK;
}

int laspj_orset_concat_batch_create(laspj_ctx* ctx, uint64_t replicas, uint32_t elements,
                                    laspj_batch** out) {
    return batch_create(ctx, LASPJ_KIND_ORSET_CONCAT, replicas, elements, out);
}

int laspj_orset_product_batch_create(laspj_ctx* ctx, uint64_t replicas, uint32_t el,
                                     uint32_t er, laspj_batch** out) {
    return batch_create(ctx, LASPJ_KIND_ORSET_PRODUCT, replicas, el, out, er);
}

int laspj_orset_product_wide_batch_create(laspj_ctx* ctx, uint64_t replicas, uint32_t el,
                                          uint32_t er, laspj_batch** out) {
    return batch_create(ctx, LASPJ_KIND_ORSET_PRODUCT_WIDE, replicas, el, out, er);
}

int laspj_gset_product_batch_create(laspj_ctx* ctx, uint64_t replicas, uint32_t el,
                                    uint32_t er, laspj_batch** out) {
    return batch_create(ctx, LASPJ_KIND_GSET_PRODUCT, replicas, el, out, er);
}

int laspj_orset_intersection(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                             const laspj_batch* r) {
    if (int s = check_pair(ctx, l, r, LASPJ_KIND_ORSET, "orset_intersection")) return s;
    if (!same_ctx(ctx, dst)) return fail(ctx, LASPJ_E_INVAL, "orset_intersection: bad dst");
    if (dst->kind != LASPJ_KIND_ORSET_CONCAT)
        return fail(ctx, LASPJ_E_KIND, "orset_intersection: dst must be a CONCAT batch");
    if (dst->replicas != l->replicas || dst->elements != l->elements)
        return fail(ctx, LASPJ_E_SHAPE, "orset_intersection: dst shape differs");
    Guard g(ctx);
    LJ_HIP(ctx, laspj::launch_orset_intersection(ctx, dst, l, r));
    return LASPJ_OK;
}

static int product_check(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                         const laspj_batch* r, int32_t in_kind, int32_t out_kind,
                         const char* what) {
    if (!same_ctx(ctx, dst) || !same_ctx(ctx, l) || !same_ctx(ctx, r))
        return fail(ctx, LASPJ_E_INVAL, "%s: bad batch", what);
    bool out_ok = dst->kind == out_kind ||
                  (out_kind == LASPJ_KIND_ORSET_PRODUCT && dst->kind == LASPJ_KIND_ORSET_PRODUCT_WIDE);
    if (l->kind != in_kind || r->kind != in_kind || !out_ok)
        return fail(ctx, LASPJ_E_KIND, "%s: wrong batch kinds", what);
    if (l->replicas != r->replicas || dst->replicas != l->replicas ||
        dst->elements != l->elements || dst->elements_r != r->elements)
        return fail(ctx, LASPJ_E_SHAPE, "%s: dst must be replicas x EL x ER of l, r", what);
    return LASPJ_OK;
}

int laspj_orset_product(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                        const laspj_batch* r) {
    if (int s = product_check(ctx, dst, l, r, LASPJ_KIND_ORSET, LASPJ_KIND_ORSET_PRODUCT,
                              "orset_product"))
        return s;
    Guard g(ctx);
    if (dst->kind == LASPJ_KIND_ORSET_PRODUCT_WIDE) {
        LJ_HIP(ctx, laspj::launch_orset_product(ctx, dst, l, r, ctx->flag));
        return LASPJ_OK;
    }
    LJ_HIP(ctx, hipMemsetAsync(ctx->flag, 0, 4, ctx->stream));
    LJ_HIP(ctx, laspj::launch_orset_product(ctx, dst, l, r, ctx->flag));
    uint32_t flag = 0;
    LJ_HIP(ctx, laspj::readback(ctx, &flag, ctx->flag, 4));
    if (flag)
        return fail(ctx, LASPJ_E_RANGE,
                    "orset_product: an input element uses token slot >= 8 (4-byte cells)");
    return LASPJ_OK;
}

int laspj_orset_product_diag(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                             const laspj_batch* r) {
    if (!same_ctx(ctx, dst) || !same_ctx(ctx, l) || !same_ctx(ctx, r))
        return fail(ctx, LASPJ_E_INVAL, "orset_product_diag: bad batch");
    if (l->kind != LASPJ_KIND_ORSET || r->kind != LASPJ_KIND_ORSET ||
        dst->kind != LASPJ_KIND_ORSET_PRODUCT)
        return fail(ctx, LASPJ_E_KIND,
                    "orset_product_diag: OR-Set inputs and a PRODUCT (4-byte cell) output");
    if (l->replicas != r->replicas || l->elements != r->elements ||
        dst->replicas != l->replicas || dst->elements != l->elements || dst->elements_r != 1)
        return fail(ctx, LASPJ_E_SHAPE,
                    "orset_product_diag: inputs of one shape, output EL = E and ER = 1");
    Guard g(ctx);
    LJ_HIP(ctx, hipMemsetAsync(ctx->flag, 0, 4, ctx->stream));
    LJ_HIP(ctx, laspj::launch_orset_product_diag(ctx, dst, l, r, ctx->flag));
    uint32_t flag = 0;
    LJ_HIP(ctx, laspj::readback(ctx, &flag, ctx->flag, 4));
    if (flag)
        return fail(ctx, LASPJ_E_RANGE,
                    "orset_product_diag: an input element uses token slot >= 8 (4-byte cells)");
    return LASPJ_OK;
}

int laspj_orset_gather(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                       const laspj_buf* index) {
    if (!same_ctx(ctx, dst) || !same_ctx(ctx, src))
        return fail(ctx, LASPJ_E_INVAL, "orset_gather: bad batch");
    if (dst->kind != LASPJ_KIND_ORSET || src->kind != LASPJ_KIND_ORSET)
        return fail(ctx, LASPJ_E_KIND, "orset_gather: OR-Set batches expected");
    if (dst->replicas != src->replicas || dst->dev == src->dev)
        return fail(ctx, LASPJ_E_SHAPE, "orset_gather: replicas differ or dst aliases src");
    if (int s = check_buf(ctx, index, 4ull * dst->elements, "orset_gather")) return s;
    Guard g(ctx);
    LJ_HIP(ctx, laspj::launch_orset_gather(ctx, dst, src, static_cast<const uint32_t*>(index->dev)));
    return LASPJ_OK;
}

int laspj_gset_union(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                     const laspj_batch* r) {
    return join_impl(ctx, dst, l, r, LASPJ_KIND_GSET, "gset_union");
}

int laspj_gset_intersection(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                            const laspj_batch* r) {
    if (int s = check_pair(ctx, l, r, LASPJ_KIND_GSET, "gset_intersection")) return s;
    if (int s = check_pair(ctx, dst, l, LASPJ_KIND_GSET, "gset_intersection")) return s;
    Guard g(ctx);
    LJ_HIP(ctx, laspj::launch_and(ctx, dst->dev, l->dev, r->dev, l->replicas * l->words_per_replica));
    return LASPJ_OK;
}

int laspj_gset_filter(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                      const laspj_buf* keep) {
    if (int s = check_pair(ctx, dst, src, LASPJ_KIND_GSET, "gset_filter")) return s;
    if (int s = check_buf(ctx, keep, src->words_per_replica * 8ull, "gset_filter")) return s;
    Guard g(ctx);
    LJ_HIP(ctx, laspj::launch_gset_filter(ctx, dst, src, static_cast<const uint64_t*>(keep->dev)));
    return LASPJ_OK;
}

int laspj_gset_product(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                       const laspj_batch* r) {
    if (int s = product_check(ctx, dst, l, r, LASPJ_KIND_GSET, LASPJ_KIND_GSET_PRODUCT,
                              "gset_product"))
        return s;
    Guard g(ctx);
    LJ_HIP(ctx, laspj::launch_gset_product(ctx, dst, l, r));
    return LASPJ_OK;
}

int laspj_gset_gather(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                      const laspj_buf* index) {
    if (!same_ctx(ctx, dst) || !same_ctx(ctx, src))
        return fail(ctx, LASPJ_E_INVAL, "gset_gather: bad batch");
    if (dst->kind != LASPJ_KIND_GSET || src->kind != LASPJ_KIND_GSET)
        return fail(ctx, LASPJ_E_KIND, "gset_gather: G-Set batches expected");
    if (dst->replicas != src->replicas || dst->dev == src->dev)
        return fail(ctx, LASPJ_E_SHAPE, "gset_gather: replicas differ or dst aliases src");
    if (int s = check_buf(ctx, index, 4ull * dst->elements, "gset_gather")) return s;
    Guard g(ctx);
    LJ_HIP(ctx, laspj::launch_gset_gather(ctx, dst, src, static_cast<const uint32_t*>(index->dev)));
    return LASPJ_OK;
}

// ------------------------------------------------------------------------- riak_dt_gcounter

int laspj_gcounter_batch_create(laspj_ctx* ctx, uint64_t replicas, uint32_t actors,
                                laspj_batch** out) {
    return batch_create(ctx, LASPJ_KIND_GCOUNTER, replicas, actors, out);
}

int laspj_gcounter_join(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* a,
                        const laspj_batch* b) {
    if (int s = check_pair(ctx, a, b, LASPJ_KIND_GCOUNTER, "gcounter_join")) return s;
    if (int s = check_pair(ctx, dst, a, LASPJ_KIND_GCOUNTER, "gcounter_join")) return s;
    Guard g(ctx);
    LJ_HIP(ctx, laspj::launch_max(ctx, dst->dev, a->dev, b->dev, a->replicas * a->words_per_replica));
    return LASPJ_OK;
}

int laspj_gcounter_value(laspj_ctx* ctx, const laspj_batch* b, laspj_buf* out) {
    if (!same_ctx(ctx, b)) return fail(ctx, LASPJ_E_INVAL, "gcounter_value: bad batch");
    if (b->kind != LASPJ_KIND_GCOUNTER) return fail(ctx, LASPJ_E_KIND, "gcounter_value: kind");
    if (int s = check_buf(ctx, out, b->replicas * 8ull, "gcounter_value")) return s;
    Guard g(ctx);
    LJ_HIP(ctx, laspj::launch_gcounter_sums(ctx, b, static_cast<uint64_t*>(out->dev)));
    return LASPJ_OK;
}

int laspj_gcounter_threshold(laspj_ctx* ctx, const laspj_batch* b, uint64_t threshold,
                             int strict, laspj_buf* out) {
    if (!same_ctx(ctx, b)) return fail(ctx, LASPJ_E_INVAL, "gcounter_threshold: bad batch");
    if (b->kind != LASPJ_KIND_GCOUNTER)
        return fail(ctx, LASPJ_E_KIND, "gcounter_threshold: kind");
    if (int s = check_buf(ctx, out, b->replicas, "gcounter_threshold")) return s;
    Guard g(ctx);
    LJ_HIP(ctx, laspj::launch_gcounter_threshold(ctx, b, threshold, strict != 0,
                                                 static_cast<uint8_t*>(out->dev)));
    return LASPJ_OK;
}

int laspj_gcounter_inflation(laspj_ctx* ctx, const laspj_batch* prev, const laspj_batch* cur,
                             int strict, laspj_buf* out) {
    if (!same_ctx(ctx, prev) || !same_ctx(ctx, cur))
        return fail(ctx, LASPJ_E_INVAL, "gcounter_inflation: bad batch");
    if (prev->kind != LASPJ_KIND_GCOUNTER || cur->kind != LASPJ_KIND_GCOUNTER)
        return fail(ctx, LASPJ_E_KIND, "gcounter_inflation: kind");
    if (prev->elements != cur->elements ||
        !(prev->replicas == cur->replicas || prev->replicas == 1))
        return fail(ctx, LASPJ_E_SHAPE, "gcounter_inflation: prev must have cur's replicas or 1");
    if (int s = check_buf(ctx, out, cur->replicas, "gcounter_inflation")) return s;
    Guard g(ctx);
    LJ_HIP(ctx, laspj::launch_gcounter_inflation(ctx, prev, cur, strict != 0,
                                                 static_cast<uint8_t*>(out->dev)));
    return LASPJ_OK;
}

int laspj_gcounter_equal(laspj_ctx* ctx, const laspj_batch* a, const laspj_batch* b,
                         laspj_buf* out) {
    return equal_impl(ctx, a, b, out, LASPJ_KIND_GCOUNTER, "gcounter_equal");
}

int laspj_gcounter_apply_increments(laspj_ctx* ctx, laspj_batch* b, const laspj_incr* incs,
                                    uint64_t n) {
    if (!same_ctx(ctx, b) || (!incs && n))
        return fail(ctx, LASPJ_E_INVAL, "gcounter_apply_increments: bad argument");
    if (b->kind != LASPJ_KIND_GCOUNTER)
        return fail(ctx, LASPJ_E_KIND, "gcounter_apply_increments: kind");
    for (uint64_t i = 0; i < n; ++i) {
        if (incs[i].replica >= b->replicas || incs[i].actor >= b->elements)
            return fail(ctx, LASPJ_E_RANGE, "gcounter_apply_increments: op %llu out of range",
                        (unsigned long long)i);
        // riak_dt_gcounter:update({increment, N}, ...) takes N > 0 only (function_clause)
        if (incs[i].amount == 0)
            return fail(ctx, LASPJ_E_INVAL, "gcounter_apply_increments: op %llu amount 0",
                        (unsigned long long)i);
    }
    if (!n) return LASPJ_OK;
    Guard g(ctx);
    uint64_t need = n * sizeof(laspj_incr);
    if (ctx->scratch_bytes < need) {
        if (ctx->scratch) {
            LJ_HIP(ctx, hipStreamSynchronize(ctx->stream));
            hipFree(ctx->scratch);
            ctx->scratch = nullptr;
            ctx->scratch_bytes = 0;
        }
        if (laspj::dev_malloc(ctx, &ctx->scratch, need) != hipSuccess) {
            hipGetLastError();
            return fail(ctx, LASPJ_E_NOMEM, "gcounter_apply_increments: scratch");
        }
        ctx->scratch_bytes = need;
    }
    LJ_HIP(ctx, hipMemcpyAsync(ctx->scratch, incs, need, hipMemcpyHostToDevice, ctx->stream));
    LJ_HIP(ctx, laspj::launch_gcounter_incr(ctx, b, static_cast<const laspj_incr*>(ctx->scratch), n));
    LJ_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return LASPJ_OK;
}

int laspj_gcounter_reduce(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                          uint32_t group) {
    if (!same_ctx(ctx, dst) || !same_ctx(ctx, src))
        return fail(ctx, LASPJ_E_INVAL, "gcounter_reduce: bad batch");
    if (dst->kind != LASPJ_KIND_GCOUNTER || src->kind != LASPJ_KIND_GCOUNTER)
        return fail(ctx, LASPJ_E_KIND, "gcounter_reduce: kind");
    if (group == 0 || dst->elements != src->elements ||
        dst->replicas * (uint64_t)group != src->replicas)
        return fail(ctx, LASPJ_E_SHAPE, "gcounter_reduce: need src replicas = dst x group");
    if (dst->dev == src->dev) return fail(ctx, LASPJ_E_INVAL, "gcounter_reduce: aliasing");
    Guard g(ctx);
    LJ_HIP(ctx, laspj::launch_reduce_max(ctx, dst->dev, src->dev, dst->replicas, group,
                                         src->words_per_replica));
    return LASPJ_OK;
}

// ------------------------------------------------------------------------- events

int laspj_event_create(laspj_ctx* ctx, laspj_event** out) {
    if (!ctx || !out) return LASPJ_E_INVAL;
    *out = nullptr;
    Guard g(ctx);
    auto* ev = new (std::nothrow) laspj_event;
    if (!ev) return LASPJ_E_NOMEM;
    ev->ctx = ctx;
    if (hipEventCreate(&ev->ev) != hipSuccess) {
        delete ev;
        return fail(ctx, LASPJ_E_DEVICE, "event_create failed");
    }
    *out = ev;
    return LASPJ_OK;
}

int laspj_event_destroy(laspj_event* ev) {
    if (!ev) return LASPJ_E_INVAL;
    {
        Guard g(ev->ctx);
        hipEventDestroy(ev->ev);
    }
    delete ev;
    return LASPJ_OK;
}

int laspj_event_record(laspj_ctx* ctx, laspj_event* ev) {
    if (!ctx || !ev || ev->ctx != ctx) return LASPJ_E_INVAL;
    Guard g(ctx);
    LJ_HIP(ctx, hipEventRecord(ev->ev, ctx->stream));
    return LASPJ_OK;
}

int laspj_event_elapsed_ms(laspj_event* start, laspj_event* stop, float* ms) {
    if (!start || !stop || !ms || start->ctx != stop->ctx) return LASPJ_E_INVAL;
    laspj_ctx* ctx = start->ctx;
    Guard g(ctx);
    LJ_HIP(ctx, hipEventSynchronize(stop->ev));
    LJ_HIP(ctx, hipEventElapsedTime(ms, start->ev, stop->ev));
    return LASPJ_OK;
}

}  // extern "C"
