// Combinator kernels: the bodies lasp_core re-runs on every bind (src/lasp_core.erl:
// 460-712) over device-resident replicas.  All HBM-bound integer work (no MFMA).
//
//   intersection  per-slot select into 32-byte CONCAT cells {pL, rL, pR, rR}: the
//                 reference's token list for a kept element is Cx ++ Cy
//                 (lasp_lattice:orset_causal_union/2), so both halves are kept as is.
//   product       LDS-tiled outer product: a 256-row x 1024-column tile stages the two
//                 input strips once as packed 16-bit {p8, r8} words, then every lane
//                 writes 4 cells (16 B, dwordx4, non-temporal) per row; output is 4 B
//                 per (x, y) cell, i.e. the product is write-bound at |L|*|R|*4 B.
//   gather        map / fold: output slot o copies input slot index[o].
//   G-Set         AND / filter / outer product / bit gather on bitmaps.

#include "laspj_internal.h"

namespace laspj {

typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kB = 256;

__device__ __forceinline__ u64x2 ldnt(const u64x2* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void stnt(u64x2* p, u64x2 v) { __builtin_nontemporal_store(v, p); }

static int grid_for(const laspj_ctx* ctx, uint64_t items, int per_cu = 64) {
    uint64_t g = (items + kB - 1) / kB;
    uint64_t cap = (uint64_t)ctx->cus * per_cu;
    if (g > cap) g = cap;
    return g ? (int)g : 1;
}

// ------------------------------------------------------------------ intersection

// A wave takes 64 consecutive cells: one coalesced 1 KiB load each of L and R, then a
// lane shuffle (ds_bpermute) transposes them so each of the two 1 KiB stores writes
// consecutive 16-byte halves: lanes 2k / 2k+1 store cell k's L / R half.
__global__ __launch_bounds__(kB) void k_orset_intersection(u64x2* out, const u64x2* l,
                                                           const u64x2* r, uint64_t n) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nwaves = (uint64_t)gridDim.x * (kB / 64);
    for (uint64_t base = (((uint64_t)blockIdx.x * kB + threadIdx.x) >> 6) * 64; base < n;
         base += nwaves * 64) {
        uint64_t i = base + lane;
        u64x2 a = {0, 0}, b = {0, 0};
        if (i < n) {
            a = ldnt(l + i);
            b = ldnt(r + i);
        }
        if (!((a.x != 0) & (b.x != 0))) {      // keep X iff in L and keyfind(X, R) found
            a = u64x2{0, 0};
            b = a;
        }
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            int src = half * 32 + (int)(lane >> 1);
            u64 ax = __shfl(a.x, src, 64), ay = __shfl(a.y, src, 64);
            u64 bx = __shfl(b.x, src, 64), by = __shfl(b.y, src, 64);
            u64x2 v;
            v.x = (lane & 1) ? bx : ax;
            v.y = (lane & 1) ? by : ay;
            uint64_t u = 2 * base + half * 64 + lane;
            if (u < 2 * n) stnt(out + u, v);
        }
    }
}

hipError_t launch_orset_intersection(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                                     const laspj_batch* r) {
    uint64_t n = l->replicas * l->elements;
    hipLaunchKernelGGL(k_orset_intersection, dim3(grid_for(ctx, n)), dim3(kB), 0, ctx->stream,
                       reinterpret_cast<u64x2*>(dst->dev), reinterpret_cast<const u64x2*>(l->dev),
                       reinterpret_cast<const u64x2*>(r->dev), n);
    return hipGetLastError();
}

// ------------------------------------------------------------------ product (OR-Set)

constexpr int kPX = 256;    // rows per tile (profiles/r01_suite_product_rows.log: 256 > 128 > 64)
constexpr int kPG = 1;      // 1024-column groups per tile (default)
constexpr int kPY = 1024;   // columns per tile = 4 per lane

__device__ __forceinline__ uint32_t pack8(u64x2 c, uint32_t* flag) {
    if (c.x >> 8) atomicOr(flag, 1u);          // token slot >= 8: not expressible in 4 B
    return c.x ? (uint32_t)((c.x & 0xFFull) | ((c.y & 0xFFull) << 8)) : 0u;
}

// G column groups of 1024 per tile: a lane keeps G x 4 packed column cells in registers
// and every row is G 16-byte stores per lane (G x 4 KiB contiguous per row and block)
template <bool ALIGNED, int PX, int G>
__global__ __launch_bounds__(kB) void k_orset_product(uint32_t* out, const u64x2* L,
                                                      const u64x2* R, uint64_t reps,
                                                      uint32_t EL, uint32_t ER,
                                                      uint64_t cstride, uint32_t* flag) {
    constexpr uint32_t PY = G * kPY;
    __shared__ __attribute__((aligned(16))) uint32_t ry[PY];
    __shared__ uint32_t lx[PX];
    const uint64_t tx_n = (EL + PX - 1) / PX, ty_n = (ER + PY - 1) / PY;
    const uint64_t tiles = reps * tx_n * ty_n;
    for (uint64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
        uint64_t rep = t / (tx_n * ty_n);
        uint64_t rem = t - rep * tx_n * ty_n;
        uint32_t tx = (uint32_t)(rem / ty_n), ty = (uint32_t)(rem - (uint64_t)tx * ty_n);
        uint32_t x0 = tx * PX, y0 = ty * PY;
        for (int i = threadIdx.x; i < (int)PY; i += kB) {
            uint32_t y = y0 + i;
            ry[i] = y < ER ? pack8(ldnt(R + rep * ER + y), flag) << 16 : 0u;
        }
        for (int i = threadIdx.x; i < PX; i += kB) {
            uint32_t x = x0 + i;
            lx[i] = x < EL ? pack8(ldnt(L + rep * EL + x), flag) : 0u;
        }
        __syncthreads();
        u32x4 ryv[G];
#pragma unroll
        for (int g = 0; g < G; ++g)
            ryv[g] = *reinterpret_cast<const u32x4*>(&ry[g * kPY + threadIdx.x * 4]);
        const uint32_t rows = min((uint32_t)PX, EL - x0);
        for (uint32_t rr = 0; rr < rows; ++rr) {
            const uint32_t lv = lx[rr];
            const uint64_t rowb = rep * cstride + (uint64_t)(x0 + rr) * ER + y0;
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const u32x4 c = ryv[g];
                u32x4 v;
                v.x = (lv && c.x) ? lv | c.x : 0u;
                v.y = (lv && c.y) ? lv | c.y : 0u;
                v.z = (lv && c.z) ? lv | c.z : 0u;
                v.w = (lv && c.w) ? lv | c.w : 0u;
                const uint32_t yl = g * kPY + threadIdx.x * 4;
                const uint64_t base = rowb + yl;
                if (ALIGNED && y0 + yl + 3 < ER) {
                    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(out + base));
                } else {
                    uint32_t y = y0 + yl;
                    if (y < ER) out[base] = v.x;
                    if (y + 1 < ER) out[base + 1] = v.y;
                    if (y + 2 < ER) out[base + 2] = v.z;
                    if (y + 3 < ER) out[base + 3] = v.w;
                }
            }
        }
        __syncthreads();
    }
}

// wide form: cell (x, y) = {pX, rX, pY, rY} (32 B) for any token slots.  A block takes a
// (replica, row x, 1024-column tile): row x's cell is one broadcast load, lanes 2k /
// 2k+1 write cell k's X / Y half, so each wave store covers 1 KiB contiguously; the
// only divisions are per tile.
constexpr uint32_t kWTile = 1024;

__global__ __launch_bounds__(kB) void k_orset_product_wide(u64x2* out, const u64x2* L,
                                                           const u64x2* R, uint64_t reps,
                                                           uint32_t EL, uint32_t ER) {
    const uint64_t ty_n = (ER + kWTile - 1) / kWTile;
    const uint64_t tiles = reps * EL * ty_n;
    for (uint64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
        const uint64_t row = t / ty_n;                  // rep * EL + x
        const uint32_t y0 = (uint32_t)(t - row * ty_n) * kWTile;
        const uint64_t rep = row / EL;
        const u64x2 a = L[row];
        const u64x2* Rr = R + rep * ER;
        u64x2* o = out + (row * ER + y0) * 2;
        const uint32_t units = 2u * min(kWTile, ER - y0);
#pragma unroll 4
        for (uint32_t u = threadIdx.x; u < units; u += kB) {
            const u64x2 b = Rr[y0 + (u >> 1)];
            const bool keep = (a.x != 0) & (b.x != 0);
            stnt(o + u, keep ? ((u & 1) ? b : a) : u64x2{0, 0});
        }
    }
}

// product followed by filter(fun({X, Y}) -> X =:= Y), fused (BASELINE config 5's
// variant): over one element dictionary the pairs that pass are the slots present on
// both sides, so cell e of the output (an EL = E, ER = 1 PRODUCT batch) is the product
// cell of l[e] and r[e] — 32 B read and 4 B written per slot instead of EL x ER cells.
// Grid-stride with 4 slots per lane a stride apart (each load instruction is 1 KiB of
// consecutive cells, each store 256 B).
__global__ __launch_bounds__(kB) void k_orset_product_diag(uint32_t* out, const u64x2* L,
                                                           const u64x2* R, uint64_t n,
                                                           uint32_t* flag) {
    const uint64_t stride = (uint64_t)gridDim.x * kB;
    uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        u64x2 a[4], b[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) a[k] = ldnt(L + i + k * stride);
#pragma unroll
        for (int k = 0; k < 4; ++k) b[k] = ldnt(R + i + k * stride);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t x = pack8(a[k], flag), y = pack8(b[k], flag) << 16;
            __builtin_nontemporal_store((x && y) ? x | y : 0u, out + i + k * stride);
        }
    }
    for (; i < n; i += stride) {
        const uint32_t x = pack8(ldnt(L + i), flag), y = pack8(ldnt(R + i), flag) << 16;
        out[i] = (x && y) ? x | y : 0u;
    }
}

hipError_t launch_orset_product_diag(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                                     const laspj_batch* r, uint32_t* flag) {
    const uint64_t n = l->replicas * l->elements;
    hipLaunchKernelGGL(k_orset_product_diag, dim3(grid_for(ctx, n)), dim3(kB), 0,
                       ctx->stream, reinterpret_cast<uint32_t*>(dst->dev),
                       reinterpret_cast<const u64x2*>(l->dev),
                       reinterpret_cast<const u64x2*>(r->dev), n, flag);
    return hipGetLastError();
}

hipError_t launch_orset_product(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                                const laspj_batch* r, uint32_t* flag) {
    if (dst->kind == LASPJ_KIND_ORSET_PRODUCT_WIDE) {
        uint64_t tiles = l->replicas * (uint64_t)l->elements *
                         ((r->elements + kWTile - 1) / kWTile);
        uint64_t g = tiles < (uint64_t)ctx->cus * 32 ? tiles : (uint64_t)ctx->cus * 32;
        hipLaunchKernelGGL(k_orset_product_wide, dim3((unsigned)(g ? g : 1)), dim3(kB), 0, ctx->stream,
                           reinterpret_cast<u64x2*>(dst->dev), reinterpret_cast<const u64x2*>(l->dev),
                           reinterpret_cast<const u64x2*>(r->dev), l->replicas, l->elements,
                           r->elements);
        return hipGetLastError();
    }
    const int px = ctx->tune_product_rows > 0 ? (int)ctx->tune_product_rows : kPX;
    const int gy = ctx->tune_product_cols > 0 ? (int)(ctx->tune_product_cols / kPY) : kPG;
    uint64_t tiles = l->replicas * ((l->elements + px - 1) / px) *
                     ((r->elements + (uint64_t)gy * kPY - 1) / ((uint64_t)gy * kPY));
    uint64_t g = tiles < (uint64_t)ctx->cus * 32 ? tiles : (uint64_t)ctx->cus * 32;
    auto* o = reinterpret_cast<uint32_t*>(dst->dev);
    auto* L = reinterpret_cast<const u64x2*>(l->dev);
    auto* R = reinterpret_cast<const u64x2*>(r->dev);
    const bool al = r->elements % 4 == 0;
#define LJ_PK(PXV, GV) (al ? k_orset_product<true, PXV, GV> : k_orset_product<false, PXV, GV>)
    auto k = LJ_PK(kPX, kPG);
    if (gy == 1) {
        if (px == 256) k = LJ_PK(256, 1);
        if (px == 128) k = LJ_PK(128, 1);
        if (px == 64) k = LJ_PK(64, 1);
        if (px == 32) k = LJ_PK(32, 1);
    } else if (gy == 2) {
        if (px == 256) k = LJ_PK(256, 2);
        if (px == 128) k = LJ_PK(128, 2);
        if (px == 64) k = LJ_PK(64, 2);
        if (px == 32) k = LJ_PK(32, 2);
    } else {
        if (px == 256) k = LJ_PK(256, 4);
        if (px == 128) k = LJ_PK(128, 4);
        if (px == 64) k = LJ_PK(64, 4);
        if (px == 32) k = LJ_PK(32, 4);
    }
#undef LJ_PK
    hipLaunchKernelGGL(k, dim3((unsigned)g), dim3(kB), 0, ctx->stream, o, L, R, l->replicas,
                       l->elements, r->elements, 2 * dst->words_per_replica, flag);
    return hipGetLastError();
}

// ------------------------------------------------------------------ gather (map / fold)

// A block owns one 4096-slot segment of the output and a run of replicas: its 16
// index entries per lane are loaded once into registers, then every replica of the
// run is 16 independent gathers + 16 coalesced 16-byte stores per lane.
constexpr uint32_t kGSeg = 4096, kGPer = kGSeg / kB, kGRun = 8;

__global__ __launch_bounds__(kB) void k_orset_gather(u64x2* out, const u64x2* src,
                                                     const uint32_t* index, uint64_t reps,
                                                     uint32_t E_out, uint32_t E_in,
                                                     uint32_t nseg) {
    const uint64_t runs = (reps + kGRun - 1) / kGRun;
    for (uint64_t it = blockIdx.x; it < runs * nseg; it += gridDim.x) {
        const uint64_t run = it / nseg;
        const uint32_t o0 = (uint32_t)(it - run * nseg) * kGSeg;
        uint32_t si[kGPer];
#pragma unroll
        for (uint32_t k = 0; k < kGPer; ++k) {
            const uint32_t o = o0 + k * kB + threadIdx.x;
            si[k] = o < E_out ? index[o] : 0xFFFFFFFFu;
        }
        const uint64_t r1 = min(reps, (run + 1) * kGRun);
        for (uint64_t rep = run * kGRun; rep < r1; ++rep) {
            const u64x2* s = src + rep * E_in;
            u64x2* d = out + rep * E_out;
            u64x2 v[kGPer];
#pragma unroll
            for (uint32_t k = 0; k < kGPer; ++k)
                v[k] = si[k] < E_in ? s[si[k]] : u64x2{0, 0};
#pragma unroll
            for (uint32_t k = 0; k < kGPer; ++k) {
                const uint32_t o = o0 + k * kB + threadIdx.x;
                if (o < E_out) stnt(d + o, v[k]);
            }
        }
    }
}

hipError_t launch_orset_gather(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                               const uint32_t* index) {
    uint32_t ns = (dst->elements + kGSeg - 1) / kGSeg;
    uint64_t items = (dst->replicas + kGRun - 1) / kGRun * ns;
    uint64_t cap = (uint64_t)ctx->cus * 32;
    uint64_t g = items < cap ? items : cap;
    hipLaunchKernelGGL(k_orset_gather, dim3((unsigned)(g ? g : 1)), dim3(kB), 0, ctx->stream,
                       reinterpret_cast<u64x2*>(dst->dev), reinterpret_cast<const u64x2*>(src->dev),
                       index, dst->replicas, dst->elements, src->elements, ns);
    return hipGetLastError();
}

// ------------------------------------------------------------------ G-Set

__global__ __launch_bounds__(kB) void k_and16(u64x2* d, const u64x2* a, const u64x2* b,
                                              uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * kB;
    for (uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x; i < n; i += stride)
        stnt(d + i, ldnt(a + i) & ldnt(b + i));
}

__global__ void k_and_tail(u64* d, const u64* a, const u64* b, uint64_t idx) {
    if (threadIdx.x == 0 && blockIdx.x == 0) d[idx] = a[idx] & b[idx];
}

hipError_t launch_and(laspj_ctx* ctx, uint64_t* dst, const uint64_t* a, const uint64_t* b,
                      uint64_t words) {
    uint64_t n = words / 2;
    if (n)
        hipLaunchKernelGGL(k_and16, dim3(grid_for(ctx, n)), dim3(kB), 0, ctx->stream,
                           reinterpret_cast<u64x2*>(dst), reinterpret_cast<const u64x2*>(a),
                           reinterpret_cast<const u64x2*>(b), n);
    if (words & 1)
        hipLaunchKernelGGL(k_and_tail, dim3(1), dim3(64), 0, ctx->stream, (u64*)dst,
                           (const u64*)a, (const u64*)b, words - 1);
    return hipGetLastError();
}

__global__ __launch_bounds__(kB) void k_gset_filter(u64* d, const u64* s, const u64* keep,
                                                    uint64_t reps, uint64_t W) {
    const uint64_t n = reps * W;
    const uint64_t stride = (uint64_t)gridDim.x * kB;
    for (uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x; i < n; i += stride)
        d[i] = s[i] & keep[i % W];
}

hipError_t launch_gset_filter(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                              const uint64_t* keep) {
    uint64_t n = src->replicas * src->words_per_replica;
    hipLaunchKernelGGL(k_gset_filter, dim3(grid_for(ctx, n)), dim3(kB), 0, ctx->stream,
                       (u64*)dst->dev, (const u64*)src->dev, (const u64*)keep, src->replicas,
                       src->words_per_replica);
    return hipGetLastError();
}

// dst replica i: EL rows of WR words; row x = R's bitmap if x in L, else 0
__global__ __launch_bounds__(kB) void k_gset_product(u64* d, const u64* L, const u64* R,
                                                     uint64_t reps, uint32_t EL, uint64_t WL,
                                                     uint64_t WR) {
    const uint64_t n = reps * EL * WR;
    const uint64_t stride = (uint64_t)gridDim.x * kB;
    for (uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x; i < n; i += stride) {
        uint64_t row = i / WR, w = i - row * WR;
        uint64_t rep = row / EL;
        uint32_t x = (uint32_t)(row - rep * EL);
        bool in_l = (L[rep * WL + (x >> 6)] >> (x & 63u)) & 1ull;
        d[i] = in_l ? R[rep * WR + w] : 0ull;
    }
}

hipError_t launch_gset_product(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                               const laspj_batch* r) {
    uint64_t WR = r->words_per_replica;
    uint64_t n = l->replicas * (uint64_t)l->elements * WR;
    hipLaunchKernelGGL(k_gset_product, dim3(grid_for(ctx, n)), dim3(kB), 0, ctx->stream,
                       (u64*)dst->dev, (const u64*)l->dev, (const u64*)r->dev, l->replicas,
                       l->elements, l->words_per_replica, WR);
    return hipGetLastError();
}

// wave per destination word: lane = bit, __ballot packs
__global__ __launch_bounds__(kB) void k_gset_gather(u64* d, const u64* s, const uint32_t* index,
                                                    uint64_t reps, uint32_t E_out,
                                                    uint32_t E_in) {
    const uint64_t Wo = (E_out + 63u) / 64u, Wi = (E_in + 63u) / 64u;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nwaves = (uint64_t)gridDim.x * (kB / 64);
    for (uint64_t w = ((uint64_t)blockIdx.x * kB + threadIdx.x) >> 6; w < reps * Wo;
         w += nwaves) {
        uint64_t rep = w / Wo;
        uint32_t o = (uint32_t)(w - rep * Wo) * 64u + lane;
        bool bit = false;
        if (o < E_out) {
            uint32_t src = index[o];
            if (src < E_in) bit = (s[rep * Wi + (src >> 6)] >> (src & 63u)) & 1ull;
        }
        u64 m = __ballot(bit);
        if (lane == 0) d[w] = m;
    }
}

hipError_t launch_gset_gather(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                              const uint32_t* index) {
    uint64_t words = dst->replicas * dst->words_per_replica;
    hipLaunchKernelGGL(k_gset_gather, dim3(grid_for(ctx, words * 64)), dim3(kB), 0, ctx->stream,
                       (u64*)dst->dev, (const u64*)src->dev, index, dst->replicas, dst->elements,
                       src->elements);
    return hipGetLastError();
}

// ------------------------------------------------------------------ value of outputs

// CONCAT: visible iff the element is present and Cx ++ Cy holds a {Token, false}
__global__ __launch_bounds__(kB) void k_concat_value(const u64x2* cells, u64* out, uint64_t reps,
                                                     uint32_t E) {
    const uint32_t W = (E + 63u) / 64u;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nwaves = (uint64_t)gridDim.x * (kB / 64);
    for (uint64_t w = ((uint64_t)blockIdx.x * kB + threadIdx.x) >> 6; w < reps * W;
         w += nwaves) {
        uint64_t rep = w / W;
        uint32_t e = (uint32_t)(w - rep * W) * 64u + lane;
        bool vis = false;
        if (e < E) {
            u64x2 a = ldnt(cells + 2 * (rep * E + e)), b = ldnt(cells + 2 * (rep * E + e) + 1);
            vis = (a.x != 0) && (((a.x & ~a.y) | (b.x & ~b.y)) != 0);
        }
        u64 m = __ballot(vis);
        if (lane == 0) out[w] = m;
    }
}

// PRODUCT: visible iff x and y both hold a live token (the pair flag is Dx orelse Dy)
__global__ __launch_bounds__(kB) void k_product_value(const uint32_t* cells, u64* out,
                                                      uint64_t reps, uint64_t C,
                                                      uint64_t cstride) {
    const uint64_t W = (C + 63u) / 64u;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nwaves = (uint64_t)gridDim.x * (kB / 64);
    for (uint64_t w = ((uint64_t)blockIdx.x * kB + threadIdx.x) >> 6; w < reps * W;
         w += nwaves) {
        uint64_t rep = w / W;
        uint64_t c = (w - rep * W) * 64u + lane;
        bool vis = false;
        if (c < C) {
            uint32_t v = cells[rep * cstride + c];
            vis = ((v & ~(v >> 8)) & 0xFFu) && (((v >> 16) & ~(v >> 24)) & 0xFFu);
        }
        u64 m = __ballot(vis);
        if (lane == 0) out[w] = m;
    }
}

// PRODUCT_WIDE: visible iff x and y both hold a live token
__global__ __launch_bounds__(kB) void k_product_wide_value(const u64x2* cells, u64* out,
                                                           uint64_t reps, uint64_t C) {
    const uint64_t W = (C + 63u) / 64u;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nwaves = (uint64_t)gridDim.x * (kB / 64);
    for (uint64_t w = ((uint64_t)blockIdx.x * kB + threadIdx.x) >> 6; w < reps * W;
         w += nwaves) {
        uint64_t rep = w / W;
        uint64_t c = (w - rep * W) * 64u + lane;
        bool vis = false;
        if (c < C) {
            u64x2 a = ldnt(cells + 2 * (rep * C + c)), b = ldnt(cells + 2 * (rep * C + c) + 1);
            vis = ((a.x & ~a.y) != 0) && ((b.x & ~b.y) != 0);
        }
        u64 m = __ballot(vis);
        if (lane == 0) out[w] = m;
    }
}

hipError_t launch_combinator_value(laspj_ctx* ctx, const laspj_batch* b, uint64_t* out) {
    if (b->kind == LASPJ_KIND_ORSET_PRODUCT_WIDE) {
        uint64_t words = b->replicas * ((b->cells + 63ull) / 64ull);
        hipLaunchKernelGGL(k_product_wide_value, dim3(grid_for(ctx, words * 64, 8)), dim3(kB), 0,
                           ctx->stream, reinterpret_cast<const u64x2*>(b->dev), (u64*)out,
                           b->replicas, b->cells);
        return hipGetLastError();
    }
    uint64_t words = b->replicas * ((b->cells + 63ull) / 64ull);
    int grid = grid_for(ctx, words * 64, 8);
    if (b->kind == LASPJ_KIND_ORSET_CONCAT)
        hipLaunchKernelGGL(k_concat_value, dim3(grid), dim3(kB), 0, ctx->stream,
                           reinterpret_cast<const u64x2*>(b->dev), (u64*)out, b->replicas,
                           b->elements);
    else
        hipLaunchKernelGGL(k_product_value, dim3(grid), dim3(kB), 0, ctx->stream,
                           reinterpret_cast<const uint32_t*>(b->dev), (u64*)out, b->replicas,
                           b->cells, 2 * b->words_per_replica);
    return hipGetLastError();
}

}  // namespace laspj
