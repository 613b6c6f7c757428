// CDNA4 (gfx950) kernels of the lattice-join engine.
//
// Everything on this path is integer/boolean and HBM-bound: no MFMA.
// Design rules applied (cdna_hip_programming.md §6, MI355X_MICROARCH.md §HBM):
//   * 16 B per lane per access (global_load/store_dwordx4): one wave-instruction moves
//     1 KiB of consecutive bytes; cells are {p, r} u64 pairs so one load = one cell.
//   * grid-stride loops over 64 workgroups per CU with U cells in flight per lane,
//     non-temporal loads/stores for once-touched streams (206 GB per join batch never
//     fits the 256 MiB Infinity Cache).
//   * per-replica predicates use one wave64 per replica: lanes walk the replica's
//     cells with a 64-cell stride (coalesced), and the reduction is a __ballot or a
//     __shfl_xor tree — no LDS, no __syncthreads.
//
// Layout (include/laspj.h): OR-Set cell (i, e) = words [2(iE+e), 2(iE+e)+1] = {p, r};
// G-Set replica i = words [iW, (i+1)W), W = ceil(E/64).

#include <algorithm>

#include "laspj_internal.h"

namespace laspj {

typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

constexpr int kBlock = 256;

template <bool NT>
__device__ __forceinline__ u64x2 ld2(const u64x2* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st2(u64x2* p, u64x2 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

__device__ __forceinline__ u64 wave_sum(u64 v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// ------------------------------------------------------------------ tuning

StreamTune stream_tune(const laspj_ctx* ctx, uint64_t n16) {
    StreamTune t;
    // defaults from the bench-size sweep (profiles/r01_sweep_join.log): 64 workgroups
    // per CU x 2 cells in flight per lane reached 6.1 TB/s; 8/CU (persistent-style)
    // stayed at 5.6-5.8 TB/s.
    t.grid = ctx->tune_grid > 0 ? (int)ctx->tune_grid : ctx->cus * 64;
    t.unroll = ctx->tune_unroll > 0 ? (int)ctx->tune_unroll : 2;
    // a launch smaller than 8 cells per lane of one full wave of blocks has nothing to
    // unroll over (the bind path's single replica); it also keeps those launches apart
    // from the batched ones in kernel-trace statistics (k_or16<1, ...>)
    if (ctx->tune_unroll <= 0 && n16 < (uint64_t)ctx->cus * kBlock * 8) t.unroll = 1;
    t.nt = ctx->tune_nt < 0 ? true : ctx->tune_nt != 0;
    uint64_t need = (n16 + kBlock - 1) / kBlock;
    if (need < (uint64_t)t.grid) t.grid = need > 0 ? (int)need : 1;
    return t;
}

// ------------------------------------------------------------------ join: d = a | b

template <int U, bool NT>
__global__ __launch_bounds__(kBlock) void k_or16(u64x2* d, const u64x2* a, const u64x2* b,
                                                 uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        u64x2 x[U], y[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = ld2<NT>(a + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) y[u] = ld2<NT>(b + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) st2<NT>(d + i + u * stride, x[u] | y[u]);
    }
    for (; i < n; i += stride) st2<NT>(d + i, ld2<NT>(a + i) | ld2<NT>(b + i));
}

__global__ void k_or_tail(u64* d, const u64* a, const u64* b, uint64_t idx) {
    if (threadIdx.x == 0 && blockIdx.x == 0) d[idx] = a[idx] | b[idx];
}

template <int U, bool NT>
static void launch_or16_t(laspj_ctx* ctx, int grid, u64x2* d, const u64x2* a, const u64x2* b,
                          uint64_t n) {
    hipLaunchKernelGGL((k_or16<U, NT>), dim3(grid), dim3(kBlock), 0, ctx->stream, d, a, b, n);
}

template <bool NT>
static void launch_or16_u(laspj_ctx* ctx, const StreamTune& t, u64x2* d, const u64x2* a,
                          const u64x2* b, uint64_t n) {
    switch (t.unroll) {
        case 1: launch_or16_t<1, NT>(ctx, t.grid, d, a, b, n); break;
        case 2: launch_or16_t<2, NT>(ctx, t.grid, d, a, b, n); break;
        case 8: launch_or16_t<8, NT>(ctx, t.grid, d, a, b, n); break;
        default: launch_or16_t<4, NT>(ctx, t.grid, d, a, b, n); break;
    }
}

hipError_t launch_or(laspj_ctx* ctx, uint64_t* dst, const uint64_t* a, const uint64_t* b,
                     uint64_t words) {
    uint64_t n16 = words / 2;
    if (n16) {
        StreamTune t = stream_tune(ctx, n16);
        auto* d2 = reinterpret_cast<u64x2*>(dst);
        auto* a2 = reinterpret_cast<const u64x2*>(a);
        auto* b2 = reinterpret_cast<const u64x2*>(b);
        if (t.nt) launch_or16_u<true>(ctx, t, d2, a2, b2, n16);
        else launch_or16_u<false>(ctx, t, d2, a2, b2, n16);
    }
    if (words & 1)
        hipLaunchKernelGGL(k_or_tail, dim3(1), dim3(64), 0, ctx->stream, (u64*)dst,
                           (const u64*)a, (const u64*)b, words - 1);
    return hipGetLastError();
}

// ------------------------------------------------------------------ reduce over groups

// dst replica g = OR_{j<group} src replica (g*group + j): one block per (dst replica,
// 8192-word segment); lanes stride the segment, `group` independent loads per step.
constexpr uint64_t kRSeg = 8192;

template <bool VEC2>
__global__ __launch_bounds__(kBlock) void k_reduce_or(u64* dst, const u64* src, uint64_t groups,
                                                      uint32_t group, uint64_t wr,
                                                      uint32_t nseg) {
    const uint64_t per = VEC2 ? wr / 2 : wr;          // items per replica
    for (uint64_t it = blockIdx.x; it < groups * nseg; it += gridDim.x) {
        uint64_t g = it / nseg;
        uint64_t lo = (it - g * nseg) * kRSeg, hi = min(per, lo + kRSeg);
        if constexpr (VEC2) {
            const u64x2* s = reinterpret_cast<const u64x2*>(src) + g * group * per;
            u64x2* d = reinterpret_cast<u64x2*>(dst) + g * per;
#pragma unroll 2
            for (uint64_t i = lo + threadIdx.x; i < hi; i += kBlock) {
                u64x2 acc = ld2<true>(s + i);
                for (uint32_t j = 1; j < group; ++j) acc |= ld2<true>(s + j * per + i);
                st2<true>(d + i, acc);
            }
        } else {
            const u64* s = src + g * group * per;
            u64* d = dst + g * per;
            for (uint64_t i = lo + threadIdx.x; i < hi; i += kBlock) {
                u64 acc = s[i];
                for (uint32_t j = 1; j < group; ++j) acc |= s[j * per + i];
                d[i] = acc;
            }
        }
    }
}

// group known at compile time (the FSMs' N = 2..4): all G loads of a step are issued
// before the first OR, two steps per lane in flight
template <int G>
__global__ __launch_bounds__(kBlock) void k_reduce_or_g(u64x2* dst, const u64x2* src,
                                                        uint64_t groups, uint64_t per,
                                                        uint32_t nseg) {
    for (uint64_t it = blockIdx.x; it < groups * nseg; it += gridDim.x) {
        const uint64_t g = it / nseg;
        const uint64_t lo = (it - g * nseg) * kRSeg, hi = min(per, lo + kRSeg);
        const u64x2* s = src + g * G * per;
        u64x2* d = dst + g * per;
        uint64_t i = lo + threadIdx.x;
        for (; i + kBlock < hi; i += 2 * kBlock) {
            u64x2 x[G], y[G];
#pragma unroll
            for (int j = 0; j < G; ++j) x[j] = ld2<true>(s + j * per + i);
#pragma unroll
            for (int j = 0; j < G; ++j) y[j] = ld2<true>(s + j * per + i + kBlock);
#pragma unroll
            for (int j = 1; j < G; ++j) {
                x[0] |= x[j];
                y[0] |= y[j];
            }
            st2<true>(d + i, x[0]);
            st2<true>(d + i + kBlock, y[0]);
        }
        if (i < hi) {
            u64x2 x[G];
#pragma unroll
            for (int j = 0; j < G; ++j) x[j] = ld2<true>(s + j * per + i);
#pragma unroll
            for (int j = 1; j < G; ++j) x[0] |= x[j];
            st2<true>(d + i, x[0]);
        }
    }
}

// the join of one 64-bit word: OR for set bitmaps, unsigned max for G-Counter counts
// (riak_dt_gcounter merge)
template <bool MAX>
__device__ __forceinline__ u64 join_word(u64 x, u64 y) {
    if constexpr (MAX) return x > y ? x : y;
    else return x | y;
}

// power-of-two replica length: one flat grid-stride sweep over the destination (all
// blocks move through HBM together, as the join does), 2 cells x G loads per lane (knob
// 4; the default is k_reduce_or_tile below);
// MAX: the same sweep for the G-Counter reduce (per-actor max)
template <int G, bool MAX = false>
__global__ __launch_bounds__(kBlock) void k_reduce_or_flat(u64x2* dst, const u64x2* src,
                                                           uint64_t n, uint32_t lg) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock, mask = (1ull << lg) - 1ull;
    uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    for (; i + stride < n; i += 2 * stride) {
        const uint64_t i2 = i + stride;
        const u64x2* s = src + (((i >> lg) * G) << lg) + (i & mask);
        const u64x2* t = src + (((i2 >> lg) * G) << lg) + (i2 & mask);
        u64x2 x[G], y[G];
#pragma unroll
        for (int j = 0; j < G; ++j) x[j] = ld2<true>(s + ((uint64_t)j << lg));
#pragma unroll
        for (int j = 0; j < G; ++j) y[j] = ld2<true>(t + ((uint64_t)j << lg));
#pragma unroll
        for (int j = 1; j < G; ++j) {
            x[0].x = join_word<MAX>(x[0].x, x[j].x);
            x[0].y = join_word<MAX>(x[0].y, x[j].y);
            y[0].x = join_word<MAX>(y[0].x, y[j].x);
            y[0].y = join_word<MAX>(y[0].y, y[j].y);
        }
        st2<true>(dst + i, x[0]);
        st2<true>(dst + i2, y[0]);
    }
    if (i < n) {
        const u64x2* s = src + (((i >> lg) * G) << lg) + (i & mask);
        u64x2 x[G];
#pragma unroll
        for (int j = 0; j < G; ++j) x[j] = ld2<true>(s + ((uint64_t)j << lg));
#pragma unroll
        for (int j = 1; j < G; ++j) {
            x[0].x = join_word<MAX>(x[0].x, x[j].x);
            x[0].y = join_word<MAX>(x[0].y, x[j].y);
        }
        st2<true>(dst + i, x[0]);
    }
}

// the same reduce as tiles of T x 256 destination cells, one per block, sources read
// one at a time (as k_reduce_chunks_tile)
template <int G, bool MAX, int T>
__global__ __launch_bounds__(kBlock) void k_reduce_or_tile(u64x2* dst, const u64x2* src,
                                                           uint64_t n, uint32_t lg) {
    const uint64_t mask = (1ull << lg) - 1ull;
    const uint64_t tile = (uint64_t)T * kBlock;
    const uint64_t tiles = n / tile;
    for (uint64_t b = blockIdx.x; b < tiles; b += gridDim.x) {
        const uint64_t i0 = b * tile + threadIdx.x;
        const u64x2* sp[T];
#pragma unroll
        for (int u = 0; u < T; ++u) {
            const uint64_t i = i0 + u * kBlock;
            sp[u] = src + (((i >> lg) * G) << lg) + (i & mask);
        }
        u64x2 acc[T];
#pragma unroll
        for (int u = 0; u < T; ++u) acc[u] = ld2<true>(sp[u]);
#pragma unroll
        for (int j = 1; j < G; ++j) {
            u64x2 v[T];
#pragma unroll
            for (int u = 0; u < T; ++u) v[u] = ld2<true>(sp[u] + ((uint64_t)j << lg));
#pragma unroll
            for (int u = 0; u < T; ++u) {
                acc[u].x = join_word<MAX>(acc[u].x, v[u].x);
                acc[u].y = join_word<MAX>(acc[u].y, v[u].y);
            }
        }
#pragma unroll
        for (int u = 0; u < T; ++u) st2<true>(dst + i0 + u * kBlock, acc[u]);
    }
    for (uint64_t i = tiles * tile + (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * kBlock) {
        const u64x2* s = src + (((i >> lg) * G) << lg) + (i & mask);
        u64x2 a = ld2<true>(s);
#pragma unroll
        for (int j = 1; j < G; ++j) {
            const u64x2 v = ld2<true>(s + ((uint64_t)j << lg));
            a.x = join_word<MAX>(a.x, v.x);
            a.y = join_word<MAX>(a.y, v.y);
        }
        st2<true>(dst + i, a);
    }
}

template <int G, bool MAX = false>
static void launch_reduce_flat(laspj_ctx* ctx, u64x2* d, const u64x2* s, uint64_t n,
                               uint32_t lg) {
    // tiles by default (N = 3 OR-Set 12.6 -> 11.6 ms, N = 4 G-Counter 2.20 -> 1.81 ms,
    // profiles/r02_sweep_reduce_groups.log); knob 4: the grid-stride sweep
    if (ctx->tune_reduce != 4) {
        const uint64_t tiles = n / (4ull * kBlock);
        const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(tiles, 1u << 30));
        hipLaunchKernelGGL((k_reduce_or_tile<G, MAX, 4>), dim3(grid), dim3(kBlock), 0,
                           ctx->stream, d, s, n, lg);
        return;
    }
    StreamTune t = stream_tune(ctx, n);
    hipLaunchKernelGGL((k_reduce_or_flat<G, MAX>), dim3(t.grid), dim3(kBlock), 0, ctx->stream,
                       d, s, n, lg);
}

hipError_t launch_reduce_or(laspj_ctx* ctx, uint64_t* dst, const uint64_t* src,
                            uint64_t groups, uint32_t group, uint64_t wr) {
    if ((wr % 2) == 0 && (ctx->tune_reduce == 0 || ctx->tune_reduce == 4)) {
        const uint64_t per = wr / 2;
        if ((per & (per - 1)) == 0 && group >= 2 && group <= 4) {
            const uint32_t lg = (uint32_t)__builtin_ctzll(per);
            auto* d2 = reinterpret_cast<u64x2*>(dst);
            auto* s2 = reinterpret_cast<const u64x2*>(src);
            if (group == 2) launch_reduce_flat<2>(ctx, d2, s2, groups * per, lg);
            else if (group == 3) launch_reduce_flat<3>(ctx, d2, s2, groups * per, lg);
            else launch_reduce_flat<4>(ctx, d2, s2, groups * per, lg);
            return hipGetLastError();
        }
    }
    bool vec2 = (wr % 2) == 0;
    uint64_t per = vec2 ? wr / 2 : wr;
    uint32_t ns = (uint32_t)((per + kRSeg - 1) / kRSeg);
    uint64_t items = groups * ns, cap = (uint64_t)ctx->cus * 32;
    unsigned g = (unsigned)(items < cap ? (items ? items : 1) : cap);
    auto* d2 = reinterpret_cast<u64x2*>(dst);
    auto* s2 = reinterpret_cast<const u64x2*>(src);
    if (vec2 && group == 2 && ctx->tune_reduce != 2)
        hipLaunchKernelGGL((k_reduce_or_g<2>), dim3(g), dim3(kBlock), 0, ctx->stream, d2, s2,
                           groups, per, ns);
    else if (vec2 && group == 3 && ctx->tune_reduce != 2)
        hipLaunchKernelGGL((k_reduce_or_g<3>), dim3(g), dim3(kBlock), 0, ctx->stream, d2, s2,
                           groups, per, ns);
    else if (vec2 && group == 4 && ctx->tune_reduce != 2)
        hipLaunchKernelGGL((k_reduce_or_g<4>), dim3(g), dim3(kBlock), 0, ctx->stream, d2, s2,
                           groups, per, ns);
    else if (vec2)
        hipLaunchKernelGGL((k_reduce_or<true>), dim3(g), dim3(kBlock), 0, ctx->stream,
                           (u64*)dst, (const u64*)src, groups, group, wr, ns);
    else
        hipLaunchKernelGGL((k_reduce_or<false>), dim3(g), dim3(kBlock), 0, ctx->stream,
                           (u64*)dst, (const u64*)src, groups, group, wr, ns);
    return hipGetLastError();
}

// dst[w] = join_j src[j*n + w]: the reduce of an all-to-all receive buffer.  The join
// is the word-wise OR for set bitmaps and the per-actor (unsigned) max for G-Counter
// counts (riak_dt_gcounter merge); MAX selects the latter.
template <bool MAX>
__global__ __launch_bounds__(kBlock) void k_reduce_chunks(u64x2* dst, const u64x2* src,
                                                          uint64_t n, uint32_t nchunks) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        u64x2 acc = ld2<true>(src + i);
        for (uint32_t j = 1; j < nchunks; ++j) {
            const u64x2 v = ld2<true>(src + (uint64_t)j * n + i);
            acc.x = join_word<MAX>(acc.x, v.x);
            acc.y = join_word<MAX>(acc.y, v.y);
        }
        st2<true>(dst + i, acc);
    }
}

// chunk count known at compile time (world sizes 2..8): all NC loads of a cell are
// issued before the first join, so a lane keeps U x NC x 16 B in flight (U cells per
// lane per step, a stride apart, as the join's sweep does)
template <bool MAX, int NC, int U, bool NT>
__global__ __launch_bounds__(kBlock) void k_reduce_chunks_n(u64x2* dst, const u64x2* src,
                                                            uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        u64x2 v[U][NC];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < NC; ++j) v[u][j] = ld2<NT>(src + (uint64_t)j * n + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
            for (int j = 1; j < NC; ++j) {
                v[u][0].x = join_word<MAX>(v[u][0].x, v[u][j].x);
                v[u][0].y = join_word<MAX>(v[u][0].y, v[u][j].y);
            }
            st2<NT>(dst + i + u * stride, v[u][0]);
        }
    }
    for (; i < n; i += stride) {
        u64x2 v[NC];
#pragma unroll
        for (int j = 0; j < NC; ++j) v[j] = ld2<NT>(src + (uint64_t)j * n + i);
#pragma unroll
        for (int j = 1; j < NC; ++j) {
            v[0].x = join_word<MAX>(v[0].x, v[j].x);
            v[0].y = join_word<MAX>(v[0].y, v[j].y);
        }
        st2<NT>(dst + i, v[0]);
    }
}

// Tiled, one source at a time: a block owns T x 256 consecutive cells and reads them
// from source 0, then 1, ... (T loads in flight per lane per source), one tile per
// block and no grid stride, so the blocks in flight cover one contiguous run of every
// source.  At N = 8 (98304 x 4096 cells, 51.5 GB read + 6.4 GB written) this runs
// 10.2 ms against 11.4 ms for the grid-stride sweep with all 8 loads of a cell in
// flight (profiles/r02_sweep_reduce_tiles.log); the two-stream join gains nothing from
// the same shape (r02_sweep_join_tiles.log), so it keeps its sweep.
template <bool MAX, int NC, int T>
__global__ __launch_bounds__(kBlock) void k_reduce_chunks_tile(u64x2* dst, const u64x2* src,
                                                               uint64_t n) {
    const uint64_t tile = (uint64_t)T * kBlock;
    const uint64_t tiles = n / tile;
    for (uint64_t b = blockIdx.x; b < tiles; b += gridDim.x) {
        const uint64_t i0 = b * tile + threadIdx.x;
        u64x2 acc[T];
#pragma unroll
        for (int u = 0; u < T; ++u) acc[u] = ld2<true>(src + i0 + u * kBlock);
#pragma unroll
        for (int j = 1; j < NC; ++j) {
            u64x2 v[T];
#pragma unroll
            for (int u = 0; u < T; ++u) v[u] = ld2<true>(src + (uint64_t)j * n + i0 + u * kBlock);
#pragma unroll
            for (int u = 0; u < T; ++u) {
                acc[u].x = join_word<MAX>(acc[u].x, v[u].x);
                acc[u].y = join_word<MAX>(acc[u].y, v[u].y);
            }
        }
#pragma unroll
        for (int u = 0; u < T; ++u) st2<true>(dst + i0 + u * kBlock, acc[u]);
    }
    // the cells past the last whole tile
    for (uint64_t i = tiles * tile + (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * kBlock) {
        u64x2 a = ld2<true>(src + i);
        for (int j = 1; j < NC; ++j) {
            const u64x2 v = ld2<true>(src + (uint64_t)j * n + i);
            a.x = join_word<MAX>(a.x, v.x);
            a.y = join_word<MAX>(a.y, v.y);
        }
        st2<true>(dst + i, a);
    }
}

template <bool MAX>
static void launch_reduce_tiles(laspj_ctx* ctx, u64x2* d, const u64x2* s, uint64_t n,
                                uint32_t nchunks) {
    // T cells per lane: the unroll knob when 2, 4 or 8, else 4
    const int T = ctx->tune_unroll == 8 ? 8 : ctx->tune_unroll == 2 ? 2 : 4;
    const uint64_t tiles = n / ((uint64_t)T * kBlock);
    const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(tiles, 1u << 30));
#define LJ_RT(NC, TT)                                                                        \
    hipLaunchKernelGGL((k_reduce_chunks_tile<MAX, NC, TT>), dim3(grid), dim3(kBlock), 0,     \
                       ctx->stream, d, s, n)
#define LJ_RTN(NC)                                                                           \
    case NC:                                                                                 \
        if (T == 8) LJ_RT(NC, 8);                                                            \
        else if (T == 2) LJ_RT(NC, 2);                                                       \
        else LJ_RT(NC, 4);                                                                   \
        break
    switch (nchunks) {
        LJ_RTN(2); LJ_RTN(3); LJ_RTN(4); LJ_RTN(5); LJ_RTN(6); LJ_RTN(7); LJ_RTN(8);
    }
#undef LJ_RTN
#undef LJ_RT
}

// the same reduce over NC arbitrary source arrays (the anti-entropy round reads the
// rank's own copy in place in its state and the peers' copies from the receive buffer,
// and writes the join back into the state: no staging copies)
struct Srcs {
    const u64x2* p[8];
};

// tiles of 4 cells per lane, one per block, sources read one at a time (as
// k_reduce_chunks_tile)
template <bool MAX, int NC>
__global__ __launch_bounds__(kBlock) void k_reduce_ptrs(u64x2* dst, Srcs s, uint64_t n) {
    constexpr int T = 4;
    const uint64_t tile = (uint64_t)T * kBlock;
    const uint64_t tiles = n / tile;
    for (uint64_t b = blockIdx.x; b < tiles; b += gridDim.x) {
        const uint64_t i0 = b * tile + threadIdx.x;
        u64x2 acc[T];
#pragma unroll
        for (int u = 0; u < T; ++u) acc[u] = ld2<true>(s.p[0] + i0 + u * kBlock);
#pragma unroll
        for (int j = 1; j < NC; ++j) {
            u64x2 v[T];
#pragma unroll
            for (int u = 0; u < T; ++u) v[u] = ld2<true>(s.p[j] + i0 + u * kBlock);
#pragma unroll
            for (int u = 0; u < T; ++u) {
                acc[u].x = join_word<MAX>(acc[u].x, v[u].x);
                acc[u].y = join_word<MAX>(acc[u].y, v[u].y);
            }
        }
#pragma unroll
        for (int u = 0; u < T; ++u) st2<true>(dst + i0 + u * kBlock, acc[u]);
    }
    for (uint64_t i = tiles * tile + (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * kBlock) {
        u64x2 a = ld2<true>(s.p[0] + i);
#pragma unroll
        for (int j = 1; j < NC; ++j) {
            const u64x2 v = ld2<true>(s.p[j] + i);
            a.x = join_word<MAX>(a.x, v.x);
            a.y = join_word<MAX>(a.y, v.y);
        }
        st2<true>(dst + i, a);
    }
}

// the last word of an odd word count (a G-Set batch can have one)
template <bool MAX>
__global__ void k_reduce_ptrs_last(u64* dst, Srcs s, uint32_t nsrc, uint64_t w) {
    if (threadIdx.x != 0) return;
    u64 a = reinterpret_cast<const u64*>(s.p[0])[w];
    for (uint32_t j = 1; j < nsrc; ++j) a = join_word<MAX>(a, reinterpret_cast<const u64*>(s.p[j])[w]);
    dst[w] = a;
}

hipError_t launch_reduce_ptrs(laspj_ctx* ctx, uint64_t* dst, const uint64_t* const* srcs,
                              uint32_t nsrc, uint64_t words, bool max_join) {
    if (nsrc < 1 || nsrc > 8) return hipErrorInvalidValue;
    if (words & 1) {
        Srcs t;
        for (uint32_t j = 0; j < 8; ++j)
            t.p[j] = reinterpret_cast<const u64x2*>(srcs[j < nsrc ? j : 0]);
        if (max_join)
            hipLaunchKernelGGL(k_reduce_ptrs_last<true>, dim3(1), dim3(64), 0, ctx->stream,
                               reinterpret_cast<u64*>(dst), t, nsrc, words - 1);
        else
            hipLaunchKernelGGL(k_reduce_ptrs_last<false>, dim3(1), dim3(64), 0, ctx->stream,
                               reinterpret_cast<u64*>(dst), t, nsrc, words - 1);
        if (--words == 0) return hipGetLastError();
    }
    Srcs s;
    for (uint32_t j = 0; j < 8; ++j)
        s.p[j] = reinterpret_cast<const u64x2*>(srcs[j < nsrc ? j : 0]);
    const uint64_t n = words / 2;
    const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(n / (4 * kBlock), 1u << 30));
    auto* d = reinterpret_cast<u64x2*>(dst);
#define LJ_RP(NC)                                                                              \
    case NC:                                                                                   \
        if (max_join)                                                                          \
            hipLaunchKernelGGL((k_reduce_ptrs<true, NC>), dim3(grid), dim3(kBlock), 0,        \
                               ctx->stream, d, s, n);                                          \
        else                                                                                   \
            hipLaunchKernelGGL((k_reduce_ptrs<false, NC>), dim3(grid), dim3(kBlock), 0,       \
                               ctx->stream, d, s, n);                                          \
        break
    switch (nsrc) {
        LJ_RP(1); LJ_RP(2); LJ_RP(3); LJ_RP(4); LJ_RP(5); LJ_RP(6); LJ_RP(7); LJ_RP(8);
    }
#undef LJ_RP
    return hipGetLastError();
}

template <bool MAX>
__global__ __launch_bounds__(kBlock) void k_reduce_chunks_scalar(u64* dst, const u64* src,
                                                                 uint64_t n, uint32_t nchunks) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        u64 acc = src[i];
        for (uint32_t j = 1; j < nchunks; ++j) acc = join_word<MAX>(acc, src[(uint64_t)j * n + i]);
        dst[i] = acc;
    }
}

template <bool MAX>
static void launch_reduce_chunks_t(laspj_ctx* ctx, uint64_t* dst, const uint64_t* src,
                                   uint64_t words, uint32_t nchunks) {
    if ((words & 1) == 0) {
        StreamTune t = stream_tune(ctx, words / 2);
        auto* d2 = reinterpret_cast<u64x2*>(dst);
        auto* s2 = reinterpret_cast<const u64x2*>(src);
        const uint64_t n = words / 2;
        // cells per lane per step: the unroll knob when set (1 or 2), else 1; the
        // non-temporal knob as for the join
        const int u = ctx->tune_unroll == 2 ? 2 : 1;
#define LJ_RCN(NC)                                                                          \
    case NC:                                                                                \
        if (u == 2 && t.nt)                                                                 \
            hipLaunchKernelGGL((k_reduce_chunks_n<MAX, NC, 2, true>), dim3(t.grid),        \
                               dim3(kBlock), 0, ctx->stream, d2, s2, n);                    \
        else if (u == 2)                                                                    \
            hipLaunchKernelGGL((k_reduce_chunks_n<MAX, NC, 2, false>), dim3(t.grid),       \
                               dim3(kBlock), 0, ctx->stream, d2, s2, n);                    \
        else if (t.nt)                                                                      \
            hipLaunchKernelGGL((k_reduce_chunks_n<MAX, NC, 1, true>), dim3(t.grid),        \
                               dim3(kBlock), 0, ctx->stream, d2, s2, n);                    \
        else                                                                                \
            hipLaunchKernelGGL((k_reduce_chunks_n<MAX, NC, 1, false>), dim3(t.grid),       \
                               dim3(kBlock), 0, ctx->stream, d2, s2, n);                    \
        break
        if (ctx->tune_reduce != 2 && ctx->tune_reduce != 3 && nchunks >= 2 && nchunks <= 8) {
            launch_reduce_tiles<MAX>(ctx, d2, s2, n, nchunks);
            return;
        }
        // knob 3: the grid-stride sweep with NC compile-time loads per cell
        switch (ctx->tune_reduce == 2 ? 0u : nchunks) {
            LJ_RCN(2); LJ_RCN(3); LJ_RCN(4); LJ_RCN(5); LJ_RCN(6); LJ_RCN(7); LJ_RCN(8);
            default:
                hipLaunchKernelGGL(k_reduce_chunks<MAX>, dim3(t.grid), dim3(kBlock), 0,
                                   ctx->stream, d2, s2, n, nchunks);
        }
#undef LJ_RCN
    } else {    // odd word count: chunk starts are only 8-byte aligned
        StreamTune t = stream_tune(ctx, words);
        hipLaunchKernelGGL(k_reduce_chunks_scalar<MAX>, dim3(t.grid), dim3(kBlock), 0,
                           ctx->stream, (u64*)dst, (const u64*)src, words, nchunks);
    }
}

hipError_t launch_reduce_chunks(laspj_ctx* ctx, uint64_t* dst, const uint64_t* src,
                                uint64_t words, uint32_t nchunks, bool max_join) {
    if (max_join) launch_reduce_chunks_t<true>(ctx, dst, src, words, nchunks);
    else launch_reduce_chunks_t<false>(ctx, dst, src, words, nchunks);
    return hipGetLastError();
}

// ------------------------------------------------------------------ synthetic replicas
// DESIGN.md §5; restated in oracle/laspj_oracle.c (orc_synth_*).

__device__ __forceinline__ u64 sm64(u64 x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__device__ __forceinline__ u64 synth_replica_key(u64 seed, u64 grep) {
    return sm64(sm64(seed ^ 0x4C41535000000000ull) ^ grep);
}

__global__ __launch_bounds__(kBlock) void k_fill_orset(u64x2* cells, uint64_t R, uint32_t E,
                                                       u64 seed, u64 base, u64 tmask) {
    const uint64_t n = R * E;
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        uint64_t rep = i / E;
        uint32_t e = (uint32_t)(i - rep * E);
        u64 h = synth_replica_key(seed, base + rep);
        u64 x = sm64(h + (u64)e * 0xD1B54A32D192ED03ull);
        u64 y = sm64(x ^ 0xA5A5A5A5A5A5A5A5ull);
        u64 z = sm64(y ^ 0x5A5A5A5A5A5A5A5Aull);
        u64 w = sm64(z);
        // the full stream leaves ~5 % of elements absent; the T-token stream
        // (laspj_batch_fill_synthetic_tokens) keeps every element with 1..T tokens
        u64 p = (z % 20ull) == 0 ? 0ull : x;
        if (tmask != ~0ull) {
            p = x & tmask;
            if (p == 0) p = 1;
        }
        u64x2 c;
        c.x = p;
        c.y = p & y & w;
        cells[i] = c;
    }
}

__global__ __launch_bounds__(kBlock) void k_fill_gset(u64* words, uint64_t R, uint32_t E,
                                                      u64 seed, u64 base) {
    const uint64_t W = (E + 63ull) / 64ull;
    const uint64_t n = R * W;
    const u64 last_mask = (E % 64) ? ((1ull << (E % 64)) - 1ull) : ~0ull;
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        uint64_t rep = i / W;
        uint64_t wi = i - rep * W;
        u64 h = synth_replica_key(seed, base + rep);
        u64 x = sm64(h + wi * 0xD1B54A32D192ED03ull);
        words[i] = (wi == W - 1) ? (x & last_mask) : x;
    }
}

// G-Counter replicas: count of actor slot a = 20 low bits of the stream word (bench data)
__global__ __launch_bounds__(kBlock) void k_fill_gcounter(u64* words, uint64_t R, uint64_t W,
                                                          u64 seed, u64 base) {
    const uint64_t n = R * W;
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        uint64_t rep = i / W;
        uint64_t a = i - rep * W;
        u64 h = synth_replica_key(seed, base + rep);
        words[i] = sm64(h + a * 0xD1B54A32D192ED03ull) & 0xFFFFFull;
    }
}

hipError_t launch_fill_synthetic(laspj_ctx* ctx, laspj_batch* b, uint64_t seed,
                                 uint64_t base, uint64_t tmask) {
    if (b->kind == LASPJ_KIND_GCOUNTER) {
        StreamTune t = stream_tune(ctx, b->replicas * b->words_per_replica / 2 + 1);
        hipLaunchKernelGGL(k_fill_gcounter, dim3(t.grid), dim3(kBlock), 0, ctx->stream,
                           (u64*)b->dev, b->replicas, b->words_per_replica, (u64)seed, (u64)base);
        return hipGetLastError();
    }
    StreamTune t = stream_tune(ctx, b->replicas * b->words_per_replica / 2 + 1);
    if (b->kind == LASPJ_KIND_ORSET)
        hipLaunchKernelGGL(k_fill_orset, dim3(t.grid), dim3(kBlock), 0, ctx->stream,
                           reinterpret_cast<u64x2*>(b->dev), b->replicas, b->elements,
                           (u64)seed, (u64)base, (u64)tmask);
    else
        hipLaunchKernelGGL(k_fill_gset, dim3(t.grid), dim3(kBlock), 0, ctx->stream,
                           (u64*)b->dev, b->replicas, b->elements, (u64)seed, (u64)base);
    return hipGetLastError();
}

// ------------------------------------------------------------------ fragment / context
// value({tokens, E}) / value({fragment, E}) (lasp_orset.erl:76-89): the cell of element
// slot e of every replica; precondition_context/1 (:147-154, minimum_tokens :264-267):
// every element keeps its tokens flagged false, and drops out when none is left.

__global__ __launch_bounds__(kBlock) void k_orset_fragment(const u64x2* cells, u64x2* out,
                                                           uint64_t R, uint32_t E, uint32_t e,
                                                           uint32_t k) {
    // k {p, r} pairs per cell (wide batches): out holds replica i's pairs at i k ..
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < R * k;
         i += (uint64_t)gridDim.x * kBlock) {
        const uint64_t rep = i / k;
        out[i] = cells[(rep * E + e) * k + (i - rep * k)];
    }
}

template <int U, bool NT>
__global__ __launch_bounds__(kBlock) void k_orset_context(u64x2* d, const u64x2* a, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        u64x2 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = ld2<NT>(a + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) st2<NT>(d + i + u * stride, u64x2{x[u].x & ~x[u].y, 0});
    }
    for (; i < n; i += stride) {
        const u64x2 x = ld2<NT>(a + i);
        st2<NT>(d + i, u64x2{x.x & ~x.y, 0});
    }
}

hipError_t launch_orset_fragment(laspj_ctx* ctx, const laspj_batch* b, uint32_t e, void* out) {
    uint64_t g = (b->replicas * b->tok_words + kBlock - 1) / kBlock;
    if (g > (uint64_t)ctx->cus * 16) g = (uint64_t)ctx->cus * 16;
    hipLaunchKernelGGL(k_orset_fragment, dim3((unsigned)(g ? g : 1)), dim3(kBlock), 0, ctx->stream,
                       reinterpret_cast<const u64x2*>(b->dev), reinterpret_cast<u64x2*>(out),
                       b->replicas, b->elements, e, b->tok_words);
    return hipGetLastError();
}

hipError_t launch_orset_context(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src) {
    const uint64_t n = src->replicas * (uint64_t)src->elements * src->tok_words;   // pairs
    StreamTune t = stream_tune(ctx, n);
    auto* d = reinterpret_cast<u64x2*>(dst->dev);
    auto* a = reinterpret_cast<const u64x2*>(src->dev);
    if (t.unroll == 1) hipLaunchKernelGGL((k_orset_context<1, true>), dim3(t.grid), dim3(kBlock), 0, ctx->stream, d, a, n);
    else hipLaunchKernelGGL((k_orset_context<2, true>), dim3(t.grid), dim3(kBlock), 0, ctx->stream, d, a, n);
    return hipGetLastError();
}

// ------------------------------------------------------------------ value / removed
// One wave per 64-element word: lane l tests element 64*w + l, __ballot packs the bits.

// One wave per (replica, <= 4096-cell segment): it walks the segment's <= 64 words, 4
// words (4 x 1 KiB loads) in flight before each group of __ballot packs, lane g keeping
// word g for one coalesced store at the end; no per-cell division.
constexpr uint64_t kTicketItems = 8192;     // see the partial-record note below
static uint32_t fin_for(uint64_t items, uint32_t ns) { return items <= kTicketItems ? ns : 0u; }

// segment length for R replicas of n items: the base segment, shortened (to a multiple
// of 256 items, >= 256) when R x segments would leave the chip under ~2048 waves
static uint64_t seg_for(uint64_t R, uint64_t n, uint64_t base) {
    if (n == 0) return base;
    const uint64_t ns = (n + base - 1) / base;
    if (R * ns >= 2048) return base;
    const uint64_t want = (2048 + R - 1) / R;
    uint64_t seg = (n + want - 1) / want;
    seg = (seg + 255) & ~255ull;
    if (seg < 256) seg = 256;
    return seg < base ? seg : base;
}

constexpr uint32_t kVSeg = 4096;

template <bool REMOVED, int U>
__global__ __launch_bounds__(kBlock) void k_orset_value(const u64x2* cells, u64* out,
                                                        uint64_t R, uint32_t E, uint32_t nseg,
                                                        uint32_t seg) {
    const uint32_t W = (E + 63u) / 64u;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nwaves = (uint64_t)gridDim.x * (kBlock / 64);
    for (uint64_t it = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 6; it < R * nseg;
         it += nwaves) {
        uint64_t rep = it / nseg;
        uint32_t e0 = (uint32_t)(it - rep * nseg) * seg;
        uint32_t e1 = min(E, e0 + seg);
        const u64x2* c = cells + rep * E;
        u64* o = out + rep * W;
        // lane g keeps the segment's g-th word (segments are <= 64 words), so the words
        // leave as one coalesced store instead of one single-lane store each
        const uint32_t g0 = e0 >> 6;
        u64 mine = 0;
        for (uint32_t e = e0; e < e1; e += 64 * U) {
            u64x2 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                uint32_t x = e + u * 64 + lane;
                v[u] = x < e1 ? ld2<true>(c + x) : u64x2{0, 0};
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                bool pred = REMOVED ? (v[u].y != 0) : ((v[u].x & ~v[u].y) != 0);
                u64 m = __ballot(pred);
                if (lane == ((e + u * 64) >> 6) - g0) mine = m;
            }
        }
        if (lane < ((e1 - e0 + 63u) >> 6)) o[g0 + lane] = mine;
    }
}

hipError_t launch_combinator_value(laspj_ctx* ctx, const laspj_batch* b, uint64_t* out);

hipError_t launch_orset_value(laspj_ctx* ctx, const laspj_batch* b, uint64_t* out,
                              bool removed) {
    if (b->kind != LASPJ_KIND_ORSET) return launch_combinator_value(ctx, b, out);
    const uint32_t sg = (uint32_t)seg_for(b->replicas, b->elements, kVSeg);
    uint32_t ns = (b->elements + sg - 1) / sg;
    uint64_t items = b->replicas * ns;
    uint64_t blocks = (items + 3) / 4, cap = (uint64_t)ctx->cus * 16;
    int grid = (int)(blocks < cap ? (blocks ? blocks : 1) : cap);
    auto* cells = reinterpret_cast<const u64x2*>(b->dev);
    // words in flight per lane: 4 (default) or the stream unroll knob when it is 8
    const bool u8 = ctx->tune_unroll == 8;
    auto k = removed ? (u8 ? k_orset_value<true, 8> : k_orset_value<true, 4>)
                     : (u8 ? k_orset_value<false, 8> : k_orset_value<false, 4>);
    hipLaunchKernelGGL(k, dim3(grid), dim3(kBlock), 0, ctx->stream, cells, (u64*)out,
                       b->replicas, b->elements, ns, sg);
    return hipGetLastError();
}

// ------------------------------------------------------------------ per-replica reductions
// stats / equal / inflation reduce over each replica.  Work is cut into segments of
// kSeg cells (kSegW words for G-Sets); one wave64 reduces one (replica, segment) item
// with __ballot / __shfl_xor.  A replica that is a single segment (BASELINE config 2:
// E = 4096) is finished by its wave; longer replicas (config 4: 3M slots) combine their
// segments with atomics into a per-replica record in ctx->partials, the last segment's
// wave finishing the replica (a ticket); segments shrink when R x segments is small
// (seg_for), so a launch always has thousands of waves.

constexpr uint32_t kSeg = 4096;     // OR-Set cells per segment (64 KiB)
constexpr uint32_t kSegW = 4096;    // G-Set words per segment (32 KiB)

__device__ __forceinline__ void seg_range(uint64_t item, uint32_t nseg, uint64_t n, uint64_t seg,
                                          uint64_t* rep, uint64_t* b, uint64_t* e) {
    *rep = item / nseg;
    uint64_t sg = item - *rep * nseg;
    *b = sg * seg;
    *e = min(n, *b + seg);
}

// K per-replica sums: written directly when a replica is one segment, else accumulated
// in its record of ctx->partials and finished either by the last segment's wave
// (fin = segments: a ticket in word 3, see `emit` below) or, for large launches
// (fin = 0), by a finalize kernel; both re-zero the record
template <int K>
__device__ __forceinline__ void emit_sums(bool seg, u64* out, u64* part, uint64_t rep,
                                          const u64 (&v)[K], uint32_t fin) {
    if (!seg) {
#pragma unroll
        for (int k = 0; k < K; ++k) out[rep * K + k] = v[k];
        return;
    }
    u64* r = part + rep * 4;
#pragma unroll
    for (int k = 0; k < K; ++k)
        if (v[k]) __hip_atomic_fetch_add(r + k, v[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (fin == 0) return;                 // a finalize kernel reads and re-zeroes the record
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const u64 tk = __hip_atomic_fetch_add(r + 3, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (tk == fin - 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#pragma unroll
        for (int k = 0; k < K; ++k)
            out[rep * K + k] = __hip_atomic_load(r + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            __hip_atomic_store(r + k, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

template <int K>
__global__ void k_finalize_sums(u64* part, u64* out, uint64_t R) {
    for (uint64_t rep = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; rep < R;
         rep += (uint64_t)gridDim.x * blockDim.x) {
        u64* r = part + rep * 4;
#pragma unroll
        for (int k = 0; k < K; ++k) out[rep * K + k] = r[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) r[k] = 0;
    }
}

template <int K>
static hipError_t finalize_sums(laspj_ctx* ctx, u64* part, uint64_t* out, uint64_t R) {
    uint64_t g = (R + kBlock - 1) / kBlock;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_finalize_sums<K>, dim3((unsigned)g), dim3(kBlock), 0, ctx->stream, part,
                       (u64*)out, R);
    return hipGetLastError();
}

template <bool SEG>
__global__ __launch_bounds__(kBlock) void k_orset_stats(const u64x2* cells, u64* out,
                                                        u64* part, uint64_t R, uint32_t E,
                                                        uint32_t nseg, uint64_t sg,
                                                        uint32_t fin) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nwaves = (uint64_t)gridDim.x * (kBlock / 64);
    for (uint64_t it = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 6; it < R * nseg;
         it += nwaves) {
        uint64_t rep, b, e;
        seg_range(it, nseg, E, sg, &rep, &b, &e);
        const u64x2* c = cells + rep * E;
        u64 elems = 0, adds = 0, rems = 0;
#pragma unroll 8
        for (uint64_t i = b + lane; i < e; i += 64) {
            u64x2 v = ld2<true>(c + i);
            elems += v.x != 0;
            adds += __popcll(v.x & ~v.y);
            rems += __popcll(v.y);
        }
        elems = wave_sum(elems);
        adds = wave_sum(adds);
        rems = wave_sum(rems);
        if (lane == 0) {
            const u64 v[3] = {elems, adds, rems};
            emit_sums<3>(SEG, out, part, rep, v, fin);
        }
    }
}

template <bool SEG>
__global__ __launch_bounds__(kBlock) void k_gset_stats(const u64* words, u64* out, u64* part,
                                                       uint64_t R, uint64_t W, uint32_t nseg,
                                                       uint64_t sg, uint32_t fin) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nwaves = (uint64_t)gridDim.x * (kBlock / 64);
    for (uint64_t it = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 6; it < R * nseg;
         it += nwaves) {
        uint64_t rep, b, e;
        seg_range(it, nseg, W, sg, &rep, &b, &e);
        u64 n = 0;
        for (uint64_t w = b + lane; w < e; w += 64) n += __popcll(words[rep * W + w]);
        n = wave_sum(n);
        if (lane == 0) {
            const u64 v[1] = {n};
            emit_sums<1>(SEG, out, part, rep, v, fin);
        }
    }
}

static uint32_t nseg_of(uint64_t n, uint64_t seg) { return (uint32_t)((n + seg - 1) / seg); }

static int seg_grid(const laspj_ctx* ctx, uint64_t items) {
    uint64_t blocks = (items + 3) / 4;
    uint64_t cap = (uint64_t)ctx->cus * 16;
    if (blocks > cap) blocks = cap;
    return blocks ? (int)blocks : 1;
}

static hipError_t partials(laspj_ctx* ctx, uint64_t R, u64** out);

hipError_t launch_orset_stats(laspj_ctx* ctx, const laspj_batch* b, uint64_t* out) {
    const uint64_t sg = seg_for(b->replicas, b->elements, kSeg);
    uint32_t ns = nseg_of(b->elements, sg);
    int grid = seg_grid(ctx, b->replicas * ns);
    auto* cells = reinterpret_cast<const u64x2*>(b->dev);
    if (ns == 1) {
        hipLaunchKernelGGL(k_orset_stats<false>, dim3(grid), dim3(kBlock), 0, ctx->stream, cells,
                           (u64*)out, nullptr, b->replicas, b->elements, ns, sg, 0u);
    } else {
        u64* part = nullptr;
        hipError_t e = partials(ctx, b->replicas, &part);
        if (e != hipSuccess) return e;
        const uint32_t fin = fin_for(b->replicas * ns, ns);
        hipLaunchKernelGGL(k_orset_stats<true>, dim3(grid), dim3(kBlock), 0, ctx->stream, cells,
                           (u64*)out, part, b->replicas, b->elements, ns, sg, fin);
        if (!fin) return finalize_sums<3>(ctx, part, out, b->replicas);
    }
    return hipGetLastError();
}

hipError_t launch_gset_stats(laspj_ctx* ctx, const laspj_batch* b, uint64_t* out) {
    const uint64_t W = b->words_per_replica;
    const uint64_t sg = seg_for(b->replicas, W, kSegW);
    uint32_t ns = nseg_of(W, sg);
    int grid = seg_grid(ctx, b->replicas * ns);
    if (ns == 1) {
        hipLaunchKernelGGL(k_gset_stats<false>, dim3(grid), dim3(kBlock), 0, ctx->stream,
                           (const u64*)b->dev, (u64*)out, nullptr, b->replicas, W, ns, sg, 0u);
    } else {
        u64* part = nullptr;
        hipError_t e = partials(ctx, b->replicas, &part);
        if (e != hipSuccess) return e;
        const uint32_t fin = fin_for(b->replicas * ns, ns);
        hipLaunchKernelGGL(k_gset_stats<true>, dim3(grid), dim3(kBlock), 0, ctx->stream,
                           (const u64*)b->dev, (u64*)out, part, b->replicas, W, ns, sg, fin);
        if (!fin) return finalize_sums<1>(ctx, part, out, b->replicas);
    }
    return hipGetLastError();
}

// per-replica partial record for segmented reductions: {flags, count P, count C, ticket}.
// Records are all-zero between launches: zeroed once when allocated, and re-zeroed by
// whoever finishes them.  Small launches (<= kTicketItems segment items, e.g. one long
// replica on the bind path) finish in the same launch: the wave whose ticket reads
// fin - 1 computes the result.  Its agent-scope release / acquire fences write back and
// invalidate the XCD's L2, which is cheap for a few hundred waves but not for 750k
// (config 4), so large launches accumulate with plain atomics and a finalize kernel
// reads and re-zeroes the records.

constexpr u64 kViol = 1, kChanged = 2;

static hipError_t partials(laspj_ctx* ctx, uint64_t R, u64** out) {
    uint64_t need = R * 32;
    if (ctx->partials_bytes < need) {
        if (ctx->partials) {
            hipError_t e = hipStreamSynchronize(ctx->stream);
            if (e != hipSuccess) return e;
            hipFree(ctx->partials);
            ctx->partials = nullptr;
            ctx->partials_bytes = 0;
        }
        hipError_t e = dev_malloc(ctx, &ctx->partials, need);
        if (e != hipSuccess) return e;
        ctx->partials_bytes = need;
        e = hipMemsetAsync(ctx->partials, 0, need, ctx->stream);
        if (e != hipSuccess) return e;
    }
    *out = static_cast<u64*>(ctx->partials);
    return hipSuccess;
}

// mode 0: equal (= no difference), 1: inflation, 2: strict inflation, 3: G-Counter strict
// inflation (value(Prev) < value(Cur)), 4 / 5: G-Counter threshold t =< sum / t < sum
__device__ __forceinline__ bool seg_result(int mode, u64 f, u64 np, u64 nc, u64 t) {
    if (mode == 0) return !(f & kViol);
    if (mode == 3) return np < nc;
    if (mode == 4) return t <= np;
    if (mode == 5) return t < np;
    return !(f & kViol) && (mode == 1 || (f & kChanged) || np < nc);
}

__device__ __forceinline__ void emit(bool seg, uint8_t* out, u64* part, uint64_t rep,
                                     u64 flags, u64 np, u64 nc, int mode, uint32_t fin,
                                     u64 t = 0) {
    if (!seg) {
        out[rep] = seg_result(mode, flags, np, nc, t) ? 1 : 0;
        return;
    }
    u64* r = part + rep * 4;
    if (flags) __hip_atomic_fetch_or(r, flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (np) __hip_atomic_fetch_add(r + 1, np, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (nc) __hip_atomic_fetch_add(r + 2, nc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (fin == 0) return;                 // a finalize kernel reads and re-zeroes the record
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const u64 tk = __hip_atomic_fetch_add(r + 3, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (tk == fin - 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        const u64 f = __hip_atomic_load(r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const u64 a = __hip_atomic_load(r + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const u64 b = __hip_atomic_load(r + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        out[rep] = seg_result(mode, f, a, b, t) ? 1 : 0;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            __hip_atomic_store(r + k, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ void k_finalize(u64* part, uint8_t* out, uint64_t R, int mode, u64 t) {
    for (uint64_t rep = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; rep < R;
         rep += (uint64_t)gridDim.x * blockDim.x) {
        u64* r = part + rep * 4;
        out[rep] = seg_result(mode, r[0], r[1], r[2], t) ? 1 : 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) r[k] = 0;
    }
}

static hipError_t finalize(laspj_ctx* ctx, u64* part, uint8_t* out, uint64_t R, int mode,
                           u64 t = 0) {
    uint64_t g = (R + kBlock - 1) / kBlock;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_finalize, dim3((unsigned)g), dim3(kBlock), 0, ctx->stream, part, out, R,
                       mode, t);
    return hipGetLastError();
}



// ------------------------------------------------------------------ equal
// equal/2 (lasp_orset.erl:136-138, lasp_gset.erl:103-105): every word equal.

template <bool SEG, bool VEC2>
__global__ __launch_bounds__(kBlock) void k_equal(const u64* a, const u64* b, uint8_t* out,
                                                  u64* part, uint64_t R, uint64_t wr,
                                                  uint32_t nseg, uint64_t seg, uint32_t fin) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nwaves = (uint64_t)gridDim.x * (kBlock / 64);
    const uint64_t n = VEC2 ? wr / 2 : wr;
    for (uint64_t it = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 6; it < R * nseg;
         it += nwaves) {
        uint64_t rep, lo, hi;
        seg_range(it, nseg, n, seg, &rep, &lo, &hi);
        bool diff = false;
        if constexpr (VEC2) {
            const u64x2* a2 = reinterpret_cast<const u64x2*>(a + rep * wr);
            const u64x2* b2 = reinterpret_cast<const u64x2*>(b + rep * wr);
#pragma unroll 4
            for (uint64_t w = lo + lane; w < hi; w += 64) {
                u64x2 x = ld2<true>(a2 + w), y = ld2<true>(b2 + w);
                diff |= (x.x != y.x) | (x.y != y.y);
            }
        } else {
            for (uint64_t w = lo + lane; w < hi; w += 64) diff |= a[rep * wr + w] != b[rep * wr + w];
        }
        bool any = __ballot(diff) != 0;
        if (lane == 0) emit(SEG, out, part, rep, any ? kViol : 0, 0, 0, 0, fin);
    }
}

hipError_t launch_equal(laspj_ctx* ctx, const laspj_batch* a, const laspj_batch* b,
                        uint8_t* out) {
    bool vec2 = (a->words_per_replica & 1) == 0;
    uint64_t n = vec2 ? a->words_per_replica / 2 : a->words_per_replica;
    const uint64_t sg = seg_for(a->replicas, n, kSeg);
    uint32_t ns = nseg_of(n, sg);
    int grid = seg_grid(ctx, a->replicas * ns);
    u64* part = nullptr;
    if (ns > 1) {
        hipError_t e = partials(ctx, a->replicas, &part);
        if (e != hipSuccess) return e;
    }
#define LJ_EQ(S, V)                                                                        \
    hipLaunchKernelGGL((k_equal<S, V>), dim3(grid), dim3(kBlock), 0, ctx->stream,          \
                       (const u64*)a->dev, (const u64*)b->dev, out, part, a->replicas,     \
                       a->words_per_replica, ns, sg, fin)
    const uint32_t fin = ns > 1 ? fin_for(a->replicas * ns, ns) : 0u;
    if (ns > 1) {
        if (vec2) LJ_EQ(true, true); else LJ_EQ(true, false);
        if (!fin) return finalize(ctx, part, out, a->replicas, 0);
        return hipGetLastError();
    }
    if (vec2) LJ_EQ(false, true); else LJ_EQ(false, false);
#undef LJ_EQ
    return hipGetLastError();
}

// ------------------------------------------------------------------ inflation

// lasp_lattice.erl:153-161 (non-strict): every Prev element is in Cur with every Prev
// token  <=>  for all e: (pP & ~pC) == 0   (an absent Cur element has pC == 0).
// lasp_lattice.erl:235-253 (strict): [] -> non-empty is true; otherwise
// inflation && (some element of Prev found in Cur with a different token dict
//               || length(Prev) < length(Cur)).
template <bool STRICT, bool SEG>
__global__ __launch_bounds__(kBlock) void k_orset_inflation(const u64x2* prev,
                                                            const u64x2* cur, uint8_t* out,
                                                            u64* part, uint64_t R, uint32_t E,
                                                            bool prev_bcast, uint32_t nseg,
                                                            uint64_t seg, uint32_t fin) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nwaves = (uint64_t)gridDim.x * (kBlock / 64);
    for (uint64_t it = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 6; it < R * nseg;
         it += nwaves) {
        uint64_t rep, lo, hi;
        seg_range(it, nseg, E, seg, &rep, &lo, &hi);
        const u64x2* P = prev + (prev_bcast ? 0 : rep * E);
        const u64x2* C = cur + rep * E;
        bool viol = false, changed = false;
        u64 np = 0, nc = 0;
#pragma unroll 4
        for (uint64_t e = lo + lane; e < hi; e += 64) {
            u64x2 p = ld2<false>(P + e), c = ld2<true>(C + e);
            viol |= (p.x & ~c.x) != 0;
            if constexpr (STRICT) {
                changed |= (p.x != 0) & (c.x != 0) & ((p.x != c.x) | (p.y != c.y));
                np += p.x != 0;
                nc += c.x != 0;
            }
        }
        u64 flags = (__ballot(viol) != 0) ? kViol : 0;
        if constexpr (STRICT) {
            if (__ballot(changed) != 0) flags |= kChanged;
            np = wave_sum(np);
            nc = wave_sum(nc);
        }
        if (lane == 0) emit(SEG, out, part, rep, flags, np, nc, STRICT ? 2 : 1, fin);
    }
}

// A dataflow stage whose output is threshold-checked in the same pass (BASELINE config
// 4's map -> filter -> fold -> {strict, Prev} read, fused): dst = src gathered through
// index (map / filter / fold compose into one index on the host: the fold's slot o takes
// filtered slot f[o], which is mapped slot f[o] when kept, which is src slot m[f[o]]),
// and out[i] = is_(strict_)inflation(prev[i], dst[i]) — lasp_lattice.erl:153-161,
// 235-253 — over the cells just written.  A block owns a 4096-slot segment of the output
// and a run of 8 replicas (its 16 index entries per lane stay in registers); the block's
// 4 waves combine their ballots in LDS and emit one partial per (replica, segment).
//
// KEYED: output keys may repeat across source slots (a collapsing map such as X div 3, a
// fold whose F(X) lists overlap).  The reference finds each Prev entry's key in Cur with
// lists:keyfind — the FIRST entry of Cur carrying that key — so an entry is compared with
// whatever entry of its key comes first in Cur, not with its own position.  head[o] is
// the first output slot with o's key, next[o] the following one (list order, kNone after
// the last); the walk takes the first present Cur slot of the chain.  Tokens of distinct
// source elements are distinct terms (every token Lasp mints is fresh, unique/1), so a
// match with another source slot is never ids_inflated and always `=/=`.  The walk only
// moves forward inside [0, E_out), so a malformed chain cannot loop.
constexpr uint32_t kFSeg = 4096, kFPer = kFSeg / kBlock, kFRun = 8, kNone = 0xFFFFFFFFu;

template <bool STRICT, bool SEG, bool KEYED>
__global__ __launch_bounds__(kBlock) void k_gather_inflation(u64x2* out, const u64x2* src,
                                                             const u64x2* prev,
                                                             const uint32_t* index,
                                                             const uint32_t* head,
                                                             const uint32_t* next,
                                                             uint8_t* res, u64* part,
                                                             uint64_t reps, uint32_t E_out,
                                                             uint32_t E_in, uint32_t nseg,
                                                             uint32_t fin, bool bcast) {
    __shared__ u64 s_f[kBlock / 64], s_np[kBlock / 64], s_nc[kBlock / 64];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t runs = (reps + kFRun - 1) / kFRun;
    for (uint64_t it = blockIdx.x; it < runs * nseg; it += gridDim.x) {
        const uint64_t run = it / nseg;
        const uint32_t o0 = (uint32_t)(it - run * nseg) * kFSeg;
        uint32_t si[kFPer], hd[KEYED ? kFPer : 1];
#pragma unroll
        for (uint32_t k = 0; k < kFPer; ++k) {
            const uint32_t o = o0 + k * kBlock + threadIdx.x;
            si[k] = o < E_out ? index[o] : kNone;
            if constexpr (KEYED) hd[k] = o < E_out ? head[o] : kNone;
        }
        const uint64_t r1 = min(reps, (run + 1) * kFRun);
        for (uint64_t rep = run * kFRun; rep < r1; ++rep) {
            const u64x2* s = src + rep * E_in;
            const u64x2* P = prev + (bcast ? 0 : rep * E_out);
            u64x2* d = out + rep * E_out;
            u64x2 v[kFPer];
#pragma unroll
            for (uint32_t k = 0; k < kFPer; ++k)
                v[k] = si[k] < E_in ? s[si[k]] : u64x2{0, 0};
            bool viol = false, changed = false;
            u64 np = 0, nc = 0;
#pragma unroll
            for (uint32_t k = 0; k < kFPer; ++k) {
                const uint32_t o = o0 + k * kBlock + threadIdx.x;
                if (o < E_out) {
                    __builtin_nontemporal_store(v[k], d + o);
                    const u64x2 p = __builtin_nontemporal_load(P + o);
                    u64x2 c = v[k];
                    bool other = false;             // keyfind matched another source slot
                    if constexpr (KEYED) {
                        if (p.x != 0 && (hd[k] != o || c.x == 0)) {
                            // lists:keyfind(Key, 1, Cur): first present slot of the chain
                            c = u64x2{0, 0};
                            uint32_t j = hd[k] < E_out ? hd[k] : o;
                            for (;;) {
                                const uint32_t sj = j == o ? si[k] : index[j];
                                const u64x2 cj = j == o ? v[k] : (sj < E_in ? s[sj] : u64x2{0, 0});
                                if (cj.x != 0) {
                                    c = cj;
                                    other = sj != si[k];
                                    break;
                                }
                                const uint32_t nj = next[j];
                                if (nj == kNone || nj <= j || nj >= E_out) break;
                                j = nj;
                            }
                        }
                    }
                    viol |= (p.x != 0) & ((c.x == 0) | other | ((p.x & ~c.x) != 0));
                    if constexpr (STRICT) {
                        changed |= (p.x != 0) & (c.x != 0) &
                                   (other | (p.x != c.x) | (p.y != c.y));
                        np += p.x != 0;
                        nc += v[k].x != 0;
                    }
                }
            }
            u64 f = (__ballot(viol) != 0) ? kViol : 0;
            if constexpr (STRICT) {
                if (__ballot(changed) != 0) f |= kChanged;
                np = wave_sum(np);
                nc = wave_sum(nc);
            }
            if (lane == 0) {
                s_f[wv] = f;
                s_np[wv] = np;
                s_nc[wv] = nc;
            }
            __syncthreads();
            if (threadIdx.x == 0) {
                u64 F = 0, NP = 0, NC = 0;
#pragma unroll
                for (int w = 0; w < kBlock / 64; ++w) F |= s_f[w], NP += s_np[w], NC += s_nc[w];
                emit(SEG, res, part, rep, F, NP, NC, STRICT ? 2 : 1, fin);
            }
            __syncthreads();
        }
    }
}

hipError_t launch_gather_inflation(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                                   const uint32_t* index, const uint32_t* head,
                                   const uint32_t* next, const laspj_batch* prev, bool strict,
                                   uint8_t* res) {
    const uint32_t ns = (dst->elements + kFSeg - 1) / kFSeg;
    const uint64_t items = (dst->replicas + kFRun - 1) / kFRun * ns;
    // one (run, segment) item per block, no grid stride: 21.5 ms against 22.5 ms with 32
    // blocks per CU striding (profiles/r02_sweep_c4_grid.log)
    const uint64_t cap = ctx->tune_grid > 0 ? (uint64_t)ctx->tune_grid : (1ull << 30);
    const uint64_t g = items < cap ? items : cap;
    const bool bc = prev->replicas == 1 && dst->replicas != 1;
    u64* part = nullptr;
    if (ns > 1) {
        hipError_t e = partials(ctx, dst->replicas, &part);
        if (e != hipSuccess) return e;
    }
    const uint32_t fin = ns > 1 ? fin_for(dst->replicas * ns, ns) : 0u;
    const bool keyed = head != nullptr;
#define LJ_GI(ST, SG, KY)                                                                    \
    hipLaunchKernelGGL((k_gather_inflation<ST, SG, KY>), dim3((unsigned)(g ? g : 1)),        \
                       dim3(kBlock), 0, ctx->stream, reinterpret_cast<u64x2*>(dst->dev),     \
                       reinterpret_cast<const u64x2*>(src->dev),                             \
                       reinterpret_cast<const u64x2*>(prev->dev), index, head, next, res,    \
                       part, dst->replicas, dst->elements, src->elements, ns, fin, bc)
#define LJ_GI2(SG)                                                                           \
    do {                                                                                     \
        if (keyed) {                                                                         \
            if (strict) LJ_GI(true, SG, true); else LJ_GI(false, SG, true);                 \
        } else {                                                                             \
            if (strict) LJ_GI(true, SG, false); else LJ_GI(false, SG, false);               \
        }                                                                                    \
    } while (0)
    if (ns > 1) {
        LJ_GI2(true);
        if (!fin) return finalize(ctx, part, res, dst->replicas, strict ? 2 : 1);
        return hipGetLastError();
    }
    LJ_GI2(false);
#undef LJ_GI2
#undef LJ_GI
    return hipGetLastError();
}

// lasp_lattice.erl:137-140 / :212-215: subset, and strict adds "sets differ".
template <bool STRICT, bool SEG>
__global__ __launch_bounds__(kBlock) void k_gset_inflation(const u64* prev, const u64* cur,
                                                           uint8_t* out, u64* part, uint64_t R,
                                                           uint64_t W, bool prev_bcast,
                                                           uint32_t nseg, uint64_t seg,
                                                           uint32_t fin) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nwaves = (uint64_t)gridDim.x * (kBlock / 64);
    for (uint64_t it = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 6; it < R * nseg;
         it += nwaves) {
        uint64_t rep, lo, hi;
        seg_range(it, nseg, W, seg, &rep, &lo, &hi);
        const u64* P = prev + (prev_bcast ? 0 : rep * W);
        const u64* C = cur + rep * W;
        bool viol = false, diff = false;
        for (uint64_t w = lo + lane; w < hi; w += 64) {
            u64 p = P[w], c = C[w];
            viol |= (p & ~c) != 0;
            diff |= p != c;
        }
        u64 flags = (__ballot(viol) != 0) ? kViol : 0;
        if (__ballot(diff) != 0) flags |= kChanged;
        // strict = subset and differs: "differs" plays the role of `changed`, and
        // np = nc = 0 so the length test never fires
        if (lane == 0) emit(SEG, out, part, rep, flags, 0, 0, STRICT ? 2 : 1, fin);
    }
}

hipError_t launch_orset_inflation(laspj_ctx* ctx, const laspj_batch* prev,
                                  const laspj_batch* cur, bool strict, uint8_t* out) {
    const uint64_t sg = seg_for(cur->replicas, cur->elements, kSeg);
    uint32_t ns = nseg_of(cur->elements, sg);
    int grid = seg_grid(ctx, cur->replicas * ns);
    bool bc = prev->replicas == 1 && cur->replicas != 1;
    auto* P = reinterpret_cast<const u64x2*>(prev->dev);
    auto* C = reinterpret_cast<const u64x2*>(cur->dev);
    u64* part = nullptr;
    if (ns > 1) {
        hipError_t e = partials(ctx, cur->replicas, &part);
        if (e != hipSuccess) return e;
    }
#define LJ_INF(ST, SG)                                                                      \
    hipLaunchKernelGGL((k_orset_inflation<ST, SG>), dim3(grid), dim3(kBlock), 0, ctx->stream, \
                       P, C, out, part, cur->replicas, cur->elements, bc, ns, sg, fin)
    const uint32_t fin = ns > 1 ? fin_for(cur->replicas * ns, ns) : 0u;
    if (ns > 1) {
        if (strict) LJ_INF(true, true); else LJ_INF(false, true);
        if (!fin) return finalize(ctx, part, out, cur->replicas, strict ? 2 : 1);
        return hipGetLastError();
    }
    if (strict) LJ_INF(true, false); else LJ_INF(false, false);
#undef LJ_INF
    return hipGetLastError();
}

hipError_t launch_gset_inflation(laspj_ctx* ctx, const laspj_batch* prev,
                                 const laspj_batch* cur, bool strict, uint8_t* out) {
    uint64_t W = cur->words_per_replica;
    const uint64_t sg = seg_for(cur->replicas, W, kSegW);
    uint32_t ns = nseg_of(W, sg);
    int grid = seg_grid(ctx, cur->replicas * ns);
    bool bc = prev->replicas == 1 && cur->replicas != 1;
    u64* part = nullptr;
    if (ns > 1) {
        hipError_t e = partials(ctx, cur->replicas, &part);
        if (e != hipSuccess) return e;
    }
#define LJ_GINF(ST, SG)                                                                     \
    hipLaunchKernelGGL((k_gset_inflation<ST, SG>), dim3(grid), dim3(kBlock), 0, ctx->stream, \
                       (const u64*)prev->dev, (const u64*)cur->dev, out, part, cur->replicas, \
                       W, bc, ns, sg, fin)
    const uint32_t fin = ns > 1 ? fin_for(cur->replicas * ns, ns) : 0u;
    if (ns > 1) {
        if (strict) LJ_GINF(true, true); else LJ_GINF(false, true);
        if (!fin) return finalize(ctx, part, out, cur->replicas, strict ? 2 : 1);
        return hipGetLastError();
    }
    if (strict) LJ_GINF(true, false); else LJ_GINF(false, false);
#undef LJ_GINF
    return hipGetLastError();
}

// ------------------------------------------------------------------ riak_dt_gcounter
// merge = per-actor max; value = sum (riak_dt, restated in oracle/core.py _GCounter)

template <int U>
__global__ __launch_bounds__(kBlock) void k_max16(u64x2* d, const u64x2* a, const u64x2* b,
                                                  uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        u64x2 x[U], y[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = ld2<true>(a + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) y[u] = ld2<true>(b + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            u64x2 m;
            m.x = x[u].x > y[u].x ? x[u].x : y[u].x;
            m.y = x[u].y > y[u].y ? x[u].y : y[u].y;
            st2<true>(d + i + u * stride, m);
        }
    }
    for (; i < n; i += stride) {
        u64x2 x = ld2<true>(a + i), y = ld2<true>(b + i), m;
        m.x = x.x > y.x ? x.x : y.x;
        m.y = x.y > y.y ? x.y : y.y;
        st2<true>(d + i, m);
    }
}

__global__ void k_max_tail(u64* d, const u64* a, const u64* b, uint64_t idx) {
    if (threadIdx.x == 0 && blockIdx.x == 0) d[idx] = a[idx] > b[idx] ? a[idx] : b[idx];
}

hipError_t launch_max(laspj_ctx* ctx, uint64_t* dst, const uint64_t* a, const uint64_t* b,
                      uint64_t words) {
    uint64_t n16 = words / 2;
    if (n16) {
        StreamTune t = stream_tune(ctx, n16);
        hipLaunchKernelGGL(k_max16<2>, dim3(t.grid), dim3(kBlock), 0, ctx->stream,
                           reinterpret_cast<u64x2*>(dst), reinterpret_cast<const u64x2*>(a),
                           reinterpret_cast<const u64x2*>(b), n16);
    }
    if (words & 1)
        hipLaunchKernelGGL(k_max_tail, dim3(1), dim3(64), 0, ctx->stream, (u64*)dst,
                           (const u64*)a, (const u64*)b, words - 1);
    return hipGetLastError();
}

__global__ __launch_bounds__(kBlock) void k_reduce_max(u64* dst, const u64* src, uint64_t groups,
                                                       uint32_t group, uint64_t wr) {
    const uint64_t n = groups * wr;
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        uint64_t g = i / wr, w = i - g * wr;
        uint64_t base = g * group * wr + w;
        u64 acc = src[base];
        for (uint32_t j = 1; j < group; ++j) {
            u64 v = src[base + j * wr];
            acc = v > acc ? v : acc;
        }
        dst[i] = acc;
    }
}

hipError_t launch_reduce_max(laspj_ctx* ctx, uint64_t* dst, const uint64_t* src,
                             uint64_t groups, uint32_t group, uint64_t wr) {
    if ((wr % 2) == 0 && (ctx->tune_reduce == 0 || ctx->tune_reduce == 4)) {   // as the OR reduce
        const uint64_t per = wr / 2;
        if ((per & (per - 1)) == 0 && group >= 2 && group <= 4) {
            const uint32_t lg = (uint32_t)__builtin_ctzll(per);
            auto* d2 = reinterpret_cast<u64x2*>(dst);
            auto* s2 = reinterpret_cast<const u64x2*>(src);
            if (group == 2) launch_reduce_flat<2, true>(ctx, d2, s2, groups * per, lg);
            else if (group == 3) launch_reduce_flat<3, true>(ctx, d2, s2, groups * per, lg);
            else launch_reduce_flat<4, true>(ctx, d2, s2, groups * per, lg);
            return hipGetLastError();
        }
    }
    StreamTune t = stream_tune(ctx, groups * wr);
    hipLaunchKernelGGL(k_reduce_max, dim3(t.grid), dim3(kBlock), 0, ctx->stream, (u64*)dst,
                       (const u64*)src, groups, group, wr);
    return hipGetLastError();
}

// per replica: sum of counts (mode 3 partial np/nc or plain sums)
template <bool SEG>
__global__ __launch_bounds__(kBlock) void k_gcounter_sums(const u64* c, u64* sums, u64* part,
                                                          uint64_t R, uint64_t W, uint32_t nseg,
                                                          uint64_t sg, uint32_t fin) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nwaves = (uint64_t)gridDim.x * (kBlock / 64);
    for (uint64_t it = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 6; it < R * nseg;
         it += nwaves) {
        uint64_t rep, lo, hi;
        seg_range(it, nseg, W, sg, &rep, &lo, &hi);
        u64 s = 0;
        for (uint64_t w = lo + lane; w < hi; w += 64) s += c[rep * W + w];
        s = wave_sum(s);
        if (lane == 0) {
            const u64 v[1] = {s};
            emit_sums<1>(SEG, sums, part, rep, v, fin);
        }
    }
}

hipError_t launch_gcounter_sums(laspj_ctx* ctx, const laspj_batch* b, uint64_t* sums) {
    const uint64_t W = b->words_per_replica;
    const uint64_t sg = seg_for(b->replicas, W, kSegW);
    uint32_t ns = nseg_of(W, sg);
    int grid = seg_grid(ctx, b->replicas * ns);
    if (ns == 1) {
        hipLaunchKernelGGL(k_gcounter_sums<false>, dim3(grid), dim3(kBlock), 0, ctx->stream,
                           (const u64*)b->dev, (u64*)sums, nullptr, b->replicas, W, ns, sg, 0u);
    } else {
        u64* part = nullptr;
        hipError_t e = partials(ctx, b->replicas, &part);
        if (e != hipSuccess) return e;
        const uint32_t fin = fin_for(b->replicas * ns, ns);
        hipLaunchKernelGGL(k_gcounter_sums<true>, dim3(grid), dim3(kBlock), 0, ctx->stream,
                           (const u64*)b->dev, (u64*)sums, part, b->replicas, W, ns, sg, fin);
        if (!fin) return finalize_sums<1>(ctx, part, sums, b->replicas);
    }
    return hipGetLastError();
}

// threshold_met(riak_dt_gcounter, V, T) (lasp_lattice.erl:87-90): sum per replica
// compared with T in the same launch (the last segment of a replica decides)
template <bool SEG>
__global__ __launch_bounds__(kBlock) void k_gcounter_threshold(const u64* c, uint8_t* out,
                                                               u64* part, uint64_t R,
                                                               uint64_t W, uint32_t nseg,
                                                               uint64_t seg, u64 t, int mode,
                                                               uint32_t fin) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nwaves = (uint64_t)gridDim.x * (kBlock / 64);
    for (uint64_t it = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 6; it < R * nseg;
         it += nwaves) {
        uint64_t rep, lo, hi;
        seg_range(it, nseg, W, seg, &rep, &lo, &hi);
        u64 s = 0;
        for (uint64_t w = lo + lane; w < hi; w += 64) s += c[rep * W + w];
        s = wave_sum(s);
        if (lane == 0) emit(SEG, out, part, rep, 0, s, 0, mode, fin, t);
    }
}

hipError_t launch_gcounter_threshold(laspj_ctx* ctx, const laspj_batch* b, uint64_t t,
                                     bool strict, uint8_t* out) {
    const uint64_t W = b->words_per_replica;
    const uint64_t sg = seg_for(b->replicas, W, kSegW);
    const uint32_t ns = nseg_of(W, sg);
    const int grid = seg_grid(ctx, b->replicas * ns);
    const int mode = strict ? 5 : 4;
    if (ns == 1) {
        hipLaunchKernelGGL(k_gcounter_threshold<false>, dim3(grid), dim3(kBlock), 0, ctx->stream,
                           (const u64*)b->dev, out, nullptr, b->replicas, W, ns, sg, (u64)t, mode,
                           0u);
        return hipGetLastError();
    }
    u64* part = nullptr;
    hipError_t e = partials(ctx, b->replicas, &part);
    if (e != hipSuccess) return e;
    const uint32_t fin = fin_for(b->replicas * ns, ns);
    hipLaunchKernelGGL(k_gcounter_threshold<true>, dim3(grid), dim3(kBlock), 0, ctx->stream,
                       (const u64*)b->dev, out, part, b->replicas, W, ns, sg, (u64)t, mode, fin);
    if (!fin) return finalize(ctx, part, out, b->replicas, mode, (u64)t);
    return hipGetLastError();
}

// lasp_lattice.erl:169-179: for all actors Count(Prev) =< Count(Cur) (absent = 0);
// :273-275 strict: value(Prev) < value(Cur) only (the reference's "massive shortcut")
template <bool STRICT, bool SEG>
__global__ __launch_bounds__(kBlock) void k_gcounter_inflation(const u64* prev, const u64* cur,
                                                               uint8_t* out, u64* part,
                                                               uint64_t R, uint64_t W,
                                                               bool bcast, uint32_t nseg,
                                                               uint64_t seg, uint32_t fin) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nwaves = (uint64_t)gridDim.x * (kBlock / 64);
    for (uint64_t it = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 6; it < R * nseg;
         it += nwaves) {
        uint64_t rep, lo, hi;
        seg_range(it, nseg, W, seg, &rep, &lo, &hi);
        const u64* P = prev + (bcast ? 0 : rep * W);
        const u64* C = cur + rep * W;
        bool viol = false;
        u64 sp = 0, sc = 0;
        for (uint64_t w = lo + lane; w < hi; w += 64) {
            u64 p = P[w], c = C[w];
            viol |= p > c;
            sp += p;
            sc += c;
        }
        u64 flags = __ballot(viol) != 0 ? kViol : 0;
        if constexpr (STRICT) {
            sp = wave_sum(sp);
            sc = wave_sum(sc);
        }
        if (lane == 0) emit(SEG, out, part, rep, flags, sp, sc, STRICT ? 3 : 1, fin);
    }
}

hipError_t launch_gcounter_inflation(laspj_ctx* ctx, const laspj_batch* prev,
                                     const laspj_batch* cur, bool strict, uint8_t* out) {
    uint64_t W = cur->words_per_replica;
    const uint64_t sg = seg_for(cur->replicas, W, kSegW);
    uint32_t ns = nseg_of(W, sg);
    int grid = seg_grid(ctx, cur->replicas * ns);
    bool bc = prev->replicas == 1 && cur->replicas != 1;
    u64* part = nullptr;
    if (ns > 1) {
        hipError_t e = partials(ctx, cur->replicas, &part);
        if (e != hipSuccess) return e;
    }
#define LJ_GC(ST, SG)                                                                          \
    hipLaunchKernelGGL((k_gcounter_inflation<ST, SG>), dim3(grid), dim3(kBlock), 0, ctx->stream, \
                       (const u64*)prev->dev, (const u64*)cur->dev, out, part, cur->replicas,    \
                       W, bc, ns, sg, fin)
    const uint32_t fin = ns > 1 ? fin_for(cur->replicas * ns, ns) : 0u;
    if (ns > 1) {
        if (strict) LJ_GC(true, true); else LJ_GC(false, true);
        if (!fin) return finalize(ctx, part, out, cur->replicas, strict ? 3 : 1);
        return hipGetLastError();
    }
    if (strict) LJ_GC(true, false); else LJ_GC(false, false);
#undef LJ_GC
    return hipGetLastError();
}

__global__ __launch_bounds__(kBlock) void k_gcounter_incr(u64* c, uint64_t W,
                                                          const laspj_incr* incs, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * kBlock)
        atomicAdd(c + incs[i].replica * W + incs[i].actor, (u64)incs[i].amount);
}

hipError_t launch_gcounter_incr(laspj_ctx* ctx, laspj_batch* b, const laspj_incr* incs,
                                uint64_t n) {
    uint64_t g = (n + kBlock - 1) / kBlock;
    if (g > (uint64_t)ctx->cus * 16) g = (uint64_t)ctx->cus * 16;
    hipLaunchKernelGGL(k_gcounter_incr, dim3((unsigned)(g ? g : 1)), dim3(kBlock), 0, ctx->stream,
                       (u64*)b->dev, b->words_per_replica, incs, n);
    return hipGetLastError();
}

// ------------------------------------------------------------------ update ops
// lasp_orset:update/3 (lasp_orset.erl:99-117).  The op list is grouped by replica
// (validated on the host); the thread owning the first op of a replica's run applies
// that run in order, one update/3 call at a time: a call whose remove finds its
// element absent (and not added earlier in the same call) is rolled back as a whole —
// the reference returns {error,{precondition,{not_present,E}}} and keeps the state.

__global__ __launch_bounds__(kBlock) void k_apply_ops(u64* state, uint64_t wr, int32_t kind,
                                                      const laspj_op* ops, uint64_t nops,
                                                      int32_t* status) {
    uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= nops) return;
    const uint64_t rep = ops[i].replica;
    if (i > 0 && ops[i - 1].replica == rep) return;
    uint64_t end = i + 1;
    while (end < nops && ops[end].replica == rep) ++end;
    u64* s = state + rep * wr;
    uint64_t c0 = i;
    while (c0 < end) {
        uint64_t c1 = c0 + 1;
        while (c1 < end && !(ops[c1].flags & LASPJ_OP_FLAG_NEW_CALL)) ++c1;
        uint64_t bad = ~0ull;
        int32_t why = LASPJ_OPST_NOT_PRESENT;
        if (kind == LASPJ_KIND_ORSET) {
            for (uint64_t k = c0; k < c1 && bad == ~0ull; ++k) {
                const uint32_t e = ops[k].element;
                if (ops[k].kind == LASPJ_OP_REMOVE) {
                    bool present = s[2ull * e] != 0;
                    for (uint64_t j = c0; j < k && !present; ++j)
                        present = ops[j].kind != LASPJ_OP_REMOVE && ops[j].element == e;
                    if (!present) bad = k;
                } else if (ops[k].kind == LASPJ_OP_INSERT) {
                    const uint8_t t = ops[k].slot;
                    bool exists = (s[2ull * e] >> t) & 1ull;
                    for (uint64_t j = c0; j < k && !exists; ++j)
                        exists = ops[j].kind != LASPJ_OP_REMOVE && ops[j].element == e &&
                                 ops[j].slot == t;
                    if (exists) {
                        bad = k;
                        why = LASPJ_OPST_KEY_EXISTS;
                    }
                }
            }
        }
        if (bad != ~0ull) {
            for (uint64_t k = c0; k < c1; ++k)
                status[k] = k == bad ? why : LASPJ_OPST_ROLLED_BACK;
        } else {
            for (uint64_t k = c0; k < c1; ++k) {
                const laspj_op& o = ops[k];
                if (kind == LASPJ_KIND_ORSET) {
                    u64* cell = s + 2ull * o.element;
                    if (o.kind != LASPJ_OP_REMOVE) {
                        // orddict:store(Token, false, Tokens) — present, flag false
                        cell[0] |= 1ull << o.slot;
                        cell[1] &= ~(1ull << o.slot);
                    } else {
                        cell[1] = cell[0];  // every token of Elem := true
                    }
                } else {
                    s[o.element >> 6] |= 1ull << (o.element & 63u);
                }
                status[k] = LASPJ_OPST_APPLIED;
            }
        }
        c0 = c1;
    }
}

hipError_t launch_apply_ops(laspj_ctx* ctx, laspj_batch* b, const laspj_op* ops, uint64_t nops,
                            int32_t* status) {
    uint64_t grid = (nops + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(k_apply_ops, dim3((unsigned)grid), dim3(kBlock), 0, ctx->stream,
                       (u64*)b->dev, b->words_per_replica, b->kind, ops, nops, status);
    return hipGetLastError();
}

// ------------------------------------------------------------------ combinators

// union (lasp_core.erl:616-618): keep-left select per cell
template <bool NT>
__global__ __launch_bounds__(kBlock) void k_orset_union(u64x2* d, const u64x2* l,
                                                        const u64x2* r, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        u64x2 x = ld2<NT>(l + i), y = ld2<NT>(r + i);
        st2<NT>(d + i, x.x != 0 ? x : y);
    }
}

hipError_t launch_orset_union(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                              const laspj_batch* r) {
    uint64_t n = l->replicas * l->elements;
    StreamTune t = stream_tune(ctx, n);
    hipLaunchKernelGGL(k_orset_union<true>, dim3(t.grid), dim3(kBlock), 0, ctx->stream,
                       reinterpret_cast<u64x2*>(dst->dev), reinterpret_cast<const u64x2*>(l->dev),
                       reinterpret_cast<const u64x2*>(r->dev), n);
    return hipGetLastError();
}

// filter (lasp_core.erl:681-712): keep cell iff the element's predicate bit is set
// one block per (replica, 4096-cell segment); lanes stride the segment by 256 cells
__global__ __launch_bounds__(kBlock) void k_orset_filter(u64x2* d, const u64x2* s,
                                                         const u64* keep, uint64_t R,
                                                         uint32_t E, uint32_t nseg) {
    for (uint64_t it = blockIdx.x; it < R * nseg; it += gridDim.x) {
        uint64_t rep = it / nseg;
        uint32_t e0 = (uint32_t)(it - rep * nseg) * kVSeg;
        uint32_t e1 = min(E, e0 + kVSeg);
        const u64x2* src = s + rep * E;
        u64x2* dst = d + rep * E;
#pragma unroll 4
        for (uint32_t e = e0 + threadIdx.x; e < e1; e += kBlock) {
            bool k = (keep[e >> 6] >> (e & 63u)) & 1ull;
            u64x2 v = ld2<true>(src + e);
            u64x2 z = {0, 0};
            st2<true>(dst + e, k ? v : z);
        }
    }
}

static int seg_blocks(const laspj_ctx* ctx, uint64_t items) {
    uint64_t cap = (uint64_t)ctx->cus * 32;
    return (int)(items < cap ? (items ? items : 1) : cap);
}

hipError_t launch_orset_filter(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                               const uint64_t* keep) {
    uint32_t ns = (src->elements + kVSeg - 1) / kVSeg;
    hipLaunchKernelGGL(k_orset_filter, dim3(seg_blocks(ctx, src->replicas * ns)), dim3(kBlock), 0,
                       ctx->stream, reinterpret_cast<u64x2*>(dst->dev),
                       reinterpret_cast<const u64x2*>(src->dev), (const u64*)keep, src->replicas,
                       src->elements, ns);
    return hipGetLastError();
}

}  // namespace laspj
