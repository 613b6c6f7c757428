// List-faithful values on the device (include/laspj.h "list values").
//
// lasp_core's combinator bodies bind lists that are not orddicts (intersection
// `Cx ++ Cy`, reversed product token pairs, reordered / repeated map and fold keys, the
// G-Set `L ++ R`), and every re-run merges its new output into the old one with
// orddict:merge / ordsets:union run as written — a two-finger merge over unsorted
// lists.  A LIST batch keeps such a value exactly; the kernels below restate the list
// operations of the path over it.
//
// Execution shape: one wave64 workgroup per replica (the bind path holds one replica
// per variable; batched callers get one wave per replica).  Work that is a sequential
// chain in the reference — the two-finger walk of orddict:merge / ordsets:union over
// keys that need not ascend — runs on lane 0 over key ranks precomputed lane-parallel
// into scratch (L1-resident, read in order); everything else (token merges per merged
// entry, prefix sums for output positions, keyfind through a per-replica hash table,
// ballots for the predicates) is lane-parallel.  Output positions come from wave
// prefix sums, so each kernel runs twice: a size pass (WRITE = false) whose per-replica
// {entries, tokens} the runtime reads back to size dst, then the write pass.
//
// Term order comes from host-built rank tables (krank per element slot, grank per token
// slot), so a comparison is one integer compare and `==` is rank equality.

#include <cstring>
#include <new>
#include <type_traits>
#include <vector>

#include "laspj_internal.h"

namespace laspj {

namespace {

typedef unsigned long long u64;

constexpr u64 kPair = 1ull << 62;
constexpr u64 kCompound = 1ull << 62;
constexpr u64 kRemoved = 1ull << 63;
constexpr u64 kIdMask = 0x7FFFFFFFull;
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr u64 kEmpty = ~0ull;

// flag bits (ctx->flag[1])
constexpr uint32_t kErrRange = 1;    // an output ran past dst's capacity
constexpr uint32_t kErrId = 2;       // an item's slot is outside the rank tables
constexpr uint32_t kErrNested = 4;   // product of product outputs (nested pairs)
constexpr uint32_t kErrTable = 8;    // a map / filter / fold table index out of range
constexpr uint32_t kErrFun = 16;     // the fun failed on a key present in the list
constexpr uint32_t kInfoWalkFell = 256;  // (not an error) the chunked walk gave up

struct LV {
    uint32_t* hdr;     // [R][2] {entries, tokens}
    u64* key;          // [R][ce]
    u64* tok;          // [R][ct]
    uint32_t* toff;    // [R][ce + 1]
    uint32_t ce, ct;
    __device__ uint32_t n(u64 r) const { return hdr[2 * r]; }
    __device__ uint32_t nt(u64 r) const { return hdr[2 * r + 1]; }
    __device__ u64* K(u64 r) const { return key + r * ce; }
    __device__ u64* T(u64 r) const { return tok + r * (u64)ct; }
    __device__ uint32_t* O(u64 r) const { return toff + r * ((u64)ce + 1); }
};

struct RK {
    const uint32_t* krank;
    const uint32_t* grank;
    uint32_t nk, ng;
    uint32_t* flag;
};

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// exclusive prefix sum over the wave; *total = the wave's sum
__device__ __forceinline__ uint32_t wave_excl(uint32_t v, uint32_t* total) {
    uint32_t x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t y = __shfl_up(x, off, 64);
        if ((int)lane_id() >= off) x += y;
    }
    *total = __shfl(x, 63, 64);
    return x - v;
}

__device__ __forceinline__ void lraise(uint32_t* flag, uint32_t bit) { atomicOr(flag, bit); }

// term order of a key item: slots by krank, {X, Y} pairs element-wise after them
__device__ __forceinline__ u64 key_ord(u64 it, const RK& rk) {
    if (it & kPair) {
        const uint32_t x = (uint32_t)((it >> 31) & kIdMask), y = (uint32_t)(it & kIdMask);
        if (x >= rk.nk || y >= rk.nk) {
            lraise(rk.flag, kErrId);
            return 0;
        }
        return (1ull << 63) | ((u64)rk.krank[x] << 31) | rk.krank[y];
    }
    const uint32_t e = (uint32_t)(it & kIdMask);
    if (e >= rk.nk) {
        lraise(rk.flag, kErrId);
        return 0;
    }
    return rk.krank[e];
}

// term order of a token item (flag ignored): [Tx, Ty] element-wise, below binaries
__device__ __forceinline__ u64 tok_ord(u64 it, const RK& rk) {
    if (it & kCompound) {
        const uint32_t x = (uint32_t)((it >> 31) & kIdMask), y = (uint32_t)(it & kIdMask);
        if (x >= rk.ng || y >= rk.ng) {
            lraise(rk.flag, kErrId);
            return 0;
        }
        return ((u64)rk.grank[x] << 31) | rk.grank[y];
    }
    const uint32_t g = (uint32_t)(it & kIdMask);
    if (g >= rk.ng) {
        lraise(rk.flag, kErrId);
        return 0;
    }
    return (1ull << 62) | rk.grank[g];
}

// ---------------------------------------------------------------- per-replica hash
// keyfind / member through an open-addressing table of key ranks -> first index
// (size a power of two >= 2 x entries, so probes always end)

__device__ __forceinline__ uint32_t hmix(u64 k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    return (uint32_t)k;
}

// Slots hold ~key and ~first index, so a zeroed table is empty (one memset with the
// kernels' other zeroed words): no real key is ~0, no index is 0xFFFFFFFF, and the first
// index is the largest ~index (atomicMax).
__device__ __forceinline__ void h_insert(u64* hk, uint32_t* hi, uint32_t mask, u64 key,
                                         uint32_t idx) {
    uint32_t h = hmix(key) & mask;
    const u64 nk = ~key;
    for (;;) {
        const u64 prev = atomicCAS(hk + h, 0ull, nk);
        if (prev == 0ull || prev == nk) {
            atomicMax(hi + h, ~idx);
            return;
        }
        h = (h + 1) & mask;
    }
}

__device__ __forceinline__ uint32_t h_find(const u64* hk, const uint32_t* hi, uint32_t mask,
                                           u64 key) {
    uint32_t h = hmix(key) & mask;
    const u64 nk = ~key;
    for (;;) {
        const u64 k = __hip_atomic_load(const_cast<u64*>(hk + h), __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
        if (k == nk)
            return ~__hip_atomic_load(const_cast<uint32_t*>(hi + h), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
        if (k == 0ull) return kNone;
        h = (h + 1) & mask;
    }
}

// orddict:merge over two token runs (inner clause of lasp_orset:merge/2): count or write
template <bool W>
__device__ uint32_t inner_merge(const u64* ta, uint32_t la, const u64* tb, uint32_t lb,
                                u64* to, const RK& rk) {
    uint32_t x = 0, y = 0, n = 0;
    while (x < la && y < lb) {
        const u64 A = ta[x], B = tb[y];
        const u64 oa = tok_ord(A, rk), ob = tok_ord(B, rk);
        if (oa < ob) {
            if (W) to[n] = A;
            ++x;
        } else if (oa > ob) {
            if (W) to[n] = B;
            ++y;
        } else {                       // {Token, BoolA or BoolB}, key of the first
            if (W) to[n] = A | (B & kRemoved);
            ++x, ++y;
        }
        ++n;
    }
    for (; x < la; ++x, ++n)
        if (W) to[n] = ta[x];
    for (; y < lb; ++y, ++n)
        if (W) to[n] = tb[y];
    return n;
}

// ================================================================ kernels

// ---------------------------------------------------------------- merges
// lasp_orset:merge/2 (MODE 0), the OR-Set union body = orddict:merge keeping the left
// value (MODE 1), lasp_gset:merge/2 = OTP 17 ordsets:union (MODE 2).
//
// The reference runs a two-finger walk.  Its outer chain is sequential only when keys do
// not ascend: on lists whose key ranks are non-decreasing (every canonical value, an
// intersection output, a filter or monotone map of one) the walk passes through the
// point (i(v), j(v)) = (first index of A with key >= v, same in B) for EVERY key v — all
// keys below v are consumed before any key >= v.  So the walk splits at such points into
// independent pieces: merge-path diagonals (A first on ties) moved back to the first
// element equal to the smallest unconsumed key.  A block owns a tile of kMTile diagonal
// steps (its window staged in LDS), each thread a sub-piece of it; counts go through
// block scans and a per-replica scan of tile totals.  Within a key, the walk pairs the
// k-th copy of A with the k-th copy of B and emits the longer side's surplus alone, as
// the clauses do.  ordsets:union's argument switch only decides which side's item a
// pair emits: after a single-side step the walk's first argument is that side (a
// smaller head of the second argument makes it switch; a smaller head of the first
// keeps it), so the item of a pair is the side of the last single step before it (A
// at the start) — carried across threads and tiles by "last non-none" scans.
// Replicas whose ranks descend anywhere take a one-wave walk (merge_runs_replica, run by k_merge_tile_scan).
// Token runs of the planned entries (inner orddict:merge with `or`, or a copy) are then
// counted, scanned and written one entry per thread over the whole grid.

constexpr uint32_t kMT = 256;           // threads per block of the merge kernels
constexpr uint32_t kMTile = 2048;       // diagonal steps per tile
constexpr uint32_t kMWin = 4096;        // LDS window (u64) for a tile's A and B keys

struct MS {
    u64* sa;           // [R][ce_a] key ranks of A
    u64* sb;           // [R][ce_b]
    u64* plan;         // [R][ce_a + ce_b] output entries: ia | jb << 32 (MODE 0/1),
                       //                 idx | side << 32 (MODE 2)
    uint32_t* tcnt;    // [R][ce_a + ce_b] tokens per output entry
    uint32_t* tile;    // [R][ntiles] entries per tile -> exclusive offsets
    uint32_t* tside;   // [R][ntiles] MODE 2: last single side in the tile -> side at its start
    uint32_t* tsplit;  // [R][ntiles][4] the tile's merge-path start and end (i, j), found by
                       // the counting pass, read by the writing pass
    uint32_t* chunk;   // [R][nchunks] tokens per chunk of kMT entries -> exclusive offsets
    uint32_t* nout;    // [R] output entries
    uint32_t* ntok;    // [R] output tokens
    uint32_t* unsorted;// [R] 1: a side's ranks descend somewhere (lane-0 walk)
    uint32_t* aweak;   // [R] 1: a's keys are not strictly ascending (a tie or a descent)
    uint32_t ce_a, ce_b, ntiles, nchunks;
    uint32_t spec = 0; // 1: k_merge_spec walks the replicas whose ranks descend
    // [R][nba] / [R][nbb] the largest rank of each 256-entry block of A / B (k_merge_ranks
    // stores every one: no clearing), or null: a walk's long run of one side skips the
    // 1024-entry chunks (nca / ncb, four blocks each) that cannot end it
    u64* amax = nullptr;
    u64* bmax = nullptr;
    uint32_t nca = 0, ncb = 0, nba = 0, nbb = 0;
};

// exclusive prefix sum / running max over a block of kMT threads (s_w: kMT/64 words)
__device__ __forceinline__ uint32_t block_excl(uint32_t v, uint32_t* total, uint32_t* s_w) {
    uint32_t wt;
    const uint32_t x = wave_excl(v, &wt), w = threadIdx.x >> 6;
    __syncthreads();
    if (lane_id() == 0) s_w[w] = wt;
    __syncthreads();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (uint32_t k = 0; k < kMT / 64; ++k) {
        base += k < w ? s_w[k] : 0u;
        tot += s_w[k];
    }
    *total = tot;
    return base + x;
}

__device__ __forceinline__ uint32_t wave_excl_max(uint32_t v, uint32_t* all) {
    uint32_t x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if ((int)lane_id() >= off) x = x > y ? x : y;
    }
    *all = __shfl(x, 63, 64);
    const uint32_t e = __shfl_up(x, 1, 64);
    return lane_id() ? e : 0u;
}

__device__ __forceinline__ uint32_t block_excl_max(uint32_t v, uint32_t* all, uint32_t* s_w) {
    uint32_t wa;
    const uint32_t x = wave_excl_max(v, &wa), w = threadIdx.x >> 6;
    __syncthreads();
    if (lane_id() == 0) s_w[w] = wa;
    __syncthreads();
    uint32_t base = 0, mx = 0;
#pragma unroll
    for (uint32_t k = 0; k < kMT / 64; ++k) {
        if (k < w) base = base > s_w[k] ? base : s_w[k];
        mx = mx > s_w[k] ? mx : s_w[k];
    }
    *all = mx;
    return base > x ? base : x;
}

// first index in X[lo, hi) whose key is >= v (hi when none)
__device__ __forceinline__ uint32_t lower_bound(const u64* X, uint32_t lo, uint32_t hi, u64 v) {
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (X[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// the merge-path point on diagonal d of non-decreasing X[0, nx), Y[0, ny) (A first on
// ties), moved back to (i(v), j(v)) for the smallest unconsumed key v: a point the
// two-finger walk passes through
__device__ void mp_split(const u64* X, uint32_t nx, const u64* Y, uint32_t ny, uint32_t d,
                         uint32_t* pi, uint32_t* pj) {
    uint32_t lo = d > ny ? d - ny : 0, hi = d < nx ? d : nx;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (X[mid] <= Y[d - 1 - mid]) lo = mid + 1;
        else hi = mid;
    }
    const uint32_t i = lo, j = d - lo;
    if (i >= nx && j >= ny) {
        *pi = nx;
        *pj = ny;
        return;
    }
    const u64 v = i >= nx ? Y[j] : (j >= ny ? X[i] : (X[i] < Y[j] ? X[i] : Y[j]));
    *pi = lower_bound(X, 0, i, v);
    *pj = lower_bound(Y, 0, j, v);
}

// The first k in [lo, hi) with pred(k) true (hi when none) for a predicate that is false
// then true, with every thread of the block probing: 256 candidates per step, so a range
// of 10^5 takes three steps of one load each instead of ~17 dependent loads on one
// thread.  Block-uniform arguments; s: one word of LDS.
template <class P>
__device__ uint32_t block_first_true(uint32_t lo, uint32_t hi, P pred, uint32_t* s) {
    while (hi > lo) {
        const uint32_t step = (hi - lo + kMT - 1) / kMT;           // >= 1
        const uint32_t c = lo + threadIdx.x * step;
        const bool f = c < hi && pred(c);
        if (threadIdx.x == 0) s[0] = kMT;
        __syncthreads();
        const u64 bal = __ballot(f);
        if (bal && lane_id() == 0)
            atomicMin(s, (threadIdx.x & ~63u) + (uint32_t)__ffsll((long long)bal) - 1u);
        __syncthreads();
        const uint32_t t = s[0];
        __syncthreads();                                            // s read before reuse
        if (t == kMT) {
            // every probe below hi is false: the answer is past the last of them
            lo = lo + ((hi - 1 - lo) / step) * step + 1;
        } else {
            hi = lo + t * step;                                     // pred(hi) holds
            if (t) lo = lo + (t - 1) * step + 1;                    // pred(probe t-1) fails
        }
    }
    return lo;
}

// mp_split with the whole block searching (block-uniform arguments, every thread gets the
// result)
__device__ void mp_split_block(const u64* X, uint32_t nx, const u64* Y, uint32_t ny, uint32_t d,
                               uint32_t* pi, uint32_t* pj, uint32_t* s) {
    const uint32_t lo = d > ny ? d - ny : 0, hi = d < nx ? d : nx;
    const uint32_t i = block_first_true(lo, hi, [&](uint32_t k) { return X[k] > Y[d - 1 - k]; }, s);
    const uint32_t j = d - i;
    if (i >= nx && j >= ny) {
        *pi = nx;
        *pj = ny;
        return;
    }
    const u64 v = i >= nx ? Y[j] : (j >= ny ? X[i] : (X[i] < Y[j] ? X[i] : Y[j]));
    // moved back over keys equal to v: none there (the usual case: distinct keys) is one
    // load, not a search
    *pi = i == 0 || X[i - 1] < v ? i : block_first_true(0, i, [&](uint32_t k) { return X[k] >= v; }, s);
    *pj = j == 0 || Y[j - 1] < v ? j : block_first_true(0, j, [&](uint32_t k) { return Y[k] >= v; }, s);
}

// key ranks of both sides, and whether either descends
__global__ __launch_bounds__(kMT) void k_merge_ranks(LV a, LV b, RK rk, MS m, uint64_t R) {
    for (u64 r = blockIdx.y; r < R; r += gridDim.y) {
        const uint32_t na = a.n(r), nb = b.n(r);
        const uint32_t i = blockIdx.x * kMT + threadIdx.x;
        bool desc = false, weak = false;
        if (i < na) {
            const u64 x = key_ord(a.K(r)[i], rk);
            m.sa[r * m.ce_a + i] = x;
            const u64 px = i > 0 ? key_ord(a.K(r)[i - 1], rk) : 0;
            desc |= i > 0 && px > x;
            weak = i > 0 && px >= x;
        }
        if (i < nb) {
            const u64 y = key_ord(b.K(r)[i], rk);
            m.sb[r * m.ce_b + i] = y;
            desc |= i > 0 && key_ord(b.K(r)[i - 1], rk) > y;
        }
        if (__syncthreads_or(desc) && threadIdx.x == 0) atomicOr(m.unsorted + r, 1u);
        if (__syncthreads_or(weak) && threadIdx.x == 0) atomicOr(m.aweak + r, 1u);
        if (m.amax) {
            // this block's 256 ranks of each side -> their maximum (0 past a side's end)
            __shared__ u64 s_mx[2][kMT / 64];
            u64 xa = i < na ? m.sa[r * m.ce_a + i] : 0ull, xb = i < nb ? m.sb[r * m.ce_b + i] : 0ull;
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                const u64 ya = __shfl_xor(xa, off, 64), yb = __shfl_xor(xb, off, 64);
                xa = ya > xa ? ya : xa;
                xb = yb > xb ? yb : xb;
            }
            if (lane_id() == 0) {
                s_mx[0][threadIdx.x >> 6] = xa;
                s_mx[1][threadIdx.x >> 6] = xb;
            }
            __syncthreads();
            if (threadIdx.x < 2) {
                u64 v = 0;
#pragma unroll
                for (uint32_t k = 0; k < kMT / 64; ++k) v = s_mx[threadIdx.x][k] > v ? s_mx[threadIdx.x][k] : v;
                if (threadIdx.x == 0 && blockIdx.x < m.nba) m.amax[r * m.nba + blockIdx.x] = v;
                if (threadIdx.x == 1 && blockIdx.x < m.nbb) m.bmax[r * m.nbb + blockIdx.x] = v;
            }
            __syncthreads();
        }
    }
}

template <int MODE>
__device__ void merge_runs_replica(const LV& a, const LV& b, const MS& m, u64 r);

// one replica's tile counts -> exclusive offsets, its output entry count, and (MODE 2) the
// pair side at every tile's start (the last single side before it, A at the start); WALK:
// a replica whose ranks descend takes the run-jumping walk on the block's first wave
// instead.  Tile words are read with relaxed atomic loads: in the fused form (the
// counting pass's last block) other blocks of the same launch wrote them.
template <int MODE, bool WALK>
__device__ void tile_scan_replica(const LV& a, const LV& b, const MS& m, u64 r, uint32_t* s_w,
                                  uint32_t* s_sd) {
    if (m.unsorted[r]) {
        if (WALK && !m.spec && threadIdx.x < 64) merge_runs_replica<MODE>(a, b, m, r);
        return;
    }
    const uint32_t n = a.n(r) + b.n(r), nt = (n + kMTile - 1) / kMTile;
    uint32_t* tile = m.tile + r * m.ntiles;
    uint32_t* tside = m.tside + r * m.ntiles;
    uint32_t carry = 0, side = 1;
    for (uint32_t c0 = 0; c0 < nt; c0 += kMT) {
        const uint32_t k = c0 + threadIdx.x;
        const uint32_t v = k < nt ? __atomic_load_n(tile + k, __ATOMIC_RELAXED) : 0u;
        uint32_t tot;
        const uint32_t off = carry + block_excl(v, &tot, s_w);
        uint32_t mx = 0, pv = 0;
        if (MODE == 2) {
            const uint32_t sd = k < nt ? __atomic_load_n(tside + k, __ATOMIC_RELAXED) : 0u;
            s_sd[threadIdx.x] = sd;                          // the tiles' own last sides
            pv = block_excl_max(sd ? threadIdx.x + 1 : 0u, &mx, s_w);
        }
        if (k < nt) {
            tile[k] = off;
            if (MODE == 2) tside[k] = pv ? s_sd[pv - 1] : side;
        }
        if (MODE == 2 && mx) side = s_sd[mx - 1];
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) m.nout[r] = carry;
}

// the last block of a launch to finish (agent-scope ticket, zero on entry and left zero)
__device__ __forceinline__ bool last_block(uint32_t* ticket, uint32_t* s_flag) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        *s_flag = atomicAdd(ticket, 1u) == gridDim.x * gridDim.y - 1u;
    }
    __syncthreads();
    const bool last = *s_flag != 0;
    if (last) {
        __threadfence();
        if (threadIdx.x == 0) *ticket = 0;
    }
    return last;
}

// one tile of the merge path per block: WRITE = false counts the tile's entries (and,
// MODE 2, its last single side); WRITE = true writes its plan entries
// ticket (the counting pass of a merge of few replicas): the last block to finish also
// runs the tile scan (and the walk of replicas whose ranks descend) — k_merge_tile_scan's
// work, one launch fewer
template <int MODE, bool WRITE>
__global__ __launch_bounds__(kMT) void k_merge_tiles(LV a, LV b, MS m, uint64_t R,
                                                     uint32_t* ticket) {
    __shared__ u64 s_win[kMWin];
    __shared__ uint32_t s_si[kMT + 1], s_sj[kMT + 1], s_last[kMT], s_w[kMT / 64], s_s[1];
    __shared__ uint32_t s_sd[kMT];
    for (u64 r = blockIdx.y; r < R; r += gridDim.y) {
        const uint32_t na = a.n(r), nb = b.n(r), n = na + nb;
        const uint32_t d0 = blockIdx.x * kMTile;
        if (m.unsorted[r] || d0 >= n) continue;              // uniform over the block
        const u64* X = m.sa + r * m.ce_a;
        const u64* Y = m.sb + r * m.ce_b;
        uint32_t* sp = m.tsplit + 4ull * (r * m.ntiles + blockIdx.x);
        uint32_t i0, j0, i1, j1;
        if (!WRITE) {
            // the tile's start and end on the merge path, the whole block searching; kept
            // for the writing pass
            mp_split_block(X, na, Y, nb, d0, &i0, &j0, s_s);
            mp_split_block(X, na, Y, nb, d0 + kMTile < n ? d0 + kMTile : n, &i1, &j1, s_s);
            if (threadIdx.x == 0) {
                sp[0] = i0;
                sp[1] = j0;
                sp[2] = i1;
                sp[3] = j1;
            }
        } else {
            i0 = sp[0];
            j0 = sp[1];
            i1 = sp[2];
            j1 = sp[3];
        }
        const uint32_t wa = i1 - i0, wb = j1 - j0, w = wa + wb;
        const u64* WX = X + i0;
        const u64* WY = Y + j0;
        if (w <= kMWin) {                                    // stage the window in LDS
            for (uint32_t k = threadIdx.x; k < wa; k += kMT) s_win[k] = WX[k];
            for (uint32_t k = threadIdx.x; k < wb; k += kMT) s_win[wa + k] = WY[k];
            WX = s_win;
            WY = s_win + wa;
        }
        __syncthreads();
        {
            uint32_t si, sj;
            mp_split(WX, wa, WY, wb, (uint32_t)((u64)threadIdx.x * w / kMT), &si, &sj);
            s_si[threadIdx.x] = si;
            s_sj[threadIdx.x] = sj;
            if (threadIdx.x == 0) {
                s_si[kMT] = wa;
                s_sj[kMT] = wb;
            }
        }
        __syncthreads();
        const uint32_t ei = s_si[threadIdx.x + 1], ej = s_sj[threadIdx.x + 1];
        // pass 1: count and the last single-event side (1 = A, 2 = B)
        uint32_t i = s_si[threadIdx.x], j = s_sj[threadIdx.x], c = 0, last = 0;
        while (i < ei || j < ej) {
            if (i < ei && j < ej) {
                const u64 x = WX[i], y = WY[j];
                if (x < y) ++i, last = 1;
                else if (x > y) ++j, last = 2;
                else ++i, ++j;
            } else if (i < ei) {
                ++i, last = 1;
            } else {
                ++j, last = 2;
            }
            ++c;
        }
        uint32_t total;
        const uint32_t base = block_excl(c, &total, s_w);
        uint32_t* tile = m.tile + r * m.ntiles + blockIdx.x;
        uint32_t* tside = m.tside + r * m.ntiles + blockIdx.x;
        if (MODE == 2) s_last[threadIdx.x] = last;
        uint32_t lastidx;
        const uint32_t prev = MODE == 2 ? block_excl_max(last ? threadIdx.x + 1 : 0u, &lastidx, s_w)
                                        : 0u;
        if (!WRITE) {
            if (threadIdx.x == 0) {
                *tile = total;
                if (MODE == 2) *tside = lastidx ? s_last[lastidx - 1] : 0u;
            }
            __syncthreads();
            continue;
        }
        // pass 2: the plan entries, at the tile's offset
        u64* plan = m.plan + r * ((u64)m.ce_a + m.ce_b) + *tile + base;
        uint32_t side = MODE == 2 ? (prev ? s_last[prev - 1] : *tside) : 0u;
        i = s_si[threadIdx.x], j = s_sj[threadIdx.x];
        for (uint32_t k = 0; k < c; ++k) {
            u64 e;
            if (i < ei && j < ej && WX[i] == WY[j]) {
                if (MODE == 2) e = side == 2 ? (u64)(j0 + j) | (1ull << 32) : (u64)(i0 + i);
                else e = (u64)(i0 + i) | ((u64)(j0 + j) << 32);
                ++i, ++j;
            } else if (i < ei && (j >= ej || WX[i] < WY[j])) {
                e = MODE == 2 ? (u64)(i0 + i) : (u64)(i0 + i) | ((u64)kNone << 32);
                ++i, side = 1;
            } else {
                e = MODE == 2 ? (u64)(j0 + j) | (1ull << 32) : (u64)kNone | ((u64)(j0 + j) << 32);
                ++j, side = 2;
            }
            plan[k] = e;
        }
        __syncthreads();
    }
    if (!WRITE && ticket && last_block(ticket, s_s))
        for (u64 r = 0; r < R; ++r) tile_scan_replica<MODE, true>(a, b, m, r, s_w, s_sd);
}

// per replica: exclusive offsets of the tile counts, the output entry count, and (MODE 2)
// the pair side at every tile's start (the last single side before it, A at the start)
// WALK: a replica whose ranks descend takes the run-jumping walk on the block's first
// wave instead (merge_runs_replica: the walk in this launch)
template <int MODE, bool WALK>
__global__ __launch_bounds__(kMT) void k_merge_tile_scan(LV a, LV b, MS m, uint64_t R) {
    __shared__ uint32_t s_w[kMT / 64], s_sd[kMT];
    for (u64 r = blockIdx.x; r < R; r += gridDim.x)
        tile_scan_replica<MODE, WALK>(a, b, m, r, s_w, s_sd);
}

// replicas whose keys do not ascend: the clauses' walk on lane 0 (over precomputed ranks)
// The clauses' walk for replicas whose ranks descend somewhere (no merge-path split).
// One wave walks a replica: the next 64 ranks of each side sit one per lane in
// registers and are read at the cursor with v_readlane (no memory round trip per step),
// and plan entries are gathered one per lane and leave 64 at a time — the walk is the
// same sequence of decisions, each step now ~a dozen instructions instead of two
// dependent L2 loads.
__device__ __forceinline__ u64 rd64(u64 v, uint32_t l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)l);
    return ((u64)hi << 32) | lo;
}
__device__ __forceinline__ u64 wr64(u64 old, u64 v, uint32_t l) {
    return lane_id() == l ? v : old;
}

struct Win64 {
    const u64* src;
    uint32_t n, base;   // lanes hold src[base + lane] (base: a multiple of 64)
    u64 v;
    __device__ void load(uint32_t at) {
        base = at & ~63u;
        const uint32_t k = base + lane_id();
        v = k < n ? src[k] : 0;
    }
    __device__ u64 get(uint32_t at) {
        if (at - base >= 64u) load(at);
        return rd64(v, at - base);
    }
};

struct PlanOut {
    u64* plan;
    uint32_t o = 0;
    u64 buf = 0;
    __device__ void put(u64 e) {
        buf = wr64(buf, e, o & 63u);
        if ((++o & 63u) == 0) plan[o - 64 + lane_id()] = buf;
    }
    __device__ void flush() {
        const uint32_t k = o & 63u;
        if (lane_id() < k) plan[o - k + lane_id()] = buf;
    }
};

template <int MODE>
__global__ __launch_bounds__(64) void k_merge_serial(LV a, LV b, MS m, uint64_t R) {
    for (u64 r = blockIdx.x; r < R; r += gridDim.x) {
        if (!m.unsorted[r]) continue;
        const uint32_t na = a.n(r), nb = b.n(r);
        Win64 A{m.sa + r * m.ce_a, na, 0, 0}, B{m.sb + r * m.ce_b, nb, 0, 0};
        A.load(0);
        B.load(0);
        PlanOut P{m.plan + r * ((u64)m.ce_a + m.ce_b)};
        uint32_t i = 0, j = 0;
        if (MODE != 2) {
            // merge(F,[{K1,_}=E1|D1],[{K2,_}=E2|D2]) when K1 < K2 -> [E1|merge(F,D1,[E2|D2])];
            //   ... when K1 > K2 -> [E2|merge(F,[E1|D1],D2)];  equal -> F on both;
            // merge(F,[],D2) -> D2;  merge(F,D1,[]) -> D1.
            while (i < na && j < nb) {
                const u64 x = A.get(i), y = B.get(j);
                if (x < y) P.put((u64)i++ | ((u64)kNone << 32));
                else if (x > y) P.put((u64)kNone | ((u64)j++ << 32));
                else P.put((u64)i++ | ((u64)j++ << 32));
            }
            P.flush();
            // the tails, lane-parallel
            for (uint32_t k = lane_id(); k < na - i; k += 64)
                P.plan[P.o + k] = (u64)(i + k) | ((u64)kNone << 32);
            P.o += na - i;
            for (uint32_t k = lane_id(); k < nb - j; k += 64)
                P.plan[P.o + k] = (u64)kNone | ((u64)(j + k) << 32);
            P.o += nb - j;
        } else {
            // union([E1|Es1],[E2|_]=S2) when E1 < E2 -> [E1|union(Es1,S2)];
            // union([E1|_]=S1,[E2|Es2]) when E1 > E2 -> [E2|union(Es2,S1)];  (switch)
            // union([E1|Es1],[_|Es2]) -> [E1|union(Es1,Es2)];  tails as they are.
            // i / j index A / B; sx says which of them is the walk's first argument X.
            uint32_t sx = 0;
            while (i < na && j < nb) {
                const u64 va = A.get(i), vb = B.get(j);
                const u64 x = sx ? vb : va, y = sx ? va : vb;
                const uint32_t ix = sx ? j : i, iy = sx ? i : j;
                if (x < y) {
                    P.put((u64)ix | ((u64)sx << 32));
                    if (sx) ++j; else ++i;
                } else if (x > y) {
                    P.put((u64)iy | ((u64)(sx ^ 1u) << 32));
                    if (sx) ++i; else ++j;             // Y's head taken, then Y becomes X
                    sx ^= 1u;
                } else {
                    P.put((u64)ix | ((u64)sx << 32));
                    ++i, ++j;
                }
            }
            P.flush();
            // tails: the rest of X, then the rest of Y (one of them is empty)
            const uint32_t nx = sx ? nb - j : na - i, x0 = sx ? j : i;
            for (uint32_t k = lane_id(); k < nx; k += 64)
                P.plan[P.o + k] = (u64)(x0 + k) | ((u64)sx << 32);
            P.o += nx;
            const uint32_t ny = sx ? na - i : nb - j, y0 = sx ? i : j;
            for (uint32_t k = lane_id(); k < ny; k += 64)
                P.plan[P.o + k] = (u64)(y0 + k) | ((u64)(sx ^ 1u) << 32);
            P.o += ny;
        }
        if (lane_id() == 0) m.nout[r] = P.o;
    }
}

// Run-jumping walk (round 4) for replicas whose ranks descend somewhere.  Every clause
// emits the smaller head, or both heads on a tie (ordsets:union's switch only decides
// which side a tie's item comes from: the side of the last single step, see above), and
// step kinds come in runs: A's head while A[i] < B[j] (B's head fixed), B's while
// B[j] < A[i], ties while A[i+k] == B[j+k].  The wave holds each side's next 256 ranks
// in registers (a window based at its cursor, position base + 64 t + lane in v[t]) and
// finds how far the current run extends with four ballots; a run that reaches the
// window's end continues as a streaming scan over the precomputed ranks (1024 per wave
// iteration, coalesced).  The run's plan entries are index ranges, written
// lane-parallel.  So the reversed re-bind (one tie run, then one side's rest) costs
// ~n/1024 iterations where the step walk took n dependent steps, and an interleaving of
// short runs still costs one step per run.
struct Win256 {
    const u64* src;
    uint32_t n, base;
    u64 v[4];
    __device__ void load(uint32_t at) {
        base = at;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const uint32_t k = at + 64u * t + lane_id();
            v[t] = k < n ? src[k] : ~0ull;
        }
    }
    // rank at position p, base <= p < base + 256 (wave-uniform)
    __device__ u64 at(uint32_t p) const {
        const uint32_t q = p - base, t = q >> 6;
        return rd64(t == 0 ? v[0] : t == 1 ? v[1] : t == 2 ? v[2] : v[3], q & 63u);
    }
};

// first failing position at or after window offset s: kind 0 = tie (A.v == B.v, windows
// aligned), 1 = A.v < y, 2 = B.v < y; 256 when none in the window (positions >= n fail)
template <int KIND>
__device__ __forceinline__ uint32_t win_fail(const Win256& A, const Win256& B, uint32_t s, u64 y) {
    const Win256& W = KIND == 2 ? B : A;
#pragma unroll
    for (uint32_t t = 0; t < 4; ++t) {
        const uint32_t q = 64u * t + lane_id();
        bool ok;
        if (KIND == 0) ok = W.base + q < W.n && B.base + q < B.n && A.v[t] == B.v[t];
        else ok = W.base + q < W.n && W.v[t] < y;
        const u64 f = __ballot(q >= s && !ok);
        if (f) return 64u * t + (uint32_t)__ffsll((long long)f) - 1u;
    }
    return 256u;
}

// the run's length from positions p (and q for ties) onwards over global ranks, to the
// first failure or the end of a side
// (software-pipelined: the next 1024 ranks of each side are in flight while the current
// ones are tested, so a long run costs one memory round trip per 1024, not two)
template <int KIND>
__device__ uint32_t stream_run(const u64* X, uint32_t nx, uint32_t p, const u64* Y, uint32_t ny,
                               uint32_t q, u64 y) {
    uint32_t L = 0;
    u64 vx[16], vy[16];
    auto load = [&](uint32_t at, u64 (&ax)[16], u64 (&ay)[16]) {
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const uint32_t k = at + 64u * t + lane_id();
            ax[t] = p + k < nx ? X[p + k] : ~0ull;
            if (KIND == 0) ay[t] = q + k < ny ? Y[q + k] : ~0ull;
        }
    };
    load(0, vx, vy);
    for (;;) {
        u64 nxv[16], nyv[16];
        const bool more = p + L + 1024u < nx && (KIND != 0 || q + L + 1024u < ny);
        if (more) load(L + 1024u, nxv, nyv);
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const uint32_t k = L + 64u * t + lane_id();
            const bool ok = KIND == 0 ? (p + k < nx && q + k < ny && vx[t] == vy[t])
                                      : (p + k < nx && vx[t] < y);
            const u64 f = __ballot(!ok);
            if (f) return L + 64u * t + (uint32_t)__ffsll((long long)f) - 1u;
        }
        L += 1024;
        if (!more) load(L, nxv, nyv);          // (all past the end: the next test fails)
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            vx[t] = nxv[t];
            if (KIND == 0) vy[t] = nyv[t];
        }
    }
}

// the largest rank of 1024-entry chunk c: the maximum of its four blocks' maxima
__device__ __forceinline__ u64 chunk_max(const u64* bm, uint32_t nb, uint32_t c) {
    u64 v = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t q = 4u * c + k;
        const u64 x = q < nb ? bm[q] : 0ull;
        v = x > v ? x : v;
    }
    return v;
}

// stream_run<1> (X[p ..] < y: the length of the run from p) with the chunk maxima of X:
// the rest of p's 1024-entry chunk, then straight to the first later chunk whose maximum
// reaches y (a ballot over 64 chunk maxima at a time), then that chunk — three memory
// round trips for a run of any length instead of one per 1024 entries
__device__ uint32_t stream_run_max(const u64* X, uint32_t nx, uint32_t p, u64 y, const u64* mx,
                                   uint32_t nbk, uint32_t nc, u64 mreg) {
    if (!mx) return stream_run<1>(X, nx, p, nullptr, 0, 0, y);
    auto scan = [&](uint32_t from, uint32_t to) -> uint32_t {    // first q in [from, to): X >= y
        for (uint32_t b0 = from; b0 < to; b0 += 1024u) {
            u64 v[16];
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const uint32_t k = b0 + 64u * t + lane_id();
                v[t] = k < to ? X[k] : ~0ull;
            }
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const u64 f = __ballot(v[t] >= y);
                if (f) return b0 + 64u * t + (uint32_t)__ffsll((long long)f) - 1u;
            }
        }
        return to;
    };
    if (p >= nx) return 0;
    const uint32_t ce = min(nx, ((p >> 10) + 1u) << 10);
    uint32_t q = scan(p, ce);
    if (q < ce) return q - p;
    for (uint32_t c0 = (ce >> 10) & ~63u; c0 < nc; c0 += 64u) {
        // (chunks 0 .. 63: the maxima the walk holds in registers, mreg = chunk lane's)
        const uint32_t c = c0 + lane_id();
        const u64 v = c0 == 0 ? mreg : (c < nc ? chunk_max(mx, nbk, c) : 0ull);
        const u64 f = __ballot(c >= (ce >> 10) && c < nc && v >= y);
        if (f) {
            const uint32_t cf = c0 + (uint32_t)__ffsll((long long)f) - 1u;
            q = scan(cf << 10, min(nx, (cf + 1u) << 10));
            return q - p;
        }
    }
    return nx - p;
}

// one replica's walk by one wave (its lanes); k_merge_tile_scan runs it on its first wave
// for a replica whose ranks descend, so the scan and the walk are one launch
template <int MODE>
__device__ void merge_runs_replica(const LV& a, const LV& b, const MS& m, u64 r) {
    {
        const uint32_t na = a.n(r), nb = b.n(r);
        const u64* SA = m.sa + r * m.ce_a;
        const u64* SB = m.sb + r * m.ce_b;
        Win256 A{SA, na, 0, {}}, B{SB, nb, 0, {}};
        A.load(0);
        B.load(0);
        // the first 64 chunk maxima of each side, one per lane (stream_run_max)
        const u64 mra = m.amax && lane_id() < m.nca ? chunk_max(m.amax + r * m.nba, m.nba, lane_id())
                                                    : 0ull;
        const u64 mrb = m.bmax && lane_id() < m.ncb ? chunk_max(m.bmax + r * m.nbb, m.nbb, lane_id())
                                                    : 0ull;
        u64* plan = m.plan + r * ((u64)m.ce_a + m.ce_b);
        uint32_t i = 0, j = 0, o = 0, sx = 0;        // sx: the last single step was B's
        while (i < na && j < nb) {
            if (i - A.base >= 192u) A.load(i);
            if (j - B.base >= 192u) B.load(j);
            const u64 x = A.at(i), y = B.at(j);
            uint32_t L;
            if (x == y) {
                if (i - A.base != j - B.base) {
                    A.load(i);
                    B.load(j);
                }
                const uint32_t s = i - A.base;
                L = win_fail<0>(A, B, s, 0) - s;
                if (L == 256u - s) L += stream_run<0>(SA, na, i + L, SB, nb, j + L, 0);
                // merge(F, [{K1,V1}|D1], [{_,V2}|D2]) -> [{K1, F(K1,V1,V2)} | ...];
                // union: the item of the walk's first argument
                for (uint32_t k = lane_id(); k < L; k += 64)
                    plan[o + k] = MODE == 2 ? (sx ? (u64)(j + k) | (1ull << 32) : (u64)(i + k))
                                            : (u64)(i + k) | ((u64)(j + k) << 32);
                i += L, j += L;
            } else if (x < y) {
                const uint32_t s = i - A.base;
                L = win_fail<1>(A, B, s, y) - s;
                if (L == 256u - s)
                    L += stream_run_max(SA, na, i + L, y, m.amax ? m.amax + r * m.nba : nullptr, m.nba,
                                        m.nca, mra);
                for (uint32_t k = lane_id(); k < L; k += 64)
                    plan[o + k] = MODE == 2 ? (u64)(i + k) : (u64)(i + k) | ((u64)kNone << 32);
                i += L;
                sx = 0;
            } else {
                const uint32_t s = j - B.base;
                L = win_fail<2>(A, B, s, x) - s;
                if (L == 256u - s)
                    L += stream_run_max(SB, nb, j + L, x, m.bmax ? m.bmax + r * m.nbb : nullptr, m.nbb,
                                        m.ncb, mrb);
                for (uint32_t k = lane_id(); k < L; k += 64)
                    plan[o + k] = MODE == 2 ? (u64)(j + k) | (1ull << 32)
                                            : (u64)kNone | ((u64)(j + k) << 32);
                j += L;
                sx = 1;
            }
            o += L;
        }
        // the rest of the side left over (merge(F,[],D2) -> D2; merge(F,D1,[]) -> D1;
        // the union's tails as they are), tagged with its side
        for (uint32_t k = lane_id(); k < na - i; k += 64)
            plan[o + k] = MODE == 2 ? (u64)(i + k) : (u64)(i + k) | ((u64)kNone << 32);
        o += na - i;
        for (uint32_t k = lane_id(); k < nb - j; k += 64)
            plan[o + k] = MODE == 2 ? (u64)(j + k) | (1ull << 32)
                                    : (u64)kNone | ((u64)(j + k) << 32);
        o += nb - j;
        if (lane_id() == 0) m.nout[r] = o;
    }
}

// ---------------------------------------------------------------- chunked walk
// The clauses' walk for replicas whose keys descend, spread over the chip (k_merge_spec).
// Row i of A is emitted at the first column f >= j(i) with B[f] >= A[i] — B[j(i) .. f)
// go first, alone; B[f] == A[i] pairs with it — and the next row starts at
// j(i+1) = f + [pair].  So the walk is a chain of monotone maps j -> j' over rows, and
// two walks of the same rows from different columns meet and then agree.  A wave takes
// a chunk of L rows and walks it from a guessed column (round 0: proportional), then from
// the previous chunk's exit of the round before, until no chunk's exit changes — that
// round's walks are then one consistent walk from (0, 0), i.e. the clauses' own (chunk 0
// always starts right, so round k has chunks 0 .. k right; reversed lists and lists
// shuffled alike — tie runs — settle in 2).  Each round ends at a barrier over the replica's blocks (one u64 per
// round: arrivals | blocks changed << 32, so every block reads the same decision).  Keys
// shuffled independently on both sides do not meet (measured: 4 chunks of 16k rows took
// 5 rounds, one chunk settling per round), so when most blocks still change after round
// 1, or after kSpRounds rounds, the one-wave walk runs instead.
// Chunk words (double-buffered by round) carry exit | pairs << 32 | last single side <<
// 52 | round tag << 56.  Then every wave writes its chunk's plan entries at
// i0 + entry - (pairs before the chunk), ordsets:union's item of a pair from the side of
// the last single step (carried over chunks).
constexpr uint32_t kSpW = 4;                // chunks (waves) per block
constexpr uint32_t kSpRounds = 16;
constexpr uint32_t kSpWords = kSpRounds + 2;  // per replica: round words, done ticket
struct SP {
    u64* w;            // [R][kSpWords] zero on entry, left zero
    u64* cw;           // [R][2][C] chunk words, zero on entry, left zero
    uint32_t* fr;      // [R][ce_a] per row: f | pair << 31
    uint32_t L, C;     // rows per chunk, chunks per replica (gridDim.x * kSpW)
    uint32_t* flag;    // the call's flag word (kInfoWalkFell)
};

__device__ __forceinline__ u64 sp_load(const u64* p) {
    return __hip_atomic_load(const_cast<u64*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// chunk c's word of round `round` (waits for it)
__device__ __forceinline__ u64 sp_word(const SP& sp, u64 r, uint32_t round, uint32_t c) {
    const u64* p = sp.cw + (r * 2 + (round & 1)) * sp.C + c;
    for (;;) {
        const u64 v = sp_load(p);
        if ((uint32_t)(v >> 56) == round + 1) return v;
        __builtin_amdgcn_s_sleep(1);
    }
}

template <int MODE>
__global__ __launch_bounds__(64 * kSpW) void k_merge_spec(LV a, LV b, MS m, SP sp, uint64_t R) {
    const uint32_t wv = threadIdx.x >> 6, lane = lane_id();
    for (u64 r = blockIdx.y; r < R; r += gridDim.y) {
        if (!m.unsorted[r]) continue;                    // (uniform over the replica's grid)
        const uint32_t na = a.n(r), nb = b.n(r);
        const u64* SA = m.sa + r * m.ce_a;
        const u64* SB = m.sb + r * m.ce_b;
        const uint32_t c = blockIdx.x * kSpW + wv;
        const uint32_t nc = (na + sp.L - 1) / sp.L;      // chunks with rows
        const uint32_t i0 = c < nc ? c * sp.L : na, i1 = c < nc ? min(na, i0 + sp.L) : na;
        u64* w = sp.w + r * kSpWords;
        uint32_t* fr = sp.fr + r * m.ce_a;
        uint32_t round = 0, entry = 0;
        bool fallback = false;
        for (;;) {
            bool changed = false;
            if (c < nc) {
                if (c == 0) entry = 0;
                else if (round == 0) entry = (uint32_t)((u64)i0 * nb / na);
                else entry = (uint32_t)sp_word(sp, r, round - 1, c - 1);
                // the walk of rows [i0, i1) from column `entry`, a run at a time (as
                // merge_runs_replica): rows of an A run take f = j, a tie run f = j + k
                // with the pair bit, a B run moves j
                Win256 A{SA, i1, 0, {}}, B{SB, nb, 0, {}};
                A.load(i0);
                B.load(entry);
                uint32_t i = i0, j = entry, pairs = 0, side = 0;
                while (i < i1) {
                    uint32_t L;
                    if (j >= nb) {                                  // B is done: rows alone
                        L = i1 - i;
                        for (uint32_t k = lane; k < L; k += 64) fr[i + k] = nb;
                        i = i1;
                        side = 1;
                        break;
                    }
                    if (i - A.base >= 192u) A.load(i);
                    if (j - B.base >= 192u) B.load(j);
                    const u64 x = A.at(i), y = B.at(j);
                    if (x == y) {
                        if (i - A.base != j - B.base) {
                            A.load(i);
                            B.load(j);
                        }
                        const uint32_t s0 = i - A.base;
                        L = win_fail<0>(A, B, s0, 0) - s0;
                        if (L == 256u - s0) L += stream_run<0>(SA, i1, i + L, SB, nb, j + L, 0);
                        L = min(L, i1 - i);
                        for (uint32_t k = lane; k < L; k += 64) fr[i + k] = (j + k) | 0x80000000u;
                        pairs += L;
                        i += L;
                        j += L;
                    } else if (x < y) {
                        const uint32_t s0 = i - A.base;
                        L = win_fail<1>(A, B, s0, y) - s0;
                        if (L == 256u - s0) L += stream_run<1>(SA, i1, i + L, nullptr, 0, 0, y);
                        L = min(L, i1 - i);
                        for (uint32_t k = lane; k < L; k += 64) fr[i + k] = j;
                        i += L;
                        side = 1;
                    } else {
                        const uint32_t s0 = j - B.base;
                        L = win_fail<2>(A, B, s0, x) - s0;
                        if (L == 256u - s0) L += stream_run<1>(SB, nb, j + L, nullptr, 0, 0, x);
                        j += L;
                        side = 2;
                    }
                }
                if (round > 0) changed = (uint32_t)sp_word(sp, r, round - 1, c) != j;
                if (lane == 0)
                    __hip_atomic_store(sp.cw + (r * 2 + (round & 1)) * sp.C + c,
                                       (u64)j | ((u64)pairs << 32) | ((u64)side << 52) |
                                           ((u64)(round + 1) << 56),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            // the round's barrier over the replica's blocks, with its decision
            __shared__ uint32_t s_ch;
            if (threadIdx.x == 0) s_ch = 0;
            __syncthreads();
            if (lane == 0 && changed) atomicOr(&s_ch, 1u);
            __syncthreads();
            __shared__ u64 s_word;
            if (threadIdx.x == 0) {
                u64* rw = w + round;
                __hip_atomic_fetch_add(rw, 1ull | ((u64)s_ch << 32), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                u64 v;
                while ((uint32_t)(v = sp_load(rw)) < gridDim.x) __builtin_amdgcn_s_sleep(1);
                s_word = v;
            }
            __syncthreads();
            if (round > 0 && (uint32_t)(s_word >> 32) == 0) break;   // settled
            // walks that do not meet (keys shuffled independently on both sides: the gap
            // between two walks closes only when a row's key tops every B key in it) change
            // most chunks every round: the one-wave walk then, without more rounds
            if (++round == kSpRounds || (round > 1 && 2 * (uint32_t)(s_word >> 32) > gridDim.x)) {
                fallback = true;
                break;
            }
        }
        if (fallback) {
            if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(sp.flag, kInfoWalkFell);
            if (blockIdx.x == 0 && wv == 0) merge_runs_replica<MODE>(a, b, m, r);
        } else if (c < nc || (c == 0 && nc == 0)) {
            // the plan entries of this chunk (the final round's walk, from fr)
            uint32_t before = 0, sidx = 0;                // pairs before; last sided chunk + 1
            for (uint32_t k = lane; k < c; k += 64) {
                const u64 v = sp_word(sp, r, round, k);
                before += (uint32_t)(v >> 32) & 0xFFFFFu;
                if ((v >> 52) & 3u) sidx = k + 1 > sidx ? k + 1 : sidx;
            }
            for (int off = 32; off > 0; off >>= 1) {
                before += __shfl_xor(before, off, 64);
                const uint32_t o2 = __shfl_xor(sidx, off, 64);
                sidx = o2 > sidx ? o2 : sidx;
            }
            uint32_t side = 1;                                  // A at the start
            if (MODE == 2 && sidx) side = (uint32_t)(sp_word(sp, r, round, sidx - 1) >> 52) & 3u;
            u64* plan = m.plan + r * ((u64)m.ce_a + m.ce_b);
            // 64 rows at a time, a row per lane: its entry column (the row before's f +
            // pair), its place i + j - (pairs before), its B run, its own entry; ordsets:
            // union's pair item from the last single side before it (a wave max-scan)
            uint32_t j = entry, pbefore = before;
            for (uint32_t g = i0; g < i1; g += 64) {
                const uint32_t i = g + lane;
                const bool live = i < i1;
                const uint32_t e = live ? fr[i] : 0u;
                const uint32_t f = e & 0x7FFFFFFFu;
                const uint32_t pr = live ? e >> 31 : 0u;
                uint32_t jn = __shfl_up(f + pr, 1, 64);          // the row before's exit
                if (lane == 0) jn = j;
                uint32_t ptot;
                const uint32_t pex = wave_excl(pr, &ptot);
                const uint32_t o = i + jn - (pbefore + pex);     // this row's B run starts here
                const uint32_t run = live ? f - jn : 0u;
                auto bent = [&](uint32_t k) {
                    return MODE == 2 ? (u64)k | (1ull << 32) : (u64)kNone | ((u64)k << 32);
                };
                if (run <= 32)
                    for (uint32_t k = 0; k < run; ++k) plan[o + k] = bent(jn + k);
                for (u64 longs = __ballot(run > 32); longs; longs &= longs - 1) {
                    const int l = __builtin_ctzll(longs);            // a long run: wave-wide
                    const uint32_t lo = __shfl(o, l, 64), lj = __shfl(jn, l, 64),
                                   lr = __shfl(run, l, 64);
                    for (uint32_t k = lane; k < lr; k += 64) plan[lo + k] = bent(lj + k);
                }
                // ordsets:union's item of a pair: the side before this row's own entry —
                // B when its run went first, else the last row before it that set one (A
                // alone, or a B run), else the carried side
                const uint32_t setter = live ? (!pr ? 1u : (run ? 2u : 0u)) : 0u;
                uint32_t allmax;
                const uint32_t prev_idx = wave_excl_max(setter ? lane + 1 : 0u, &allmax);
                const uint32_t prev_side = __shfl(setter, prev_idx ? prev_idx - 1 : 0, 64);
                if (live) {
                    u64 ent;
                    if (MODE == 2) {
                        const uint32_t sd = run ? 2u : (prev_idx ? prev_side : side);
                        ent = pr && sd == 2 ? (u64)f | (1ull << 32) : (u64)i;
                    } else {
                        ent = (u64)i | ((u64)(pr ? f : kNone) << 32);
                    }
                    plan[o + run] = ent;
                }
                // carry: the last live row's exit, pairs, and the side after the group
                const uint32_t last = min(63u, i1 - 1 - g);
                j = __shfl(f + pr, last, 64);
                pbefore += ptot;
                if (MODE == 2 && allmax) side = __shfl(setter, allmax - 1, 64);
            }
            uint32_t o = i1 + j - pbefore;
            if (c + 1 >= nc) {                                   // the last chunk: B's tail
                for (uint32_t k = lane; k < nb - j; k += 64)
                    plan[o + k] = MODE == 2 ? (u64)(j + k) | (1ull << 32)
                                            : (u64)kNone | ((u64)(j + k) << 32);
                if (lane == 0) m.nout[r] = o + (nb - j);
            }
        }
        // the replica's words back to zero (the block that finishes last)
        __syncthreads();
        __shared__ uint32_t s_last;
        if (threadIdx.x == 0)
            s_last = __hip_atomic_fetch_add(w + kSpRounds + 1, 1ull, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
        __syncthreads();
        if (s_last) {
            for (uint32_t k = threadIdx.x; k < 2 * sp.C; k += 64 * kSpW) sp.cw[r * 2 * sp.C + k] = 0;
            for (uint32_t k = threadIdx.x; k < kSpWords; k += 64 * kSpW) w[k] = 0;
        }
    }
}

// the token count of planned entry o (inner orddict:merge, or the run it copies)
template <int MODE>
__device__ __forceinline__ uint32_t entry_tokens(const LV& a, const LV& b, u64 r, u64 p,
                                                 const RK& rk, uint32_t* ia, uint32_t* jb) {
    *ia = kNone, *jb = kNone;
    if (MODE == 2) {
        if (p >> 32) *jb = (uint32_t)p;
        else *ia = (uint32_t)p;
        return 0;
    }
    *ia = (uint32_t)p;
    *jb = (uint32_t)(p >> 32);
    const uint32_t* OA = a.O(r);
    const uint32_t* OB = b.O(r);
    if (*ia != kNone && *jb != kNone)
        return MODE == 0 ? inner_merge<false>(a.T(r) + OA[*ia], OA[*ia + 1] - OA[*ia],
                                              b.T(r) + OB[*jb], OB[*jb + 1] - OB[*jb], nullptr, rk)
                         : OA[*ia + 1] - OA[*ia];
    if (*ia != kNone) return OA[*ia + 1] - OA[*ia];
    return OB[*jb + 1] - OB[*jb];
}

// one replica's chunk token counts -> exclusive offsets; need = {entries, tokens}
// (relaxed loads: in the fused form other blocks of the same launch wrote the counts)
__device__ void chunk_scan_replica(const MS& m, u64 r, uint32_t* need, uint32_t* s_w) {
    const uint32_t nc = (m.nout[r] + kMT - 1) / kMT;
    uint32_t* ch = m.chunk + r * m.nchunks;
    uint32_t carry = 0;
    for (uint32_t c0 = 0; c0 < nc; c0 += kMT) {
        const uint32_t k = c0 + threadIdx.x;
        uint32_t tot;
        const uint32_t off =
            carry + block_excl(k < nc ? __atomic_load_n(ch + k, __ATOMIC_RELAXED) : 0u, &tot, s_w);
        if (k < nc) ch[k] = off;
        carry += tot;
    }
    if (threadIdx.x == 0) {
        m.ntok[r] = carry;
        need[2 * r] = m.nout[r];
        need[2 * r + 1] = carry;
    }
}

// ticket (few replicas): the last block to finish also scans the chunk counts
// (k_merge_chunk_scan's work, one launch fewer)
template <int MODE>
__global__ __launch_bounds__(kMT) void k_merge_tok_count(LV a, LV b, RK rk, MS m, uint64_t R,
                                                         uint32_t* ticket, uint32_t* need) {
    __shared__ uint32_t s_w[kMT / 64], s_s[1];
    for (u64 r = blockIdx.y; r < R; r += gridDim.y) {
        const uint32_t nout = m.nout[r], o0 = blockIdx.x * kMT;
        if (o0 >= nout) continue;
        const uint32_t o = o0 + threadIdx.x;
        uint32_t cnt = 0, ia, jb;
        if (o < nout) {
            cnt = entry_tokens<MODE>(a, b, r, m.plan[r * ((u64)m.ce_a + m.ce_b) + o], rk, &ia, &jb);
            m.tcnt[r * ((u64)m.ce_a + m.ce_b) + o] = cnt;
        }
        uint32_t tot;
        block_excl(cnt, &tot, s_w);
        if (threadIdx.x == 0) m.chunk[r * m.nchunks + blockIdx.x] = tot;
    }
    if (ticket && last_block(ticket, s_s))
        for (u64 r = 0; r < R; ++r) chunk_scan_replica(m, r, need, s_w);
}

// per replica: exclusive offsets of the chunk token counts; need = {entries, tokens}
__global__ __launch_bounds__(kMT) void k_merge_chunk_scan(MS m, uint64_t R, uint32_t* need) {
    __shared__ uint32_t s_w[kMT / 64];
    for (u64 r = blockIdx.x; r < R; r += gridDim.x) chunk_scan_replica(m, r, need, s_w);
}

// list_bind: the merged list's keyfind table filled by the write pass itself (the keys it
// writes, their ranks from the rank pass) for the replicas whose check runs (used[r]) —
// k_linf_insert's work without its launch
struct Ins {
    u64* hk;
    uint32_t* hi;
    uint32_t hsize;
    const uint32_t* used;
};

// the write pass: one planned entry per thread
template <int MODE>
__global__ __launch_bounds__(kMT) void k_merge_write(LV a, LV b, LV out, RK rk, MS m, uint64_t R,
                                                     Ins ins) {
    __shared__ uint32_t s_w[kMT / 64];
    for (u64 r = blockIdx.y; r < R; r += gridDim.y) {
        const uint32_t nout = m.nout[r], nt = m.ntok[r], o0 = blockIdx.x * kMT;
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            if (nout > out.ce || nt > out.ct) {
                lraise(rk.flag, kErrRange);
            } else {
                out.hdr[2 * r] = nout;
                out.hdr[2 * r + 1] = nt;
                if (MODE != 2) out.O(r)[nout] = nt;
            }
        }
        if (o0 >= nout || nout > out.ce || nt > out.ct) continue;
        const uint32_t o = o0 + threadIdx.x;
        const u64 row = r * ((u64)m.ce_a + m.ce_b);
        const uint32_t cnt = o < nout ? m.tcnt[row + o] : 0u;
        uint32_t tot;
        const uint32_t tpos = m.chunk[r * m.nchunks + blockIdx.x] + block_excl(cnt, &tot, s_w);
        if (o >= nout) continue;
        uint32_t ia, jb;
        const u64 p = m.plan[row + o];
        if (MODE == 2) {
            if (p >> 32) jb = (uint32_t)p, ia = kNone;
            else ia = (uint32_t)p, jb = kNone;
        } else {
            ia = (uint32_t)p;
            jb = (uint32_t)(p >> 32);
        }
        out.K(r)[o] = ia != kNone ? a.K(r)[ia] : b.K(r)[jb];
        if (ins.hk && ins.used[r])
            h_insert(ins.hk + r * ins.hsize, ins.hi + r * ins.hsize, ins.hsize - 1,
                     ia != kNone ? m.sa[r * m.ce_a + ia] : m.sb[r * m.ce_b + jb], o);
        if (MODE == 2) continue;
        out.O(r)[o] = tpos;
        u64* to = out.T(r) + tpos;
        const uint32_t* OA = a.O(r);
        const uint32_t* OB = b.O(r);
        if (MODE == 0 && ia != kNone && jb != kNone) {
            inner_merge<true>(a.T(r) + OA[ia], OA[ia + 1] - OA[ia], b.T(r) + OB[jb],
                              OB[jb + 1] - OB[jb], to, rk);
        } else {
            const u64* from = ia != kNone ? a.T(r) + OA[ia] : b.T(r) + OB[jb];
            for (uint32_t k = 0; k < cnt; ++k) to[k] = from[k];
        }
    }
}

// `case Value0 of Value` (=:=): same entries, keys, token runs and flags
__global__ __launch_bounds__(64) void k_list_equal(LV a, LV b, RK rk, uint8_t* out) {
    const u64 r = blockIdx.x;
    const uint32_t n = a.n(r), nt = a.nt(r);
    bool diff = n != b.n(r) || nt != b.nt(r);
    if (!diff) {
        const u64 *KA = a.K(r), *KB = b.K(r), *TA = a.T(r), *TB = b.T(r);
        const uint32_t *OA = a.O(r), *OB = b.O(r);
        for (uint32_t i = lane_id(); i < n && !diff; i += 64)
            diff = key_ord(KA[i], rk) != key_ord(KB[i], rk) || OA[i] != OB[i];
        for (uint32_t t = lane_id(); t < nt && !diff; t += 64)
            diff = tok_ord(TA[t], rk) != tok_ord(TB[t], rk) ||
                   ((TA[t] ^ TB[t]) & kRemoved) != 0;
        diff = __ballot(diff) != 0;
    }
    if (lane_id() == 0) out[r] = diff ? 0 : 1;
}

// the same spread over a (chunk, replica) grid for the bind path's few long replicas:
// diff[r] (zeroed) gets a bit at the first difference any block sees
// (list_bind: also zeroes the keyfind tables of the replicas whose inflation check used
// them — used[r] != 0 — so the next bind finds them empty without a memset; and the block
// that finishes last writes bind/3's answer into pinned host memory (BindFin))
constexpr uint32_t kViolBit = 1, kChangedBit = 2;   // the inflation check's flag bits
struct BindFin {
    uint32_t* words;         // [flag | unsorted R | tickets 2 | aweak R | flags R | diff R |
                             //  ticket], zero on entry, left zero
    const uint32_t* need;    // [R][2] the merge's {entries, tokens}
    uint32_t* hneed;         // host: need, then status R bytes, then the flag word
    uint32_t R;
};
__global__ __launch_bounds__(256) void k_list_equal_grid(LV a, LV b, RK rk, uint32_t* diff,
                                                         uint64_t R, u64* hk, uint32_t* hi,
                                                         uint32_t hsize, const uint32_t* used,
                                                         BindFin fin) {
    for (u64 r = blockIdx.y; r < R; r += gridDim.y) {
        if (used && used[r]) {
            u64* k0 = hk + r * hsize;
            uint32_t* i0 = hi + r * hsize;
            for (uint32_t x = blockIdx.x * 256u + threadIdx.x; x < hsize; x += gridDim.x * 256u) {
                k0[x] = 0;
                i0[x] = 0;
            }
        }
        const uint32_t n = a.n(r), nt = a.nt(r);
        if (n != b.n(r) || nt != b.nt(r)) {
            if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(diff + r, 1u);
            continue;
        }
        const u64 *KA = a.K(r), *KB = b.K(r), *TA = a.T(r), *TB = b.T(r);
        const uint32_t *OA = a.O(r), *OB = b.O(r);
        bool d = false;
        const uint32_t stride = gridDim.x * 256u;
        for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n && !d; i += stride)
            d = key_ord(KA[i], rk) != key_ord(KB[i], rk) || OA[i] != OB[i];
        for (uint32_t t = blockIdx.x * 256u + threadIdx.x; t < nt && !d; t += stride)
            d = tok_ord(TA[t], rk) != tok_ord(TB[t], rk) || ((TA[t] ^ TB[t]) & kRemoved) != 0;
        if (__ballot(d) != 0 && lane_id() == 0) atomicOr(diff + r, 1u);
    }
    if (!fin.words) return;
    // bind/3's answer per replica (the non-strict rule: no violation): 0 = equal (no-op), 1 = the merge
    // inflates Value0 (written), 2 = it does not; then every word zeroed for the next call
    __shared__ uint32_t s_last;
    const uint32_t n = fin.R;
    uint32_t* w = fin.words;
    uint32_t* ticket = w + 4 * n + 3;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        s_last = atomicAdd(ticket, 1u) == gridDim.x * gridDim.y - 1;
    }
    __syncthreads();
    if (!s_last) return;
    __threadfence();
    uint8_t* hst = reinterpret_cast<uint8_t*>(fin.hneed + 2 * n);
    for (uint32_t r = threadIdx.x; r < n; r += 256) {
        const uint32_t dv = __atomic_load_n(w + 3 * n + 3 + r, __ATOMIC_RELAXED);
        const uint32_t lf = __atomic_load_n(w + 2 * n + 3 + r, __ATOMIC_RELAXED);
        hst[r] = !dv ? 0 : ((lf & kViolBit) ? 2 : 1);
        fin.hneed[2 * r] = fin.need[2 * r];
        fin.hneed[2 * r + 1] = fin.need[2 * r + 1];
        w[1 + r] = 0;                                          // unsorted
        w[n + 3 + r] = 0;                                      // aweak
        w[2 * n + 3 + r] = 0;                                  // inflation flags
        w[3 * n + 3 + r] = 0;                                  // diff
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        fin.hneed[2 * n + (n + 3) / 4] = __atomic_load_n(w, __ATOMIC_RELAXED);
        w[0] = 0;
        *ticket = 0;
        __threadfence_system();
    }
}

// ---------------------------------------------------------------- list_bind, ascending
// When both lists' keys strictly ascend in term order (plain keys: every orddict and
// ordset, an intersection / filter output of one, a merge of two), orddict:merge's and
// ordsets:union's two-finger walk visits the keys in rank order and pairs equal keys:
// the merged list has one entry per rank that either side holds — both sides: the inner
// token merge (merge/2's F), ordsets:union's equal elements being one slot — in rank
// order.  So this bind needs no merge path, no plan and no per-entry scans:
//   k_lbf_prep   entry i of each side -> its rank's cell of a rank-indexed map (tagged
//                with the call's epoch, so the maps are never cleared), the ascent
//                checked against the lane below, every token id checked, and
//                `Value0 =:= Value` over the grid
//   k_lbf_write  256 ranks per block (one per thread): entry present?, token count (inner
//                merge or run); offsets from a block scan and a decoupled look-back over
//                the rank tiles; the merged list written; each replica's last tile writes
//                its part of bind/3's answer
// is_inflation(Value0, Merged) holds by construction when Value0 ascends (k_linf_probe's
// skip, below), so the answer is equal ? 0 : 1.  A replica that does not ascend (or
// carries product pairs, or an id outside the rank tables) answers 3 and the call runs
// the merge path instead, which reports the errors.  No tickets, no fences: tiles are
// block indices (dispatched in order), the look-back words carry their whole payload,
// and the words a call uses are zeroed by the NEXT call (two parities), so nothing
// waits for the whole grid to finish.
constexpr uint32_t kLfT = 256;              // threads per block
constexpr uint32_t kLfPer = 1;              // ranks per thread (4 measured slower: 42 vs 31 us;
                                            // runs loaded into registers up front: 56 us)
constexpr uint32_t kLfTile = kLfT * kLfPer; // ranks per tile
struct LF {
    u64* ia;          // [R][nk] epoch << 32 | index of the entry of A (Value0) with rank v
    u64* ib;          // [R][nk] the same for B (Value)
    uint32_t* w;      // this call's words [diff R | bad R], zero on entry
    u64* st;          // this call's look-back words [R][ntiles]: state << 62 | entries << 32
                      // | tokens, zero on entry
    uint32_t* wz;     // the previous call's words and look-back words, zeroed here
    uint64_t nwz;     //   (32-bit words)
    uint32_t* hneed;  // host answer: need [R][2], then status R bytes
    uint32_t epoch, nk, ntiles, R;
};

__device__ __forceinline__ bool tok_ok(u64 it, const RK& rk) {
    if (it & kCompound)
        return (uint32_t)((it >> 31) & kIdMask) < rk.ng && (uint32_t)(it & kIdMask) < rk.ng;
    return (uint32_t)(it & kIdMask) < rk.ng;
}

// a side's entry i: its rank into the map when the keys ascend, else bad |= bit
__device__ __forceinline__ uint32_t lbf_side(const LV& x, u64 r, uint32_t i, uint32_t n,
                                             const RK& rk, const LF& f, u64* map,
                                             uint32_t bit, u64* rank_out) {
    u64 rank = ~0ull;
    bool ok = true;
    if (i < n) {
        const u64 it = x.K(r)[i];
        const uint32_t e = (uint32_t)(it & kIdMask);
        if ((it & kPair) || e >= rk.nk) ok = false;         // (pairs: no rank universe)
        else rank = rk.krank[e];
        if (rank >= f.nk) ok = false;
    }
    u64 prev = __shfl_up(rank, 1, 64);                      // the previous entry's rank
    if (lane_id() == 0 && i > 0 && i < n) {
        const u64 it = x.K(r)[i - 1];
        const uint32_t e = (uint32_t)(it & kIdMask);
        prev = (it & kPair) || e >= rk.nk ? ~0ull : (u64)rk.krank[e];
    }
    if (i < n && i > 0 && !(prev < rank)) ok = false;
    if (i < n && ok) map[r * f.nk + rank] = ((u64)f.epoch << 32) | i;
    *rank_out = rank;
    return i < n && !ok ? bit : 0u;
}

template <bool GSET>
__global__ __launch_bounds__(256) void k_lbf_prep(LV a, LV b, RK rk, LF f, uint64_t R) {
    for (u64 r = blockIdx.y; r < R; r += gridDim.y) {
        const uint32_t na = a.n(r), nb = b.n(r), nta = a.nt(r), ntb = b.nt(r);
        const uint32_t i = blockIdx.x * 256u + threadIdx.x;
        u64 ra, rb;
        uint32_t bad = lbf_side(a, r, i, na, rk, f, f.ia, 1u, &ra);
        bad |= lbf_side(b, r, i, nb, rk, f, f.ib, 2u, &rb);
        // every token id inside the rank tables (the write pass reads ranks unchecked)
        if (!GSET) {
            if (i < nta && !tok_ok(a.T(r)[i], rk)) bad |= 1u;
            if (i < ntb && !tok_ok(b.T(r)[i], rk)) bad |= 2u;
        }
        // `Value0 =:= Value` (k_list_equal_grid's comparisons)
        bool d = false;
        if (na != nb || nta != ntb) {
            d = i == 0;
        } else {
            if (i < na) d = ra != rb || a.O(r)[i] != b.O(r)[i];
            if (!GSET && i < nta) {
                const u64 x = a.T(r)[i], y = b.T(r)[i];
                if (tok_ok(x, rk) && tok_ok(y, rk))
                    d = d || tok_ord(x, rk) != tok_ord(y, rk) || ((x ^ y) & kRemoved) != 0;
            }
        }
        for (int off = 32; off > 0; off >>= 1) bad |= __shfl_xor(bad, off, 64);
        if (__ballot(d) && lane_id() == 0) atomicOr(f.w + r, 1u);
        if (bad && lane_id() == 0) atomicOr(f.w + R + r, bad);
    }
}

__device__ __forceinline__ u64 wave_excl64(u64 v, u64* total) {
    u64 x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const u64 y = __shfl_up(x, off, 64);
        if ((int)lane_id() >= off) x += y;
    }
    *total = __shfl(x, 63, 64);
    return x - v;
}

template <int MODE>
__global__ __launch_bounds__(kLfT) void k_lbf_write(LV a, LV b, LV out, RK rk, LF f) {
    __shared__ u64 s_w[kLfT / 64];
    __shared__ u64 s_base;
    constexpr u64 kVal = (1ull << 62) - 1;
    if (blockIdx.x == 0 && blockIdx.y == 0)                 // the previous call's words
        for (u64 k = threadIdx.x; k < f.nwz; k += kLfT) f.wz[k] = 0;
    const uint32_t t = blockIdx.x;
    for (u64 r = blockIdx.y; r < f.R; r += gridDim.y) {
        const uint32_t bad = f.w[f.R + r];                  // (the prep pass's, uniform)
        uint8_t* hst = reinterpret_cast<uint8_t*>(f.hneed + 2 * f.R);
        if (bad) {
            if (t == f.ntiles - 1 && threadIdx.x == 0) hst[r] = (uint8_t)(3u | (bad << 2));
            continue;
        }
        const uint32_t* OA = a.O(r);
        const uint32_t* OB = b.O(r);
        uint32_t ia[kLfPer], jb[kLfPer], cnt[kLfPer];
        u64 mine = 0;
#pragma unroll
        for (uint32_t k = 0; k < kLfPer; ++k) {
            const uint32_t v = t * kLfTile + threadIdx.x * kLfPer + k;   // (rank order = thread order)
            ia[k] = kNone, jb[k] = kNone, cnt[k] = 0;
            if (v < f.nk) {
                const u64 xa = f.ia[r * f.nk + v], xb = f.ib[r * f.nk + v];
                if ((uint32_t)(xa >> 32) == f.epoch) ia[k] = (uint32_t)xa;
                if ((uint32_t)(xb >> 32) == f.epoch) jb[k] = (uint32_t)xb;
            }
            const bool has = ia[k] != kNone || jb[k] != kNone;
            if (MODE == 2) {
                // ordsets:union's pair of equal rank from two slots (1 and 1.0): its item
                // is the side of the walk's last single step (the merge path's work).
                // G-Set lists have no tokens: the count field carries these pairs through
                // the look-back to the last tile
                cnt[k] = ia[k] != kNone && jb[k] != kNone && a.K(r)[ia[k]] != b.K(r)[jb[k]];
            } else if (has) {
                if (ia[k] != kNone && jb[k] != kNone)
                    cnt[k] = inner_merge<false>(a.T(r) + OA[ia[k]], OA[ia[k] + 1] - OA[ia[k]],
                                                b.T(r) + OB[jb[k]], OB[jb[k] + 1] - OB[jb[k]],
                                                nullptr, rk);
                else if (ia[k] != kNone) cnt[k] = OA[ia[k] + 1] - OA[ia[k]];
                else cnt[k] = OB[jb[k] + 1] - OB[jb[k]];
            }
            mine += ((u64)has << 32) | cnt[k];
        }
        // entries << 32 | tokens: one scan carries both (tokens stay below 2^32)
        u64 wt;
        const u64 x = wave_excl64(mine, &wt);
        const uint32_t wv = threadIdx.x >> 6;
        __syncthreads();
        if (lane_id() == 0) s_w[wv] = wt;
        __syncthreads();
        u64 ex = x, tot = 0;
#pragma unroll
        for (uint32_t k = 0; k < kLfT / 64; ++k) {
            ex += k < wv ? s_w[k] : 0ull;
            tot += s_w[k];
        }
        if (threadIdx.x == 0) {
            // relaxed device-scope atomics: the words carry their whole payload (acquire /
            // release would write back and invalidate the XCD's L2 at every step)
            u64* st = f.st + r * f.ntiles;
            u64 prefix = 0;
            if (t == 0) {
                __hip_atomic_store(st, (2ull << 62) | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                __hip_atomic_store(st + t, (1ull << 62) | tot, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                for (int64_t j = (int64_t)t - 1; j >= 0;) {
                    const u64 sj = __hip_atomic_load(st + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (!(sj >> 62)) {                              // not published yet
                        __builtin_amdgcn_s_sleep(1);
                        continue;
                    }
                    prefix += sj & kVal;
                    if ((sj >> 62) == 2) break;
                    --j;
                }
                __hip_atomic_store(st + t, (2ull << 62) | (prefix + tot), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
            s_base = prefix;
        }
        __syncthreads();
        u64 pos = s_base + ex;
#pragma unroll
        for (uint32_t k = 0; k < kLfPer; ++k) {
            if (ia[k] == kNone && jb[k] == kNone) continue;
            const uint32_t o = (uint32_t)(pos >> 32), tp = (uint32_t)pos;
            out.K(r)[o] = ia[k] != kNone ? a.K(r)[ia[k]] : b.K(r)[jb[k]];
            if (MODE != 2) {
                out.O(r)[o] = tp;
                u64* to = out.T(r) + tp;
                if (ia[k] != kNone && jb[k] != kNone) {
                    inner_merge<true>(a.T(r) + OA[ia[k]], OA[ia[k] + 1] - OA[ia[k]],
                                      b.T(r) + OB[jb[k]], OB[jb[k] + 1] - OB[jb[k]], to, rk);
                } else {
                    const u64* from = ia[k] != kNone ? a.T(r) + OA[ia[k]] : b.T(r) + OB[jb[k]];
                    for (uint32_t q = 0; q < cnt[k]; ++q) to[q] = from[q];
                }
            }
            pos += (1ull << 32) | cnt[k];
        }
        if (t == f.ntiles - 1 && threadIdx.x == 0) {
            // the last tile: the totals, and this replica's answer (0 = Value0 =:= Value,
            // 1 = merged: the inflation holds, 3 | bad << 2 = retry on the merge path)
            const u64 all = s_base + tot;
            const uint32_t nout = (uint32_t)(all >> 32);
            const uint32_t ntok = MODE == 2 ? 0u : (uint32_t)all;
            const bool pairs2 = MODE == 2 && (uint32_t)all != 0;
            out.hdr[2 * r] = nout;
            out.hdr[2 * r + 1] = ntok;
            if (MODE != 2) out.O(r)[nout] = ntok;
            f.hneed[2 * r] = nout;
            f.hneed[2 * r + 1] = ntok;
            hst[r] = pairs2 ? (uint8_t)(3u | (16u << 2)) : (f.w[r] ? 1 : 0);
        }
        __syncthreads();
    }
}

// is_lattice_inflation / is_lattice_strict_inflation (lasp_lattice.erl:137-161,
// 212-215, 235-253, 277-285), spread over the grid (a 50k-entry list is 200 blocks, not
// one wave): k_linf_insert builds, per replica, an open-addressing table of Cur's key
// ranks -> first index (= lists:keyfind's first match; G-Set strict also Prev's keys),
// k_linf_probe checks one Prev (and, G-Set strict, one Cur) entry per thread and ORs
// violation / change bits into a per-replica word, k_linf_final turns them into the
// answer.  The tables start zeroed (empty, see h_insert) by one memset with the flags.
// skip (list_bind's non-strict check of Value0 against merge(Value0, Value), or null): a
// replica with skip[r] == 0 — Value0's keys strictly ascending — has nothing to check:
// orddict:merge's two-finger walk emits every entry of its first list, alone or with the
// other list's equal key, and before any later entry of that key (the first list ascends,
// so no earlier emitted key equals it), so keyfind finds it; the inner merge emits every
// token of the first list likewise (ids_inflated asks presence only); ordsets:union
// keeps every element of its first set.  The inflation then holds by construction.

template <bool GSET, bool STRICT>
__global__ __launch_bounds__(256) void k_linf_insert(LV prev, LV cur, RK rk, u64* hk,
                                                     uint32_t* hi, uint32_t hsize, bool bcast,
                                                     uint64_t R, const uint32_t* skip) {
    const uint32_t mask = hsize - 1;
    for (u64 r = blockIdx.y; r < R; r += gridDim.y) {
        if (skip && !skip[r]) continue;
        const u64 pr = bcast ? 0 : r;
        const uint32_t i = blockIdx.x * 256 + threadIdx.x;
        u64* hk0 = hk + r * (GSET && STRICT ? 2ull : 1ull) * hsize;
        uint32_t* hi0 = hi + r * (GSET && STRICT ? 2ull : 1ull) * hsize;
        if (i < cur.n(r)) h_insert(hk0, hi0, mask, key_ord(cur.K(r)[i], rk), i);
        if (GSET && STRICT && i < prev.n(pr))
            h_insert(hk0 + hsize, hi0 + hsize, mask, key_ord(prev.K(pr)[i], rk), i);
    }
}

template <bool GSET, bool STRICT>
__global__ __launch_bounds__(256) void k_linf_probe(LV prev, LV cur, RK rk, const u64* hk,
                                                    const uint32_t* hi, uint32_t hsize,
                                                    bool bcast, uint64_t R, uint32_t* flags,
                                                    const uint32_t* skip) {
    const uint32_t mask = hsize - 1;
    for (u64 r = blockIdx.y; r < R; r += gridDim.y) {
        if (skip && !skip[r]) continue;
        const u64 pr = bcast ? 0 : r;
        const uint32_t np = prev.n(pr), nc = cur.n(r);
        const uint32_t i = blockIdx.x * 256 + threadIdx.x;
        const u64* hk0 = hk + r * (GSET && STRICT ? 2ull : 1ull) * hsize;
        const uint32_t* hi0 = hi + r * (GSET && STRICT ? 2ull : 1ull) * hsize;
        bool viol = false, changed = false;
        if (GSET) {
            // sets:is_subset(from_list(Prev), from_list(Cur))
            if (i < np) viol = h_find(hk0, hi0, mask, key_ord(prev.K(pr)[i], rk)) == kNone;
            // usort(Prev) =/= usort(Cur): with Prev ⊆ Cur, some Cur key is not in Prev
            if (STRICT && i < nc)
                changed = h_find(hk0 + hsize, hi0 + hsize, mask, key_ord(cur.K(r)[i], rk)) == kNone;
        } else if (i < np) {
            // lists:keyfind(Element, 1, Current): the first entry with an equal key
            const uint32_t j = h_find(hk0, hi0, mask, key_ord(prev.K(pr)[i], rk));
            if (j == kNone) {
                viol = true;
            } else {
                const uint32_t* OP = prev.O(pr);
                const uint32_t* OC = cur.O(r);
                const u64* tp = prev.T(pr) + OP[i];
                const u64* tc = cur.T(r) + OC[j];
                const uint32_t lp = OP[i + 1] - OP[i], lc = OC[j + 1] - OC[j];
                // ids_inflated: every Prev token keyfind-s among Cur's (flags ignored)
                for (uint32_t x = 0; x < lp && !viol; ++x) {
                    const u64 ox = tok_ord(tp[x], rk);
                    bool found = false;
                    for (uint32_t y = 0; y < lc && !found; ++y) found = tok_ord(tc[y], rk) == ox;
                    viol = !found;
                }
                // DeletedElements: Ids =/= Ids1 (order- and flag-sensitive)
                if (STRICT) {
                    if (lp != lc) {
                        changed = true;
                    } else {
                        for (uint32_t x = 0; x < lp && !changed; ++x)
                            changed = tok_ord(tp[x], rk) != tok_ord(tc[x], rk) ||
                                      ((tp[x] ^ tc[x]) & kRemoved) != 0;
                    }
                }
            }
        }
        const uint32_t f = (viol ? kViolBit : 0u) | (changed ? kChangedBit : 0u);
        const u64 any = __ballot(f != 0);
        uint32_t wf = f;
        for (int off = 32; off > 0; off >>= 1) wf |= __shfl_xor(wf, off, 64);
        if (any && lane_id() == 0) atomicOr(flags + r, wf);
    }
}

template <bool GSET, bool STRICT>
__global__ void k_linf_final(LV prev, LV cur, bool bcast, uint64_t R, const uint32_t* flags,
                             uint8_t* out) {
    for (u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x; r < R; r += (u64)gridDim.x * blockDim.x) {
        const uint32_t np = prev.n(bcast ? 0 : r), nc = cur.n(r), f = flags[r];
        bool res = !(f & kViolBit);
        if (STRICT) {
            const bool changed = (f & kChangedBit) != 0;
            if (GSET) res = res && changed;
            else if (np == 0 && nc != 0) res = true;       // ([], Current) when Current =/= []
            else res = res && (changed || np < nc);        // NewElements: length/1
        }
        out[r] = res ? 1 : 0;
    }
}

// ---------------------------------------------------------------- tiled producers
// Every producer below emits, per replica, a compaction of one input sequence in order:
// item i of replica r emits ne_i entries and nt_i tokens at the exclusive prefix sums of
// the items before it.  A pass runs over a (tile, replica) grid of kPTile items per
// block, so a single long replica (the bind path's one variable) spreads over the chip
// instead of one wave:
//   k_tp_count  per tile {ne, nt} sums -> tc[r][t]
//   k_tp_scan   per replica, the exclusive scan of its tile sums in place; totals -> need
//   k_tp_write  (write pass) each tile re-counts its items, one block scan gives every
//               item's positions after the tile's offset, the functor writes; tile 0
//               writes the header and the token-offset sentinel.
// The functors restate the reference bodies item by item:
//   PFromSet      canonical cells -> list (elements ascending in term order, tokens likewise)
//   PValue        value/1: keys of entries with a {_, false} token (lasp_orset.erl:67-73)
//   PConcat       G-Set union body L ++ R (lasp_core.erl:602-627)
//   PIsect        intersection body: per entry of L in order, keyfind (OR-Set) / member
//                 (G-Set) in R, tokens Cx ++ Cy (lasp_core.erl:546-589,
//                 lasp_lattice.erl:311-312)
//   PProduct      product body: entry (x, y) x-major, tokens orset_causal_product(Cx, Cy)
//                 (lasp_core.erl:499-533, lasp_lattice.erl:303-308)
//   PMap / PFilter / PFold   map / filter / fold bodies over host-evaluated fun tables
//                 (lasp_core.erl:641-667, 681-712, 460-486)
constexpr uint32_t kPT = 256;             // threads per tile block
constexpr uint32_t kPI = 4;               // items per thread
constexpr uint32_t kPTile = kPT * kPI;

// {entries, tokens} of an item, a tile or a replica prefix (64-bit sums: a total past
// the list's 32-bit counts is caught by the scan, never wrapped)
struct C2 {
    u64 e, t;
    __device__ C2& operator+=(const C2& o) {
        e += o.e;
        t += o.t;
        return *this;
    }
    __device__ bool any() const { return (e | t) != 0; }
};
__device__ __forceinline__ C2 operator+(C2 a, const C2& b) { return a += b; }
__device__ __forceinline__ C2 pk2(uint32_t ne, uint32_t nt) { return C2{ne, nt}; }

// exclusive block scan of {ne, nt}
__device__ __forceinline__ C2 block_scan_pk(C2 v, C2* lds, C2* total) {
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    C2 x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const C2 y{__shfl_up(x.e, off, 64), __shfl_up(x.t, off, 64)};
        if ((int)lane >= off) x += y;
    }
    if (lane == 63) lds[w] = x;
    __syncthreads();
    C2 before{0, 0}, all{0, 0};
#pragma unroll
    for (uint32_t i = 0; i < kPT / 64; ++i) {
        const C2 t = lds[i];
        if (i < w) before += t;
        all += t;
    }
    __syncthreads();
    *total = all;
    return C2{before.e + x.e - v.e, before.t + x.t - v.t};
}

template <class P>
__global__ __launch_bounds__(kPT) void k_tp_count(P p, C2* tc, uint32_t ntile, uint64_t R) {
    __shared__ C2 lds[kPT / 64];
    const uint32_t t = blockIdx.x;
    for (uint64_t r = blockIdx.y; r < R; r += gridDim.y) {
        const u64 n = p.items(r), i0 = (u64)t * kPTile;
        C2 sum{0, 0};
        if (i0 < n) {
#pragma unroll
            for (uint32_t k = 0; k < kPI; ++k) {
                const u64 i = i0 + k * kPT + threadIdx.x;
                if (i < n) sum += p.count(r, i);
            }
        }
        C2 tot;
        block_scan_pk(sum, lds, &tot);
        if (threadIdx.x == 0) tc[r * ntile + t] = tot;
    }
}

__global__ __launch_bounds__(kPT) void k_tp_scan(C2* tc, uint32_t ntile, uint64_t R,
                                                 uint32_t* need, uint32_t* flag) {
    __shared__ C2 lds[kPT / 64];
    for (uint64_t r = blockIdx.x; r < R; r += gridDim.x) {
        C2* c = tc + r * ntile;
        C2 carry{0, 0};
        for (uint32_t t0 = 0; t0 < ntile; t0 += kPT) {
            const uint32_t t = t0 + threadIdx.x;
            const C2 v = t < ntile ? c[t] : C2{0, 0};
            C2 tot;
            const C2 ex = block_scan_pk(v, lds, &tot);
            if (t < ntile) c[t] = carry + ex;
            carry += tot;
        }
        if (threadIdx.x == 0) {
            // a list counts entries and tokens in 32 bits
            if (carry.e > 0xFFFFFFFFull || carry.t > 0xFFFFFFFFull) lraise(flag, kErrRange);
            need[2 * r] = (uint32_t)min(carry.e, 0xFFFFFFFFull);
            need[2 * r + 1] = (uint32_t)min(carry.t, 0xFFFFFFFFull);
        }
    }
}

template <class P>
__global__ __launch_bounds__(kPT) void k_tp_write(P p, LV out, const C2* tc, uint32_t ntile,
                                                  uint64_t R, const uint32_t* need,
                                                  uint32_t* flag) {
    __shared__ C2 lds[kPT / 64];
    const uint32_t t = blockIdx.x;
    for (uint64_t r = blockIdx.y; r < R; r += gridDim.y) {
        const u64 n = p.items(r), i0 = (u64)t * kPTile + (u64)threadIdx.x * kPI;
        if (t == 0 && threadIdx.x == 0) {
            const uint32_t ne = need[2 * r], nt = need[2 * r + 1];
            if (ne > out.ce || nt > out.ct) {
                lraise(flag, kErrRange);
            } else {
                out.hdr[2 * r] = ne;
                out.hdr[2 * r + 1] = nt;
                out.O(r)[ne] = nt;
            }
        }
        if ((u64)t * kPTile >= n) continue;        // block-uniform: no barrier skipped
        C2 c[kPI], mine{0, 0};
#pragma unroll
        for (uint32_t k = 0; k < kPI; ++k) {
            c[k] = i0 + k < n ? p.count(r, i0 + k) : C2{0, 0};
            mine += c[k];
        }
        C2 tot;
        C2 at = tc[r * ntile + t] + block_scan_pk(mine, lds, &tot);
#pragma unroll
        for (uint32_t k = 0; k < kPI; ++k) {
            if (c[k].any()) {
                if (at.e + c[k].e > out.ce || at.t + c[k].t > out.ct)
                    lraise(flag, kErrRange);
                else
                    p.write(r, i0 + k, (uint32_t)at.e, (uint32_t)at.t, out);
            }
            at += c[k];
        }
    }
}

template <bool GSET>
struct PFromSet {
    const u64* src;
    uint64_t wpr;
    const uint32_t* order;
    uint32_t nord, E;
    const uint8_t* tord;
    uint32_t* flag;
    __device__ u64 items(u64) const { return nord; }
    __device__ void cell(u64 r, u64 i, uint32_t& e, u64& p, u64& rm) const {
        e = order[i];
        p = rm = 0;
        if (e >= E) {
            lraise(flag, kErrId);
            return;
        }
        const u64* s = src + r * wpr;
        if (GSET) {
            p = (s[e >> 6] >> (e & 63)) & 1ull;
        } else {
            p = s[2ull * e];
            rm = s[2ull * e + 1];
        }
    }
    __device__ C2 count(u64 r, u64 i) const {
        uint32_t e;
        u64 p, rm;
        cell(r, i, e, p, rm);
        return p ? pk2(1, GSET ? 0u : (uint32_t)__popcll(p)) : C2{0, 0};
    }
    __device__ void write(u64 r, u64 i, uint32_t pos, uint32_t tpos, LV out) const {
        uint32_t e;
        u64 p, rm;
        cell(r, i, e, p, rm);
        out.K(r)[pos] = e;
        if (GSET) return;
        out.O(r)[pos] = tpos;
        u64* T = out.T(r);
        const uint8_t* to = tord + 64ull * e;
        for (int j = 0; j < 64; ++j) {
            const uint32_t k = to[j];
            if (k >= 64) break;
            if ((p >> k) & 1ull) T[tpos++] = (64ull * e + k) | (((rm >> k) & 1ull) << 63);
        }
    }
};

struct PValue {
    LV src;
    __device__ u64 items(u64 r) const { return src.n(r); }
    __device__ C2 count(u64 r, u64 i) const {
        const uint32_t* O = src.O(r);
        const u64* T = src.T(r);
        for (uint32_t t = O[i]; t < O[i + 1]; ++t)
            if (!(T[t] & kRemoved)) return pk2(1, 0);
        return C2{0, 0};
    }
    __device__ void write(u64 r, u64 i, uint32_t pos, uint32_t, LV out) const {
        out.K(r)[pos] = src.K(r)[i];
    }
};

struct PConcat {
    LV l, rr;
    __device__ u64 items(u64 r) const { return (u64)l.n(r) + rr.n(r); }
    __device__ C2 count(u64, u64) const { return pk2(1, 0); }
    __device__ void write(u64 r, u64 i, uint32_t pos, uint32_t, LV out) const {
        const uint32_t nl = l.n(r);
        out.K(r)[pos] = i < nl ? l.K(r)[i] : rr.K(r)[i - nl];
    }
};

// R's keys -> first index, built before the count pass (k_isect_hash)
template <bool GSET>
struct PIsect {
    LV l, rr;
    RK rk;
    const u64* hk;
    const uint32_t* hi;
    uint32_t hsize;
    __device__ uint32_t find(u64 r, u64 i) const {
        return h_find(hk + r * (u64)hsize, hi + r * (u64)hsize, hsize - 1,
                      key_ord(l.K(r)[i], rk));
    }
    __device__ u64 items(u64 r) const { return l.n(r); }
    __device__ C2 count(u64 r, u64 i) const {
        const uint32_t j = find(r, i);
        if (j == kNone) return C2{0, 0};
        if (GSET) return pk2(1, 0);
        const uint32_t* OL = l.O(r);
        const uint32_t* OR = rr.O(r);
        return pk2(1, (OL[i + 1] - OL[i]) + (OR[j + 1] - OR[j]));
    }
    __device__ void write(u64 r, u64 i, uint32_t pos, uint32_t tpos, LV out) const {
        out.K(r)[pos] = l.K(r)[i];
        if (GSET) return;
        const uint32_t j = find(r, i);
        const uint32_t* OL = l.O(r);
        const uint32_t* OR = rr.O(r);
        out.O(r)[pos] = tpos;
        u64* to = out.T(r) + tpos;
        const u64* tl = l.T(r) + OL[i];
        const uint32_t ll = OL[i + 1] - OL[i], lr = OR[j + 1] - OR[j];
        for (uint32_t k = 0; k < ll; ++k) to[k] = tl[k];        // Cx ++ Cy
        const u64* tr = rr.T(r) + OR[j];
        for (uint32_t k = 0; k < lr; ++k) to[ll + k] = tr[k];
    }
};

// the intersection body with a canonical right side (an OR-Set / G-Set batch): keyfind /
// member of X in R's list form (one entry per present slot, tokens in term order) is R's
// cell of X's slot — no conversion of R into a list, no hash.  (The Store's dictionaries
// give distinct slots distinct ranks, codec.EqualTerms, so the slot is the only match.)
template <bool GSET>
struct PIsectSet {
    LV l;
    const u64* src;
    uint64_t wpr;
    uint32_t E;
    const uint8_t* tord;
    __device__ bool cell(u64 r, u64 i, uint32_t& e, u64& p, u64& rm) const {
        const u64 it = l.K(r)[i];
        p = rm = 0;
        e = (uint32_t)(it & kIdMask);
        if ((it & kPair) || e >= E) return false;      // not an element of the set
        const u64* s = src + r * wpr;
        if (GSET) {
            p = (s[e >> 6] >> (e & 63)) & 1ull;
        } else {
            p = s[2ull * e];
            rm = s[2ull * e + 1];
        }
        return p != 0;
    }
    __device__ u64 items(u64 r) const { return l.n(r); }
    __device__ C2 count(u64 r, u64 i) const {
        uint32_t e;
        u64 p, rm;
        if (!cell(r, i, e, p, rm)) return C2{0, 0};
        if (GSET) return pk2(1, 0);
        const uint32_t* OL = l.O(r);
        return pk2(1, (OL[i + 1] - OL[i]) + (uint32_t)__popcll(p));
    }
    __device__ void write(u64 r, u64 i, uint32_t pos, uint32_t tpos, LV out) const {
        uint32_t e;
        u64 p, rm;
        cell(r, i, e, p, rm);
        out.K(r)[pos] = l.K(r)[i];
        if (GSET) return;
        const uint32_t* OL = l.O(r);
        out.O(r)[pos] = tpos;
        u64* to = out.T(r) + tpos;
        const u64* tl = l.T(r) + OL[i];
        const uint32_t ll = OL[i + 1] - OL[i];
        for (uint32_t k = 0; k < ll; ++k) to[k] = tl[k];            // Cx ++ Cy
        uint32_t n = ll;
        const uint8_t* ot = tord + 64ull * e;
        for (int j = 0; j < 64; ++j) {
            const uint32_t k = ot[j];
            if (k >= 64) break;
            if ((p >> k) & 1ull) to[n++] = (64ull * e + k) | (((rm >> k) & 1ull) << 63);
        }
    }
};

template <bool GSET>
__global__ __launch_bounds__(256) void k_isect_hash(LV rr, RK rk, u64* hk, uint32_t* hi,
                                                    uint32_t hsize, uint64_t R) {
    for (uint64_t r = blockIdx.y; r < R; r += gridDim.y) {
        const uint32_t nr = rr.n(r);
        const u64* KR = rr.K(r);
        for (uint32_t j = blockIdx.x * 256 + threadIdx.x; j < nr; j += gridDim.x * 256)
            h_insert(hk + r * (u64)hsize, hi + r * (u64)hsize, hsize - 1, key_ord(KR[j], rk), j);
    }
}

template <bool GSET>
struct PProduct {
    LV l, rr;
    uint32_t* flag;
    __device__ u64 items(u64 r) const { return (u64)l.n(r) * rr.n(r); }
    __device__ C2 count(u64 r, u64 o) const {
        // entries and tokens of the whole output must fit the list's 32-bit counts
        if (items(r) > 0xFFFFFFFFull || (!GSET && (u64)l.nt(r) * rr.nt(r) > 0xFFFFFFFFull)) {
            lraise(flag, kErrRange);
            return C2{0, 0};
        }
        if (GSET) return pk2(1, 0);
        const uint32_t nr = rr.n(r);
        const uint32_t xi = (uint32_t)(o / nr), yi = (uint32_t)(o - (u64)xi * nr);
        const uint32_t lx = l.O(r)[xi + 1] - l.O(r)[xi], ly = rr.O(r)[yi + 1] - rr.O(r)[yi];
        return pk2(1, lx * ly);
    }
    __device__ void write(u64 r, u64 o, uint32_t pos, uint32_t tpos, LV out) const {
        const uint32_t nr = rr.n(r);
        const uint32_t xi = (uint32_t)(o / nr), yi = (uint32_t)(o - (u64)xi * nr);
        const u64 kx = l.K(r)[xi], ky = rr.K(r)[yi];
        if ((kx & kPair) || (ky & kPair)) {
            lraise(flag, kErrNested);
            return;
        }
        out.K(r)[pos] = kPair | ((kx & kIdMask) << 31) | (ky & kIdMask);
        if (GSET) return;
        const uint32_t* OL = l.O(r);
        const uint32_t* OR = rr.O(r);
        const uint32_t lx = OL[xi + 1] - OL[xi], ly = OR[yi + 1] - OR[yi];
        out.O(r)[pos] = tpos;
        u64* to = out.T(r) + tpos;
        const u64* tx = l.T(r) + OL[xi];
        const u64* ty = rr.T(r) + OR[yi];
        uint32_t k = 0;
        for (uint32_t a = lx; a-- > 0;) {           // reversed foldl: Xs backwards
            const u64 X = tx[a];
            for (uint32_t b = ly; b-- > 0;) {       // ... and Ys backwards
                const u64 Y = ty[b];
                if ((X & kCompound) || (Y & kCompound)) {
                    lraise(flag, kErrNested);
                    ++k;
                    continue;
                }
                to[k++] = kCompound | ((X & kIdMask) << 31) | (Y & kIdMask) |
                          ((X | Y) & kRemoved);     // XDeleted orelse YDeleted
            }
        }
    }
};

__device__ __forceinline__ uint32_t tab_index(u64 key, uint64_t i, int per_entry, uint32_t ntab,
                                              uint32_t* flag) {
    if (!per_entry && (key & kPair)) {
        lraise(flag, kErrTable);
        return kNone;
    }
    const u64 idx = per_entry ? i : (key & kIdMask);
    if (idx >= ntab) {
        lraise(flag, kErrTable);
        return kNone;
    }
    return (uint32_t)idx;
}

// map body: {F(X), C} / F(X) in list order — keys replaced, tokens kept
struct PMap {
    LV src;
    const u64* tab;
    uint32_t ntab;
    int per_entry;
    uint32_t* flag;
    __device__ u64 items(u64 r) const { return src.n(r); }
    __device__ C2 count(u64 r, u64 i) const {
        return pk2(1, src.O(r)[i + 1] - src.O(r)[i]);
    }
    __device__ void write(u64 r, u64 i, uint32_t pos, uint32_t tpos, LV out) const {
        const uint32_t idx = tab_index(src.K(r)[i], i, per_entry, ntab, flag);
        const u64 k = idx == kNone ? 0 : tab[idx];
        if (k == kEmpty) lraise(flag, kErrFun);     // Function(X) raised
        out.K(r)[pos] = k;
        out.O(r)[pos] = tpos;
        const uint32_t* O = src.O(r);
        const u64* from = src.T(r) + O[i];
        for (uint32_t t = 0; t < O[i + 1] - O[i]; ++t) out.T(r)[tpos + t] = from[t];
    }
};

// filter body: keep {X, C} / X when F(X) =:= true (tombstoned entries included)
struct PFilter {
    LV src;
    const uint8_t* keep;
    uint32_t ntab;
    int per_entry;
    uint32_t* flag;
    __device__ u64 items(u64 r) const { return src.n(r); }
    __device__ C2 count(u64 r, u64 i) const {
        const uint32_t idx = tab_index(src.K(r)[i], i, per_entry, ntab, flag);
        if (idx == kNone) return C2{0, 0};
        if (keep[idx] == 2) lraise(flag, kErrFun);   // Function(V) raised
        if (keep[idx] != 1) return C2{0, 0};
        return pk2(1, src.O(r)[i + 1] - src.O(r)[i]);
    }
    __device__ void write(u64 r, u64 i, uint32_t pos, uint32_t tpos, LV out) const {
        const uint32_t* O = src.O(r);
        out.K(r)[pos] = src.K(r)[i];
        out.O(r)[pos] = tpos;
        const u64* from = src.T(r) + O[i];
        for (uint32_t t = 0; t < O[i + 1] - O[i]; ++t) out.T(r)[tpos + t] = from[t];
    }
};

// fold body: [{V, C} || V <- F(X)] / F(X), concatenated in list order
struct PFold {
    LV src;
    const uint32_t* off;
    const u64* keys;
    uint32_t ntab;
    int per_entry;
    uint32_t* flag;
    __device__ u64 items(u64 r) const { return src.n(r); }
    __device__ C2 count(u64 r, u64 i) const {
        const uint32_t idx = tab_index(src.K(r)[i], i, per_entry, ntab, flag);
        if (idx == kNone) return C2{0, 0};
        const uint32_t k = off[idx + 1] - off[idx], len = src.O(r)[i + 1] - src.O(r)[i];
        for (uint32_t v = 0; v < k; ++v)
            if (keys[off[idx] + v] == kEmpty) lraise(flag, kErrFun);
        if ((u64)k * len > 0xFFFFFFFFull) {
            lraise(flag, kErrRange);
            return C2{0, 0};
        }
        return pk2(k, k * len);
    }
    __device__ void write(u64 r, u64 i, uint32_t pos, uint32_t tpos, LV out) const {
        const uint32_t idx = tab_index(src.K(r)[i], i, per_entry, ntab, flag);
        const uint32_t* O = src.O(r);
        const uint32_t k = off[idx + 1] - off[idx], len = O[i + 1] - O[i];
        const u64* from = src.T(r) + O[i];
        for (uint32_t v = 0; v < k; ++v) {
            out.K(r)[pos + v] = keys[off[idx] + v];
            out.O(r)[pos + v] = tpos + v * len;
            for (uint32_t t = 0; t < len; ++t) out.T(r)[tpos + v * len + t] = from[t];
        }
    }
};

}  // namespace

}  // namespace laspj

// ================================================================ runtime + C ABI

using laspj::fail;
using namespace laspj;

namespace {

struct LGuard {
    std::lock_guard<std::mutex> lk;
    explicit LGuard(laspj_ctx* c) : lk(c->mu) { hipSetDevice(c->device); }
};

uint64_t list_wpr(uint32_t ce, uint32_t ct) {
    return (8ull + 8ull * ce + 8ull * ct + 4ull * ((uint64_t)ce + 1) + 7ull) / 8ull;
}

LV view(const laspj_batch* b) {
    LV v;
    char* base = reinterpret_cast<char*>(b->dev);
    const uint64_t R = b->replicas;
    v.hdr = reinterpret_cast<uint32_t*>(base);
    base += R * 8ull;
    v.key = reinterpret_cast<u64*>(base);
    base += R * 8ull * b->cap_e;
    v.tok = reinterpret_cast<u64*>(base);
    base += R * 8ull * b->cap_t;
    v.toff = reinterpret_cast<uint32_t*>(base);
    v.ce = b->cap_e;
    v.ct = b->cap_t;
    return v;
}

// (re)allocate a list batch's device memory for caps (ce, ct); contents: empty lists
// zero: clear the new block (empty lists); otherwise its contents are undefined until the
// caller's write pass (known counts = the capacities until then)
int list_alloc(laspj_ctx* ctx, laspj_batch* b, uint32_t ce, uint32_t ct, bool zero = true) {
    if (ce == 0) ce = 1;
    if (ct == 0) ct = 1;
    const uint64_t wpr = list_wpr(ce, ct);
    if (b->replicas > (~0ull / 8ull) / wpr)
        return fail(ctx, LASPJ_E_SHAPE, "list: size overflow");
    const uint64_t bytes = b->replicas * wpr * 8ull;
    void* p = nullptr;
    hipError_t e = laspj::dev_alloc(ctx, bytes, &p);
    if (e != hipSuccess) {
        hipGetLastError();
        return fail(ctx, LASPJ_E_NOMEM, "list: hipMalloc(%llu): %s", (unsigned long long)bytes,
                    hipGetErrorString(e));
    }
    if (zero) e = hipMemsetAsync(p, 0, bytes, ctx->stream);
    if (e != hipSuccess) {
        laspj::dev_release(ctx, p, bytes);
        return fail(ctx, LASPJ_E_DEVICE, "list: memset: %s", hipGetErrorString(e));
    }
    if (b->dev) laspj::dev_release(ctx, b->dev, laspj::bytes_of(b));
    b->dev = static_cast<uint64_t*>(p);
    b->cap_e = ce;
    b->cap_t = ct;
    b->known_e = zero ? 0 : ce;
    b->known_t = zero ? 0 : ct;
    b->not_asc = false;
    b->no_spec = false;
    b->words_per_replica = wpr;
    b->elements = ce;
    b->cells = ce;
    return LASPJ_OK;
}

void* lscratch(laspj_ctx* ctx, uint64_t bytes) {
    if (bytes == 0) bytes = 8;
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

int check_list(laspj_ctx* ctx, const laspj_batch* b, const char* what) {
    if (!b || b->ctx != ctx) return fail(ctx, LASPJ_E_INVAL, "%s: null batch or other context", what);
    if (!laspj_is_list(b->kind)) return fail(ctx, LASPJ_E_KIND, "%s: not a list batch", what);
    return LASPJ_OK;
}

int ranks(laspj_ctx* ctx, const laspj_list_order* ord, bool need_tokens, RK* rk,
          const char* what) {
    if (!ord || !ord->krank || ord->krank->ctx != ctx)
        return fail(ctx, LASPJ_E_INVAL, "%s: rank tables missing", what);
    if ((uint64_t)ord->nkeys * 4ull > ord->krank->bytes)
        return fail(ctx, LASPJ_E_RANGE, "%s: krank holds fewer than %u ranks", what, ord->nkeys);
    rk->krank = static_cast<const uint32_t*>(ord->krank->dev);
    rk->nk = ord->nkeys;
    rk->grank = nullptr;
    rk->ng = 0;
    if (ord->grank) {
        if (ord->grank->ctx != ctx) return fail(ctx, LASPJ_E_INVAL, "%s: grank context", what);
        if ((uint64_t)ord->ntokens * 4ull > ord->grank->bytes)
            return fail(ctx, LASPJ_E_RANGE, "%s: grank holds fewer than %u ranks", what,
                        ord->ntokens);
        rk->grank = static_cast<const uint32_t*>(ord->grank->dev);
        rk->ng = ord->ntokens;
    } else if (need_tokens) {
        return fail(ctx, LASPJ_E_INVAL, "%s: OR-Set lists need token ranks", what);
    }
    rk->flag = ctx->flag + 1;
    return LASPJ_OK;
}

uint32_t pow2_at_least(uint64_t n) {
    uint64_t h = 64;
    while (h < n) h <<= 1;
    return (uint32_t)h;
}

int flag_status(laspj_ctx* ctx, uint32_t f, const char* what) {
    if (f & kErrFun)
        return fail(ctx, LASPJ_E_FUN, "%s: the fun failed on a key of the list", what);
    if (f & kErrNested)
        return fail(ctx, LASPJ_E_UNSUPPORTED, "%s: product of product outputs (nested pairs)",
                    what);
    if (f & kErrId) return fail(ctx, LASPJ_E_RANGE, "%s: item outside the rank tables", what);
    if (f & kErrTable) return fail(ctx, LASPJ_E_RANGE, "%s: table index out of range", what);
    if (f & kErrRange) return fail(ctx, LASPJ_E_RANGE, "%s: output capacity exceeded", what);
    return LASPJ_OK;
}

int read_flag(laspj_ctx* ctx, const char* what) {
    uint32_t f = 0;
    LJ_HIP(ctx, laspj::readback(ctx, &f, ctx->flag + 1, 4));
    return flag_status(ctx, f, what);
}

// run a size pass, size dst from the per-replica maxima, then the write pass
template <class SizeFn, class WriteFn>
int sized(laspj_ctx* ctx, laspj_batch* dst, uint32_t* need, SizeFn size_pass, WriteFn write_pass,
          const char* what) {
    const uint64_t R = dst->replicas;
    size_pass();
    LJ_LAUNCHED(ctx);
    std::vector<uint32_t> h(2 * R);
    uint32_t f = 0;
    const laspj::ReadPiece rp[2] = {{h.data(), need, 8ull * R}, {&f, ctx->flag + 1, 4}};
    LJ_HIP(ctx, laspj::readback(ctx, rp, 2));
    if (int s = flag_status(ctx, f, what)) return s;
    uint32_t ce = 0, ct = 0;
    for (uint64_t i = 0; i < R; ++i) {
        ce = h[2 * i] > ce ? h[2 * i] : ce;
        ct = h[2 * i + 1] > ct ? h[2 * i + 1] : ct;
    }
    if (ce > dst->cap_e || ct > dst->cap_t)
        if (int s = list_alloc(ctx, dst, ce > dst->cap_e ? ce : dst->cap_e,
                               ct > dst->cap_t ? ct : dst->cap_t))
            return s;
    write_pass(view(dst));
    LJ_LAUNCHED(ctx);
    dst->known_e = ce;
    dst->known_t = ct;
    return read_flag(ctx, what);
}

// a tiled producer (k_tp_*): `pre` carves its own scratch from the front of the block
// (pre_bytes), enqueues whatever must run first and returns the functor.
// ub_e / ub_t (0: none): upper bounds of the output's entries / tokens per replica the
// host knows, true in the usual case: dst sized to them, the count, scan and write passes
// run back to back and one readback brings the sizes and the flag.  When the write pass
// finds dst short after all (kErrRange: the bound did not hold), dst is sized from the
// counts, which are still in the scratch, and the write pass runs again.
template <class P, class Pre>
int tiled(laspj_ctx* ctx, laspj_batch* dst, uint64_t max_items, uint64_t pre_bytes, Pre pre,
          const char* what, uint64_t ub_e = 0, uint64_t ub_t = 0) {
    const uint64_t R = dst->replicas;
    const uint64_t nt64 = max_items ? (max_items + kPTile - 1) / kPTile : 1;
    if (nt64 > 0x7FFFFFFFull) return fail(ctx, LASPJ_E_RANGE, "%s: lists too long", what);
    const uint32_t ntile = (uint32_t)nt64;
    const uint64_t pb = (pre_bytes + 63) & ~63ull;
    char* base = static_cast<char*>(lscratch(ctx, pb + sizeof(C2) * R * ntile + 8ull * R));
    if (!base) return fail(ctx, LASPJ_E_NOMEM, "%s: scratch", what);
    C2* tc = reinterpret_cast<C2*>(base + pb);
    auto* need = reinterpret_cast<uint32_t*>(base + pb + sizeof(C2) * R * ntile);
    uint32_t* flag = ctx->flag + 1;
    LJ_HIP(ctx, hipMemsetAsync(flag, 0, 4, ctx->stream));
    const P p = pre(base);
    const dim3 grid(ntile, (unsigned)(R < 65535 ? R : 65535));
    const unsigned sg = (unsigned)(R < 65535 ? R : 65535);
    if (ub_e && ub_t && ub_e <= 0xFFFFFFF0ull && ub_t <= 0xFFFFFFF0ull) {
        const bool gs = dst->kind == LASPJ_KIND_GSET_LIST;
        if (ub_e > dst->cap_e || ub_t > dst->cap_t)
            if (int s = list_alloc(ctx, dst, ub_e > dst->cap_e ? (uint32_t)ub_e : dst->cap_e,
                                   ub_t > dst->cap_t ? (uint32_t)ub_t : dst->cap_t, gs))
                return s;
        hipLaunchKernelGGL((k_tp_count<P>), grid, dim3(kPT), 0, ctx->stream, p, tc, ntile, R);
        hipLaunchKernelGGL(k_tp_scan, dim3(sg), dim3(kPT), 0, ctx->stream, tc, ntile, R, need,
                           flag);
        hipLaunchKernelGGL((k_tp_write<P>), grid, dim3(kPT), 0, ctx->stream, p, view(dst), tc,
                           ntile, R, need, flag);
        LJ_LAUNCHED(ctx);
        std::vector<uint32_t> h(2 * R);
        uint32_t f = 0;
        const laspj::ReadPiece rp[2] = {{h.data(), need, 8ull * R}, {&f, flag, 4}};
        LJ_HIP(ctx, laspj::readback(ctx, rp, 2));
        uint32_t ce = 0, ct = 0;
        for (uint64_t i = 0; i < R; ++i) {
            ce = h[2 * i] > ce ? h[2 * i] : ce;
            ct = h[2 * i + 1] > ct ? h[2 * i + 1] : ct;
        }
        if (f == kErrRange && ce < 0xFFFFFFFFu && ct < 0xFFFFFFFFu &&
            (ce > dst->cap_e || ct > dst->cap_t)) {
            // the bound did not hold: dst from the counts, the write pass again
            if (int s = list_alloc(ctx, dst, ce > dst->cap_e ? ce : dst->cap_e,
                                   ct > dst->cap_t ? ct : dst->cap_t, gs))
                return s;
            LJ_HIP(ctx, hipMemsetAsync(flag, 0, 4, ctx->stream));
            hipLaunchKernelGGL((k_tp_write<P>), grid, dim3(kPT), 0, ctx->stream, p, view(dst),
                               tc, ntile, R, need, flag);
            LJ_LAUNCHED(ctx);
            LJ_HIP(ctx, laspj::readback(ctx, &f, flag, 4));
        }
        if (int s = flag_status(ctx, f, what)) {
            dst->known_e = dst->cap_e, dst->known_t = dst->cap_t;      // contents undefined
            return s;
        }
        dst->known_e = ce;
        dst->known_t = ct;
        return LASPJ_OK;
    }
    return sized(
        ctx, dst, need,
        [&] {
            hipLaunchKernelGGL((k_tp_count<P>), grid, dim3(kPT), 0, ctx->stream, p, tc, ntile, R);
            hipLaunchKernelGGL(k_tp_scan, dim3(sg), dim3(kPT), 0, ctx->stream, tc, ntile, R, need,
                               flag);
        },
        [&](LV out) {
            hipLaunchKernelGGL((k_tp_write<P>), grid, dim3(kPT), 0, ctx->stream, p, out, tc, ntile,
                               R, need, flag);
        },
        what);
}

}  // namespace

extern "C" {

int laspj_list_batch_create(laspj_ctx* ctx, int32_t kind, uint64_t replicas,
                            uint32_t cap_entries, uint32_t cap_tokens, laspj_batch** out) {
    if (!ctx || !out) return fail(ctx, LASPJ_E_INVAL, "list_batch_create: null argument");
    *out = nullptr;
    if (!laspj_is_list(kind)) return fail(ctx, LASPJ_E_KIND, "list_batch_create: kind");
    if (replicas == 0) return fail(ctx, LASPJ_E_SHAPE, "list_batch_create: no replicas");
    if (replicas > 0x7FFFFFFFull)
        return fail(ctx, LASPJ_E_SHAPE, "list_batch_create: at most 2^31-1 replicas");
    LGuard g(ctx);
    auto* b = new (std::nothrow) laspj_batch;
    if (!b) return fail(ctx, LASPJ_E_NOMEM, "list_batch_create: host allocation");
    b->ctx = ctx;
    b->kind = kind;
    b->replicas = replicas;
    if (int s = list_alloc(ctx, b, cap_entries, kind == LASPJ_KIND_GSET_LIST ? 1 : cap_tokens)) {
        delete b;
        return s;
    }
    *out = b;
    return LASPJ_OK;
}

int laspj_list_counts(laspj_ctx* ctx, const laspj_batch* b, uint32_t* out) {
    if (int s = check_list(ctx, b, "list_counts")) return s;
    if (!out) return fail(ctx, LASPJ_E_INVAL, "list_counts: null output");
    LGuard g(ctx);
    LJ_HIP(ctx, laspj::readback(ctx, out, b->dev, 8ull * b->replicas));
    return LASPJ_OK;
}

int laspj_list_upload(laspj_ctx* ctx, laspj_batch* b, uint64_t replica, uint32_t n,
                      const uint64_t* keys, const uint32_t* toff, const uint64_t* toks) {
    if (int s = check_list(ctx, b, "list_upload")) return s;
    const bool gs = b->kind == LASPJ_KIND_GSET_LIST;
    if (replica >= b->replicas) return fail(ctx, LASPJ_E_RANGE, "list_upload: replica");
    if ((n && !keys) || (!gs && !toff))
        return fail(ctx, LASPJ_E_INVAL, "list_upload: null arrays");
    uint32_t nt = 0;
    if (!gs) {
        if (toff[0] != 0) return fail(ctx, LASPJ_E_INVAL, "list_upload: toff[0] != 0");
        for (uint32_t i = 0; i < n; ++i)
            if (toff[i + 1] < toff[i])
                return fail(ctx, LASPJ_E_INVAL, "list_upload: toff not ascending");
        nt = toff[n];
        if (nt && !toks) return fail(ctx, LASPJ_E_INVAL, "list_upload: null tokens");
    }
    LGuard g(ctx);
    if (n > b->cap_e || nt > b->cap_t) {
        // keep the other replicas: only a 1-replica batch grows here
        if (b->replicas != 1)
            return fail(ctx, LASPJ_E_RANGE, "list_upload: list exceeds the batch capacity");
        if (int s = list_alloc(ctx, b, n > b->cap_e ? n : b->cap_e, nt > b->cap_t ? nt : b->cap_t))
            return s;
    }
    b->not_asc = false;                    // (hints: list_bind tries the ascending path,
    b->no_spec = false;                    //  merges the chunked walk)
    if (b->replicas == 1) {
        b->known_e = n;
        b->known_t = nt;
    } else {
        b->known_e = n > b->known_e ? n : b->known_e;
        b->known_t = nt > b->known_t ? nt : b->known_t;
    }
    LV v = view(b);
    uint32_t hdr[2] = {n, nt};
    LJ_HIP(ctx, hipMemcpyAsync(v.hdr + 2 * replica, hdr, 8, hipMemcpyHostToDevice, ctx->stream));
    if (n)
        LJ_HIP(ctx, hipMemcpyAsync(v.key + replica * v.ce, keys, 8ull * n, hipMemcpyHostToDevice,
                                   ctx->stream));
    if (!gs) {
        LJ_HIP(ctx, hipMemcpyAsync(v.toff + replica * ((uint64_t)v.ce + 1), toff, 4ull * (n + 1),
                                   hipMemcpyHostToDevice, ctx->stream));
        if (nt)
            LJ_HIP(ctx, hipMemcpyAsync(v.tok + replica * (uint64_t)v.ct, toks, 8ull * nt,
                                       hipMemcpyHostToDevice, ctx->stream));
    }
    LJ_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return LASPJ_OK;
}

int laspj_list_download(laspj_ctx* ctx, const laspj_batch* b, uint64_t replica, uint64_t* keys,
                        uint32_t* toff, uint64_t* toks) {
    if (int s = check_list(ctx, b, "list_download")) return s;
    if (replica >= b->replicas) return fail(ctx, LASPJ_E_RANGE, "list_download: replica");
    const bool gs = b->kind == LASPJ_KIND_GSET_LIST;
    LGuard g(ctx);
    LV v = view(b);
    uint32_t hdr[2];
    LJ_HIP(ctx, laspj::readback(ctx, hdr, v.hdr + 2 * replica, 8));
    if ((hdr[0] && !keys) || (!gs && (!toff || (hdr[1] && !toks))))
        return fail(ctx, LASPJ_E_INVAL, "list_download: null arrays");
    if (hdr[0])
        LJ_HIP(ctx, hipMemcpyAsync(keys, v.key + replica * v.ce, 8ull * hdr[0],
                                   hipMemcpyDeviceToHost, ctx->stream));
    if (!gs) {
        LJ_HIP(ctx, hipMemcpyAsync(toff, v.toff + replica * ((uint64_t)v.ce + 1),
                                   4ull * (hdr[0] + 1), hipMemcpyDeviceToHost, ctx->stream));
        if (hdr[1])
            LJ_HIP(ctx, hipMemcpyAsync(toks, v.tok + replica * (uint64_t)v.ct, 8ull * hdr[1],
                                       hipMemcpyDeviceToHost, ctx->stream));
    }
    LJ_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return LASPJ_OK;
}

int laspj_list_from_set(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                        const laspj_buf* elem_order, uint32_t nslots, const laspj_buf* tok_order) {
    if (int s = check_list(ctx, dst, "list_from_set")) return s;
    if (!src || src->ctx != ctx) return fail(ctx, LASPJ_E_INVAL, "list_from_set: src");
    const bool gs = src->kind == LASPJ_KIND_GSET;
    if (!(src->kind == LASPJ_KIND_ORSET || gs) ||
        dst->kind != (gs ? LASPJ_KIND_GSET_LIST : LASPJ_KIND_ORSET_LIST))
        return fail(ctx, LASPJ_E_KIND, "list_from_set: OR-Set -> OR-Set list, G-Set -> G-Set list");
    if (dst->replicas != src->replicas) return fail(ctx, LASPJ_E_SHAPE, "list_from_set: replicas");
    if (!elem_order || elem_order->ctx != ctx || (uint64_t)nslots * 4 > elem_order->bytes ||
        nslots > src->elements)
        return fail(ctx, LASPJ_E_RANGE, "list_from_set: element order");
    if (!gs && (!tok_order || tok_order->ctx != ctx ||
                tok_order->bytes < 64ull * src->elements))
        return fail(ctx, LASPJ_E_RANGE, "list_from_set: token order (64 bytes per slot)");
    if ((uint64_t)src->elements * 64ull > kIdMask)
        return fail(ctx, LASPJ_E_RANGE, "list_from_set: too many element slots for token ids");
    // element slots in elem_order must be < E: the kernels raise kErrId (E_RANGE) on one
    // that is not, so no copy of the order comes back to the host
    LGuard g(ctx);
    const auto* ordp = static_cast<const uint32_t*>(elem_order->dev);
    const auto* tordp = gs ? nullptr : static_cast<const uint8_t*>(tok_order->dev);
    const auto* sp = reinterpret_cast<const u64*>(src->dev);
    const uint64_t wpr = src->words_per_replica;
    const uint32_t E = src->elements;
    uint32_t* flag = ctx->flag + 1;
    // one entry per slot at most, 64 tokens per entry at most: exact bounds, used for a
    // single pass while the tokens' block stays small (256 MiB)
    const uint64_t R = src->replicas, ub_e = nslots ? nslots : 1;
    const uint64_t ub_t = gs ? 1 : 64ull * ub_e;
    const bool one = R * ub_t * 8ull <= (256ull << 20);
    if (gs)
        return tiled<PFromSet<true>>(ctx, dst, nslots, 0, [&](char*) {
            return PFromSet<true>{sp, wpr, ordp, nslots, E, tordp, flag};
        }, "list_from_set", one ? ub_e : 0, one ? ub_t : 0);
    return tiled<PFromSet<false>>(ctx, dst, nslots, 0, [&](char*) {
        return PFromSet<false>{sp, wpr, ordp, nslots, E, tordp, flag};
    }, "list_from_set", one ? ub_e : 0, one ? ub_t : 0);
}

static int pair_checks(laspj_ctx* ctx, const laspj_batch* dst, const laspj_batch* a,
                       const laspj_batch* b, const char* what) {
    if (int s = check_list(ctx, dst, what)) return s;
    if (int s = check_list(ctx, a, what)) return s;
    if (int s = check_list(ctx, b, what)) return s;
    if (a->kind != b->kind || dst->kind != a->kind)
        return fail(ctx, LASPJ_E_KIND, "%s: list kinds differ", what);
    if (a->replicas != b->replicas || dst->replicas != a->replicas)
        return fail(ctx, LASPJ_E_SHAPE, "%s: replica counts differ", what);
    if (dst == a || dst == b) return fail(ctx, LASPJ_E_INVAL, "%s: dst aliases an input", what);
    return LASPJ_OK;
}

// The merge proper, with the context's lock held and the arguments checked.  A merge has
// at most the entries and the tokens of both inputs together, so dst is sized from the
// inputs' known counts and the size pass and the write pass run back to back: the caller
// synchronises once, reading `need` (per replica {entries, tokens}), the error flag and
// whatever it enqueued after (the bind's equality and inflation bytes).  eq (R bytes, or
// null): `cur =:= val` per replica, launched first.
// words (or null: the scratch and ctx's error word): 2R + 3 words of the caller's,
// zeroed here in one memset — [rk.flag (the caller points rk.flag at words[0]) |
// unsorted R | tickets 2 | aweak R] — for a caller that reads them after other users of
// the scratch (list_bind's inflation reads `aweak`: words + R + 3)
static int grow_block(laspj_ctx* ctx, void** p, uint64_t* have, uint64_t bytes, bool zero,
                      const char* what);

// spec: replicas whose keys descend take the chunked walk (k_merge_spec) — asked for when
// an input is known not to ascend (laspj_batch::not_asc), as it costs a launch otherwise
static int merge_enqueue(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* a,
                         const laspj_batch* b, const RK& rk, bool keep_left, uint32_t* need,
                         uint8_t* eq, const char* what, uint32_t* words = nullptr,
                         uint64_t words_bytes = 0, const Ins* ins = nullptr,
                         bool spec = false) {
    // (words_bytes == 0 with words: they are known zero already, no memset)
    const bool gs = a->kind == LASPJ_KIND_GSET_LIST;
    const uint64_t R = a->replicas;
    const uint64_t ce = (uint64_t)a->cap_e + b->cap_e;
    if (ce > 0xFFFFFFF0ull) return fail(ctx, LASPJ_E_RANGE, "%s: lists too long", what);
    const uint64_t be = (uint64_t)a->known_e + b->known_e;
    const uint64_t bt = gs ? 1ull : (uint64_t)a->known_t + b->known_t;
    if (be > 0xFFFFFFF0ull || bt > 0xFFFFFFF0ull)
        return fail(ctx, LASPJ_E_RANGE, "%s: lists too long", what);
    // OR-Set lists: the write pass writes every word a reader looks at (header, keys,
    // token offsets, tokens), so a fresh block is not cleared; G-Set lists keep zero token
    // offsets, which the write pass does not write (k_list_equal compares them)
    if (be > dst->cap_e || bt > dst->cap_t)
        if (int s = list_alloc(ctx, dst, be > dst->cap_e ? (uint32_t)be : dst->cap_e,
                               bt > dst->cap_t ? (uint32_t)bt : dst->cap_t, gs))
            return s;
    MS m;
    m.ce_a = a->cap_e;
    m.ce_b = b->cap_e;
    m.ntiles = (uint32_t)((ce + kMTile - 1) / kMTile);
    m.nchunks = (uint32_t)((ce + kMT - 1) / kMT);
    // scratch: ranks, plan, token counts, tile / chunk scans, per-replica words
    const uint64_t sz_sa = R * 8ull * m.ce_a, sz_sb = R * 8ull * m.ce_b, sz_pl = R * 8ull * ce,
                   sz_tc = R * 4ull * ce, sz_t = R * 4ull * m.ntiles, sz_c = R * 4ull * m.nchunks,
                   sz_r = R * 4ull;
    // the chunked walk: L rows per chunk, C chunks (a multiple of kSpW, at most 1024)
    const bool fuse0 = R <= 4 && ctx->tune_list_walk != 1;
    uint32_t spL = 256, spC = 0;
    if (((spec && !a->no_spec && !b->no_spec) || ctx->tune_list_walk == 3) && fuse0 &&
        a->known_e) {
        spL = (uint32_t)std::max<uint64_t>(ctx->tune_list_chunk ? ctx->tune_list_chunk : 1024,
                                           (a->known_e + 1023) / 1024);
        spC = (uint32_t)((((uint64_t)a->known_e + spL - 1) / spL + kSpW - 1) / kSpW * kSpW);
        if (spL >= (1u << 20)) spC = 0;
    }
    const uint64_t sz_fr = spC ? R * 4ull * m.ce_a : 0;
    // chunk maxima for the one-wave walk's long runs, when an input is known not to ascend
    const bool maxima = (spec || ctx->tune_list_walk == 3) && ctx->tune_list_walk != 1;
    const uint32_t nca = (m.ce_a + 1023u) / 1024u, ncb = (m.ce_b + 1023u) / 1024u;
    const uint32_t nba = (m.ce_a + kMT - 1) / kMT, nbb = (m.ce_b + kMT - 1) / kMT;
    const uint64_t sz_mx = maxima ? R * 8ull * ((uint64_t)nba + nbb) : 0;
    const uint64_t total = sz_sa + sz_sb + sz_pl + sz_tc + 6 * sz_t + sz_c + 5 * sz_r + 72 + sz_fr +
                           sz_mx + 16;
    char* base = static_cast<char*>(lscratch(ctx, total));
    if (!base) return fail(ctx, LASPJ_E_NOMEM, "%s: scratch", what);
    char* q = base;
    auto take = [&](uint64_t bytes) {
        char* p = q;
        q += (bytes + 7) & ~7ull;
        return p;
    };
    m.sa = reinterpret_cast<u64*>(take(sz_sa));
    m.sb = reinterpret_cast<u64*>(take(sz_sb));
    m.plan = reinterpret_cast<u64*>(take(sz_pl));
    m.tcnt = reinterpret_cast<uint32_t*>(take(sz_tc));
    m.tile = reinterpret_cast<uint32_t*>(take(sz_t));
    m.tside = reinterpret_cast<uint32_t*>(take(sz_t));
    m.tsplit = reinterpret_cast<uint32_t*>(take(4 * sz_t));
    m.chunk = reinterpret_cast<uint32_t*>(take(sz_c));
    m.nout = reinterpret_cast<uint32_t*>(take(sz_r));
    m.ntok = reinterpret_cast<uint32_t*>(take(sz_r));
    if (maxima) {
        m.amax = reinterpret_cast<u64*>(take(sz_mx));
        m.bmax = m.amax + R * nba;
        m.nca = nca;
        m.ncb = ncb;
        m.nba = nba;
        m.nbb = nbb;
    }
    SP sp{};
    if (spC) {
        sp.fr = reinterpret_cast<uint32_t*>(take(sz_fr));
        sp.L = spL;
        sp.C = spC;
        const uint64_t zb = R * 8ull * (kSpWords + 2ull * spC);
        if (int s = grow_block(ctx, &ctx->lspec, &ctx->lspec_bytes, std::max<uint64_t>(zb, 1 << 16),
                               ctx->lspec_dirty, what))
            return s;
        sp.w = static_cast<u64*>(ctx->lspec);
        sp.flag = rk.flag;
        sp.cw = sp.w + R * kSpWords;
        m.spec = 1;
    }
    // [unsorted R | tickets 2 | aweak R], zeroed together
    m.unsorted = words ? words + 1 : reinterpret_cast<uint32_t*>(take(2 * sz_r + 8));
    uint32_t* tickets = m.unsorted + R;
    m.aweak = m.unsorted + R + 2;
    // few replicas: the tile scan rides in the counting pass's last block (one launch
    // fewer); many: its own launch, one block per replica
    const bool fuse = R <= 4 && ctx->tune_list_walk != 1;
    const LV A = view(a), B = view(b), OUT = view(dst);
    const unsigned ry = (unsigned)(R < 65535 ? R : 65535);
    const unsigned rx = (unsigned)(R < (1u << 20) ? R : (1u << 20));
    const uint32_t cmax = m.ce_a > m.ce_b ? m.ce_a : m.ce_b;
    const unsigned gr = cmax ? (cmax + kMT - 1) / kMT : 1u;
    if (words) {
        if (rk.flag != words) return fail(ctx, LASPJ_E_INVAL, "%s: error word", what);
        if (words_bytes) {
            const uint64_t wb = std::max<uint64_t>(words_bytes, (4 + 2 * sz_r + 8 + 15) & ~15ull);
            LJ_HIP(ctx, hipMemsetAsync(words, 0, wb, ctx->stream));
        }
    } else {
        LJ_HIP(ctx, hipMemsetAsync(ctx->flag + 1, 0, 4, ctx->stream));
    }
    if (eq)
        hipLaunchKernelGGL(k_list_equal, dim3(R), dim3(64), 0, ctx->stream, A, B, rk, eq);
    auto passes = [&](auto mode) {
        constexpr int MODE = decltype(mode)::value;
        if (!words) hipMemsetAsync(m.unsorted, 0, 2 * sz_r + 8, ctx->stream);
        hipLaunchKernelGGL(k_merge_ranks, dim3(gr, ry), dim3(kMT), 0, ctx->stream, A, B,
                           rk, m, R);
        if (spC) {
            // (its last block per replica zeroes the words again)
            hipLaunchKernelGGL(k_merge_spec<MODE>, dim3(spC / kSpW, ry), dim3(64 * kSpW), 0,
                               ctx->stream, A, B, m, sp, R);
        }
        hipLaunchKernelGGL((k_merge_tiles<MODE, false>), dim3(m.ntiles ? m.ntiles : 1, ry),
                           dim3(kMT), 0, ctx->stream, A, B, m, R,
                           fuse ? tickets : (uint32_t*)nullptr);
        // keys that descend somewhere: the run-jumping walk, in the scan's launch
        // (LASPJ_TUNE_LIST_WALK 1: the step-by-step walk it replaced, a launch of its own)
        if (ctx->tune_list_walk == 1) {
            hipLaunchKernelGGL((k_merge_tile_scan<MODE, false>), dim3(rx), dim3(kMT), 0,
                               ctx->stream, A, B, m, R);
            hipLaunchKernelGGL(k_merge_serial<MODE>, dim3(rx), dim3(64), 0, ctx->stream, A, B,
                               m, R);
        } else if (!fuse) {
            hipLaunchKernelGGL((k_merge_tile_scan<MODE, true>), dim3(rx), dim3(kMT), 0,
                               ctx->stream, A, B, m, R);
        }
        hipLaunchKernelGGL((k_merge_tiles<MODE, true>), dim3(m.ntiles ? m.ntiles : 1, ry),
                           dim3(kMT), 0, ctx->stream, A, B, m, R, (uint32_t*)nullptr);
        // (the chunk scan in the token count's last block measured slower: every one of
        // its ~400 blocks pays the ticket's agent-scope fence — profiles/r04t_*)
        hipLaunchKernelGGL((k_merge_tok_count<MODE>), dim3(m.nchunks ? m.nchunks : 1, ry),
                           dim3(kMT), 0, ctx->stream, A, B, rk, m, R, (uint32_t*)nullptr, need);
        hipLaunchKernelGGL(k_merge_chunk_scan, dim3(rx), dim3(kMT), 0, ctx->stream, m, R, need);
        // the write pass (it raises kErrRange rather than write past dst's capacity)
        hipLaunchKernelGGL((k_merge_write<MODE>), dim3(m.nchunks ? m.nchunks : 1, ry), dim3(kMT),
                           0, ctx->stream, A, B, OUT, rk, m, R,
                           ins ? *ins : Ins{nullptr, nullptr, 0, nullptr});
    };
    if (gs) passes(std::integral_constant<int, 2>{});
    else if (keep_left) passes(std::integral_constant<int, 1>{});
    else passes(std::integral_constant<int, 0>{});
    LJ_LAUNCHED(ctx);
    return LASPJ_OK;
}

// dst's known counts from the per-replica {entries, tokens} a merge read back
static void set_known(laspj_batch* dst, const uint32_t* h, uint64_t R) {
    uint32_t ce = 0, ct = 0;
    for (uint64_t i = 0; i < R; ++i) {
        ce = h[2 * i] > ce ? h[2 * i] : ce;
        ct = h[2 * i + 1] > ct ? h[2 * i + 1] : ct;
    }
    dst->known_e = ce;
    dst->known_t = ct;
    dst->not_asc = false;
    dst->no_spec = false;
}

static int merge_impl(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* a,
                      const laspj_batch* b, const laspj_list_order* ord, bool keep_left,
                      const char* what) {
    if (int s = pair_checks(ctx, dst, a, b, what)) return s;
    RK rk;
    if (int s = ranks(ctx, ord, a->kind != LASPJ_KIND_GSET_LIST, &rk, what)) return s;
    LGuard g(ctx);
    const uint64_t R = a->replicas;
    void* dev = nullptr;
    if (laspj::dev_alloc(ctx, 8 * R, &dev) != hipSuccess) {
        hipGetLastError();
        return fail(ctx, LASPJ_E_NOMEM, "%s: sizes", what);
    }
    auto* need = static_cast<uint32_t*>(dev);
    int s = merge_enqueue(ctx, dst, a, b, rk, keep_left, need, nullptr, what, nullptr, 0, nullptr,
                          a->not_asc || b->not_asc);
    std::vector<uint32_t> h(2 * R);
    if (s == LASPJ_OK) {
        uint32_t f = 0;
        const laspj::ReadPiece rp[2] = {{h.data(), need, 8ull * R}, {&f, ctx->flag + 1, 4}};
        const hipError_t e = laspj::readback(ctx, rp, 2);
        s = e != hipSuccess ? fail(ctx, LASPJ_E_DEVICE, "%s: readback: %s", what,
                                   hipGetErrorString(e))
                            : flag_status(ctx, f, what);
        if (f & kInfoWalkFell) a->no_spec = b->no_spec = true;
    }
    laspj::dev_release(ctx, dev, 8 * R);
    if (s != LASPJ_OK) {
        dst->known_e = dst->cap_e, dst->known_t = dst->cap_t;     // contents undefined
        return s;
    }
    set_known(dst, h.data(), R);
    return LASPJ_OK;
}

// list_bind's keyfind tables: ctx->ltab, at least `bytes`, all zero (zeroed here when new
// or when a call may have left them used); marked in use until the caller's clean-up is
// enqueued.  Null (and the context's error set) when it cannot be allocated.
static char* bind_tables(laspj_ctx* ctx, uint64_t bytes, const char* what) {
    if (ctx->ltab_bytes < bytes || ctx->ltab_dirty) {
        if (ctx->ltab_bytes < bytes) {
            if (ctx->ltab) {
                hipStreamSynchronize(ctx->stream);
                hipFree(ctx->ltab);
                ctx->ltab = nullptr;
                ctx->ltab_bytes = 0;
            }
            if (laspj::dev_malloc(ctx, &ctx->ltab, bytes) != hipSuccess) {
                hipGetLastError();
                fail(ctx, LASPJ_E_NOMEM, "%s: keyfind tables", what);
                return nullptr;
            }
            ctx->ltab_bytes = bytes;
        }
        if (hipMemsetAsync(ctx->ltab, 0, ctx->ltab_bytes, ctx->stream) != hipSuccess) {
            fail(ctx, LASPJ_E_DEVICE, "%s: keyfind tables memset", what);
            return nullptr;
        }
    }
    ctx->ltab_dirty = true;
    return static_cast<char*>(ctx->ltab);
}

// the inflation kernels of prev -> cur into o (R bytes); clear_flag: start from a clean
// error flag (the fused bind keeps the merge's bits and reads them with o)
// final = false: the answer is left to the caller, which gets the flag words through
// *flag_words (list_bind: its equality pass's last block)
static int inflation_launch(laspj_ctx* ctx, const laspj_batch* prev, const laspj_batch* cur,
                            int strict, const RK& rk, uint8_t* o, bool clear_flag,
                            const char* what, uint32_t** zeroed_words = nullptr,
                            bool final = true, const uint32_t** flag_words = nullptr,
                            const uint32_t* skip = nullptr, uint32_t* zeroed_flags = nullptr,
                            u64** tab_k = nullptr, uint32_t** tab_i = nullptr,
                            uint32_t* tab_size = nullptr) {
    const bool gs = cur->kind == LASPJ_KIND_GSET_LIST;
    const bool bcast = prev->replicas == 1 && cur->replicas != 1;
    const uint64_t R = cur->replicas;
    const uint32_t cmax = cur->cap_e > prev->cap_e ? cur->cap_e : prev->cap_e;
    const uint32_t hsize = pow2_at_least(2ull * cmax);
    // (a second table only for the G-Set strict check's Prev keys)
    const uint64_t ntab = gs && strict ? 2 : 1;
    const uint64_t tbytes = R * ntab * hsize * 12ull;
    // [tables | flag words | R more zeroed words for the caller (zeroed_words)]
    // (a multiple of 256 bytes: the runtime fills an unaligned tail with a second kernel)
    const uint64_t zbytes = (tbytes + 4ull * R * (zeroed_words ? 2 : 1) + 255) & ~255ull;
    char* base = nullptr;
    uint32_t* flags = nullptr;
    if (zeroed_flags) {
        // list_bind: the tables kept zeroed in ctx->ltab (the caller's last kernel zeroes
        // what this check used) — acquired by the caller already when *tab_k is set (its
        // merge's write pass filled them: no insert launch), the flag words the caller's,
        // zeroed with its own
        if (tab_k && *tab_k) {
            base = reinterpret_cast<char*>(*tab_k);
            if (*tab_size != hsize) return fail(ctx, LASPJ_E_INVAL, "%s: table size", what);
        } else {
            base = bind_tables(ctx, tbytes, what);
            if (!base) return LASPJ_E_NOMEM;
        }
        flags = zeroed_flags;
        if (zeroed_words) *zeroed_words = flags + R;
    } else {
        base = static_cast<char*>(lscratch(ctx, zbytes));
        if (!base) return fail(ctx, LASPJ_E_NOMEM, "%s: scratch", what);
        flags = reinterpret_cast<uint32_t*>(base + tbytes);
        if (zeroed_words) *zeroed_words = flags + R;
        if (clear_flag) LJ_HIP(ctx, hipMemsetAsync(ctx->flag + 1, 0, 4, ctx->stream));
        // the tables (empty = zero) and the per-replica flag words, one memset
        LJ_HIP(ctx, hipMemsetAsync(base, 0, zbytes, ctx->stream));
    }
    u64* hk = reinterpret_cast<u64*>(base);
    auto* hi = reinterpret_cast<uint32_t*>(base + R * ntab * hsize * 8ull);
    if (flag_words) *flag_words = flags;
    const bool inserted = tab_k && *tab_k;
    if (tab_k) *tab_k = hk;
    if (tab_i) *tab_i = hi;
    if (tab_size) *tab_size = hsize;
    const LV P = view(prev), C = view(cur);
    const dim3 grid(cmax ? (cmax + 255) / 256 : 1, (unsigned)(R < 65535 ? R : 65535));
    const unsigned fg = (unsigned)((R + 255) / 256 < 4096 ? (R + 255) / 256 : 4096);
#define LJ_INFL(G, S)                                                                         \
    do {                                                                                      \
        if (!inserted)                                                                        \
            hipLaunchKernelGGL((k_linf_insert<G, S>), grid, dim3(256), 0, ctx->stream, P, C,   \
                               rk, hk, hi, hsize, bcast, R, skip);                            \
        hipLaunchKernelGGL((k_linf_probe<G, S>), grid, dim3(256), 0, ctx->stream, P, C, rk,    \
                           hk, hi, hsize, bcast, R, flags, skip);                             \
        if (final)                                                                            \
            hipLaunchKernelGGL((k_linf_final<G, S>), dim3(fg), dim3(256), 0, ctx->stream, P,   \
                               C, bcast, R, flags, o);                                        \
    } while (0)
    if (gs) {
        if (strict) LJ_INFL(true, true); else LJ_INFL(true, false);
    } else {
        if (strict) LJ_INFL(false, true); else LJ_INFL(false, false);
    }
#undef LJ_INFL
    LJ_LAUNCHED(ctx);
    return LASPJ_OK;
}

int laspj_list_merge(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* a,
                     const laspj_batch* b, const laspj_list_order* ord) {
    return merge_impl(ctx, dst, a, b, ord, false, "list_merge");
}

int laspj_list_union(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                     const laspj_batch* r, const laspj_list_order* ord) {
    if (l && l->kind == LASPJ_KIND_GSET_LIST) {
        if (int s = pair_checks(ctx, dst, l, r, "list_union")) return s;
        LGuard g(ctx);
        const LV L = view(l), Rr = view(r);
        return tiled<PConcat>(ctx, dst, (uint64_t)l->cap_e + r->cap_e, 0,
                              [&](char*) { return PConcat{L, Rr}; }, "list_union",
                              std::max<uint64_t>(1, (uint64_t)l->known_e + r->known_e), 1);
    }
    return merge_impl(ctx, dst, l, r, ord, true, "list_union");
}

int laspj_list_equal(laspj_ctx* ctx, const laspj_batch* a, const laspj_batch* b,
                     const laspj_list_order* ord, laspj_buf* out) {
    if (int s = check_list(ctx, a, "list_equal")) return s;
    if (int s = check_list(ctx, b, "list_equal")) return s;
    if (a->kind != b->kind) return fail(ctx, LASPJ_E_KIND, "list_equal: kinds differ");
    if (a->replicas != b->replicas) return fail(ctx, LASPJ_E_SHAPE, "list_equal: replicas");
    if (!out || out->ctx != ctx || out->bytes < a->replicas)
        return fail(ctx, LASPJ_E_RANGE, "list_equal: output buffer");
    RK rk;
    if (int s = ranks(ctx, ord, a->kind == LASPJ_KIND_ORSET_LIST, &rk, "list_equal")) return s;
    LGuard g(ctx);
    LJ_HIP(ctx, hipMemsetAsync(ctx->flag + 1, 0, 4, ctx->stream));
    hipLaunchKernelGGL(k_list_equal, dim3(a->replicas), dim3(64), 0, ctx->stream, view(a),
                       view(b), rk, static_cast<uint8_t*>(out->dev));
    LJ_LAUNCHED(ctx);
    return read_flag(ctx, "list_equal");
}

int laspj_list_inflation(laspj_ctx* ctx, const laspj_batch* prev, const laspj_batch* cur,
                         int strict, const laspj_list_order* ord, laspj_buf* out) {
    if (int s = check_list(ctx, prev, "list_inflation")) return s;
    if (int s = check_list(ctx, cur, "list_inflation")) return s;
    if (prev->kind != cur->kind) return fail(ctx, LASPJ_E_KIND, "list_inflation: kinds differ");
    const bool bcast = prev->replicas == 1 && cur->replicas != 1;
    if (!bcast && prev->replicas != cur->replicas)
        return fail(ctx, LASPJ_E_SHAPE, "list_inflation: replicas");
    if (!out || out->ctx != ctx || out->bytes < cur->replicas)
        return fail(ctx, LASPJ_E_RANGE, "list_inflation: output buffer");
    RK rk;
    if (int s = ranks(ctx, ord, cur->kind != LASPJ_KIND_GSET_LIST, &rk, "list_inflation"))
        return s;
    LGuard g(ctx);
    if (int s = inflation_launch(ctx, prev, cur, strict, rk, static_cast<uint8_t*>(out->dev),
                                 true, "list_inflation"))
        return s;
    return read_flag(ctx, "list_inflation");
}

// list_bind's answer block: pinned, coherent host memory the last block writes into
static int bind_answer(laspj_ctx* ctx, uint64_t hbytes) {
    if (ctx->lbind_h_bytes < hbytes) {
        if (ctx->lbind_h) {
            hipStreamSynchronize(ctx->stream);
            hipHostFree(ctx->lbind_h);
            ctx->lbind_h = nullptr;
            ctx->lbind_h_bytes = 0;
        }
        if (hipHostMalloc(&ctx->lbind_h, hbytes, hipHostMallocCoherent) != hipSuccess) {
            hipGetLastError();
            ctx->lbind_h = nullptr;
            return fail(ctx, LASPJ_E_NOMEM, "list_bind: pinned answer");
        }
        ctx->lbind_h_bytes = hbytes;
        LJ_HIP(ctx, hipHostGetDevicePointer(&ctx->lbind_hd, ctx->lbind_h, 0));
    }
    return LASPJ_OK;
}

// a device block of at least `bytes` in *p (grown), zeroed when new or `zero`
static int grow_block(laspj_ctx* ctx, void** p, uint64_t* have, uint64_t bytes, bool zero,
                      const char* what) {
    if (*have < bytes) {
        if (*p) {
            hipStreamSynchronize(ctx->stream);
            hipFree(*p);
            *p = nullptr;
            *have = 0;
        }
        if (laspj::dev_malloc(ctx, p, bytes) != hipSuccess) {
            hipGetLastError();
            *p = nullptr;
            return fail(ctx, LASPJ_E_NOMEM, "%s: device block", what);
        }
        *have = bytes;
        zero = true;
    }
    if (zero) LJ_HIP(ctx, hipMemsetAsync(*p, 0, *have, ctx->stream));
    return LASPJ_OK;
}

constexpr int kLfRetry = 1;     // list_bind_ascending: take the merge path instead

// list_bind over the rank universe when both lists' keys strictly ascend (k_lbf_*):
// LASPJ_OK with status / dst set, kLfRetry when a replica does not ascend (the lists are
// marked not_asc, so the next bind of them goes straight to the merge path), or an error
static int list_bind_ascending(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* cur,
                               const laspj_batch* val, const RK& rk, uint8_t* status) {
    const bool gs = cur->kind == LASPJ_KIND_GSET_LIST;
    const uint64_t R = cur->replicas, nk = rk.nk;
    const uint64_t be = (uint64_t)cur->known_e + val->known_e;
    const uint64_t bt = gs ? 1ull : (uint64_t)cur->known_t + val->known_t;
    if (be > dst->cap_e || bt > dst->cap_t)
        if (int s = list_alloc(ctx, dst, be > dst->cap_e ? (uint32_t)be : dst->cap_e,
                               bt > dst->cap_t ? (uint32_t)bt : dst->cap_t, gs))
            return s;
    const uint32_t ntiles = (uint32_t)std::max<uint64_t>(1, (nk + kLfTile - 1) / kLfTile);
    // this call's half of the zeroed block: [diff R | bad R] words, then the look-back words
    const uint64_t wbytes = (8 * R + 7) & ~7ull;
    const uint64_t use = wbytes + 8ull * R * ntiles;
    if (ctx->lfz_bytes < 2 * use || ctx->lfz_dirty) {
        const uint64_t want = std::max<uint64_t>({2 * use, ctx->lfz_bytes, 1 << 16});
        if (int s = grow_block(ctx, &ctx->lfz, &ctx->lfz_bytes, want, true, "list_bind"))
            return s;
        ctx->lf_prev_use = 0;                               // all zero now
    }
    const uint64_t ibytes = 16ull * R * std::max<uint64_t>(nk, 1);
    const bool grew = ctx->lfi_bytes < ibytes;
    if (++ctx->lf_epoch == 0 || grew) ctx->lf_epoch = 1;   // (a new block is all zero: epoch 0)
    if (int s = grow_block(ctx, &ctx->lfi, &ctx->lfi_bytes, ibytes, ctx->lf_epoch == 1 && !grew,
                           "list_bind"))
        return s;
    const uint64_t hbytes = 8 * R + 4 * ((R + 3) / 4) + 4;
    if (int s = bind_answer(ctx, hbytes)) return s;
    const uint64_t half = (ctx->lfz_bytes / 2) & ~7ull;
    const uint32_t par = ctx->lf_parity ^ 1u;
    char* mine = static_cast<char*>(ctx->lfz) + par * half;
    char* prev = static_cast<char*>(ctx->lfz) + (par ^ 1u) * half;
    LF f;
    f.ia = static_cast<u64*>(ctx->lfi);
    f.ib = f.ia + R * nk;
    f.w = reinterpret_cast<uint32_t*>(mine);
    f.st = reinterpret_cast<u64*>(mine + wbytes);
    f.wz = reinterpret_cast<uint32_t*>(prev);
    f.nwz = ctx->lf_prev_use / 4;
    f.hneed = static_cast<uint32_t*>(ctx->lbind_hd);
    f.epoch = ctx->lf_epoch;
    f.nk = (uint32_t)nk;
    f.ntiles = ntiles;
    f.R = (uint32_t)R;
    const LV A = view(cur), B = view(val), OUT = view(dst);
    const uint64_t span = std::max<uint64_t>(
        {cur->known_e, val->known_e, gs ? 0 : cur->known_t, gs ? 0 : val->known_t, 1});
    const unsigned ry = (unsigned)(R < 65535 ? R : 65535);
    ctx->lfz_dirty = true;
    const dim3 gp((unsigned)((span + 255) / 256), ry), gw(ntiles, ry);
    if (gs) {
        hipLaunchKernelGGL(k_lbf_prep<true>, gp, dim3(256), 0, ctx->stream, A, B, rk, f, R);
        hipLaunchKernelGGL(k_lbf_write<2>, gw, dim3(kLfT), 0, ctx->stream, A, B, OUT, rk, f);
    } else {
        hipLaunchKernelGGL(k_lbf_prep<false>, gp, dim3(256), 0, ctx->stream, A, B, rk, f, R);
        hipLaunchKernelGGL(k_lbf_write<0>, gw, dim3(kLfT), 0, ctx->stream, A, B, OUT, rk, f);
    }
    if (hipGetLastError() != hipSuccess) return fail(ctx, LASPJ_E_DEVICE, "list_bind: launch");
    ctx->lf_parity = par;
    ctx->lf_prev_use = use;
    const hipError_t e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess)
        return fail(ctx, LASPJ_E_DEVICE, "list_bind: synchronise: %s", hipGetErrorString(e));
    ctx->lfz_dirty = false;                 // the next call zeroes what this one used
    const auto* hb = static_cast<const uint8_t*>(ctx->lbind_h);
    bool retry = false;
    for (uint64_t r = 0; r < R; ++r) {
        const uint8_t st = hb[8 * R + r];
        if ((st & 3u) == 3u) {
            retry = true;
            if (st & 4u) cur->not_asc = true;
            if (st & 8u) val->not_asc = true;
        }
    }
    if (retry) return kLfRetry;
    set_known(dst, reinterpret_cast<const uint32_t*>(hb), R);
    std::memcpy(status, hb + 8 * R, R);
    return LASPJ_OK;
}

int laspj_list_bind(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* cur,
                    const laspj_batch* val, const laspj_list_order* ord, uint8_t* status) {
    if (int s = check_list(ctx, dst, "list_bind")) return s;
    if (int s = check_list(ctx, cur, "list_bind")) return s;
    if (int s = check_list(ctx, val, "list_bind")) return s;
    if (!status) return fail(ctx, LASPJ_E_INVAL, "list_bind: null status");
    if (int s = pair_checks(ctx, dst, cur, val, "list_bind")) return s;
    RK rk;
    if (int s = ranks(ctx, ord, cur->kind != LASPJ_KIND_GSET_LIST, &rk, "list_bind")) return s;
    const uint64_t R = cur->replicas;
    LGuard g(ctx);
    // both lists ascending (tried unless a list is known not to, and while the rank universe
    // is not much larger than the lists): the rank-indexed bind, two launches
    if (!cur->not_asc && !val->not_asc && ctx->tune_list_walk != 2 && R <= 1024 &&
        R * (uint64_t)rk.nk <= (1ull << 22) &&
        rk.nk <= 16ull * ((uint64_t)cur->known_e + val->known_e) + 65536 &&
        (uint64_t)cur->known_e + val->known_e < (1ull << 30) &&
        (uint64_t)cur->known_t + val->known_t <= 0xFFFFFFF0ull) {
        const int s = list_bind_ascending(ctx, dst, cur, val, rk, status);
        if (s != kLfRetry) return s;
    }
    // the context's bind block (device): [words 4R + 4 (BindFin): the error word the
    // kernels raise into, the merge's per-replica flags and tickets, the inflation's flags,
    // the equality's words, the final ticket | ... | need 8R at the block's end], the words
    // kept zero between calls (at offset 0 and need at the end, so one call's need never
    // lies where another call's words do, whatever their R) —
    // and the answer, written by the last block into pinned host memory: [need 8R |
    // status R (to a word) | flag]: no memset, no copy, one synchronisation
    const uint64_t nwords = 4 * R + 4, bytes = 4 * nwords + 8 * R;
    const uint64_t hbytes = 8 * R + 4 * ((R + 3) / 4) + 4;
    bool fresh = false;
    if (ctx->lbind_bytes < bytes) {
        if (ctx->lbind) {
            hipStreamSynchronize(ctx->stream);
            hipFree(ctx->lbind);
            ctx->lbind = nullptr;
            ctx->lbind_bytes = 0;
        }
        if (laspj::dev_malloc(ctx, &ctx->lbind, bytes) != hipSuccess) {
            hipGetLastError();
            return fail(ctx, LASPJ_E_NOMEM, "list_bind: bind block");
        }
        ctx->lbind_bytes = bytes;
        fresh = true;
    }
    if (int st = bind_answer(ctx, hbytes)) return st;
    void* hdev = ctx->lbind_hd;
    auto* mw = static_cast<uint32_t*>(ctx->lbind);
    auto* need = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(ctx->lbind) +
                                             ctx->lbind_bytes - 8 * R);
    // words not known zero (a fresh block, or a call that stopped before its last kernel
    // was enqueued): the merge zeroes them (the whole block's words) first
    const uint64_t wzero = fresh || ctx->lbind_dirty ? 4 * nwords : 0;
    ctx->lbind_dirty = true;
    // Type:merge and is_inflation(Value0, Merged) enqueued back to back (the merge sized
    // from the inputs' known counts), `Value0 =:= Value` over the grid, whose last block
    // writes the answer
    uint32_t* dd = nullptr;
    const uint32_t* fw = nullptr;
    rk.flag = mw;
    // the merged list's keyfind table, filled by the merge's write pass (Ins): sized as
    // inflation_launch sizes it, from the capacities the merge leaves dst with
    const uint64_t be = (uint64_t)cur->known_e + val->known_e;
    const uint32_t dce = be > dst->cap_e ? (uint32_t)std::min<uint64_t>(be, 0xFFFFFFFFull)
                                         : dst->cap_e;
    const uint32_t tsz0 = pow2_at_least(2ull * (dce > cur->cap_e ? dce : cur->cap_e));
    char* tb = bind_tables(ctx, R * tsz0 * 12ull, "list_bind");
    if (!tb) return LASPJ_E_NOMEM;
    u64* tk = reinterpret_cast<u64*>(tb);
    uint32_t* ti = reinterpret_cast<uint32_t*>(tb + R * tsz0 * 8ull);
    uint32_t tsz = tsz0;
    const Ins ins{tk, ti, tsz0, mw + R + 3};
    int s = merge_enqueue(ctx, dst, cur, val, rk, false, need, nullptr, "list_bind", mw, wzero,
                          &ins, cur->not_asc || val->not_asc);
    // (Value0's replicas whose keys strictly ascend skip the check: see k_linf_insert)
    if (s == LASPJ_OK)
        s = inflation_launch(ctx, cur, dst, 0, rk, nullptr, false, "list_bind", &dd, false, &fw,
                             mw + R + 3, mw + 2 * R + 3, &tk, &ti, &tsz);
    if (s == LASPJ_OK) {
        const uint32_t cmax = cur->cap_e > val->cap_e ? cur->cap_e : val->cap_e;
        const uint32_t tmax = cur->cap_t > val->cap_t ? cur->cap_t : val->cap_t;
        const uint32_t span = cmax > tmax ? cmax : tmax;
        const unsigned gx = (unsigned)std::min<uint64_t>((span + 2047) / 2048 + 1, 1024);
        const BindFin fin{mw, need, static_cast<uint32_t*>(hdev), (uint32_t)R};
        hipLaunchKernelGGL(k_list_equal_grid, dim3(gx, (unsigned)(R < 65535 ? R : 65535)),
                           dim3(256), 0, ctx->stream, view(cur), view(val), rk, dd, R, tk, ti,
                           tsz, mw + R + 3, fin);
        s = hipGetLastError() == hipSuccess ? LASPJ_OK
                                            : fail(ctx, LASPJ_E_DEVICE, "list_bind: launch");
        if (s == LASPJ_OK) {
            ctx->ltab_dirty = false;          // the clean-ups are enqueued
            ctx->lbind_dirty = false;
        }
    }
    const auto* hb = static_cast<const uint8_t*>(ctx->lbind_h);
    if (s == LASPJ_OK) {
        const hipError_t e = hipStreamSynchronize(ctx->stream);
        uint32_t f = 0;
        if (e == hipSuccess) std::memcpy(&f, hb + 8 * R + 4 * ((R + 3) / 4), 4);
        s = e != hipSuccess ? fail(ctx, LASPJ_E_DEVICE, "list_bind: synchronise: %s",
                                   hipGetErrorString(e))
                            : flag_status(ctx, f, "list_bind");
        if (f & kInfoWalkFell) cur->no_spec = val->no_spec = true;
    }
    if (s != LASPJ_OK) {
        dst->known_e = dst->cap_e, dst->known_t = dst->cap_t;
        return s;
    }
    set_known(dst, reinterpret_cast<const uint32_t*>(hb), R);
    // status: 0 = cur =:= val (no-op), 1 = the merge inflates cur (written), 2 = it does not
    std::memcpy(status, hb + 8 * R, R);
    return LASPJ_OK;
}

int laspj_list_value(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src) {
    if (int s = check_list(ctx, dst, "list_value")) return s;
    if (int s = check_list(ctx, src, "list_value")) return s;
    if (src->kind != LASPJ_KIND_ORSET_LIST || dst->kind != LASPJ_KIND_GSET_LIST)
        return fail(ctx, LASPJ_E_KIND, "list_value: OR-Set list -> G-Set list");
    if (dst->replicas != src->replicas) return fail(ctx, LASPJ_E_SHAPE, "list_value: replicas");
    LGuard g(ctx);
    const LV S = view(src);
    return tiled<PValue>(ctx, dst, src->cap_e, 0, [&](char*) { return PValue{S}; },
                         "list_value", src->known_e ? src->known_e : 1, 1);
}

int laspj_list_intersection(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                            const laspj_batch* r, const laspj_list_order* ord) {
    if (int s = pair_checks(ctx, dst, l, r, "list_intersection")) return s;
    const bool gs = l->kind == LASPJ_KIND_GSET_LIST;
    RK rk;
    if (int s = ranks(ctx, ord, !gs, &rk, "list_intersection")) return s;
    LGuard g(ctx);
    const uint64_t R = l->replicas;
    const uint32_t hsize = pow2_at_least(2ull * r->cap_e);
    const uint64_t hbytes = R * hsize * 12ull;
    const LV L = view(l), Rr = view(r);
    const dim3 hg((r->cap_e + 255) / 256 ? (r->cap_e + 255) / 256 : 1,
                  (unsigned)(R < 65535 ? R : 65535));
    auto pre = [&](auto gtag) {
        constexpr bool G = decltype(gtag)::value;
        return [&, hg](char* base) {
            u64* hk = reinterpret_cast<u64*>(base);
            auto* hi = reinterpret_cast<uint32_t*>(base + R * hsize * 8ull);
            hipMemsetAsync(base, 0, hbytes, ctx->stream);           // empty tables
            hipLaunchKernelGGL((k_isect_hash<G>), hg, dim3(256), 0, ctx->stream, Rr, rk, hk, hi,
                               hsize, R);
            return PIsect<G>{L, Rr, rk, hk, hi, hsize};
        };
    };
    if (gs)
        return tiled<PIsect<true>>(ctx, dst, l->cap_e, hbytes, pre(std::true_type{}),
                                   "list_intersection", std::max<uint32_t>(1, l->known_e), 1);
    // (tokens Cx ++ Cy: within l's and r's together unless l repeats a key of r)
    return tiled<PIsect<false>>(ctx, dst, l->cap_e, hbytes, pre(std::false_type{}),
                                "list_intersection", std::max<uint32_t>(1, l->known_e),
                                std::max<uint64_t>(1, (uint64_t)l->known_t + r->known_t));
}

int laspj_list_intersection_set(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                                const laspj_batch* r, const laspj_buf* tok_order) {
    if (int s = check_list(ctx, dst, "list_intersection_set")) return s;
    if (int s = check_list(ctx, l, "list_intersection_set")) return s;
    if (!r || r->ctx != ctx) return fail(ctx, LASPJ_E_INVAL, "list_intersection_set: r");
    const bool gs = l->kind == LASPJ_KIND_GSET_LIST;
    if (r->kind != (gs ? LASPJ_KIND_GSET : LASPJ_KIND_ORSET) || dst->kind != l->kind)
        return fail(ctx, LASPJ_E_KIND,
                    "list_intersection_set: OR-Set list x OR-Set, G-Set list x G-Set");
    if (r->replicas != l->replicas || dst->replicas != l->replicas)
        return fail(ctx, LASPJ_E_SHAPE, "list_intersection_set: replicas");
    if (!gs && (!tok_order || tok_order->ctx != ctx || tok_order->bytes < 64ull * r->elements))
        return fail(ctx, LASPJ_E_RANGE, "list_intersection_set: token order (64 bytes per slot)");
    LGuard g(ctx);
    const LV L = view(l);
    const auto* sp = reinterpret_cast<const u64*>(r->dev);
    const auto* tordp = gs ? nullptr : static_cast<const uint8_t*>(tok_order->dev);
    if (gs)
        return tiled<PIsectSet<true>>(ctx, dst, l->cap_e, 0, [&](char*) {
            return PIsectSet<true>{L, sp, r->words_per_replica, r->elements, tordp};
        }, "list_intersection_set", std::max<uint32_t>(1, l->known_e), 1);
    // (tokens Cx ++ Cy: l's run and at most 64 of the cell's)
    return tiled<PIsectSet<false>>(ctx, dst, l->cap_e, 0, [&](char*) {
        return PIsectSet<false>{L, sp, r->words_per_replica, r->elements, tordp};
    }, "list_intersection_set", std::max<uint32_t>(1, l->known_e),
       std::max<uint64_t>(1, (uint64_t)l->known_t + 64ull * l->known_e));
}

int laspj_list_product(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                       const laspj_batch* r) {
    if (int s = pair_checks(ctx, dst, l, r, "list_product")) return s;
    const bool gs = l->kind == LASPJ_KIND_GSET_LIST;
    LGuard g(ctx);
    const LV L = view(l), Rr = view(r);
    uint32_t* flag = ctx->flag + 1;
    const uint64_t mx = (uint64_t)l->cap_e * r->cap_e;
    if (gs)
        return tiled<PProduct<true>>(ctx, dst, mx, 0,
                                     [&](char*) { return PProduct<true>{L, Rr, flag}; },
                                     "list_product");
    return tiled<PProduct<false>>(ctx, dst, mx, 0,
                                  [&](char*) { return PProduct<false>{L, Rr, flag}; },
                                  "list_product");
}

static int unary_checks(laspj_ctx* ctx, const laspj_batch* dst, const laspj_batch* src,
                        const laspj_buf* tab, uint64_t tab_bytes, const char* what) {
    if (int s = check_list(ctx, dst, what)) return s;
    if (int s = check_list(ctx, src, what)) return s;
    if (dst->kind != src->kind) return fail(ctx, LASPJ_E_KIND, "%s: kinds differ", what);
    if (dst->replicas != src->replicas) return fail(ctx, LASPJ_E_SHAPE, "%s: replicas", what);
    if (dst == src) return fail(ctx, LASPJ_E_INVAL, "%s: dst aliases src", what);
    if (!tab || tab->ctx != ctx || tab->bytes < tab_bytes)
        return fail(ctx, LASPJ_E_RANGE, "%s: table buffer too small", what);
    return LASPJ_OK;
}

int laspj_list_map(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                   const laspj_buf* keys, uint32_t nidx, int per_entry) {
    if (int s = unary_checks(ctx, dst, src, keys, 8ull * nidx, "list_map")) return s;
    LGuard g(ctx);
    const LV S = view(src);
    const auto* tab = static_cast<const u64*>(keys->dev);
    uint32_t* flag = ctx->flag + 1;
    return tiled<PMap>(ctx, dst, src->cap_e, 0,
                       [&](char*) { return PMap{S, tab, nidx, per_entry, flag}; }, "list_map");
}

int laspj_list_filter(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                      const laspj_buf* keep, uint32_t nidx, int per_entry) {
    if (int s = unary_checks(ctx, dst, src, keep, nidx, "list_filter")) return s;
    LGuard g(ctx);
    const LV S = view(src);
    const auto* tab = static_cast<const uint8_t*>(keep->dev);
    uint32_t* flag = ctx->flag + 1;
    return tiled<PFilter>(ctx, dst, src->cap_e, 0,
                          [&](char*) { return PFilter{S, tab, nidx, per_entry, flag}; },
                          "list_filter");
}

int laspj_list_fold(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                    const laspj_buf* off, const laspj_buf* keys, uint32_t nidx, int per_entry) {
    if (int s = unary_checks(ctx, dst, src, off, 4ull * ((uint64_t)nidx + 1), "list_fold"))
        return s;
    if (!keys || keys->ctx != ctx) return fail(ctx, LASPJ_E_INVAL, "list_fold: keys buffer");
    LGuard g(ctx);
    // the CSR offsets must stay inside the keys buffer
    std::vector<uint32_t> h((uint64_t)nidx + 1);
    LJ_HIP(ctx, laspj::readback(ctx, h.data(), off->dev, 4ull * h.size()));
    for (uint32_t i = 0; i < nidx; ++i)
        if (h[i + 1] < h[i]) return fail(ctx, LASPJ_E_INVAL, "list_fold: offsets not ascending");
    if (8ull * h[nidx] > keys->bytes)
        return fail(ctx, LASPJ_E_RANGE, "list_fold: keys buffer too small");
    const LV S = view(src);
    const auto* po = static_cast<const uint32_t*>(off->dev);
    const auto* pk = static_cast<const u64*>(keys->dev);
    uint32_t* flag = ctx->flag + 1;
    return tiled<PFold>(ctx, dst, src->cap_e, 0,
                        [&](char*) { return PFold{S, po, pk, nidx, per_entry, flag}; },
                        "list_fold");
}

}  // extern "C"
