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
// feeding a device exclusive scan (k_scan_*) into the caller's offsets, then a writer:
//   k_orset_etf_write_rec   every token image the same length (Lasp's 20-byte tokens):
//                           host-built record templates, records OR-ed into 16-byte
//                           aligned LDS windows as byte-shifted dwords (below);
//   k_orset_etf_write       mixed image lengths, few tokens per element: one thread
//                           stages its element byte by byte;
//   k_orset_etf_write_wave  mixed image lengths, many tokens: a wave per element;
//   k_gset_etf_write        G-Set lists.
// Elements go in term order; a block scan of their sizes places them.  The path is
// write-bound: a payload is ~15-70x the bytes of its cells.

#include <algorithm>
#include <atomic>
#include <cstring>
#include <new>
#include <vector>

#include "laspj_internal.h"

// a token image that is BINARY_EXT of exactly the rest of its bytes
static inline bool tok_is_binary(const uint8_t* p, uint32_t len) {
    return len >= 5u && p[0] == 109 &&
           (((uint32_t)p[1] << 24) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 8) | p[4]) == len - 5u;
}

struct laspj_etf_dict {
    laspj_ctx* ctx = nullptr;
    uint32_t elements = 0;
    bool has_tokens = false;
    uint32_t tok_uniform = 0;     // every used token image has this length (0: mixed)
    uint32_t tok_max = 0;         // most token slots any element uses
    void* block = nullptr;        // one device allocation holding the arrays below
    uint64_t block_bytes = 0;     // (from the context's block cache: dev_alloc / dev_release)
    const uint8_t* elem_blob = nullptr;
    const uint32_t* elem_off = nullptr;    // E + 1
    const uint32_t* elem_order = nullptr;  // E
    const uint8_t* elem_byte = nullptr;    // E: 1 = image is SMALL_INTEGER_EXT (97, v)
    const uint8_t* tok_blob = nullptr;     // null: not kept on the device
    const uint32_t* tok_off = nullptr;     // 64E + 1 (mixed image lengths only)
    const uint8_t* tok_order = nullptr;    // 64E
    const uint64_t* tok_mask = nullptr;    // E: token slots with an image
    // the same images again, each starting on a 16-byte boundary (wide loads)
    const uint8_t* elem_pad = nullptr;
    const uint32_t* elem_poff = nullptr;   // E
    const uint8_t* tok_pad = nullptr;
    const uint32_t* tok_poff = nullptr;    // 64E (null: not kept on the device)
    // per element, tokens in term order: k | image length << 8 | padded offset << 32
    // (k = 0xFF after the last one) — one load per (element, rank)
    const uint64_t* tok_desc = nullptr;    // 64E
    // record templates for the uniform-token kernel (every token image rec_len - 2 bytes):
    // element e, term rank j at rec_pad + (e * tok_max + j) * rec_stride holds
    // 104 2 <token image>;  element e's header prefix 104 2 <elem image> 108 at
    // ehdr_pad + ehdr_poff[e]
    uint32_t rec_len = 0, rec_stride = 0;  // rec_len 0: no templates (mixed token lengths)
    bool bin_tokens = false;               // every token a BINARY_EXT of rec_len - 7 bytes
    uint32_t big_elems = 0;                // elements holding more than kSmallTok tokens
    const uint8_t* rec_pad = nullptr;
    const uint8_t* ehdr_pad = nullptr;
    const uint32_t* ehdr_poff = nullptr;   // E
    uint32_t ehdr_max = 0;                 // longest element header template
    // from_binary tables by element rank (term order), see ReadTabs; null when some
    // element's tokens share every bucket choice (from_binary then scans serially)
    const void* rd_desc = nullptr;         // E x {slot, header length, 0, token ranks}
    const uint8_t* rd_hdr = nullptr;       // E x 64 header template bytes
    const uint16_t* rd_tb = nullptr;       // E x tok_max token buckets (see ReadTabs)
    const uint8_t* rd_ros = nullptr;       // E x 64: token slot -> token rank (0xFF: none)
    // header template hash -> rank + 1 (segment mode's first element; with rd_*)
    const uint32_t* rd_htab = nullptr;
    uint32_t rd_hmask = 0;
    uint64_t rd_hlens = 0;                 // bit hl - 1: a header template of hl <= 64 bytes
    // G-Set from_binary: element image hash (FNV-1a) -> slot + 1; term rank per slot
    // (equal terms share one); slot + 1 of the SMALL_INTEGER_EXT image of each byte value
    const uint32_t* gs_htab = nullptr;
    uint32_t gs_hmask = 0;
    const uint32_t* gs_rank = nullptr;     // E
    const uint32_t* gs_byte = nullptr;     // 256
    // integer elements (minimal SMALL_INTEGER / INTEGER images) by value: entry v - gs_ilo
    // = slot + 1 | rank << 32 (0: no element), so the decoder finds an integer element with
    // one load instead of a hash probe and an image compare; null when no integer element
    // or their values are too spread out
    const uint64_t* gs_itab = nullptr;
    int64_t gs_ilo = 0;
    uint32_t gs_in = 0;
    // host-side state for laspj::etf_dict_patch (dictionaries built with token headroom,
    // the NIF path's): slot -> rank, each token slot's padded image offset (0xFFFFFFFF:
    // none), where the patched arrays sit in the block, the padded-image area's use
    bool patchable = false;
    std::vector<uint32_t> h_rank, h_tpoff;
    uint64_t o_mask = 0, o_tord = 0, o_tpad = 0, o_tdesc = 0, o_rpad = 0, o_rd = 0;
    uint64_t tpad_used = 0, tpad_cap = 0;
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
    const uint8_t* elem_pad;
    const uint32_t* elem_poff;
    const uint8_t* tok_pad;
    const uint32_t* tok_poff;
    const uint64_t* tok_desc;
    uint32_t tok_max, rec_len, rec_stride;
    const uint8_t* rec_pad;
    const uint8_t* ehdr_pad;
    const uint32_t* ehdr_poff;
    uint32_t ehdr_max;
};

DictView view(const laspj_etf_dict* d) {
    return {d->elem_blob, d->elem_off,  d->elem_order, d->elem_byte,  d->tok_blob,
            d->tok_off,   d->tok_order, d->tok_mask,   d->tok_uniform, d->elem_pad,
            d->elem_poff, d->tok_pad,   d->tok_poff,   d->tok_desc,    d->tok_max,
            d->rec_len,   d->rec_stride, d->rec_pad,   d->ehdr_pad,    d->ehdr_poff,
            d->ehdr_max};
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

__device__ __forceinline__ uint8_t* put_be32(uint8_t* o, uint32_t v) {
    o[0] = (uint8_t)(v >> 24);
    o[1] = (uint8_t)(v >> 16);
    o[2] = (uint8_t)(v >> 8);
    o[3] = (uint8_t)v;
    return o + 4;
}

__constant__ uint8_t kAtomTrue[7] = {100, 0, 4, 't', 'r', 'u', 'e'};
__constant__ uint8_t kAtomFalse[8] = {100, 0, 5, 'f', 'a', 'l', 's', 'e'};

// ---------------------------------------------------------------- staging windows
// The write kernels assemble a replica chunk by chunk (256 elements in term order) and
// each chunk window by window: the bytes of [w0, w0 + wl) (chunk-relative) are staged
// in LDS by whichever threads own them, then the block copies the window out with
// 16-byte non-temporal stores (LDS and HBM alignment made equal mod 16).  Byte-level
// work stays in LDS; HBM sees whole 1 KiB wave stores.
constexpr uint32_t kWin = 16384;

struct Win {
    uint8_t* buf;      // window byte x at buf[x]
    uint32_t w0, wl;   // chunk-relative window [w0, w0 + wl)
    __device__ __forceinline__ bool hits(uint32_t q, uint32_t n) const {
        return q < w0 + wl && q + n > w0;
    }
    __device__ __forceinline__ void put(uint32_t q, uint8_t b) const {
        uint32_t x = q - w0;
        if (x < wl) buf[x] = b;
    }
    __device__ __forceinline__ void span(uint32_t q, const uint8_t* src, uint32_t n) const {
        uint32_t lo = q > w0 ? q : w0, hi = min(q + n, w0 + wl);
        for (uint32_t y = lo; y < hi; ++y) buf[y - w0] = src[y - q];
    }
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// n <= 48 bytes of a 16-byte-aligned padded image into LDS bytes dst[0 .. n): up to three
// 16-byte loads issued together, then byte stores from registers
__device__ __forceinline__ void lds_put48(uint8_t* dst, const uint8_t* src16, uint32_t n) {
    const u32x4* s = reinterpret_cast<const u32x4*>(src16);
    const u32x4 z = {0, 0, 0, 0};
    const u32x4 a = s[0], b = n > 16 ? s[1] : z, c = n > 32 ? s[2] : z;
    const uint32_t wd[12] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w};
#pragma unroll
    for (uint32_t i = 0; i < 48; ++i)
        if (i < n) dst[i] = (uint8_t)(wd[i >> 2] >> ((i & 3u) * 8u));
}

__device__ __forceinline__ bool inside(const Win& w, uint32_t q, uint32_t n) {
    return q >= w.w0 && q + n <= w.w0 + w.wl;
}

// 104 2 <elem image> 108 <n:32>: 7 + el bytes at q
__device__ __forceinline__ void stage_elem_header(const Win& w, const DictView& d, uint32_t e,
                                                  uint32_t n, uint32_t q) {
    const uint32_t el = d.elem_off[e + 1] - d.elem_off[e];
    if (!w.hits(q, 7u + el)) return;
    if (el <= 48 && inside(w, q, 7u + el)) {
        uint8_t* o = w.buf + (q - w.w0);
        o[0] = 104;
        o[1] = 2;
        lds_put48(o + 2, d.elem_pad + d.elem_poff[e], el);
        o += 2 + el;
        o[0] = 108;
        o[1] = (uint8_t)(n >> 24);
        o[2] = (uint8_t)(n >> 16);
        o[3] = (uint8_t)(n >> 8);
        o[4] = (uint8_t)n;
        return;
    }
    w.put(q, 104);
    w.put(q + 1, 2);
    w.span(q + 2, d.elem_blob + d.elem_off[e], el);
    q += 2u + el;
    w.put(q, 108);
    w.put(q + 1, (uint8_t)(n >> 24));
    w.put(q + 2, (uint8_t)(n >> 16));
    w.put(q + 3, (uint8_t)(n >> 8));
    w.put(q + 4, (uint8_t)n);
}

// record from a term-order descriptor: image of L bytes at tok_pad + poff
__device__ __forceinline__ void stage_record_desc(const Win& w, const DictView& d, uint32_t L,
                                                  uint32_t poff, bool removed, uint32_t q,
                                                  uint32_t rl) {
    if (!w.hits(q, rl)) return;
    const uint8_t* img = d.tok_pad + poff;
    if (L <= 48 && inside(w, q, rl)) {
        uint8_t* o = w.buf + (q - w.w0);
        o[0] = 104;
        o[1] = 2;
        lds_put48(o + 2, img, L);
        o += 2 + L;
        o[0] = 100;
        o[1] = 0;
        o[2] = removed ? 4 : 5;
        o[3] = removed ? 't' : 'f';
        o[4] = removed ? 'r' : 'a';
        o[5] = removed ? 'u' : 'l';
        o[6] = removed ? 'e' : 's';
        if (!removed) o[7] = 'e';
        return;
    }
    w.put(q, 104);
    w.put(q + 1, 2);
    w.span(q + 2, img, L);
    if (removed) w.span(q + 2 + L, kAtomTrue, 7);
    else w.span(q + 2 + L, kAtomFalse, 8);
}

// one thread stages its whole element (few tokens per element)
__device__ void stage_elem_thread(const Win& w, const DictView& d, uint32_t e, u64 p, u64 r,
                                  uint32_t pos, uint32_t sz) {
    if (!w.hits(pos, sz)) return;
    stage_elem_header(w, d, e, (uint32_t)__popcll(p), pos);
    uint32_t q = pos + 7u + (d.elem_off[e + 1] - d.elem_off[e]);
    const uint64_t* desc = d.tok_desc + (u64)d.tok_max * e;
    for (uint32_t j = 0; j < d.tok_max; ++j) {
        const uint64_t ds = desc[j];
        const uint32_t k = (uint32_t)(ds & 0xFFu);
        if (k >= 64) break;
        if (!((p >> k) & 1ull)) continue;
        const bool rm = (r >> k) & 1ull;
        const uint32_t L = (uint32_t)(ds >> 8) & 0xFFFFFFu, rl = 2u + L + (rm ? 7u : 8u);
        stage_record_desc(w, d, L, (uint32_t)(ds >> 32), rm, q, rl);
        q += rl;
    }
    w.put(q, 106);
}

// copy window bytes buf[sh .. sh + wl) to out[g .. g + wl), (g - sh) % 16 == 0
__device__ __forceinline__ void copy_out(const uint8_t* buf, uint32_t sh, uint32_t wl,
                                         uint8_t* out, u64 g) {
    uint32_t a = (16u - sh) & 15u;
    if (a > wl) a = wl;
    for (uint32_t x = threadIdx.x; x < a; x += kBlock) out[g + x] = buf[sh + x];
    const uint32_t nv = (wl - a) >> 4;
    const u32x4* src = reinterpret_cast<const u32x4*>(buf + sh + a);
    u32x4* dst = reinterpret_cast<u32x4*>(out + g + a);
    for (uint32_t v = threadIdx.x; v < nv; v += kBlock) __builtin_nontemporal_store(src[v], dst + v);
    for (uint32_t x = a + 16u * nv + threadIdx.x; x < wl; x += kBlock) out[g + x] = buf[sh + x];
}

__device__ __forceinline__ void write_list_header(uint8_t* out, u64 base, uint32_t hdr, int tag,
                                                  int vers, uint8_t list_tag, uint32_t n) {
    uint8_t* o = out + base;
    if (hdr) {
        o[0] = (uint8_t)tag;
        o[1] = (uint8_t)vers;
    }
    o[hdr] = 131;
    o[hdr + 1] = list_tag;
    if (list_tag == 108) put_be32(o + hdr + 2, n);
    else if (list_tag == 107) {
        o[hdr + 2] = (uint8_t)(n >> 8);
        o[hdr + 3] = (uint8_t)n;
    }
}

// few tokens per element and mixed token image lengths: one thread stages its whole
// element into the block's window
__global__ __launch_bounds__(kBlock) void k_orset_etf_write(const u64x2* cells, uint64_t R,
                                                            uint32_t E, DictView d, int tag,
                                                            int vers, const u64* offs,
                                                            uint8_t* out, u64 ocap) {
    if (offs[R] > ocap) return;              // the payloads do not fit: the host re-sizes
    __shared__ uint32_t lds4[kBlock / 64];
    __shared__ __attribute__((aligned(16))) uint8_t buf[kWin + 16];
    const uint32_t hdr = tag >= 0 ? 2u : 0u;
    for (uint64_t rep = blockIdx.x; rep < R; rep += gridDim.x) {
        const u64x2* c = cells + rep * E;
        const u64 base = offs[rep], end = offs[rep + 1];
        u64 cursor = base + hdr + 6u;
        uint32_t n = 0;
        for (uint32_t c0 = 0; c0 < E; c0 += kBlock) {
            const uint32_t i = c0 + threadIdx.x;
            const uint32_t e = i < E ? d.elem_order[i] : 0u;
            const u64x2 v = i < E ? c[e] : u64x2{0, 0};
            const uint32_t sz = v.x ? orset_elem_size(d, e, v.x, v.y) : 0u;
            uint32_t tot, cnt;
            const uint32_t pos = block_excl_scan(sz, lds4, &tot);
            block_excl_scan(v.x ? 1u : 0u, lds4, &cnt);
            if (cursor + tot + 1u > end) break;          // sizes disagree: never overrun
            for (uint32_t w0 = 0; w0 < tot; w0 += kWin) {
                const uint32_t wl = min(kWin, tot - w0);
                const u64 g = cursor + w0;
                const uint32_t sh = (uint32_t)(g & 15u);
                const Win win{buf + sh, w0, wl};
                if (v.x) stage_elem_thread(win, d, e, v.x, v.y, pos, sz);
                __syncthreads();
                copy_out(buf, sh, wl, out, g);
                __syncthreads();
            }
            cursor += tot;
            n += cnt;
        }
        if (threadIdx.x == 0) {
            write_list_header(out, base, hdr, tag, vers, n ? 108 : 106, n);
            if (n && cursor < end) out[cursor] = 106;
        }
        __syncthreads();
    }
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Many tokens per element: each wave assembles whole elements on its own (lane j owns
// the element's j-th token in term order) in a private LDS buffer and stores them with
// 16-byte stores; only the chunk scan that places elements is block-wide.
constexpr uint32_t kWB = 4096;

__global__ __launch_bounds__(kBlock) void k_orset_etf_write_wave(const u64x2* cells, uint64_t R,
                                                                 uint32_t E, DictView d, int tag,
                                                                 int vers, const u64* offs,
                                                                 uint8_t* out, u64 ocap) {
    if (offs[R] > ocap) return;
    __shared__ uint32_t lds4[kBlock / 64];
    __shared__ __attribute__((aligned(16))) uint8_t wbuf[kBlock / 64][kWB + 16];
    __shared__ uint32_t s_e[kBlock], s_pos[kBlock], s_sz[kBlock];
    __shared__ u64 s_p[kBlock], s_r[kBlock];
    const uint32_t hdr = tag >= 0 ? 2u : 0u;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint8_t* mine = wbuf[wave];
    for (uint64_t rep = blockIdx.x; rep < R; rep += gridDim.x) {
        const u64x2* c = cells + rep * E;
        const u64 base = offs[rep], end = offs[rep + 1];
        u64 cursor = base + hdr + 6u;
        uint32_t n = 0;
        for (uint32_t c0 = 0; c0 < E; c0 += kBlock) {
            const uint32_t i = c0 + threadIdx.x;
            const uint32_t e = i < E ? d.elem_order[i] : 0u;
            const u64x2 v = i < E ? c[e] : u64x2{0, 0};
            const uint32_t sz = v.x ? orset_elem_size(d, e, v.x, v.y) : 0u;
            uint32_t tot, cnt;
            const uint32_t pos = block_excl_scan(sz, lds4, &tot);
            block_excl_scan(v.x ? 1u : 0u, lds4, &cnt);
            if (cursor + tot + 1u > end) break;          // sizes disagree: never overrun
            s_e[threadIdx.x] = e;
            s_p[threadIdx.x] = v.x;
            s_r[threadIdx.x] = v.y;
            s_pos[threadIdx.x] = pos;
            s_sz[threadIdx.x] = sz;
            __syncthreads();
            for (int j = wave; j < kBlock; j += kBlock / 64) {
                const uint32_t js = s_sz[j];
                if (!js) continue;
                const uint32_t je = s_e[j];
                const u64 jp = s_p[j], jr = s_r[j];
                const u64 g0 = cursor + s_pos[j];
                const uint64_t ds = lane < d.tok_max ? d.tok_desc[(u64)d.tok_max * je + lane]
                                                     : 0xFFull;
                const uint32_t k = (uint32_t)(ds & 0xFFu);
                const bool here = k < 64 && ((jp >> k) & 1ull);
                const bool rm = here && ((jr >> k) & 1ull);
                const uint32_t L = (uint32_t)(ds >> 8) & 0xFFFFFFu;
                const uint32_t rl = here ? 2u + L + (rm ? 7u : 8u) : 0u;
                uint32_t x = rl;
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    uint32_t y = __shfl_up(x, off, 64);
                    if (lane >= off) x += y;
                }
                const uint32_t q = 7u + (d.elem_off[je + 1] - d.elem_off[je]) + (x - rl);
                for (uint32_t w0 = 0; w0 < js; w0 += kWB) {
                    const uint32_t wl = min(kWB, js - w0);
                    const u64 g = g0 + w0;
                    const uint32_t sh = (uint32_t)(g & 15u);
                    const Win win{mine + sh, w0, wl};
                    if (lane == 0) {
                        stage_elem_header(win, d, je, (uint32_t)__popcll(jp), 0u);
                        win.put(js - 1u, 106);
                    }
                    if (here) stage_record_desc(win, d, L, (uint32_t)(ds >> 32), rm, q, rl);
                    wave_sync();
                    uint32_t a = (16u - sh) & 15u;
                    if (a > wl) a = wl;
                    if ((uint32_t)lane < a) out[g + lane] = mine[sh + lane];
                    const uint32_t nv = (wl - a) >> 4;
                    const u32x4* src = reinterpret_cast<const u32x4*>(mine + sh + a);
                    u32x4* dst = reinterpret_cast<u32x4*>(out + g + a);
                    for (uint32_t vi = lane; vi < nv; vi += 64)
                        __builtin_nontemporal_store(src[vi], dst + vi);
                    for (uint32_t xx = a + 16u * nv + lane; xx < wl; xx += 64) out[g + xx] = mine[sh + xx];
                    wave_sync();
                }
            }
            __syncthreads();
            cursor += tot;
            n += cnt;
        }
        if (threadIdx.x == 0) {
            write_list_header(out, base, hdr, tag, vers, n ? 108 : 106, n);
            if (n && cursor < end) out[cursor] = 106;
        }
        __syncthreads();
    }
}


// ------------------------------------------------------- uniform-token record kernel
// Every token image of the dictionary has the same length (Lasp's tokens are the
// 20-byte binaries of unique/1 or add_by_token), so a record's position follows from
// its element's position and its rank among the element's present tokens alone.  A
// block assembles a replica 256 elements (one chunk) at a time:
//   A  thread per element: the cell's token bits permuted into term order, its byte
//      size and record count; one block scan places elements and numbers records.
//   B  per LDS window (16 KiB (16-byte aligned in the output): threads stage element
//      headers and, spread over all lanes, the chunk's records (record -> element by a
//      binary search of the record prefix, -> token by rank select), each piece as
//      byte-shifted dwords OR-ed into the zeroed window (ds_or_b32; neighbours share
//      edge dwords); then whole 16-byte chunks go out with non-temporal stores and the
//      trailing partial chunk is carried to the next window.
// Lanes are busy on records whatever the tokens per element; no byte-wise LDS work.

__device__ __forceinline__ uint32_t select64(u64 m, uint32_t k) {
    uint32_t pos = 0, c = (uint32_t)__popc((uint32_t)m);
    if (k >= c) { k -= c; m >>= 32; pos = 32; }
    uint32_t lo = (uint32_t)m;
    c = (uint32_t)__popc(lo & 0xFFFFu);
    if (k >= c) { k -= c; lo >>= 16; pos += 16; }
    c = (uint32_t)__popc(lo & 0xFFu);
    if (k >= c) { k -= c; lo >>= 8; pos += 8; }
    c = (uint32_t)__popc(lo & 0xFu);
    if (k >= c) { k -= c; lo >>= 4; pos += 4; }
    c = (uint32_t)__popc(lo & 0x3u);
    if (k >= c) { k -= c; lo >>= 2; pos += 2; }
    if (k >= (lo & 1u)) pos += 1;
    return pos;
}

__device__ __forceinline__ void lds_or(uint32_t* p, uint32_t v) {
    __hip_atomic_fetch_or(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The window has kGuard bytes of slack on both sides, so a piece that overlaps it can be
// written whole: bytes that land in the guards are dropped when the window goes out.
constexpr int32_t kGuard = 64;

template <uint32_t WIN>
__device__ __forceinline__ bool overlaps(int32_t rel, uint32_t n) {
    return rel < (int32_t)WIN && rel + (int32_t)n > 0;
}

// OR a piece of n <= min(nmax, 4 * NW) bytes, little-endian in w[] (zero past n), into
// the window at window-relative byte rel (the piece must overlap the window).  With
// d0 = floor((rel - 1) / 4) and sh = rel - 4 d0 in [1, 4], window dword d0 + i receives
// bytes 4i - sh .. 4i - sh + 3 of the piece = alignbyte(w[i], w[i - 1], 4 - sh): one
// VALU op and one ds_or_b32 per dword, dwords past nmax skipped on a uniform branch.
template <int NW>
__device__ __forceinline__ void or_piece(uint32_t* win, int32_t rel, const uint32_t (&w)[NW],
                                         uint32_t nmax) {
    const int32_t rm1 = rel - 1;
    const uint32_t a = 3u - ((uint32_t)rm1 & 3u);
    uint32_t* q = win + (rm1 >> 2);
#pragma unroll
    for (int i = 0; i <= NW; ++i) {
        if (4u * (uint32_t)i <= nmax + 3u) {
            const uint32_t hi = i < NW ? w[i] : 0u, lo = i > 0 ? w[i - 1] : 0u;
            lds_or(q + i, __builtin_amdgcn_alignbyte(hi, lo, a));
        }
    }
}

// n bytes of a 16-byte-aligned zero-padded image (n <= 48) as a piece
__device__ __forceinline__ void load_piece48(uint32_t (&w)[12], const uint8_t* src16, uint32_t n) {
    const u32x4* s = reinterpret_cast<const u32x4*>(src16);
    const u32x4 z = {0, 0, 0, 0};
    const u32x4 a = s[0], b = n > 16 ? s[1] : z, c = n > 32 ? s[2] : z;
    w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
    w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
    w[8] = c.x; w[9] = c.y; w[10] = c.z; w[11] = c.w;
}

template <uint32_t WIN>
__device__ __forceinline__ void or_bytes_slow(uint32_t* win, int32_t rel, const uint8_t* src,
                                              uint32_t n) {
    for (uint32_t x = 0; x < n; ++x) {
        const int32_t b = rel + (int32_t)x;
        if (b >= 0 && b < (int32_t)WIN) lds_or(win + (b >> 2), (uint32_t)src[x] << (8 * (b & 3)));
    }
}

__device__ __forceinline__ u64 block_excl_scan64(u64 v, u64* lds4, u64* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    u64 x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        u64 y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    if (lane == 63) lds4[w] = x;
    __syncthreads();
    u64 before = 0, all = 0;
#pragma unroll
    for (int i = 0; i < kBlock / 64; ++i) {
        u64 s = lds4[i];
        if (i < w) before += s;
        all += s;
    }
    __syncthreads();
    *total = all;
    return before + x - v;
}

// Split mode (few long payloads, e.g. the NIF's one merged 10k-element value): the
// chunks of 256 term-order elements of a payload are written by different blocks.
// k_etf_chunk_sizes gives every chunk its byte size and present-element count (packed
// size | count << 40, the same per-element sizes as orset_elem_size), k_etf_chunk_scan
// turns them into per-payload exclusive offsets (entry nch = the payload's totals), and
// each block of the writer then starts at its chunk's byte offset with a fresh window:
// bytes below its first byte belong to the previous chunk's block and are left alone
// (byte stores at both ends of a block's range, as at payload ends).
constexpr u64 kChunkCnt = 1ull << 40;

__global__ __launch_bounds__(kBlock) void k_etf_chunk_sizes(const u64x2* cells, uint64_t R,
                                                            uint32_t E, DictView d, uint32_t nch,
                                                            u64* coff, uint32_t* flag) {
    __shared__ u64 lds4[kBlock / 64];
    for (uint64_t it = blockIdx.x; it < R * nch; it += gridDim.x) {
        const uint64_t rep = it / nch;
        const uint32_t c = (uint32_t)(it - rep * nch), i = c * kBlock + threadIdx.x;
        u64 v = 0;
        if (i < E) {
            const uint32_t e = d.elem_order[i];
            const u64x2 x = cells[rep * E + e];
            if (x.x) {
                // as k_orset_etf_size: a present slot without an image is an error
                if (d.elem_off[e + 1] == d.elem_off[e] || (x.x & ~d.tok_mask[e]) != 0) {
                    if (flag) atomicOr(flag, 1u);
                } else {
                    v = orset_elem_size(d, e, x.x, x.y) + kChunkCnt;
                }
            }
        }
        u64 tot;
        block_excl_scan64(v, lds4, &tot);
        if (threadIdx.x == 0) coff[rep * (nch + 1ull) + c] = tot;
    }
}

__global__ __launch_bounds__(kBlock) void k_etf_chunk_scan(u64* coff, uint64_t R, uint32_t nch) {
    __shared__ u64 lds4[kBlock / 64];
    for (uint64_t rep = blockIdx.x; rep < R; rep += gridDim.x) {
        u64* c = coff + rep * (nch + 1ull);
        u64 carry = 0;
        for (uint32_t t0 = 0; t0 <= nch; t0 += kBlock) {
            const uint32_t t = t0 + threadIdx.x;
            const u64 v = t < nch ? c[t] : 0;
            u64 tot;
            const u64 ex = block_excl_scan64(v, lds4, &tot);
            if (t <= nch) c[t] = carry + ex;
            carry += tot;
        }
    }
}

// The NIF path's merge (laspj_nif.hip): lasp_orset:merge/2 of replica i of `a` and of `b`
// (the slot-wise OR of canonical cells) written to `z`, fused with the split-mode size
// pass over z, and the operands' cells cleared behind it (the next call's decoders then
// start from new() without a memset).  Same chunk totals as k_etf_chunk_sizes.
// With `ticket` (few replicas: the NIF's single merges) the block that finishes last also
// scans the chunk totals and writes the payload offsets (k_etf_chunk_scan_offsets' work),
// so the whole size pass is one launch; ticket is zero on entry and left zero.
// With `chain` (the segment decoder's chain check deferred, ChainJob): the last
// (cj.nrep + 3) / 4 blocks check the decoded payloads' segment chains instead, one wave
// per payload, beside the join (its answer is only used when every chain held: the caller
// decodes serially and joins again when a status comes back kDecRedo).
struct SegRes;
__device__ int32_t chain_verdict(const uint8_t* payload, u64 base, u64 len, uint32_t g0,
                                 uint32_t ns, uint32_t S, const SegRes* res, uint32_t lane);
struct ChainArgs {
    const uint8_t* payload;
    const u64* offs;
    const uint32_t* segbase;
    const SegRes* res;
    int32_t* status;
    uint32_t nrep, S;
    SegRes* hres;       // (or null) a failed payload's segment results copied here too
};
// the checking wave of payload r: its segment results into cj.hres when its verdict failed
__device__ void chain_publish(const ChainArgs& cj, uint32_t r, int32_t st, uint32_t lane);
ChainArgs chain_args(const ChainJob* chain) {
    if (!chain || !chain->armed) return ChainArgs{nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0, nullptr};
    return ChainArgs{chain->payload, chain->offs, chain->segbase,
                     static_cast<const SegRes*>(chain->res), chain->status, chain->nrep, chain->S,
                     static_cast<SegRes*>(chain->hres)};
}
__global__ __launch_bounds__(kBlock) void k_etf_join_chunk_sizes(u64x2* a, u64x2* b, u64x2* z,
                                                                 uint64_t R, uint32_t E,
                                                                 DictView d, uint32_t nch,
                                                                 u64* coff, uint32_t* flag,
                                                                 uint32_t* ticket, uint32_t hdr,
                                                                 u64* offs, ChainArgs cj) {
    __shared__ u64 lds4[kBlock / 64];
    __shared__ uint32_t s_last;
    const uint32_t cblocks = cj.status ? (cj.nrep + 3u) / 4u : 0u;
    const uint32_t jblocks = gridDim.x - cblocks;
    if (blockIdx.x >= jblocks) {
        const uint32_t r = (blockIdx.x - jblocks) * 4u + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
        if (r < cj.nrep) {
            const u64 base = cj.offs[r];
            const int32_t st = chain_verdict(cj.payload, base, cj.offs[r + 1] - base,
                                             cj.segbase[r], cj.segbase[r + 1] - cj.segbase[r],
                                             cj.S, cj.res, lane);
            if (lane == 0) cj.status[r] = st;
            chain_publish(cj, r, st, lane);
        }
    }
    for (uint64_t it = blockIdx.x; blockIdx.x < jblocks && it < R * nch; it += jblocks) {
        const uint64_t rep = it / nch;
        const uint32_t c = (uint32_t)(it - rep * nch), i = c * kBlock + threadIdx.x;
        u64 v = 0;
        if (i < E) {
            const uint32_t e = d.elem_order[i];
            const uint64_t at = rep * E + e;
            const u64x2 x = a[at] | b[at];
            z[at] = x;
            a[at] = u64x2{0, 0};
            b[at] = u64x2{0, 0};
            if (x.x) {
                if (d.elem_off[e + 1] == d.elem_off[e] || (x.x & ~d.tok_mask[e]) != 0) {
                    if (flag) atomicOr(flag, 1u);
                } else {
                    v = orset_elem_size(d, e, x.x, x.y) + kChunkCnt;
                }
            }
        }
        u64 tot;
        block_excl_scan64(v, lds4, &tot);
        if (threadIdx.x == 0) coff[rep * (nch + 1ull) + c] = tot;
    }
    if (!ticket) return;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();                                   // this block's totals, visible
        s_last = atomicAdd(ticket, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!s_last) return;
    __threadfence();                                       // every block's totals, seen
    u64 ocarry = 0;
    for (uint64_t rep = 0; rep < R; ++rep) {
        u64* cp = coff + rep * (nch + 1ull);
        u64 carry = 0;
        for (uint32_t t0 = 0; t0 <= nch; t0 += kBlock) {
            const uint32_t t = t0 + threadIdx.x;
            const u64 v = t < nch ? __atomic_load_n(cp + t, __ATOMIC_RELAXED) : 0;
            u64 tot;
            const u64 ex = block_excl_scan64(v, lds4, &tot);
            if (t <= nch) cp[t] = carry + ex;
            carry += tot;
        }
        const u64 n = carry / kChunkCnt, sum = carry & (kChunkCnt - 1);
        if (threadIdx.x == 0) offs[rep] = ocarry;
        ocarry += hdr + 1u + (n ? 5u + sum + 1u : 1u);
    }
    if (threadIdx.x == 0) {
        offs[R] = ocarry;
        *ticket = 0;
    }
}

// k_etf_chunk_scan, then (the block that finishes last, by an agent-scope ticket) the
// payload offsets as k_etf_offsets_from_chunks: one launch instead of two.  ticket is zero
// on entry and left zero.
__global__ __launch_bounds__(kBlock) void k_etf_chunk_scan_offsets(u64* coff, uint64_t R,
                                                                   uint32_t nch, uint32_t hdr,
                                                                   u64* offs, uint32_t* ticket) {
    __shared__ u64 lds4[kBlock / 64];
    __shared__ uint32_t s_last;
    for (uint64_t rep = blockIdx.x; rep < R; rep += gridDim.x) {
        u64* c = coff + rep * (nch + 1ull);
        u64 carry = 0;
        for (uint32_t t0 = 0; t0 <= nch; t0 += kBlock) {
            const uint32_t t = t0 + threadIdx.x;
            const u64 v = t < nch ? c[t] : 0;
            u64 tot;
            const u64 ex = block_excl_scan64(v, lds4, &tot);
            if (t <= nch) c[t] = carry + ex;
            carry += tot;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();                                   // this block's totals, visible
        s_last = atomicAdd(ticket, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!s_last) return;
    __threadfence();                                       // every block's totals, seen
    u64 carry = 0;
    for (uint64_t t0 = 0; t0 < R; t0 += kBlock) {
        const uint64_t rep = t0 + threadIdx.x;
        u64 v = 0;
        if (rep < R) {
            const u64 t = __atomic_load_n(coff + rep * (nch + 1ull) + nch, __ATOMIC_RELAXED);
            const u64 n = t / kChunkCnt, sum = t & (kChunkCnt - 1);
            v = hdr + 1u + (n ? 5u + sum + 1u : 1u);
        }
        u64 tot;
        const u64 ex = block_excl_scan64(v, lds4, &tot);
        if (rep < R) offs[rep] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) {
        offs[R] = carry;
        *ticket = 0;
    }
}

// LB (the NIF's single merge, laspj_nif.hip): merge/2's join and the size pass folded into
// the writer.  One block per 256-element chunk of the one answer: it ORs the operands'
// cells (clearing them behind it), sizes its elements, publishes its chunk's {bytes,
// elements} and looks back over its predecessors' (decoupled look-back: a word per chunk,
// 1 = own totals, 2 = inclusive prefix) for its offset, then writes as split mode does.
// The list header's element count is not known to chunk 0: it writes a placeholder and the
// block that finishes last (ticket) writes the count (or the empty list 131 106), the
// answer's offsets {0, total} and — extra blocks after the chunks' — the segment decoder's
// chain checks (as k_etf_join_chunk_sizes does beside the join).  A total past ocap: the
// chunks write nothing, the caller re-runs with room.
struct LBJoin {
    u64x2* a;          // the operands' cells (cleared behind)
    u64x2* b;
    u64* st;           // a look-back word per chunk, zero on entry
    uint32_t* ticket;  // zero on entry, left zero
    u64* offs_out;     // {0, total}
    ChainArgs cj;      // chain checks (cj.status null: none)
    // (or null) nonzero: the decoders took tokens the images lack (NewTok) — nothing is
    // written, the operands are kept for a second launch once the images know them
    const uint32_t* skip;
};
constexpr u64 kLBCnt = 1ull << 40;              // look-back word: bytes | elements << 40
constexpr u64 kLBVal = (1ull << 62) - 1;

__device__ void lb_finish(const LBJoin& lb, uint32_t nch, uint32_t hdr, uint8_t* out) {
    __shared__ uint32_t s_lb_last;
    __syncthreads();
    if (threadIdx.x == 0) {
        // chunk 0's header bytes (host memory) land before the last block rewrites them;
        // the other blocks' bytes are ordered by the kernel's end
        if (blockIdx.x == 0) __threadfence_system();
        s_lb_last = atomicAdd(lb.ticket, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!s_lb_last || threadIdx.x != 0) return;
    if (lb.skip && *lb.skip) {
        lb.offs_out[0] = 0;
        lb.offs_out[1] = 0;
        *lb.ticket = 0;
        __threadfence_system();
        return;
    }
    u64 w;
    for (;;) {                             // the last chunk's inclusive word (relaxed)
        w = __hip_atomic_load(lb.st + nch - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((w >> 62) == 2) break;
        __builtin_amdgcn_s_sleep(1);
    }
    const u64 bytes = w & (kLBCnt - 1), n = (w & kLBVal) >> 40;
    u64 total;
    if (n) {
        out[hdr + 2] = (uint8_t)(n >> 24);
        out[hdr + 3] = (uint8_t)(n >> 16);
        out[hdr + 4] = (uint8_t)(n >> 8);
        out[hdr + 5] = (uint8_t)n;
        total = hdr + 6 + bytes + 1;
    } else {
        out[hdr + 1] = 106;                 // 131 106: []
        total = hdr + 2;
    }
    lb.offs_out[0] = 0;
    lb.offs_out[1] = total;
    *lb.ticket = 0;
    __threadfence_system();
}

// EPAR (few token slots per element): each element's thread also stages its own records
// (no record -> element search, no rank select); otherwise records are spread over lanes.
// coff != nullptr: split mode (above), block b writes chunks [g cper, (g + 1) cper) of
// payload b / ngroups.
template <uint32_t WIN, bool EPAR, bool LB = false>
__global__ __launch_bounds__(kBlock) void k_orset_etf_write_rec(const u64x2* cells, uint64_t R,
                                                                uint32_t E, DictView d, int tag,
                                                                int vers, const u64* offs,
                                                                uint8_t* out, const u64* coff,
                                                                uint32_t cper, u64 ocap,
                                                                LBJoin lb) {
    if (!LB && offs[R] > ocap) return;
    __shared__ __attribute__((aligned(16))) uint32_t winbuf[(WIN + 2 * kGuard) / 4];
    __shared__ uint32_t s_e[kBlock], s_pos[kBlock + 1], s_rec[kBlock + 1], s_hl[kBlock];
    __shared__ u64 s_p[kBlock], s_r[kBlock], lds4[kBlock / 64];
    uint32_t* win = winbuf + kGuard / 4;
    u32x4* win4 = reinterpret_cast<u32x4*>(win);
    const uint32_t tid = threadIdx.x, hdr = tag >= 0 ? 2u : 0u;
    const uint32_t RL = d.rec_len, RS = d.rec_stride, RK = d.tok_max;
    // a block owns a contiguous run of replicas, whose payloads are contiguous too: the
    // carry flows from one payload into the next and only the run's two ends need
    // byte stores
    const uint32_t nch = (E + kBlock - 1) / kBlock;
    const uint32_t ngroups = coff ? (nch + cper - 1) / cper : 1u;
    uint64_t r_begin, r_end;
    uint32_t c_begin = 0, c_end = E;             // element positions [c_begin, c_end)
    if (LB && blockIdx.x >= nch) {
        // the chain checks: a wave per decoded operand
        const uint32_t r = (blockIdx.x - nch) * 4u + (tid >> 6), lane = tid & 63u;
        if (r < lb.cj.nrep) {
            const u64 base = lb.cj.offs[r];
            const int32_t st = chain_verdict(lb.cj.payload, base, lb.cj.offs[r + 1] - base,
                                             lb.cj.segbase[r], lb.cj.segbase[r + 1] - lb.cj.segbase[r],
                                             lb.cj.S, lb.cj.res, lane);
            if (lane == 0) lb.cj.status[r] = st;
            chain_publish(lb.cj, r, st, lane);
        }
        lb_finish(lb, nch, hdr, out);
        return;
    }
    if (LB && lb.skip && *lb.skip) {
        lb_finish(lb, nch, hdr, out);
        return;
    }
    if (LB) {
        r_begin = 0;
        r_end = 1;
        c_begin = blockIdx.x * kBlock;
        c_end = min(E, c_begin + kBlock);
    } else if (coff) {
        r_begin = blockIdx.x / ngroups;
        r_end = r_begin + 1;
        const uint32_t g = blockIdx.x - (uint32_t)(r_begin * ngroups);
        c_begin = g * cper * kBlock;
        c_end = min(E, (g + 1) * cper * kBlock);
    } else {
        const uint64_t per_blk = (R + gridDim.x - 1) / gridDim.x;
        r_begin = (uint64_t)blockIdx.x * per_blk;
        r_end = r_begin + per_blk < R ? r_begin + per_blk : R;
    }
    if (r_begin >= R) return;
    for (uint32_t x = tid; x < (WIN + 2 * kGuard) / 16; x += kBlock)
        reinterpret_cast<u32x4*>(winbuf)[x] = u32x4{0, 0, 0, 0};
    __syncthreads();
    const u64* cw = reinterpret_cast<const u64*>(cells);
    // one chunk per replica: the element, its term-order token slots, header template
    // and the next replica's cell stay in registers across the run
    const bool single = E <= kBlock;
    uint32_t e_c = 0, hl_c = 0;
    u32x4 o_c = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu}, h_c = {0, 0, 0, 0};
    u64x2 v_next = {0, 0};
    if (single && tid < E) {
        e_c = d.elem_order[tid];
        hl_c = d.elem_off[e_c + 1] - d.elem_off[e_c] + 3u;
        o_c = *reinterpret_cast<const u32x4*>(d.tok_order + 64ull * e_c);
        if (hl_c <= 16) h_c = *reinterpret_cast<const u32x4*>(d.ehdr_pad + d.ehdr_poff[e_c]);
        v_next = cells[r_begin * E + e_c];
    }
    u64 mask_lo = LB ? 0 : offs[r_begin];    // output bytes below this belong to another block
    uint32_t n_split = 0;
    u64 cur_split = 0;
    if (coff) {
        // this block's first byte: the payload's header for chunk 0, else its chunk's
        const u64* co = coff + r_begin * (nch + 1ull);
        n_split = (uint32_t)(co[nch] / kChunkCnt);
        cur_split = mask_lo + hdr + (n_split ? 6u : 2u) + (co[c_begin / kBlock] & (kChunkCnt - 1));
        if (c_begin) mask_lo = cur_split;
    }
    u64 seg_lo = mask_lo;           // bytes [floor16(seg_lo), seg_lo) are the carry in win[0..4)
    for (uint64_t rep = r_begin; rep < r_end; ++rep) {
        const u64x2* c = cells + rep * E;
        const u64 base = LB ? 0 : offs[rep], end = LB ? ocap : offs[rep + 1];
        if (!coff && !LB && seg_lo != base) {
            // the previous payload broke off (sizes disagreed): flush, restart at base
            if (tid < 16) {
                const u64 g = (seg_lo & ~15ull) + tid;
                if (g >= mask_lo && g < seg_lo)
                    out[g] = (uint8_t)(win[tid >> 2] >> (8 * (tid & 3)));
            }
            __syncthreads();
            if (tid == 0) win4[0] = u32x4{0, 0, 0, 0};
            __syncthreads();
            seg_lo = mask_lo = base;
        }
        // present elements (the list header's length field): counted up front when the
        // replica spans several chunks, else taken from the one chunk's scan
        uint32_t n = n_split;
        if (!coff && !LB && E > kBlock) {
            u64 cnt = 0;
            for (uint32_t e = tid; e < E; e += kBlock) cnt += cw[2ull * (rep * E + e)] != 0;
            u64 n64;
            block_excl_scan64(cnt, lds4, &n64);
            n = (uint32_t)n64;
        }
        u64 cursor = cur_split;                     // next element byte
        for (uint32_t c0 = c_begin; c0 < c_end; c0 += kBlock) {
            const bool last = c0 + kBlock >= E;
            // ---- A: element sizes, term-order token masks, record numbering
            const uint32_t i = c0 + tid;
            uint32_t e = 0, sz = 0, nt = 0, hl = 0;
            u64 pt = 0, rt = 0;
            if (i < E) {
                e = single ? e_c : d.elem_order[i];
                u64x2 v;
                if (LB) {
                    // merge/2: the slot-wise OR of the operands' cells, cleared behind
                    const u64 at = rep * E + e;
                    v = lb.a[at] | lb.b[at];
                    lb.a[at] = u64x2{0, 0};
                    lb.b[at] = u64x2{0, 0};
                } else {
                    v = single ? v_next : c[e];
                }
                if (single && rep + 1 < r_end) v_next = c[E + e];       // next replica
                if (v.x) {
                    const u32x4* ord = reinterpret_cast<const u32x4*>(d.tok_order + 64ull * e);
                    for (uint32_t j16 = 0; j16 < RK; j16 += 16) {
                        const u32x4 o = (single && j16 == 0) ? o_c : ord[j16 >> 4];
                        const uint32_t ow[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
                        for (int b = 0; b < 16; ++b) {
                            const uint32_t k = (ow[b >> 2] >> (8 * (b & 3))) & 0xFFu;
                            if (k < 64) {
                                pt |= ((v.x >> k) & 1ull) << (j16 + b);
                                rt |= ((v.y >> k) & 1ull) << (j16 + b);
                            }
                        }
                    }
                    rt &= pt;
                    nt = (uint32_t)__popcll(pt);
                    hl = single ? hl_c : d.elem_off[e + 1] - d.elem_off[e] + 3u;
                    sz = hl + 4u + nt * (RL + 8u) - (uint32_t)__popcll(rt) + 1u;
                }
            }
            // one scan: byte size (32 bits) | records (20) | present elements (12)
            u64 tot2;
            const u64 pr = block_excl_scan64((u64)sz | ((u64)nt << 32) | ((u64)(sz != 0) << 52),
                                             lds4, &tot2);
            const uint32_t pos = (uint32_t)pr, tot = (uint32_t)tot2;
            bool closing;
            if (LB) {
                // this chunk's {bytes, elements} published, its offset looked back for
                __shared__ u64 s_pre;
                if (tid == 0) {
                    const uint32_t ch = c0 / kBlock;
                    const u64 own = (u64)tot + ((tot2 >> 52) & 0xFFFull) * kLBCnt;
                    u64 acc = 0;
                    // (the words carry their whole payload: relaxed device-scope atomics,
                    // no L2 write-back / invalidate per step as release / acquire would)
                    if (ch == 0) {
                        __hip_atomic_store(lb.st, (2ull << 62) | own, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    } else {
                        __hip_atomic_store(lb.st + ch, (1ull << 62) | own, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                        for (int32_t j = (int32_t)ch - 1; j >= 0;) {
                            const u64 w = __hip_atomic_load(lb.st + j, __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT);
                            if (!(w >> 62)) {                     // not published yet
                                __builtin_amdgcn_s_sleep(1);
                                continue;
                            }
                            acc += w & kLBVal;
                            if ((w >> 62) == 2) break;
                            --j;
                        }
                        __hip_atomic_store(lb.st + ch, (2ull << 62) | (acc + own),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                    s_pre = acc;
                }
                __syncthreads();
                const u64 pre = s_pre;
                const u64 ic = ((pre & kLBVal) >> 40) + ((tot2 >> 52) & 0xFFFull);
                n = 1;                              // (a placeholder: lb_finish writes it)
                cursor = hdr + 6u + (pre & (kLBCnt - 1));
                if (c0) mask_lo = cursor;
                seg_lo = mask_lo;
                closing = last && ic != 0;
            } else {
                if (c0 == 0) {
                    if (E <= kBlock) n = (uint32_t)(tot2 >> 52);
                    cursor = base + hdr + (n ? 6u : 2u);
                }
                closing = last && n;
            }
            s_e[tid] = e;
            s_p[tid] = pt;
            s_r[tid] = rt;
            s_hl[tid] = hl;
            s_pos[tid] = pos;
            s_rec[tid] = (uint32_t)(pr >> 32) & 0xFFFFFu;
            if (tid == kBlock - 1) {
                s_pos[kBlock] = tot;
                s_rec[kBlock] = (uint32_t)(tot2 >> 32) & 0xFFFFFu;
            }
            const u64 seg_hi = cursor + tot + (closing ? 1u : 0u);
            if (seg_hi > end) break;                      // sizes disagree: never overrun
            __syncthreads();
            const uint32_t nrec = s_rec[kBlock];
            // ---- B: windows over [floor16(seg_lo), seg_hi)
            for (u64 A = seg_lo & ~15ull; seg_lo < seg_hi && A < seg_hi; A += WIN) {
                const int32_t cur_rel = (int32_t)(int64_t)(cursor - A);  // chunk byte 0, window-relative
                if (c0 == 0 && tid == 0) {                        // 131 108 <n:32> | 131 106
                    uint32_t w[3] = {0, 0, 0};
                    uint32_t nb = 0;
                    auto put = [&](uint32_t byte) { w[nb >> 2] |= byte << (8 * (nb & 3)); ++nb; };
                    if (hdr) { put((uint32_t)tag & 0xFFu); put((uint32_t)vers & 0xFFu); }
                    put(131);
                    if (n) {
                        put(108); put(n >> 24); put((n >> 16) & 0xFFu); put((n >> 8) & 0xFFu);
                        put(n & 0xFFu);
                    } else {
                        put(106);
                    }
                    const int32_t rel = (int32_t)(int64_t)(base - A);
                    if (overlaps<WIN>(rel, nb)) or_piece<3>(win, rel, w, 8);
                }
                if (closing && tid == 0) {
                    const uint32_t w[1] = {106u};
                    const int32_t rel = cur_rel + (int32_t)tot;
                    if (overlaps<WIN>(rel, 1)) or_piece<1>(win, rel, w, 1);
                }
                // element headers 104 2 <elem> 108 <n:32> and closing 106
                if (sz) {
                    const int32_t r0 = cur_rel + (int32_t)pos;
                    if (overlaps<WIN>(r0, sz)) {
                        if (hl <= 16) {
                            if (overlaps<WIN>(r0, hl)) {
                                const u32x4 h = single ? h_c : *reinterpret_cast<const u32x4*>(
                                    d.ehdr_pad + d.ehdr_poff[e]);
                                const uint32_t w[4] = {h.x, h.y, h.z, h.w};
                                or_piece<4>(win, r0, w, 16);
                            }
                        } else if (hl <= 48) {
                            if (overlaps<WIN>(r0, hl)) {
                                uint32_t w[12];
                                load_piece48(w, d.ehdr_pad + d.ehdr_poff[e], hl);
                                or_piece<12>(win, r0, w, 48);
                            }
                        } else {
                            uint8_t pre[2] = {104, 2};
                            or_bytes_slow<WIN>(win, r0, pre, 2);
                            or_bytes_slow<WIN>(win, r0 + 2, d.elem_blob + d.elem_off[e], hl - 3u);
                            uint8_t post[1] = {108};
                            or_bytes_slow<WIN>(win, r0 + hl - 1, post, 1);
                        }
                        const uint32_t wn[1] = {__builtin_bswap32(nt)};
                        if (overlaps<WIN>(r0 + (int32_t)hl, 4)) or_piece<1>(win, r0 + (int32_t)hl, wn, 4);
                        const uint32_t wc[1] = {106u};
                        if (overlaps<WIN>(r0 + (int32_t)sz - 1, 1)) or_piece<1>(win, r0 + (int32_t)sz - 1, wc, 1);
                    }
                }
                if (EPAR) {
                    // this thread's element: its records in term order, one after another
                    if (sz && overlaps<WIN>(cur_rel + (int32_t)pos, sz)) {
                        int32_t rel = cur_rel + (int32_t)(pos + hl + 4u);
                        for (u64 m = pt; m; m &= m - 1) {
                            const uint32_t rank = (uint32_t)__ffsll((long long)m) - 1u;
                            const bool rm = (rt >> rank) & 1ull;
                            if (overlaps<WIN>(rel, RL)) {
                                uint32_t w[12];
                                load_piece48(w, d.rec_pad + ((u64)e * RK + rank) * RS, RL);
                                or_piece<12>(win, rel, w, RL);
                            }
                            const uint32_t wa[2] = {rm ? 0x74040064u : 0x66050064u,
                                                    rm ? 0x00657572u : 0x65736c61u};
                            if (overlaps<WIN>(rel + (int32_t)RL, 8))
                                or_piece<2>(win, rel + (int32_t)RL, wa, 8);
                            rel += (int32_t)(RL + (rm ? 7u : 8u));
                        }
                    }
                } else {
                    // records whose element intersects the window
                    // jlo = first element ending after the window start, jhi = first one
                    // starting at or past its end (both monotone: one ballot per 64 elements)
                    uint32_t jlo = kBlock, jhi = kBlock;
                    {
                        const uint32_t lane = tid & 63u;
    #pragma unroll
                        for (uint32_t k = 0; k < kBlock / 64; ++k) {
                            const uint32_t m = 64u * k + lane;
                            const u64 b1 = __ballot(cur_rel + (int32_t)s_pos[m + 1] > 0);
                            const u64 b2 = __ballot(cur_rel + (int32_t)s_pos[m] >= (int32_t)WIN);
                            if (jlo == kBlock && b1) jlo = 64u * k + (uint32_t)__ffsll((long long)b1) - 1u;
                            if (jhi == kBlock && b2) jhi = 64u * k + (uint32_t)__ffsll((long long)b2) - 1u;
                        }
                    }
                    const uint32_t r_lo = jlo < kBlock ? s_rec[jlo] : nrec;
                    const uint32_t r_hi = s_rec[jhi];
                    // each thread takes a run of consecutive records: the element of the
                    // run's first record by binary search and its token by rank select,
                    // then the next record is the next present token (one find-first-set)
                    // or the next element's first, its position the previous end
                    const uint32_t per = (r_hi - r_lo + kBlock - 1) / kBlock;
                    uint32_t ri = r_lo + tid * per;
                    const uint32_t re = min(ri + per, r_hi);
                    if (ri < re) {
                        uint32_t lo = jlo, hi = jhi;            // last j with s_rec[j] <= ri
                        while (hi - lo > 1) {
                            const uint32_t m = (lo + hi) >> 1;
                            if (s_rec[m] <= ri) lo = m;
                            else hi = m;
                        }
                        uint32_t j = lo;
                        const uint32_t rho = ri - s_rec[j];
                        u64 pj = s_p[j], rj = s_r[j];
                        uint32_t jend = s_rec[j + 1], e = s_e[j];
                        uint32_t rank = select64(pj, rho);
                        const u64 below = rank ? (~0ull >> (64u - rank)) : 0ull;
                        int32_t rel = cur_rel + (int32_t)(s_pos[j] + s_hl[j] + 4u +
                                                          rho * (RL + 8u) -
                                                          (uint32_t)__popcll(rj & below));
                        for (;;) {
                            const bool rm = (rj >> rank) & 1ull;
                            if (overlaps<WIN>(rel, RL)) {
                                uint32_t w[12];
                                load_piece48(w, d.rec_pad + ((u64)e * RK + rank) * RS, RL);
                                or_piece<12>(win, rel, w, RL);
                            }
                            // ATOM_EXT true = 100 0 4 "true", false = 100 0 5 "false"
                            const uint32_t wa[2] = {rm ? 0x74040064u : 0x66050064u,
                                                    rm ? 0x00657572u : 0x65736c61u};
                            if (overlaps<WIN>(rel + (int32_t)RL, 8))
                                or_piece<2>(win, rel + (int32_t)RL, wa, 8);
                            if (++ri >= re) break;
                            if (ri < jend) {                     // the element's next token
                                rel += (int32_t)(RL + (rm ? 7u : 8u));
                                rank = (uint32_t)__ffsll((long long)(pj & (~1ull << rank))) - 1u;
                            } else {                             // the next element's first
                                do ++j; while (s_rec[j + 1] <= ri);
                                pj = s_p[j];
                                rj = s_r[j];
                                jend = s_rec[j + 1];
                                e = s_e[j];
                                rank = (uint32_t)__ffsll((long long)pj) - 1u;
                                rel = cur_rel + (int32_t)(s_pos[j] + s_hl[j] + 4u);
                            }
                        }
                    }
                }
                __syncthreads();
                // whole 16-byte chunks out; the partial one below seg_hi stays as the carry
                const u64 wend = A + WIN < seg_hi ? A + WIN : seg_hi;
                const uint32_t full = (uint32_t)((wend - A) >> 4);
                for (uint32_t m = tid; m < full; m += kBlock) {
                    const u64 g = A + 16ull * m;
                    const u32x4 v = win4[m];
                    if (g >= mask_lo) {
                        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(out + g));
                    } else {
                        const uint32_t vw[4] = {v.x, v.y, v.z, v.w};
                        for (uint32_t b = (uint32_t)(mask_lo - g); b < 16; ++b)
                            out[g + b] = (uint8_t)(vw[b >> 2] >> (8 * (b & 3)));
                    }
                    win4[m] = u32x4{0, 0, 0, 0};
                }
                if (tid == 0 && full > 0 && wend == seg_hi && (seg_hi & 15u)) {
                    win4[0] = win4[full];
                    win4[full] = u32x4{0, 0, 0, 0};
                }
                if (tid >= kBlock - 2 * kGuard / 16) {          // clear both guards
                    const uint32_t gi = tid - (kBlock - 2 * kGuard / 16);
                    const uint32_t x = gi < kGuard / 16 ? gi : (kGuard + WIN) / 16 + gi - kGuard / 16;
                    reinterpret_cast<u32x4*>(winbuf)[x] = u32x4{0, 0, 0, 0};
                }
                __syncthreads();
            }
            seg_lo = seg_hi;
            cursor += tot;
        }
    }
    // flush the carry at the end of the run: bytes [floor16(seg_lo), seg_lo)
    if (tid < 16) {
        const u64 g = (seg_lo & ~15ull) + tid;
        if (g >= mask_lo && g < seg_lo) out[g] = (uint8_t)(win[tid >> 2] >> (8 * (tid & 3)));
    }
    if (LB) lb_finish(lb, nch, hdr, out);
}

// One wave per G-Set payload: lanes over element slots, 64 per word, the payload's words
// held in registers (lane j: word j of each group of 64) and four words' worth of
// dictionary loads in flight at a time (a loop over each lane's set bits waited for one
// load per element).  Per payload: element count, image bytes, whether every element is
// a byte integer (STRING_EXT), and a present slot without an image or a bit past E (the
// error flag).
struct GsCount {
    u64 sum = 0;               // image bytes of the present elements
    uint32_t n = 0, nb = 0;    // present elements, of them not byte integers
    bool bad = false;          // a present slot without an image, or a bit past E
};

template <bool SUM>
__device__ __forceinline__ GsCount gs_count(const u64* w, uint32_t E, uint32_t W,
                                            const DictView& d, uint32_t lane) {
    GsCount r;
    for (uint32_t g0 = 0; g0 < W; g0 += 64) {
        const uint32_t wi = g0 + lane;
        const u64 wv = wi < W ? w[wi] : 0ull;
        if (wi >= (E >> 6) && wv) {
            const u64 past = wi == (E >> 6) ? wv & ~((1ull << (E & 63u)) - 1ull) : wv;
            r.bad |= past != 0;
        }
        const uint32_t nw = min(64u, W - g0);
        for (uint32_t j0 = 0; j0 < nw; j0 += 4) {
            uint32_t el[4], by[4];
            bool hr[4];
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) {
                const uint32_t jj = j0 + j;
                const u64 word = __shfl(wv, (int)min(jj, 63u), 64);
                const uint32_t e = (g0 + jj) * 64u + lane;
                hr[j] = jj < nw && e < E && ((word >> lane) & 1ull);
                el[j] = 0;
                by[j] = 1;
                if (hr[j]) {
                    if (SUM) el[j] = d.elem_off[e + 1] - d.elem_off[e];
                    by[j] = d.elem_byte[e];
                }
            }
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j)
                if (hr[j]) {
                    if (SUM) {
                        r.bad |= el[j] == 0;
                        r.sum += el[j];
                    }
                    r.nb += by[j] == 0;
                    ++r.n;
                }
        }
    }
    return r;
}

__global__ __launch_bounds__(kBlock) void k_gset_etf_size(const u64* words, uint64_t R,
                                                          uint32_t E, uint32_t W, DictView d,
                                                          uint32_t hdr, u64* sizes,
                                                          uint32_t* flag) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t waves = (uint64_t)gridDim.x * (kBlock / 64);
    for (uint64_t rep = (uint64_t)blockIdx.x * (kBlock / 64) + threadIdx.x / 64; rep < R;
         rep += waves) {
        const GsCount c = gs_count<true>(words + rep * W, E, W, d, lane);
        const u64 sum = wave_sum(c.sum), n = wave_sum((u64)c.n), nb = wave_sum((u64)c.nb);
        const bool any_bad = __ballot(c.bad) != 0;
        if (lane == 0) {
            const u64 body = n == 0 ? 1u : (nb == 0 && n < 65536u) ? 3u + n : 5u + sum + 1u;
            sizes[rep] = hdr + 1u + body;
            if (any_bad) atomicOr(flag, 1u);
        }
    }
}

__global__ __launch_bounds__(kBlock) void k_gset_etf_write(const u64* words, uint64_t R,
                                                           uint32_t E, uint32_t W, DictView d,
                                                           int tag, int vers, const u64* offs,
                                                           uint8_t* out, u64 ocap) {
    if (offs[R] > ocap) return;
    __shared__ uint32_t lds4[kBlock / 64];
    __shared__ __attribute__((aligned(16))) uint8_t buf[kWin + 16];
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
            const uint32_t i = c0 + threadIdx.x;
            const uint32_t e = i < E ? d.elem_order[i] : 0u;
            const bool here = i < E && ((w[e >> 6] >> (e & 63u)) & 1ull);
            const uint32_t el = d.elem_off[e + 1] - d.elem_off[e];
            const uint32_t sz = here ? (str ? 1u : el) : 0u;
            uint32_t tot;
            const uint32_t pos = block_excl_scan(sz, lds4, &tot);
            if (cursor + tot + (str ? 0u : 1u) > end) break;
            for (uint32_t w0 = 0; w0 < tot; w0 += kWin) {
                const uint32_t wl = min(kWin, tot - w0);
                const u64 g = cursor + w0;
                const uint32_t sh = (uint32_t)(g & 15u);
                const Win win{buf + sh, w0, wl};
                if (here) {
                    const uint8_t* src = d.elem_blob + d.elem_off[e];
                    if (str) win.put(pos, src[1]);
                    else if (el <= 48 && inside(win, pos, el))
                        lds_put48(win.buf + (pos - w0), d.elem_pad + d.elem_poff[e], el);
                    else win.span(pos, src, el);
                }
                __syncthreads();
                copy_out(buf, sh, wl, out, g);
                __syncthreads();
            }
            cursor += tot;
        }
        if (threadIdx.x == 0) {
            write_list_header(out, base, hdr, tag, vers, n == 0 ? 106 : str ? 107 : 108, n);
            if (n && !str && cursor < end) out[cursor] = 106;
        }
        __syncthreads();
    }
}

// One wave per G-Set payload (the payloads are short: a few bytes per element): lanes
// take 64 element slots at a time in term order, a wave prefix sum of their image
// lengths places them, and each lane stores its image bytes straight into the payload
// (byte stores of consecutive lanes fill consecutive bytes of a line).  Same bytes as
// k_gset_etf_write: 131 107 <n:16> <bytes> (STRING_EXT, every element a byte integer,
// n < 65536), 131 108 <n:32> <images> 106, or 131 106.
__global__ __launch_bounds__(kBlock) void k_gset_etf_write_wave(const u64* words, uint64_t R,
                                                                uint32_t E, uint32_t W,
                                                                DictView d, int tag, int vers,
                                                                const u64* offs, uint8_t* out,
                                                                u64 ocap) {
    if (offs[R] > ocap) return;
    const uint32_t lane = threadIdx.x & 63u, hdr = tag >= 0 ? 2u : 0u;
    const uint64_t nwaves = (uint64_t)gridDim.x * (kBlock / 64);
    for (uint64_t rep = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 6; rep < R;
         rep += nwaves) {
        const u64* w = words + rep * W;
        const u64 base = offs[rep], end = offs[rep + 1];
        // (a bit past E counts as not a byte integer, as the size pass refused it)
        const GsCount cnt = gs_count<false>(w, E, W, d, lane);
        const uint32_t n = (uint32_t)wave_sum((u64)cnt.n),
                       nonbyte = (uint32_t)wave_sum((u64)cnt.nb + (cnt.bad ? 1u : 0u));
        // the payload's words in registers (lane j: word j) when they fit one group
        const u64 wreg = W <= 64 && lane < W ? w[lane] : 0ull;
        const bool str = n > 0 && nonbyte == 0 && n < 65536u;
        u64 cursor = base + hdr + 1u + (str ? 3u : 5u);
        bool fits = true;
        for (uint32_t c0 = 0; c0 < E && n && fits; c0 += 64) {
            const uint32_t i = c0 + lane;
            const uint32_t e = i < E ? d.elem_order[i] : 0u;
            const u64 word = W <= 64 ? __shfl(wreg, (int)(e >> 6), 64) : w[e >> 6];
            const bool here = i < E && ((word >> (e & 63u)) & 1ull);
            const uint32_t el = here ? d.elem_off[e + 1] - d.elem_off[e] : 0u;
            const uint32_t sz = here ? (str ? 1u : el) : 0u;
            uint32_t x = sz;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t y = __shfl_up(x, off, 64);
                if ((int)lane >= off) x += y;
            }
            const uint32_t tot = __shfl(x, 63, 64), pos = x - sz;
            if (cursor + tot + (str ? 0u : 1u) > end) {        // sizes disagree: never overrun
                fits = false;
                break;
            }
            if (here) {
                uint8_t* o = out + cursor + pos;
                const uint8_t* src = d.elem_blob + d.elem_off[e];
                if (str) {
                    o[0] = src[1];
                } else if (el <= 16) {
                    const u32x4 t = *reinterpret_cast<const u32x4*>(d.elem_pad + d.elem_poff[e]);
                    const uint32_t tw[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
                    for (uint32_t b = 0; b < 16; ++b)
                        if (b < el) o[b] = (uint8_t)(tw[b >> 2] >> (8 * (b & 3)));
                } else {
                    for (uint32_t b = 0; b < el; ++b) o[b] = src[b];
                }
            }
            cursor += tot;
        }
        if (lane == 0) {
            write_list_header(out, base, hdr, tag, vers, n == 0 ? 106 : str ? 107 : 108, n);
            if (fits && n && !str && cursor < end) out[cursor] = 106;
        }
    }
}

// Split G-Set writer (few long payloads: the NIF's value/1 and merge answers, one 10k-
// element ordset each, which one wave walking 64 elements at a time wrote in ~400 us): a
// block takes a chunk of 256 slots in term order.  k_gset_chunk_sizes gives each chunk its
// image bytes and element counts {bytes, elements | non-byte-integer elements << 32};
// k_gset_chunk_scan (one block) turns them into per-payload exclusive prefixes (entry nch
// = the payload's totals) and, with `offsets`, the payload offsets (k_gset_etf_size's
// sizes, scanned); k_gset_write_chunks writes each chunk's images from its prefix (bytes,
// or elements under STRING_EXT), chunk 0 the list header, the last chunk the tail.
// the source of the present elements: SRC 0 a G-Set batch's bits; 1 an OR-Set batch's
// {p, r} cells, an element present when it has a {Token, false} (value/1's G-Set image
// written without value bits in between); 2 the OR of two G-Set batches' bits (merge/2's
// answer written without the merged bits in between)
template <int SRC>
__device__ __forceinline__ bool gs_here(const u64* words, const u64* words2, uint64_t rep,
                                        uint32_t W, uint32_t E, uint32_t e) {
    if (SRC == 1) {
        const u64x2 x = reinterpret_cast<const u64x2*>(words)[rep * E + e];
        return (x.x & ~x.y) != 0;
    }
    const u64 w = SRC == 2 ? words[rep * W + (e >> 6)] | words2[rep * W + (e >> 6)]
                           : words[rep * W + (e >> 6)];
    return (w >> (e & 63u)) & 1ull;
}

// cj.status (SRC 1: value/1 of decoded operands, the segment decoder's chain check
// deferred here, ChainJob): the first chunk's block of each payload judges its segment
// chain (chain_verdict) and stores the decode status
template <int SRC>
__global__ __launch_bounds__(kBlock) void k_gset_chunk_sizes(const u64* words, const u64* words2,
                                                             uint64_t R, uint32_t E, uint32_t W,
                                                             DictView d, uint32_t nch, u64x2* co,
                                                             uint32_t* flag, ChainArgs cj) {
    __shared__ u64 lds4[kBlock / 64];
    for (uint64_t it = blockIdx.x; it < R * nch; it += gridDim.x) {
        const uint64_t rep = it / nch;
        const uint32_t c = (uint32_t)(it - rep * nch), i = c * kBlock + threadIdx.x;
        if (SRC == 1 && cj.status && c == 0 && threadIdx.x < 64) {
            const u64 base = cj.offs[rep];
            const int32_t st = chain_verdict(cj.payload, base, cj.offs[rep + 1] - base,
                                             cj.segbase[rep], cj.segbase[rep + 1] - cj.segbase[rep],
                                             cj.S, cj.res, threadIdx.x);
            if (threadIdx.x == 0) cj.status[rep] = st;
            chain_publish(cj, (uint32_t)rep, st, threadIdx.x);
        }
        const u64* w = words + rep * W;
        u64 by = 0, cn = 0;
        if (i < E) {
            const uint32_t e = d.elem_order[i];
            if (gs_here<SRC>(words, words2, rep, W, E, e)) {
                const uint32_t el = d.elem_off[e + 1] - d.elem_off[e];
                // as k_gset_etf_size: a present slot without an image is an error
                if (el == 0 && flag) atomicOr(flag, 1u);
                by = el;
                cn = 1ull + (d.elem_byte[e] == 0 ? (1ull << 32) : 0ull);
            }
        }
        if (SRC != 1 && c == 0 && flag)              // bits of no slot (past E): an error too
            for (uint32_t wi = (E >> 6) + threadIdx.x; wi < W; wi += kBlock) {
                u64 m = w[wi] | (SRC == 2 ? words2[rep * W + wi] : 0ull);
                if (wi == (E >> 6)) m &= ~((1ull << (E & 63u)) - 1ull);
                if (m) atomicOr(flag, 1u);
            }
        u64 tb, tc;
        block_excl_scan64(by, lds4, &tb);
        block_excl_scan64(cn, lds4, &tc);
        if (threadIdx.x == 0) co[rep * (nch + 1ull) + c] = u64x2{tb, tc};
    }
}

__global__ __launch_bounds__(kBlock) void k_gset_chunk_scan(u64x2* co, uint64_t R, uint32_t nch,
                                                            uint32_t hdr, u64* offsets) {
    __shared__ u64 lds4[kBlock / 64];
    u64 run = 0;                                     // payload offset (one block: few payloads)
    for (uint64_t rep = 0; rep < R; ++rep) {
        u64x2* c = co + rep * (nch + 1ull);
        u64 cb = 0, cc = 0;
        for (uint32_t t0 = 0; t0 <= nch; t0 += kBlock) {
            const uint32_t t = t0 + threadIdx.x;
            const u64x2 v = t < nch ? c[t] : u64x2{0, 0};
            u64 tb, tc;
            const u64 eb = block_excl_scan64(v.x, lds4, &tb);
            const u64 ec = block_excl_scan64(v.y, lds4, &tc);
            if (t <= nch) c[t] = u64x2{cb + eb, cc + ec};
            cb += tb;
            cc += tc;
        }
        if (offsets) {
            const uint32_t n = (uint32_t)cc, nb = (uint32_t)(cc >> 32);
            const u64 body = n == 0 ? 1u : (nb == 0 && n < 65536u) ? 3u + n : 5u + cb + 1u;
            if (threadIdx.x == 0) offsets[rep] = run;
            run += hdr + 1u + body;
        }
    }
    if (offsets && threadIdx.x == 0) offsets[R] = run;
}

// ZERO (SRC 1 only): the source cells are cleared behind the reads (the NIF's decoded
// operand: the next call's decoder then needs no memset), whether or not the answer fits
template <int SRC, bool ZERO>
__global__ __launch_bounds__(kBlock) void k_gset_write_chunks(const u64* words, const u64* words2,
                                                              uint64_t R, uint32_t E, uint32_t W,
                                                              DictView d, int tag, int vers,
                                                              const u64* offs, uint8_t* out,
                                                              u64 ocap, const u64x2* co,
                                                              uint32_t nch) {
    static_assert(!ZERO || SRC == 1, "only cells are cleared behind the reads");
    const bool room = offs[R] <= ocap;
    if (!ZERO && !room) return;
    __shared__ u64 lds4[kBlock / 64];
    const uint32_t hdr = tag >= 0 ? 2u : 0u;
    for (uint64_t it = blockIdx.x; it < R * nch; it += gridDim.x) {
        const uint64_t rep = it / nch;
        const uint32_t c = (uint32_t)(it - rep * nch), i = c * kBlock + threadIdx.x;
        const u64x2 pre = co[rep * (nch + 1ull) + c], all = co[rep * (nch + 1ull) + nch];
        const uint32_t n = (uint32_t)all.y, nb = (uint32_t)(all.y >> 32);
        const bool str = n > 0 && nb == 0 && n < 65536u;
        const u64 base = offs[rep], end = offs[rep + 1];
        const u64 cursor = base + hdr + 1u + (str ? 3u : 5u) + (str ? (uint32_t)pre.y : pre.x);
        uint32_t e = 0, el = 0;
        bool here = false;
        if (i < E) {
            e = d.elem_order[i];
            here = gs_here<SRC>(words, words2, rep, W, E, e);
            if (ZERO) reinterpret_cast<u64x2*>(const_cast<u64*>(words))[rep * E + e] = u64x2{0, 0};
            if (here) el = d.elem_off[e + 1] - d.elem_off[e];
        }
        const u64 sz = here ? (str ? 1u : el) : 0u;
        u64 tot;
        const u64 pos = block_excl_scan64(sz, lds4, &tot);
        // sizes disagree with the offsets: never overrun the payload
        const bool fits = room && cursor + tot + (str ? 0u : 1u) <= end;
        if (fits && here) {
            uint8_t* o = out + cursor + pos;
            const uint8_t* src = d.elem_blob + d.elem_off[e];
            if (str) {
                o[0] = src[1];
            } else if (el <= 16) {
                const u32x4 t = *reinterpret_cast<const u32x4*>(d.elem_pad + d.elem_poff[e]);
                const uint32_t tw[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
                for (uint32_t b = 0; b < 16; ++b)
                    if (b < el) o[b] = (uint8_t)(tw[b >> 2] >> (8 * (b & 3)));
            } else {
                for (uint32_t b = 0; b < el; ++b) o[b] = src[b];
            }
        }
        if (threadIdx.x == 0 && room) {
            if (c == 0) write_list_header(out, base, hdr, tag, vers, n == 0 ? 106 : str ? 107 : 108, n);
            if (c == nch - 1 && fits && n && !str && cursor + tot < end) out[cursor + tot] = 106;
        }
    }
}

// ------------------------------------------------------------------ from_binary/1
// binary_to_term of OR-Set payloads into cells (lasp_orset.erl:202-214 decodes with
// riak_dt:from_binary/1 = binary_to_term/1), for dictionaries with uniform token images.
// One wave parses one replica: the payload streams through a 2 KiB LDS window; the
// element at the cursor is found by 64 lanes comparing the header templates
// `104 2 <elem image> 108` of the next 64 elements in term order, each record likewise
// by 64 lanes comparing `104 2 <token image>` of the element's next 64 token ranks,
// then the flag atom (ATOM_EXT, ATOM_UTF8_EXT or SMALL_ATOM_UTF8_EXT).  Elements and
// tokens must come in term order (an orddict), so every comparison is a forward scan.
// One wave copies nv 16-byte vectors from global memory into LDS with NL loads in flight
// per lane: a plain `for (v = lane; v < nv; v += 64) lds[v] = src[v]` loop waits for each
// load before its LDS store (checked in the ISA), one memory round trip per KiB staged.
template <uint32_t NL>
__device__ __forceinline__ void wave_copy16(uint8_t* dst, const uint8_t* src, uint32_t nv,
                                            uint32_t lane) {
    u32x4* d = reinterpret_cast<u32x4*>(dst);
    const u32x4* s = reinterpret_cast<const u32x4*>(src);
    for (uint32_t v0 = 0; v0 < nv; v0 += 64 * NL) {
        u32x4 t[NL];
#pragma unroll
        for (uint32_t j = 0; j < NL; ++j) {
            const uint32_t v = v0 + 64 * j + lane;
            if (v < nv) t[j] = s[v];
        }
#pragma unroll
        for (uint32_t j = 0; j < NL; ++j) {
            const uint32_t v = v0 + 64 * j + lane;
            if (v < nv) d[v] = t[j];
        }
    }
}

constexpr uint32_t kDWin = 2048;

struct Stage {
    uint8_t* buf;          // wave-private LDS window
    const uint8_t* src;    // the payload buffer
    u64 total;             // bytes in the payload buffer
    u64 lo, hi;            // staged [lo, hi)
    uint32_t win = kDWin;  // window bytes
};

// make [p, p + n) resident (n <= s.win - 16; wave-uniform); false past `lim`
__device__ bool stage_span(Stage& s, u64 p, uint32_t n, u64 lim) {
    if (p + n > lim) return false;
    if (p >= s.lo && p + n <= s.hi) return true;
    const u64 lo = p & ~15ull;
    const u64 hi = min(s.total, lo + s.win);
    const uint32_t lane = threadIdx.x & 63u;
    wave_sync();
    const u64 nfull = (hi - lo) >> 4;
    wave_copy16<4>(s.buf, s.src + lo, (uint32_t)nfull, lane);
    for (u64 b = lo + 16 * nfull + lane; b < hi; b += 64) s.buf[b - lo] = s.src[b];
    wave_sync();
    s.lo = lo;
    s.hi = hi;
    return true;
}

__device__ __forceinline__ uint32_t at(const Stage& s, u64 p) { return s.buf[p - s.lo]; }

// 48-byte template in registers: words of a 16-byte-aligned zero-padded image
__device__ __forceinline__ void load48(uint32_t (&w)[12], const uint8_t* t16, uint32_t L) {
    const u32x4* t = reinterpret_cast<const u32x4*>(t16);
    const u32x4 z = {0, 0, 0, 0};
    const u32x4 a = t[0], b = L > 16 ? t[1] : z, c = L > 32 ? t[2] : z;
    w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
    w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
    w[8] = c.x; w[9] = c.y; w[10] = c.z; w[11] = c.w;
}

// staged bytes [p, p + L) equal the 16-byte-aligned, zero-padded template (L <= 48)
__device__ __forceinline__ bool same48(const Stage& s, u64 p, const uint8_t* t16, uint32_t L) {
    const u32x4* t = reinterpret_cast<const u32x4*>(t16);
    const u32x4 z = {0, 0, 0, 0};
    const u32x4 a = t[0], b = L > 16 ? t[1] : z, c = L > 32 ? t[2] : z;
    const uint32_t w[12] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w};
    const uint8_t* q = s.buf + (p - s.lo);
    bool eq = true;
#pragma unroll
    for (uint32_t i = 0; i < 48; ++i)
        if (i < L) eq &= q[i] == ((w[i >> 2] >> (8 * (i & 3))) & 0xFFu);
    return eq;
}

// longer templates (element images past 45 bytes), already staged
__device__ bool same_long(const Stage& s, u64 p, const uint8_t* t, uint32_t L) {
    const uint8_t* q = s.buf + (p - s.lo);
    for (uint32_t i = 0; i < L; ++i)
        if (q[i] != t[i]) return false;
    return true;
}

__global__ __launch_bounds__(kBlock) void k_orset_etf_read_serial(const uint8_t* payload, u64 total,
                                                                  const u64* offs, uint64_t R,
                                                                  uint32_t E, DictView d, int tag,
                                                                  int vers, u64x2* cells,
                                                                  int32_t* status) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[kBlock / 64][kDWin];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t RL = d.rec_len, RS = d.rec_stride, RK = d.tok_max;
    const uint64_t nwaves = (uint64_t)gridDim.x * (kBlock / 64);
    for (uint64_t rep = (uint64_t)blockIdx.x * (kBlock / 64) + wave; rep < R; rep += nwaves) {
        Stage s{stage[wave], payload, total, 0, 0};
        const u64 base = offs[rep], end = offs[rep + 1];
        u64 p = base;
        int32_t st = LASPJ_DEC_OK;
        u64x2* c = cells + rep * E;
        do {
            if (tag >= 0) {
                if (!stage_span(s, p, 2, end) || at(s, p) != (uint32_t)(tag & 0xFF)) {
                    st = LASPJ_DEC_INVALID_BINARY;
                    break;
                }
                if (at(s, p + 1) != (uint32_t)(vers & 0xFF)) {
                    st = LASPJ_DEC_UNSUPPORTED_VERSION;
                    break;
                }
                p += 2;
            }
            if (!stage_span(s, p, 2, end) || at(s, p) != 131) {
                st = LASPJ_DEC_MALFORMED;                 // binary_to_term: badarg
                break;
            }
            uint32_t n = 0;
            bool list = false;             // LIST_EXT (also of 0 elements): its tail follows
            if (at(s, p + 1) == 106) {
                p += 2;
            } else if (at(s, p + 1) == 108 && stage_span(s, p, 6, end)) {
                n = (at(s, p + 2) << 24) | (at(s, p + 3) << 16) | (at(s, p + 4) << 8) | at(s, p + 5);
                p += 6;
                list = true;
            } else {
                st = LASPJ_DEC_MALFORMED;
                break;
            }
            int64_t prev = -1;                    // term rank of the previous element
            for (uint32_t k = 0; k < n && st == LASPJ_DEC_OK; ++k) {
                // 104 2 <elem image> 108 of the next elements in term order
                const uint32_t span = (uint32_t)min((u64)(kDWin - 16), end - p);
                if (!stage_span(s, p, span, end)) { st = LASPJ_DEC_MALFORMED; break; }
                int64_t found = -1;
                uint32_t e = 0, hl = 0;
                for (int64_t c0 = prev + 1; c0 < (int64_t)E && found < 0; c0 += 64) {
                    const int64_t r = c0 + lane;
                    bool hit = false;
                    uint32_t ec = 0, hlc = 0;
                    if (r < (int64_t)E) {
                        ec = d.elem_order[r];
                        hlc = d.elem_off[ec + 1] - d.elem_off[ec] + 3u;
                        // 104 2 <elem image> (the template's closing 108 is checked below)
                        if (hlc > 3u && hlc <= span) {
                            const uint8_t* t = d.ehdr_pad + d.ehdr_poff[ec];
                            hit = hlc - 1u <= 48 ? same48(s, p, t, hlc - 1u)
                                                 : same_long(s, p, t, hlc - 1u);
                        }
                    }
                    const u64 m = __ballot(hit);
                    if (m) {
                        const uint32_t w = (uint32_t)__ffsll((long long)m) - 1u;
                        found = c0 + w;
                        e = __shfl(ec, w, 64);
                        hl = __shfl(hlc, w, 64);
                    }
                }
                if (found < 0) { st = LASPJ_DEC_UNKNOWN_TERM; break; }
                prev = found;
                p += hl;
                if (at(s, p - 1) != 108) {                 // [] tokens: no columnar form
                    st = at(s, p - 1) == 106 ? LASPJ_DEC_UNREPRESENTABLE : LASPJ_DEC_MALFORMED;
                    break;
                }
                if (!stage_span(s, p, 4, end)) { st = LASPJ_DEC_MALFORMED; break; }  // truncated count
                const uint32_t m_tok = (at(s, p) << 24) | (at(s, p + 1) << 16) | (at(s, p + 2) << 8) |
                                       at(s, p + 3);
                p += 4;
                if (m_tok == 0 || m_tok > 64) { st = LASPJ_DEC_UNREPRESENTABLE; break; }
                u64 pb = 0, rb = 0;
                int32_t tprev = -1;
                for (uint32_t j = 0; j < m_tok; ++j) {
                    if (!stage_span(s, p, RL + 8u, end) && !stage_span(s, p, RL + 6u, end)) {
                        st = LASPJ_DEC_MALFORMED;
                        break;
                    }
                    const int32_t q = tprev + 1 + (int32_t)lane;
                    bool hit = false;
                    if (q < (int32_t)RK && p + RL <= s.hi)
                        hit = same48(s, p, d.rec_pad + ((u64)e * RK + (uint32_t)q) * RS, RL);
                    const u64 m = __ballot(hit);
                    if (!m) { st = LASPJ_DEC_UNKNOWN_TERM; break; }
                    const int32_t rank = tprev + (int32_t)__ffsll((long long)m);
                    tprev = rank;
                    p += RL;
                    // the flag: ATOM_EXT / ATOM_UTF8_EXT (100 / 118, 2-byte length) or
                    // SMALL_ATOM_UTF8_EXT (119, 1-byte length), "true" or "false"
                    const uint32_t t0 = p < s.hi ? at(s, p) : 0u;
                    uint32_t len, h;
                    if ((t0 == 100 || t0 == 118) && p + 3 <= s.hi && at(s, p + 1) == 0) {
                        len = at(s, p + 2);
                        h = 3;
                    } else if (t0 == 119 && p + 2 <= s.hi) {
                        len = at(s, p + 1);
                        h = 2;
                    } else {
                        st = LASPJ_DEC_MALFORMED;
                        break;
                    }
                    bool flag;
                    if (len == 4 && p + h + 4 <= end && stage_span(s, p, h + 4, end) &&
                        at(s, p + h) == 't' && at(s, p + h + 1) == 'r' && at(s, p + h + 2) == 'u' &&
                        at(s, p + h + 3) == 'e') {
                        flag = true;
                    } else if (len == 5 && p + h + 5 <= end && stage_span(s, p, h + 5, end) &&
                               at(s, p + h) == 'f' && at(s, p + h + 1) == 'a' &&
                               at(s, p + h + 2) == 'l' && at(s, p + h + 3) == 's' &&
                               at(s, p + h + 4) == 'e') {
                        flag = false;
                    } else {
                        st = LASPJ_DEC_MALFORMED;
                        break;
                    }
                    p += h + len;
                    const uint32_t slot = d.tok_order[64ull * e + (uint32_t)rank];
                    pb |= 1ull << slot;
                    if (flag) rb |= 1ull << slot;
                }
                if (st != LASPJ_DEC_OK) break;
                if (!stage_span(s, p, 1, end) || at(s, p) != 106) { st = LASPJ_DEC_MALFORMED; break; }
                p += 1;
                if (lane == 0) c[e] = u64x2{pb, rb};
            }
            if (st != LASPJ_DEC_OK) break;
            if (list) {
                if (!stage_span(s, p, 1, end) || at(s, p) != 106) { st = LASPJ_DEC_MALFORMED; break; }
                p += 1;
            }
            if (p != end) st = LASPJ_DEC_MALFORMED;      // trailing bytes
        } while (false);
        if (lane == 0) status[rep] = st;
    }
}

// Batched record decode (the default when the dictionary admits it, see ReadTabs).
// Elements: the next rank in term order is predicted, and what the wave needs about it
// (descriptor, the first 64 bytes of its header template, its token buckets and slot ->
// rank map, all stored by rank) is loaded while the element before it decodes; one LDS
// byte per lane then checks the header and carries the token count.  Any other element
// is found by the serial scan over 64 candidates per step.
// Records go in batches of up to 64 through a 4 KiB window.  The record chain (where
// each record starts: a record is 104 2 <token image> <flag atom> and only the flag's
// length varies) is walked ten records per step: lane (j, f) reads the flag header that
// record j would have if f of the records before it said `false` (one LDS round trip for
// all 55 cases), and the scalar walk reads the ten cases it needs with readlane.  A
// record whose flag uses another atom encoding than the batch's first takes one general
// step.  Then lane j takes record j on its own: a 32-bit word of its token image (word
// and shift chosen per element by the host so that every token of the element lands in
// its own bucket of a 1024-entry LDS table) gives the token rank, the exact compare
// against that rank's template decides, term order is the previous lane's rank, and the
// flag letters are checked.  Present and `true` ranks go to a 64-byte LDS presence table
// that the element's slot lanes read back with one ballot each.  The first failing
// record in stream order gives the status the serial scan gives (templates are distinct
// within an element, so "the first rank after the previous one whose template matches"
// is "the one rank whose template matches, if it comes after the previous one").

constexpr uint32_t kBWin = 4096;         // batched decode window
constexpr uint32_t kBuckets = 1024;      // token buckets per element
// an element's key when no bucket window separates its tokens: the batch paths find no
// bucket (its table entries are 0xFFFF) and leave it to decode_elems, which matches its
// records against each template
constexpr uint32_t kNoBuckets = 0x80000000u;

struct ReadTabs {
    const uint4* desc;      // by rank: slot, header length, word | shift << 8, token ranks
    const uint8_t* hdr;     // by rank: 64 bytes of 104 2 <elem image> 108, zero padded
    const uint16_t* tb;     // by rank r, token rank k: bucket at r * tok_max + k
    const uint8_t* ros;     // by rank r, token slot s: its token rank at 64 r + s (0xFF: none)
    NewTokArgs nt;          // (out null: unseen tokens answer UNKNOWN_TERM)
};

// bytes of the ReadTabs tables: desc, hdr, tb, ros
inline uint64_t rd_bytes(uint64_t E, uint64_t RK) { return E * (16 + 64 + 2 * RK + 64) + 64; }

// words of staged bytes [o, o + L) (L <= 48), zero past L; reads 52 bytes from o & ~3
__device__ __forceinline__ void rec_words(const uint8_t* buf, uint32_t o, uint32_t L,
                                          uint32_t (&w)[12]) {
    const uint32_t* b32 = reinterpret_cast<const uint32_t*>(buf + (o & ~3u));
    // 8 dwords cover L <= 28 (Lasp's 20-byte binary tokens: L = 27), else 13; one
    // wave-uniform branch, the loads of each side issued together
    uint32_t q[13];
    if (L <= 28u) {
#pragma unroll
        for (int i = 0; i < 8; ++i) q[i] = b32[i];
#pragma unroll
        for (int i = 8; i < 13; ++i) q[i] = 0u;
    } else {
#pragma unroll
        for (int i = 0; i < 13; ++i) q[i] = b32[i];
    }
#pragma unroll
    for (int i = 0; i < 12; ++i) {
        const uint32_t v = __builtin_amdgcn_alignbyte(q[i + 1], q[i], o & 3u);
        const int rem = (int)L - 4 * i;
        w[i] = rem >= 4 ? v : rem <= 0 ? 0u : v & ((1u << (8 * rem)) - 1u);
    }
}

// the 32-bit word of staged bytes at o (any alignment)
__device__ __forceinline__ uint32_t word_at(const uint8_t* buf, uint32_t o) {
    const uint32_t* b32 = reinterpret_cast<const uint32_t*>(buf + (o & ~3u));
    return __builtin_amdgcn_alignbyte(b32[1], b32[0], o & 3u);
}

// staged bytes [o, o + L) equal the 16-byte-aligned, zero-padded template t16 (L <= 48).
// L is wave-uniform: records of up to 28 bytes (Lasp's 20-byte binary tokens make
// 104 2 109 <len:4> <20 bytes> = 27) compare 7 words read from 8 staged dwords and two
// template loads; longer ones go through rec_words / load48.
__device__ __forceinline__ bool rec_match(const uint8_t* buf, uint32_t o, uint32_t L,
                                          const uint8_t* t16) {
    if (L <= 28u) {
        const uint32_t* b32 = reinterpret_cast<const uint32_t*>(buf + (o & ~3u));
        const u32x4* t = reinterpret_cast<const u32x4*>(t16);
        const u32x4 z = {0, 0, 0, 0};
        const u32x4 a = t[0], b = L > 16u ? t[1] : z;   // a 16-byte stride holds no t[1]
        const uint32_t tw[7] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z};
        uint32_t q[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) q[i] = b32[i];
        bool eq = true;
#pragma unroll
        for (int i = 0; i < 7; ++i) {
            const int rem = (int)L - 4 * i;
            const uint32_t m = rem >= 4 ? 0xFFFFFFFFu : rem <= 0 ? 0u : (1u << (8 * rem)) - 1u;
            eq &= (__builtin_amdgcn_alignbyte(q[i + 1], q[i], o & 3u) & m) == tw[i];
        }
        return eq;
    }
    uint32_t rw[12], tw[12];
    rec_words(buf, o, L, rw);
    load48(tw, t16, L);
    bool eq = true;
#pragma unroll
    for (int i = 0; i < 12; ++i) eq &= tw[i] == rw[i];
    return eq;
}

// New tokens (NewTokArgs): the record at o is 104 2 <BINARY_EXT of RL - 7 bytes>, the form
// of the dictionary's own token records (etf_dict_bin_tokens), so records compare bytewise
// in term order
__device__ __forceinline__ bool new_tok_image(const uint8_t* buf, uint32_t o, uint32_t RL) {
    if (RL < 8u || buf[o] != 104 || buf[o + 1] != 2 || buf[o + 2] != 109) return false;
    const uint32_t n = ((uint32_t)buf[o + 3] << 24) | ((uint32_t)buf[o + 4] << 16) |
                       ((uint32_t)buf[o + 5] << 8) | buf[o + 6];
    return n == RL - 7u;
}

// staged record at o against the 16-byte-aligned, zero-padded template t (global),
// bytewise: <0, 0, >0 — the template in three 16-byte loads issued together (a byte loop
// would be a chain of dependent global loads), then word by word, big-endian
__device__ __forceinline__ int rec_cmp(const uint8_t* buf, uint32_t o, uint32_t RL,
                                       const uint8_t* t) {
    uint32_t rw[12], tw[12];
    rec_words(buf, o, RL, rw);
    load48(tw, t, RL);
#pragma unroll
    for (int i = 0; i < 12; ++i)
        if (rw[i] != tw[i])
            return __builtin_bswap32(rw[i]) < __builtin_bswap32(tw[i]) ? -1 : 1;
    return 0;
}

// how many of an element's cnt token templates (by rank, stride RS) sort below the record
// at o; -1 when one equals it
__device__ __forceinline__ int32_t new_tok_rank(const uint8_t* buf, uint32_t o, uint32_t RL,
                                                const uint8_t* tpl, uint32_t RS, uint32_t cnt) {
    uint32_t lo = 0, hi = cnt;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        const int c = rec_cmp(buf, o, RL, tpl + (u64)mid * RS);
        if (c == 0) return -1;
        if (c > 0) lo = mid + 1;
        else hi = mid;
    }
    return (int32_t)lo;
}

// the staged record at a sorts after the one at b
__device__ __forceinline__ bool img_after(const uint8_t* buf, uint32_t a, uint32_t b,
                                          uint32_t RL) {
    for (uint32_t i = 0; i < RL; ++i)
        if (buf[a + i] != buf[b + i]) return buf[a + i] > buf[b + i];
    return false;
}

// The flag atom whose first 8 bytes are v0, v1 (little-endian): 1 = true, 2 = false,
// 0 = neither; n = its bytes.  ATOM_EXT 100 0 4 "true" / 100 0 5 "false" (what
// term_to_binary writes) is two compares; ATOM_UTF8_EXT (118, 2-byte length) and
// SMALL_ATOM_UTF8_EXT (119, 1-byte length) take the general parse.
__device__ __forceinline__ uint32_t flag_atom(uint32_t v0, uint32_t v1, uint32_t& n) {
    if (v0 == 0x74040064u && (v1 & 0xFFFFFFu) == 0x00657572u) { n = 7u; return 1u; }
    if (v0 == 0x66050064u && v1 == 0x65736C61u) { n = 8u; return 2u; }
    const uint32_t a0 = v0 & 0xFFu, a1 = (v0 >> 8) & 0xFFu;
    uint32_t gh = 0, len = 0, word = 0, c4 = 0;
    if ((a0 == 100 || a0 == 118) && a1 == 0) {
        gh = 3;
        len = (v0 >> 16) & 0xFFu;
        word = __builtin_amdgcn_alignbyte(v1, v0, 3);
        c4 = v1 >> 24;
    } else if (a0 == 119) {
        gh = 2;
        len = a1;
        word = __builtin_amdgcn_alignbyte(v1, v0, 2);
        c4 = (v1 >> 16) & 0xFFu;
    }
    n = gh + len;
    if (gh && len == 4 && word == 0x65757274u) return 1u;
    if (gh && len == 5 && word == 0x736C6166u && c4 == 'e') return 2u;
    return 0u;
}

// what the wave holds about one element rank (lane-distributed where per lane)
struct RankPre {
    uint32_t e, hl, key, cnt;   // slot, header length with the 108, word | shift << 8, tokens
    uint32_t hb;                // lane i: header template byte i
    uint32_t tb;                // lane k < cnt: bucket of token rank k
    uint32_t ros;               // lane s: token rank of slot s (0xFF: none)
};

__device__ __forceinline__ RankPre load_rank(const ReadTabs& t, uint32_t RK, int64_t r,
                                             uint32_t E, uint32_t lane) {
    RankPre x{0, 0, 0, 0, 0, 0, 0xFF};
    if (r >= (int64_t)E) return x;
    const uint4 d = t.desc[r];
    x.e = (uint32_t)__builtin_amdgcn_readfirstlane(d.x);
    x.hl = (uint32_t)__builtin_amdgcn_readfirstlane(d.y);
    x.key = (uint32_t)__builtin_amdgcn_readfirstlane(d.z);
    x.cnt = (uint32_t)__builtin_amdgcn_readfirstlane(d.w);
    x.hb = t.hdr[64ull * r + lane];
    x.tb = lane < RK ? t.tb[(u64)r * RK + lane] : 0u;
    x.ros = t.ros[64ull * r + lane];
    return x;
}

// a 64-bit wave-uniform value kept in scalar registers
__device__ __forceinline__ u64 ufl(u64 v) {
    // readfirstlane returns int: through uint32_t, or the low word would sign-extend
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
    return ((u64)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t rdlane(uint32_t v, uint32_t i) {
    return (uint32_t)__builtin_amdgcn_readlane(v, i);
}

// flag header at o (atom tag, then length): 1 | false << 1 when it is the encoding with
// atom header length h (3: ATOM_EXT / ATOM_UTF8_EXT, 2: SMALL_ATOM_UTF8_EXT) and a
// length of 4 or 5; 0 otherwise
__device__ __forceinline__ uint32_t flag_code(uint32_t v, uint32_t h) {
    const uint32_t t0 = v & 0xFFu, b1 = (v >> 8) & 0xFFu, b2 = (v >> 16) & 0xFFu;
    const uint32_t len = h == 3 ? b2 : b1;
    const bool ok = (h == 3 ? (t0 == 100 || t0 == 118) && b1 == 0 : t0 == 119) &&
                    (len == 4 || len == 5);
    return ok ? 1u | ((len == 5) << 1) : 0u;
}

struct ReadLds {
    uint8_t win[kBWin + 64];     // 64 bytes of slack: rec_words reads 52 past a start
    uint8_t tab[kBuckets];       // bucket -> token rank of the current element
    uint8_t pres[64];            // token rank -> 1 present | 2 true
    uint16_t rst[64];            // record starts found by locate_records (from the element's first)
};

// The batched decode's view of one payload: a 4 KiB LDS window over it, with every
// position inside the window a 32-bit offset (scalar arithmetic stays 32-bit)
struct PWin {
    uint8_t* buf;          // wave-private LDS window
    const uint8_t* src;    // the payload buffer
    u64 total;             // bytes in the payload buffer
    u64 aend;              // this payload's end (absolute)
    u64 lo;                // absolute position of buf[0]
    uint32_t hi;           // staged bytes [0, hi)
    uint32_t end;          // payload end relative to lo (clamped to 2^31)
};

// restage the window at the cursor; returns the cursor's offset in the new window
__device__ uint32_t refill(PWin& w, uint32_t pc) {
    const u64 a = w.lo + pc;
    const u64 lo = a & ~15ull;
    const u64 hi = min(w.total, lo + kBWin);
    const uint32_t lane = threadIdx.x & 63u;
    wave_sync();
    const uint32_t nfull = (uint32_t)((hi - lo) >> 4);
    wave_copy16<4>(w.buf, w.src + lo, nfull, lane);
    for (u64 b = lo + 16ull * nfull + lane; b < hi; b += 64) w.buf[b - lo] = w.src[b];
    wave_sync();
    w.lo = lo;
    w.hi = (uint32_t)(hi - lo);
    w.end = (uint32_t)min(w.aend - lo, (u64)0x7FFFFFFF);
    return (uint32_t)(a - lo);
}

// [pc, pc + n) resident (the caller checked pc + n <= w.end; n <= kBWin - 16)
__device__ __forceinline__ uint32_t need(PWin& w, uint32_t pc, uint32_t n) {
    return pc + n <= w.hi ? pc : refill(w, pc);
}

// a window byte every lane reads at the same offset, as a wave-uniform value
__device__ __forceinline__ uint32_t ub(const PWin& w, uint32_t o) {
    return (uint32_t)__builtin_amdgcn_readfirstlane(w.buf[o]);
}

// bytes at q equal the 16-byte-aligned, zero-padded template (L <= 48)
__device__ __forceinline__ bool eq48(const uint8_t* q, const uint8_t* t16, uint32_t L) {
    const u32x4* t = reinterpret_cast<const u32x4*>(t16);
    const u32x4 z = {0, 0, 0, 0};
    const u32x4 a = t[0], b = L > 16 ? t[1] : z, c = L > 32 ? t[2] : z;
    const uint32_t w[12] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w};
    bool eq = true;
#pragma unroll
    for (uint32_t i = 0; i < 48; ++i)
        if (i < L) eq &= q[i] == ((w[i >> 2] >> (8 * (i & 3))) & 0xFFu);
    return eq;
}

struct HdrHash {
    const uint32_t* tab;   // open addressing: rank + 1, 0 empty
    uint32_t mask;
    u64 lens;              // bit hl - 1: some header template is hl bytes (hl <= 64)
    uint32_t many = 0;     // many-token dictionaries: element batches (read_batch_many)
};

// the header-template hash (host and device agree): ceil(hl / 4) words, bytes >= hl zero
__host__ __device__ inline uint32_t hdr_mix(uint32_t h, uint32_t v) {
    h ^= v;
    h *= 0x9E3779B1u;
    return h ^ (h >> 16);
}

// Element batches, for dictionaries with few token slots per element (tok_max <= 8,
// e.g. the ad counter's 3-replica tokens): one element at a time leaves 60 of 64 lanes
// idle, so the wave walks up to 64 whole elements before checking any record.  Lane i
// holds the 64-byte header template and descriptor of rank prev + 1 + i; per element the
// scalar walk compares the bytes at the cursor with every held header at once (ballot:
// the element's rank, absent elements need no scan), reads its token count and each
// record's flag length, and checks the closing 106.  Then lane j takes record j of the
// batch: bucket -> token rank among its element's <= 8 buckets, exact template compare,
// term order against the previous record of the same element, flag letters; token bits
// are ORed into per-element LDS cells.  Only elements before the first failing record
// (or the first walk step that is not a well-formed element) are committed: the caller's
// element-at-a-time path decodes from there and gives the status.  What a batch commits
// is what that path would accept, with the same cells (element images are
// self-delimiting and distinct, so the header match is the scan's first match).
constexpr uint32_t kSmallTok = 8;
// the element-batch decoders (SMALL) for a dictionary whose elements mostly hold at most
// kSmallTok tokens: an element with more fails its batch and is decoded on its own by the
// general path (a few hot elements — re-added again and again — no longer move every
// element of the dictionary to the many-token decoders)
inline bool small_dict(const laspj_etf_dict* d) {
    return d->tok_max <= kSmallTok || 16ull * d->big_elems < d->elements;
}

__device__ __forceinline__ uint32_t ufl32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readfirstlane(v);
}

__device__ uint32_t read_batch(PWin& w, uint32_t& pc, int64_t& prev, uint32_t left, u64 stop,
                               const ReadTabs& t, const DictView& d, uint32_t E, uint32_t RL,
                               uint32_t RS, ReadLds& L, u64x2* c, uint32_t lane) {
    const uint32_t RK = d.tok_max;
    if (w.hi < w.end && pc + kBWin / 2 > w.hi) pc = refill(w, pc);
    // lane i: rank prev + 1 + i (descriptor, header template words)
    const int64_t cr = prev + 1 + (int64_t)lane;
    // (the template's other 48 bytes are loaded again for the whole-header check)
    uint32_t ce = 0, chl = 0, ckey = 0, ccnt = 0, ch[4] = {0, 0, 0, 0};
    const u32x4* hsrc = reinterpret_cast<const u32x4*>(t.hdr + 64ull * (u64)max(cr, (int64_t)0));
    if (cr < (int64_t)E) {
        const uint4 ds = t.desc[cr];
        ce = ds.x; chl = ds.y; ckey = ds.z; ccnt = ds.w;
        const u32x4 v = hsrc[0];
        ch[0] = v.x; ch[1] = v.y; ch[2] = v.z; ch[3] = v.w;
    }
    const bool cval = chl > 3u && chl <= 64u;
    // the walk tells elements apart by their first 16 header bytes (masks per lane);
    // every header is compared whole below, before anything is committed
    uint32_t mk[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int rem = (int)chl - 4 * i;
        mk[i] = rem >= 4 ? 0xFFFFFFFFu : rem <= 0 ? 0u : (1u << (8 * rem)) - 1u;
    }
    const uint32_t lim = min(w.hi, w.end);
    // elements starting at or after `stop` belong to the next segment
    const uint32_t srel = stop <= w.lo ? 0u : (uint32_t)min(stop - w.lo, (u64)0xFFFFFFFFu);
    // the walk: element lanes (start, candidate lane), record lanes (start, element,
    // atom header length, atom length)
    uint32_t x = pc, ne = 0, nr = 0, ex = 0, ec = 0, ry = 0, rel = 0, rh = 0, rlen = 0;
    int32_t fmin = -1;
    u64 cm = 0;                          // candidate lanes the walk matched
    while (ne < 64u && ne < left && x < lim && x < srel) {
        const uint32_t* b32 = reinterpret_cast<const uint32_t*>(w.buf + (x & ~3u));
        const uint32_t sh = x & 3u;
        bool hit = cval && (int32_t)lane > fmin && x + chl <= lim;
        uint32_t q0 = b32[0];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t q1 = b32[i + 1];
            hit &= (__builtin_amdgcn_alignbyte(q1, q0, sh) & mk[i]) == ch[i];
            q0 = q1;
        }
        // read beside the compare, as if this lane's rank matched: the token count and
        // the first record's flag header (clamped inside the window; used only in bounds)
        const uint32_t cws = word_at(w.buf, min(x + chl, kBWin));
        const uint32_t fws = word_at(w.buf, min(x + chl + 4u + RL, kBWin));
        const u64 m = __ballot(hit);
        if (!m) break;
        const uint32_t f = (uint32_t)__ffsll((long long)m) - 1u;
        const uint32_t hl = rdlane(chl, f), cnt = rdlane(ccnt, f);
        if (x + hl + 4u > lim) break;
        const uint32_t m_tok = __builtin_bswap32(rdlane(cws, f));
        if (m_tok == 0 || m_tok > cnt || nr + m_tok > 64u) break;
        uint32_t y = x + hl + 4u;
        bool okr = true;
        for (uint32_t j = 0; j < m_tok; ++j) {
            const uint32_t v = j ? ufl32(word_at(w.buf, y + RL)) : rdlane(fws, f);
            const uint32_t a0 = v & 0xFFu, a1 = (v >> 8) & 0xFFu, a2 = (v >> 16) & 0xFFu;
            uint32_t gh = 0, len = 0;
            if ((a0 == 100 || a0 == 118) && a1 == 0) { gh = 3; len = a2; }
            else if (a0 == 119) { gh = 2; len = a1; }
            if (!gh || (len != 4 && len != 5) || y + RL + gh + len > lim) { okr = false; break; }
            if (lane == nr + j) { ry = y; rel = ne; rh = gh; rlen = len; }
            y += RL + gh + len;
        }
        if (!okr || y + 1u > lim || ufl32(w.buf[y]) != 106) break;
        if (lane == ne) { ex = x; ec = f; }
        nr += m_tok;
        ++ne;
        fmin = (int32_t)f;
        cm |= 1ull << f;
        x = y + 1u;
    }
    if (ne == 0) return 0;
    // lane j < nr: record j
    const bool mine = lane < nr;
    const uint32_t myc = __shfl(ec, rel, 64);
    const uint32_t re = __shfl(ce, myc, 64), rkey = __shfl(ckey, myc, 64),
                   rcnt = __shfl(ccnt, myc, 64);
    uint32_t k = 0xFFu, fl = 0;
    bool ok = false;
    if (mine) {
        const u64 r = (u64)(prev + 1) + myc;
        const uint32_t kw = 4u * (rkey & 0xFFu), ksh = (rkey >> 8) & 31u;
        const uint32_t bk = (word_at(w.buf, ry + kw) >> ksh) & (kBuckets - 1u);
        for (uint32_t j = 0; j < rcnt && j < RK; ++j)
            if (t.tb[r * RK + j] == bk) k = j;
        ok = k < rcnt;
        if (ok) {                                   // exact compare
            ok = rec_match(w.buf, ry, RL, d.rec_pad + ((u64)re * RK + k) * RS);
        }
        // "true" / "false" after the atom header the walk read
        const uint32_t fo = ry + RL + rh;
        const uint32_t word = word_at(w.buf, fo), c4 = w.buf[fo + 4];
        const bool tr = rlen == 4 && word == 0x65757274u;
        const bool fa = rlen == 5 && word == 0x736C6166u && c4 == 'e';
        ok &= tr || fa;
        fl = tr;
    }
    // term order within the element
    const uint32_t pk = __shfl(k, (lane + 63u) & 63u, 64), pel = __shfl(rel, (lane + 63u) & 63u, 64);
    if (mine && lane > 0 && pel == rel && k <= pk) ok = false;
    const u64 bad = __ballot(mine && !ok);
    uint32_t commit = bad ? rdlane(rel, (uint32_t)__ffsll((long long)bad) - 1u) : ne;
    // whole headers: matched candidate lane c checks element popcount(cm below c)
    const bool cme = (cm >> lane) & 1ull;
    const uint32_t ei = (uint32_t)__popcll(cm & ((1ull << lane) - 1ull));
    const uint32_t xi = __shfl(ex, ei & 63u, 64);
    bool hok = true;
    if (cme) {
        uint32_t tw[16];
        tw[0] = ch[0]; tw[1] = ch[1]; tw[2] = ch[2]; tw[3] = ch[3];
#pragma unroll
        for (int i = 1; i < 4; ++i) {
            const u32x4 v = hsrc[i];
            tw[4 * i] = v.x; tw[4 * i + 1] = v.y; tw[4 * i + 2] = v.z; tw[4 * i + 3] = v.w;
        }
        const uint32_t* b32 = reinterpret_cast<const uint32_t*>(w.buf + (xi & ~3u));
        const uint32_t sh = xi & 3u;
        uint32_t q0 = b32[0];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint32_t q1 = b32[i + 1];
            const uint32_t v = __builtin_amdgcn_alignbyte(q1, q0, sh);
            q0 = q1;
            const int rem = (int)chl - 4 * i;
            const uint32_t msk = rem >= 4 ? 0xFFFFFFFFu : rem <= 0 ? 0u : (1u << (8 * rem)) - 1u;
            hok &= (v & msk) == tw[i];
        }
    }
    const u64 hbad = __ballot(cme && !hok);
    if (hbad) commit = min(commit, rdlane(ei, (uint32_t)__ffsll((long long)hbad) - 1u));
    if (commit == 0) return 0;
    // cells: token bits by slot, ORed per element in LDS
    unsigned long long* pc64 = reinterpret_cast<unsigned long long*>(L.tab);
    wave_sync();
    pc64[2 * lane] = 0;
    pc64[2 * lane + 1] = 0;
    wave_sync();
    if (mine && rel < commit) {
        const uint32_t slot = d.tok_order[64ull * re + k];
        atomicOr(pc64 + 2 * rel, 1ull << slot);
        if (fl) atomicOr(pc64 + 2 * rel + 1, 1ull << slot);
    }
    wave_sync();
    const uint32_t me = __shfl(ce, ec, 64);
    if (lane < commit) c[me] = u64x2{pc64[2 * lane], pc64[2 * lane + 1]};
    prev += 1 + (int64_t)rdlane(ec, commit - 1u);
    pc = commit == ne ? x : rdlane(ex, commit);
    return commit;
}

// the list header after the optional <<Tag, Vers>>: 131 106 (n = 0) or 131 108 <n:32>
// (a LIST_EXT of n elements ends in its tail: `list` says the caller checks the 106)
__device__ __forceinline__ int32_t parse_head(PWin& w, uint32_t& pc, int tag, int vers,
                                              uint32_t& n, bool& list) {
    n = 0;
    list = false;
    if (tag >= 0) {
        if (pc + 2 > w.end) return LASPJ_DEC_INVALID_BINARY;
        pc = need(w, pc, 2);
        if (ub(w, pc) != (uint32_t)(tag & 0xFF)) return LASPJ_DEC_INVALID_BINARY;
        if (ub(w, pc + 1) != (uint32_t)(vers & 0xFF)) return LASPJ_DEC_UNSUPPORTED_VERSION;
        pc += 2;
    }
    if (pc + 2 > w.end) return LASPJ_DEC_MALFORMED;                // binary_to_term: badarg
    pc = need(w, pc, 2);
    if (ub(w, pc) != 131) return LASPJ_DEC_MALFORMED;
    if (ub(w, pc + 1) == 106) {
        pc += 2;
        return LASPJ_DEC_OK;
    }
    if (ub(w, pc + 1) == 108 && pc + 6 <= w.end) {
        pc = need(w, pc, 6);
        n = (ub(w, pc + 2) << 24) | (ub(w, pc + 3) << 16) | (ub(w, pc + 4) << 8) | ub(w, pc + 5);
        pc += 6;
        list = true;
        return LASPJ_DEC_OK;
    }
    return LASPJ_DEC_MALFORMED;
}

// per-lane constants of the batched record walk: lane (lj, lf), lj < 10, lf <= lj, is
// case lj (lj + 1) / 2 + lf of a chain step
struct Cases {
    uint32_t lj, lf;
    bool on;
};

__device__ __forceinline__ Cases lane_cases(uint32_t lane) {
    uint32_t lj = 0;
    while ((lj + 1) * (lj + 2) / 2 <= lane) ++lj;
    return Cases{lj, lane - lj * (lj + 1) / 2, lane < 55};
}

// Byte-parallel search of window bytes (x0, x0 + span) for the triple `first 104 2`
// (first = 101, the `e` ending a flag atom, before a record; 106, a closing nil, before
// an element): lanes take K bytes each (a multiple of 4 with an odd dword count, so
// their dword reads hit distinct LDS banks) and test 4 positions per dword with a
// zero-byte test on the XOR with the pattern.  The offsets (from x0) of the first 63
// matches in stream order go to L.rst; returns the number of matches.
__device__ __forceinline__ uint32_t find_marks(const PWin& w, uint32_t x0, uint32_t span,
                                               uint32_t first, ReadLds& L, uint32_t lane) {
    const uint32_t a0 = x0 & ~3u;
    // a lane's mask holds 64 positions: at most K = 60 bytes per lane, i.e. 3840 bytes
    // from a0 (marks past that are not reported; callers treat a missing mark as "not
    // validated").  Without the clamp a fresh 4 KiB window gave K = 68 and every lane's
    // last 4 positions wrapped into its first 4: batches stopped at the first mark there.
    span = min(span, 3840u - (x0 - a0));
    uint32_t K = (((span + (x0 - a0) + 63u) >> 6) + 3u) & ~3u;
    if (!(K & 4u)) K += 4u;
    const uint32_t b0 = a0 + lane * K;                                   // this lane's first
    const uint32_t* w32 = reinterpret_cast<const uint32_t*>(w.buf);
    const uint32_t top = (kBWin + 60u) >> 2;                            // last dword index
    const uint32_t pa = first * 0x01010101u;
    u64 mask = 0;
    uint32_t dm1 = b0 >= 4u ? w32[min((b0 >> 2) - 1u, top)] : 0u;
    uint32_t d0 = w32[min(b0 >> 2, top)];
    for (uint32_t g = 0; g < (K >> 2); ++g) {
        const uint32_t d1 = w32[min((b0 >> 2) + g + 1u, top)];
        const uint32_t A = __builtin_amdgcn_alignbyte(d0, dm1, 3);       // b[q - 1 + k]
        const uint32_t B = __builtin_amdgcn_alignbyte(d1, d0, 1);        // b[q + 1 + k]
        const uint32_t T = (A ^ pa) | (d0 ^ 0x68686868u) | (B ^ 0x02020202u);
        const uint32_t z = ~(((T & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | T) & 0x80808080u;
        mask |= (u64)((((z >> 7) * 0x204081u) >> 21) & 0xFu) << (4u * g);
        dm1 = d0;
        d0 = d1;
    }
    // positions q = b0 + i with x0 < q < x0 + span only
    const int64_t lo = (int64_t)x0 + 1 - (int64_t)b0;
    const int64_t hi = (int64_t)x0 + (int64_t)span - (int64_t)b0;
    if (hi <= 0) mask = 0;
    else if (hi < 64) mask &= (1ull << hi) - 1ull;
    if (lo >= 64) mask = 0;
    else if (lo > 0) mask &= ~((1ull << lo) - 1ull);
    if (!__ballot((mask & (mask - 1ull)) != 0)) {
        // at most one match per lane (the usual case when records or elements are longer
        // than K bytes): a match's index is the number of lanes below with one
        const u64 has = __ballot(mask != 0);
        if (mask) {
            const uint32_t k = __builtin_amdgcn_mbcnt_hi(
                (uint32_t)(has >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)has, 0u));
            if (k < 63u) L.rst[k] = (uint16_t)(b0 + (uint32_t)__ffsll((long long)mask) - 1u - x0);
        }
        wave_sync();
        return (uint32_t)__popcll(has);
    }
    const uint32_t cnt = (uint32_t)__popcll(mask);
    uint32_t incl = cnt;
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint32_t v = __shfl_up(incl, o, 64);
        if (lane >= o) incl += v;
    }
    const uint32_t total = rdlane(incl, 63);
    uint32_t k = incl - cnt;
    while (mask && k < 63u) {
        const uint32_t i = (uint32_t)__ffsll((long long)mask) - 1u;
        mask &= mask - 1ull;
        L.rst[k++] = (uint16_t)(b0 + i - x0);
    }
    wave_sync();
    return total;
}

// Records of an element found without the scalar chain walk.  Every record after the
// first starts right after a flag atom, so its first bytes are 101 104 2 (the `e` of
// true / false, then 104 2): the lanes look for that byte triple over the element's
// span, 4 positions per dword (a zero-byte test on the XOR with the pattern), and record
// j is taken at the j-th match.  The element is committed only if every record
// validates as in the chain path and each one ends exactly where the next begins (the
// last one at the element's closing 106) — then the starts are the chain's.  Otherwise
// nothing is touched and the caller walks the chain (a token image may hold those bytes,
// and the chain gives the exact status of a malformed element).  Returns whether the
// element's records were committed (into L.pres; pc left on the closing 106).
__device__ __forceinline__ bool locate_records(PWin& w, uint32_t& pc, uint32_t m_tok,
                                               const RankPre& cur, uint32_t e, uint32_t kw,
                                               uint32_t ksh, ReadLds& L, const DictView& d,
                                               uint32_t lane) {
    const uint32_t RL = d.rec_len, RS = d.rec_stride, RK = d.tok_max;
    const uint32_t x0 = pc;
    const uint32_t lim = min(w.hi, w.end);
    if (x0 >= lim) return false;
    const uint32_t span = min(m_tok * (RL + 8u) + 1u, lim - x0);   // [x0, x0 + span)
    if (m_tok > 1) {
        const uint32_t total = find_marks(w, x0, span, 0x65u, L, lane);
        if (total + 1u < m_tok) return false;
    }
    const bool mine = lane < m_tok;
    uint32_t myx = x0, rank = 0xFFu, fl = 0, fend = 0;
    bool ok = true;
    if (mine) {
        if (lane) myx = x0 + L.rst[lane - 1];
        rank = L.tab[(word_at(w.buf, myx + kw) >> ksh) & (kBuckets - 1u)];
        ok = rank < cur.cnt;
        if (ok) {                                               // exact compare
            ok = rec_match(w.buf, myx, RL, d.rec_pad + ((u64)e * RK + rank) * RS);
        }
        const uint32_t fo = myx + RL;
        const uint32_t* f32 = reinterpret_cast<const uint32_t*>(w.buf + (fo & ~3u));
        const uint32_t v0 = __builtin_amdgcn_alignbyte(f32[1], f32[0], fo & 3u);
        const uint32_t v1 = __builtin_amdgcn_alignbyte(f32[2], f32[1], fo & 3u);
        uint32_t fn;
        const uint32_t fk = flag_atom(v0, v1, fn);
        fend = fo + fn;
        ok &= fk != 0u && fend < lim;
        fl = fk == 1u;
    }
    // term order, and each record ends where the next one starts
    const uint32_t pr = __shfl(rank, (lane + 63u) & 63u, 64);
    const uint32_t nx = __shfl(myx, (lane + 1u) & 63u, 64);
    if (mine) {
        if (lane && rank <= pr) ok = false;
        if (lane + 1u < m_tok) ok &= fend == nx;
        else ok &= w.buf[min(fend, kBWin + 63u)] == 106;
    }
    if (__ballot(mine && !ok)) return false;
    if (mine) L.pres[rank] = (uint8_t)(1u | (fl << 1));
    pc = rdlane(fend, m_tok - 1u);
    return true;
}

// The rank of the element whose header 104 2 <elem image> 108 starts at window offset s
// (hl: the header's bytes), or -1: the image's length from its tag where the tag gives it
// (integers, binaries, atoms, small bignums) -> one probe of the header hash at that
// length; other terms try every header length the dictionary has.  Exact compare against
// the rank's 64-byte header template.  Per lane (s differs between lanes).
__device__ __forceinline__ int64_t hdr_rank(const PWin& w, uint32_t s, uint32_t lim,
                                            const HdrHash& hh, const ReadTabs& t, uint32_t E,
                                            uint32_t& hl) {
    int64_t rk = -1;
    u64 lens = hh.lens;
    {
        const uint32_t b2 = w.buf[min(s + 2u, kBWin + 63u)];
        const uint32_t h0 = word_at(w.buf, min(s + 3u, kBWin + 56u));
        uint32_t il = 0;
        if (b2 == 97) il = 2;                                        // SMALL_INTEGER_EXT
        else if (b2 == 98) il = 5;                                   // INTEGER_EXT
        else if (b2 == 109) il = 5u + __builtin_bswap32(h0);         // BINARY_EXT
        else if (b2 == 100 || b2 == 118)                             // ATOM(_UTF8)_EXT
            il = 3u + (((h0 & 0xFFu) << 8) | ((h0 >> 8) & 0xFFu));
        else if (b2 == 115 || b2 == 119 || b2 == 110) il = 2u + (h0 & 0xFFu) + (b2 == 110);
        if (il) lens = il <= 61u ? lens & (1ull << (il + 2u)) : 0ull;   // hl = il + 3
    }
    while (lens && rk < 0) {
        const uint32_t L2 = (uint32_t)__ffsll((long long)lens);
        lens &= lens - 1ull;
        if (s + L2 > lim) break;
        uint32_t q[16] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
        uint32_t h = L2 * 0x85EBCA6Bu;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int rem = (int)L2 - 4 * i;          // per lane: L2 follows the lane's tag
            if (rem <= 0) break;                      // the hash covers ceil(L2 / 4) words
            const uint32_t v = word_at(w.buf, min(s + 4u * i, kBWin + 56u));
            q[i] = rem >= 4 ? v : v & ((1u << (8 * rem)) - 1u);
            h = hdr_mix(h, q[i]);
        }
        for (uint32_t i = h & hh.mask;; i = (i + 1) & hh.mask) {
            const uint32_t v = hh.tab[i];
            if (!v || v > E) break;
            const uint32_t r = v - 1u;
            // (no length check: images are self-delimiting, so an L2-byte template
            // ending in 108 matches only its own element's header)
            const u32x4* tp = reinterpret_cast<const u32x4*>(t.hdr + 64ull * r);
            bool eq = true;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if ((uint32_t)(16 * j) >= L2) break;   // the rest is zero on both sides
                const u32x4 a = tp[j];
                eq &= a.x == q[4 * j] && a.y == q[4 * j + 1] && a.z == q[4 * j + 2] &&
                      a.w == q[4 * j + 3];
            }
            if (eq) { rk = r; hl = L2; break; }
        }
    }
    return rk;
}

// Element batches without the scalar walk (few token slots per element, the ad
// counter's 3-replica tokens): every element after the first at the cursor starts right
// after the previous element's closing 106, so `106 104 2` marks element starts; lane i
// takes the element at the i-th mark, finds its rank by the hash of its header bytes
// (one probe per header length the dictionary has, exact 64-byte compare), and walks its
// own <= 8 records: token bucket -> term rank among the element's, exact template
// compare, flag atom, ascending ranks, the closing 106 — which must sit right before the
// next lane's element.  Elements before the first lane that fails any of this are
// committed (the cells the element-at-a-time path would write); that path decodes from
// the failing one and gives its status.
__device__ uint32_t read_batch_par(PWin& w, uint32_t& pc, int64_t& prev, uint32_t left, u64 stop,
                                   const ReadTabs& t, const DictView& d, const HdrHash& hh,
                                   uint32_t E, ReadLds& L, u64x2* c, uint32_t lane) {
    const uint32_t RL = d.rec_len, RS = d.rec_stride, RK = d.tok_max;
    if (w.hi < w.end && pc + kBWin / 2 > w.hi) pc = refill(w, pc);
    const uint32_t lim = min(w.hi, w.end);
    const uint32_t srel = stop <= w.lo ? 0u : (uint32_t)min(stop - w.lo, (u64)0xFFFFFFFFu);
    const uint32_t x0 = pc;
    if (x0 >= lim || x0 >= srel) return 0;
    const uint32_t total = find_marks(w, x0, lim - x0, 106u, L, lane);
    const uint32_t N = min(min(64u, total + 1u), left);
    const bool mine = lane < N;
    const uint32_t s = x0 + (lane && mine ? L.rst[lane - 1] : 0u);
    bool ok = mine && s < srel;
    // the element's rank.  First the prediction that the payload holds every element from
    // prev on (the lane's element is rank prev + 1 + lane): that rank's descriptor, header
    // template and token buckets are loaded together, and an exact match of the header
    // bytes against the template (self-delimiting images: only its own element's header
    // matches) settles it — one round of loads where the hash probe below takes three
    // (bucket, template, then descriptor and buckets)
    uint32_t hl = 0;
    int64_t rk = -1;
    const int64_t pr = prev + 1 + (int64_t)lane;
    uint4 pds = {0u, 0u, 0u, 0u};
    uint32_t ptb[kSmallTok];
    bool predicted = false;
    if (ok && pr < (int64_t)E) {
        pds = t.desc[pr];
        const u32x4* tp = reinterpret_cast<const u32x4*>(t.hdr + 64ull * pr);
        u32x4 tw[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) tw[j] = tp[j];
#pragma unroll
        for (uint32_t j = 0; j < kSmallTok; ++j) ptb[j] = t.tb[(u64)pr * RK + min(j, RK - 1u)];
        const uint32_t L2 = pds.y;
        if (L2 > 3u && L2 <= 64u && s + L2 <= lim) {
            bool eq = true;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int rem = (int)L2 - 4 * j;
                if (rem <= 0) break;
                const uint32_t v = word_at(w.buf, min(s + 4u * j, kBWin + 56u));
                const uint32_t q = rem >= 4 ? v : v & ((1u << (8 * rem)) - 1u);
                const u32x4 a = tw[j >> 2];
                const uint32_t tv = (j & 3) == 0 ? a.x : (j & 3) == 1 ? a.y : (j & 3) == 2 ? a.z : a.w;
                eq &= q == tv;
            }
            if (eq) {
                rk = pr;
                hl = L2;
                predicted = true;
            }
        }
    }
    // otherwise its header 104 2 <elem image> 108 by hash
    if (ok && !predicted) rk = hdr_rank(w, s, lim, hh, t, E, hl);
    ok = rk >= 0;
    // ranks ascend: after the previous lane's element (lane 0: after prev)
    const int64_t prk = (int64_t)(int32_t)__shfl((int32_t)rk, (lane + 63u) & 63u, 64);
    if (ok) ok = rk > (lane ? prk : prev);
    u64 pb = 0, rb = 0;
    uint32_t e = 0, y = s;
    if (ok) {
        const uint4 ds = predicted ? pds : t.desc[rk];
        e = ds.x;
        const uint32_t cnt = ds.w, kw = 4u * (ds.z & 0xFFu), ksh = (ds.z >> 8) & 31u;
        y = s + hl;
        ok = y + 4u <= lim;
        const uint32_t m = ok ? __builtin_bswap32(word_at(w.buf, y)) : 0u;
        ok = ok && m >= 1u && m <= cnt && cnt <= kSmallTok;
        y += 4u;
        // the element's token buckets (by term rank) and rank -> slot
        uint32_t tb[kSmallTok];
#pragma unroll
        for (uint32_t j = 0; j < kSmallTok; ++j)
            tb[j] = ok && j < cnt ? (predicted ? ptb[j] : t.tb[(u64)rk * RK + j]) : 0xFFFFFFFFu;
        const u64 ord = ok ? *reinterpret_cast<const u64*>(d.tok_order + 64ull * e) : 0ull;
        int32_t kprev = -1;
        for (uint32_t j = 0; ok && j < m; ++j) {
            if (y + RL + 8u > lim) { ok = false; break; }
            const uint32_t bk = (word_at(w.buf, y + kw) >> ksh) & (kBuckets - 1u);
            uint32_t k = 0xFFu;
#pragma unroll
            for (uint32_t jj = 0; jj < kSmallTok; ++jj)
                if (tb[jj] == bk) k = jj;
            if (k == 0xFFu || (int32_t)k <= kprev) { ok = false; break; }
            const bool eq = rec_match(w.buf, y, RL, d.rec_pad + ((u64)e * RK + k) * RS);
            const uint32_t fo = y + RL;
            const uint32_t v0 = word_at(w.buf, fo), v1 = word_at(w.buf, fo + 4u);
            uint32_t fn;
            const uint32_t fk = flag_atom(v0, v1, fn);
            const bool tr = fk == 1u;
            if (!eq || !fk) { ok = false; break; }
            const uint32_t slot = (uint32_t)(ord >> (8 * k)) & 0xFFu;
            pb |= 1ull << slot;
            if (tr) rb |= 1ull << slot;
            kprev = (int32_t)k;
            y += RL + fn;
        }
        ok = ok && y < lim && w.buf[y] == 106;
        y += 1u;
    }
    // each element ends where the next lane's begins
    const uint32_t nxs = __shfl(s, (lane + 1u) & 63u, 64);
    if (ok && lane + 1u < N) ok = y == nxs;
    const u64 bad = __ballot(mine && !ok);
    const uint32_t commit = bad ? (uint32_t)__ffsll((long long)bad) - 1u : N;
    if (commit == 0) return 0;
    if (lane < commit) c[e] = u64x2{pb, rb};
    prev = (int64_t)(int32_t)rdlane((uint32_t)rk, commit - 1u);
    pc = rdlane(y, commit - 1u);
    return commit;
}

// Element batches for many-token dictionaries (tok_max > 8, e.g. 64 token slots per
// element): one element at a time pays the whole per-element sequence (header match,
// bucket table, mark scan, one validation pass, presence ballot) for ~30 records, and at
// t64 that sequence, not the records, is most of the time (tools/decoder_probe.py).  So
// a batch takes up to kNT whole elements and up to kItems items at once.  Every element
// and every record starts with 104 2 (a 2-tuple header), so one byte-parallel scan of
// the window lists the items in stream order; an item whose previous byte is 106 (the
// closing nil of the element before) starts an element, every other one a record (item
// 0 is the element at the cursor).  Lanes resolve the elements' ranks by the header hash
// (ascending after prev), read their counts and set up one bucket table each; then each
// lane validates one record per half of the batch exactly as the per-element path does:
// bucket -> token rank, exact template compare, flag atom, ranks ascending within the
// element, the record ending where the next item starts (the next record, or the closing
// 106 before the next element / at the element's end), the element's m-th record being
// its last.  A token image may hold 104 2 or 106 104 2: a false item shifts the lanes
// after it, and the elements it touches fail.  Elements before the first one that fails
// anything (or is not wholly inside the batch) are committed with the cells the
// per-element path writes; that path takes the failing one and gives its status.
constexpr uint32_t kNT = 4;             // elements per batch (one bucket table each)
constexpr uint32_t kItems = 128;        // element starts and records per batch

struct ReadLdsX {
    uint8_t tab[kNT - 1][kBuckets];     // bucket tables of elements 1 .. kNT-1 (0: ReadLds)
    uint8_t pres[kNT - 1][64];
    uint16_t pos[kItems];               // item starts, relative to the batch's first
};

// Positions q in [x0, x0 + span) of the bytes 104 2, in stream order, into X.pos
// (relative to x0, the first kItems of them); returns how many the scanned span holds.
// Lane l scans K bytes from a0 + l K (K / 4 odd: the lanes' dwords fall in distinct LDS
// banks); span is clamped to 3840 bytes so that a lane's 64-bit mask holds its K <= 60
// positions.
__device__ __forceinline__ uint32_t scan_items(const PWin& w, uint32_t x0, uint32_t span,
                                               ReadLdsX& X, uint32_t lane) {
    const uint32_t a0 = x0 & ~3u;
    span = min(span, 3840u - (x0 - a0));
    uint32_t K = (((span + (x0 - a0) + 63u) >> 6) + 3u) & ~3u;
    if (!(K & 4u)) K += 4u;
    const uint32_t b0 = a0 + lane * K;
    const uint32_t* w32 = reinterpret_cast<const uint32_t*>(w.buf);
    const uint32_t top = (kBWin + 60u) >> 2;                            // last dword index
    u64 mask = 0;
    uint32_t d0 = w32[min(b0 >> 2, top)];
    for (uint32_t g = 0; g < (K >> 2); ++g) {
        const uint32_t d1 = w32[min((b0 >> 2) + g + 1u, top)];
        const uint32_t B = __builtin_amdgcn_alignbyte(d1, d0, 1);        // b[q + 1 + k]
        const uint32_t T = (d0 ^ 0x68686868u) | (B ^ 0x02020202u);
        const uint32_t z = ~(((T & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | T) & 0x80808080u;
        mask |= (u64)((((z >> 7) * 0x204081u) >> 21) & 0xFu) << (4u * g);
        d0 = d1;
    }
    const int32_t lo = (int32_t)x0 - (int32_t)b0, hi = lo + (int32_t)span;
    if (hi <= 0) mask = 0;
    else if (hi < 64) mask &= (1ull << hi) - 1ull;
    if (lo >= 64) mask = 0;
    else if (lo > 0) mask &= ~((1ull << lo) - 1ull);
    // exclusive prefix of the per-lane counts, bit plane by bit plane (104 2 cannot
    // overlap itself: at most 30 in a lane's 60 bytes)
    const uint32_t cnt = (uint32_t)__popcll(mask);
    uint32_t k = 0, total = 0;
#pragma unroll
    for (uint32_t bit = 0; bit < 5; ++bit) {
        const u64 m = __ballot((cnt >> bit) & 1u);
        k += __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                       __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)) << bit;
        total += (uint32_t)__popcll(m) << bit;
    }
    while (mask && k < kItems) {
        const uint32_t i = (uint32_t)__ffsll((long long)mask) - 1u;
        mask &= mask - 1ull;
        X.pos[k++] = (uint16_t)(b0 + i - x0);
    }
    wave_sync();
    return total;
}

__device__ uint32_t read_batch_many(PWin& w, uint32_t& pc, int64_t& prev, uint32_t left,
                                    uint32_t hint, const ReadTabs& t, const DictView& d,
                                    const HdrHash& hh, uint32_t E, ReadLds& L, ReadLdsX& X,
                                    u64x2* c, uint32_t lane) {
    const uint32_t RL = d.rec_len, RS = d.rec_stride, RK = d.tok_max;
    if (w.hi < w.end && pc + hint > w.hi) pc = refill(w, pc);
    const uint32_t lim = min(w.hi, w.end);
    const uint32_t x0 = pc;
    if (x0 + 8u > lim) return 0;
    const uint32_t NI = min(scan_items(w, x0, min(lim - x0, hint), X, lane), kItems);
    if (NI < 2u || ufl32(X.pos[0]) != 0u) return 0;
    // items of the two halves: lane l holds items l and 64 + l
    uint32_t q[2];
    bool el[2];
#pragma unroll
    for (uint32_t h = 0; h < 2; ++h) {
        const uint32_t i = 64u * h + lane;
        q[h] = i < NI ? x0 + X.pos[i] : 0u;
        el[h] = i < NI && (i == 0u || w.buf[q[h] - 1u] == 106);
    }
    const u64 em0 = __ballot(el[0]), em1 = __ballot(el[1]);
    const uint32_t ne0 = (uint32_t)__popcll(em0);
    const uint32_t nel = min(min(ne0 + (uint32_t)__popcll(em1), kNT), left);
    // lane o < nel: element o of the batch (its item index it, rank, header, count)
    uint32_t it = 0, e = 0, cnt = 0, key = 0, m = 0;
    int32_t rk = -1;
    bool eok = lane < nel;
    if (eok) {
        it = lane < ne0 ? select64(em0, lane) : 64u + select64(em1, lane - ne0);
        const uint32_t s = x0 + X.pos[it];
        uint32_t hl = 0;
        rk = (int32_t)hdr_rank(w, s, lim, hh, t, E, hl);
        eok = rk >= 0;
        if (eok) {
            const uint4 ds = t.desc[rk];
            e = ds.x;
            cnt = ds.w;
            key = ds.z;
            const uint32_t y = s + hl;
            eok = y + 4u <= lim;
            m = eok ? __builtin_bswap32(word_at(w.buf, y)) : 0u;
            // its m records are items it + 1 .. it + m, all inside the batch, the first
            // right after the count
            eok = eok && m >= 1u && m <= cnt && it + m < NI && x0 + X.pos[it + 1u] == y + 4u;
        }
    }
    // ranks ascend: after the previous element (element 0: after prev)
    const int32_t prk = __shfl(rk, (lane + 63u) & 63u, 64);
    if (eok) eok = (int64_t)rk > (lane ? (int64_t)prk : prev);
    // the elements' bucket tables and empty presence tables; their rank -> slot maps
    uint32_t ros[kNT];
    wave_sync();
#pragma unroll
    for (uint32_t o = 0; o < kNT; ++o) {
        ros[o] = 0xFFu;
        if (o >= nel) continue;
        const int32_t r = (int32_t)rdlane((uint32_t)rk, o);
        if (r < 0) continue;
        const uint32_t co = rdlane(cnt, o);
        uint8_t* tab = o ? X.tab[o - 1] : L.tab;
        uint8_t* pr = o ? X.pres[o - 1] : L.pres;
        if (lane < co) {
            const uint32_t b = t.tb[(u64)r * RK + lane];
            if (b < kBuckets) tab[b] = (uint8_t)lane;
        }
        pr[lane] = 0;
        ros[o] = t.ros[64ull * r + lane];
    }
    wave_sync();
    // lane l: record 64 h + l of the batch
    uint32_t fend[2] = {0u, 0u};
    u64 bad[2];
    int32_t obad[2] = {0x7FFFFFFF, 0x7FFFFFFF};
    uint32_t last = 0xFFu;                       // rank of item 63 (the next half's lane 0)
    bad[1] = 0;
#pragma unroll
    for (uint32_t h = 0; h < 2; ++h) {
        if (64u * h >= NI) break;
        const uint32_t i = 64u * h + lane;
        // the element the item belongs to: element items up to it, minus one
        const u64 below = lane == 63u ? ~0ull : (2ull << lane) - 1ull;
        const uint32_t oi = (h ? ne0 + (uint32_t)__popcll(em1 & below)
                               : (uint32_t)__popcll(em0 & below)) - 1u;
        const bool rec = i < NI && !el[h] && oi < nel;
        const uint32_t src = rec ? oi : 0u;
        const uint32_t it_o = (uint32_t)__shfl((int32_t)it, (int32_t)src, 64);
        const uint32_t e_o = (uint32_t)__shfl((int32_t)e, (int32_t)src, 64);
        const uint32_t key_o = (uint32_t)__shfl((int32_t)key, (int32_t)src, 64);
        const uint32_t cnt_o = (uint32_t)__shfl((int32_t)cnt, (int32_t)src, 64);
        const uint32_t m_o = (uint32_t)__shfl((int32_t)m, (int32_t)src, 64);
        const uint32_t j = i - it_o;             // 1-based record index in the element
        bool ok = rec && j <= m_o;
        uint32_t rank = 0xFFu, fl = 0;
        if (ok) {
            const uint32_t x = q[h];
            const uint8_t* tab = src ? X.tab[src - 1u] : L.tab;
            const uint32_t kw = 4u * (key_o & 0xFFu), ksh = (key_o >> 8) & 31u;
            rank = tab[(word_at(w.buf, x + kw) >> ksh) & (kBuckets - 1u)];
            ok = rank < cnt_o;
            if (ok) ok = rec_match(w.buf, x, RL, d.rec_pad + ((u64)e_o * RK + rank) * RS);
            const uint32_t fo = x + RL;
            uint32_t fn;
            const uint32_t fk = flag_atom(word_at(w.buf, fo), word_at(w.buf, fo + 4u), fn);
            fend[h] = fo + fn;
            ok &= fk != 0u && fend[h] < lim;
            fl = fk == 1u;
        }
        // term order: after the previous record of the same element
        const uint32_t pr = __shfl(rank, (lane + 63u) & 63u, 64);
        const uint32_t prv = lane ? pr : last;
        if (ok && j > 1u) ok = rank > prv;
        last = rdlane(rank, 63u);
        // the record ends where the next item starts: the next record (j < m), or the
        // closing 106 of the element's token list (j = m) before the next element
        if (ok) {
            if (i + 1u < NI) {
                const uint32_t qn = x0 + X.pos[i + 1u];
                const bool nel_n = i + 1u < 64u ? ((em0 >> (i + 1u)) & 1ull) != 0
                                                : ((em1 >> (i - 63u)) & 1ull) != 0;
                ok = j < m_o ? !nel_n && fend[h] == qn : nel_n && fend[h] + 1u == qn;
            } else {
                ok = j == m_o && w.buf[min(fend[h], kBWin + 63u)] == 106;
            }
        }
        bad[h] = __ballot(rec && !ok);
        if (bad[h]) obad[h] = (int32_t)rdlane(oi, (uint32_t)__ffsll((long long)bad[h]) - 1u);
        if (ok) {
            uint8_t* prs = src ? X.pres[src - 1u] : L.pres;
            prs[rank] = (uint8_t)(1u | (fl << 1));
        }
    }
    // commit the elements before the first failure
    const u64 ebad = __ballot(lane < nel && !eok);
    uint32_t commit = ebad ? (uint32_t)__ffsll((long long)ebad) - 1u : nel;
    commit = (uint32_t)min((int32_t)commit, min(obad[0], obad[1]));
    if (commit == 0) return 0;
    wave_sync();
#pragma unroll
    for (uint32_t o = 0; o < kNT; ++o) {
        if (o >= commit) break;
        const uint8_t* prs = o ? X.pres[o - 1] : L.pres;
        const uint32_t v = ros[o] < 64u ? prs[ros[o]] : 0u;
        const u64 pb = __ballot(v & 1u), rb = __ballot(v & 2u);
        if (lane == 0) c[rdlane(e, o)] = u64x2{pb, rb};
    }
    prev = (int64_t)(int32_t)rdlane((uint32_t)rk, commit - 1u);
    const uint32_t li = rdlane(it, commit - 1u) + rdlane(m, commit - 1u);   // its last record
    pc = (li < 64u ? rdlane(fend[0], li) : rdlane(fend[1], li - 64u)) + 1u;
    return commit;
}

// Decode elements at the cursor into cells c: at most n of them (count mode), or with
// n = ~0u every element that starts before the absolute payload position `stop`, up to
// the list's closing 106 (segment mode: *tail is set when the cursor stops on it).
// prev is the previous element's term rank, nx the rank predicted next.  Returns the
// elements decoded; st receives the first failure's LASPJ_DEC_* status.
template <bool SMALL>
__device__ __forceinline__ uint32_t decode_elems(PWin& w, uint32_t& pc, int64_t& prev,
                                                 RankPre& nx, uint32_t n, u64 stop, bool& tail,
                                                 int32_t& st, const ReadTabs& tabs,
                                                 const DictView& d, const HdrHash& hh,
                                                 uint32_t E, ReadLds& L, ReadLdsX* X,
                                                 u64x2* c, uint32_t lane, Cases cs) {
    const uint32_t RL = d.rec_len, RS = d.rec_stride, RK = d.tok_max;
    const uint32_t hmax = min(d.ehdr_max + 4u, kBWin - 16u);
    const bool seg = n == 0xFFFFFFFFu;
    const uint32_t lj = cs.lj, lf = cs.lf;
    const bool lcase = cs.on;
    const bool many = !SMALL && X && hh.tab && hh.many && !seg;
    // Element batches pay off only when they fill up (kNT small elements): after one
    // that does not, the next 16 elements go one at a time (hold); after an element of
    // more than 12 records, too (cool), until an element of <= 12 records re-arms them.
    // hint: bytes the next batch scans (kNT elements at the last batch's bytes per
    // element).
    uint32_t k = 0, cool = 0, hold = 0, hint = 1024;
    while (k < n && st == LASPJ_DEC_OK) {
        if (seg) {
            if (w.lo + pc >= stop) break;
            if (pc + 1 > w.end) { st = LASPJ_DEC_MALFORMED; break; }
            pc = need(w, pc, 1);
            if (ub(w, pc) == 106) { tail = true; break; }
        }
        if (SMALL) {
            const uint32_t got =
                hh.tab ? read_batch_par(w, pc, prev, n - k, stop, tabs, d, hh, E, L, c, lane)
                       : read_batch(w, pc, prev, n - k, stop, tabs, d, E, RL, RS, L, c, lane);
            if (got) {
                k += got;
                if (k < n) nx = load_rank(tabs, RK, prev + 1, E, lane);
                continue;
            }
        }
        if (many) {
            if (cool == 0 && hold == 0) {
                const u64 at = w.lo + pc;
                const uint32_t got = read_batch_many(w, pc, prev, n - k, hint, tabs, d, hh, E,
                                                     L, *X, c, lane);
                if (got < kNT) hold = 16;
                if (!got) hint = min(2u * hint, 3840u);
                if (got) {
                    hint = (uint32_t)min((w.lo + pc - at) / got * kNT + 256u, (u64)3840u);
                    k += got;
                    if (k < n) nx = load_rank(tabs, RK, prev + 1, E, lane);
                    continue;
                }
            } else {
                if (cool) --cool;
                if (hold) --hold;
            }
        }
        // 104 2 <elem image> 108 <count:32> of the next element in term order
        const uint32_t span = min(hmax, w.end - pc);
        pc = need(w, pc, span);
        const uint32_t byte = pc + lane < min(w.hi, w.end) ? w.buf[pc + lane] : 0x100u;
        int64_t found = -1;
        RankPre cur = nx;
        if (prev + 1 < (int64_t)E && cur.hl > 3u && cur.hl <= span && cur.hl <= 64u) {
            const bool ok = lane >= cur.hl - 1u || byte == cur.hb;
            if (!__ballot(!ok)) found = prev + 1;
        }
        if (found < 0) {
            for (int64_t c0 = prev + 1; c0 < (int64_t)E && found < 0; c0 += 64) {
                const int64_t r = c0 + lane;
                bool hit = false;
                if (r < (int64_t)E) {
                    const uint32_t ec = d.elem_order[r];
                    const uint32_t hlc = d.elem_off[ec + 1] - d.elem_off[ec] + 3u;
                    // 104 2 <elem image> (the closing 108 is checked below)
                    if (hlc > 3u && hlc <= span) {
                        const uint8_t* t = d.ehdr_pad + d.ehdr_poff[ec];
                        const uint8_t* q = w.buf + pc;
                        if (hlc - 1u <= 48) {
                            hit = eq48(q, t, hlc - 1u);
                        } else {
                            hit = true;
                            for (uint32_t i = 0; i < hlc - 1u && hit; ++i) hit = q[i] == t[i];
                        }
                    }
                }
                const u64 m = __ballot(hit);
                if (m) found = c0 + __ffsll((long long)m) - 1;
            }
            if (found < 0) { st = LASPJ_DEC_UNKNOWN_TERM; break; }
            cur = load_rank(tabs, RK, found, E, lane);
        }
        prev = found;
        nx = load_rank(tabs, RK, found + 1, E, lane);
        const uint32_t e = cur.e, hl = cur.hl;
        pc += hl;
        const uint32_t close = hl <= 64u ? rdlane(byte, hl - 1u) : ub(w, pc - 1);
        if (close != 108) {                        // [] tokens: no columnar form
            st = close == 106 ? LASPJ_DEC_UNREPRESENTABLE : LASPJ_DEC_MALFORMED;
            break;
        }
        if (pc + 4 > w.end) { st = LASPJ_DEC_MALFORMED; break; }    // truncated count
        uint32_t m_tok;
        if (hl + 4u <= 64u) {
            m_tok = (rdlane(byte, hl) << 24) | (rdlane(byte, hl + 1u) << 16) |
                    (rdlane(byte, hl + 2u) << 8) | rdlane(byte, hl + 3u);
        } else {
            pc = need(w, pc, 4);
            m_tok = (ub(w, pc) << 24) | (ub(w, pc + 1) << 16) | (ub(w, pc + 2) << 8) |
                    ub(w, pc + 3);
        }
        pc += 4;
        if (m_tok == 0 || m_tok > 64) { st = LASPJ_DEC_UNREPRESENTABLE; break; }
        if (many) {
            if (m_tok <= 12u) cool = 0;
            else if (cool < 16u) cool = 16;
        }
        // the element's bucket table and an empty presence table
        const uint32_t kw = 4u * (cur.key & 0xFFu), ksh = (cur.key >> 8) & 31u;
        wave_sync();
        const bool nobk = (cur.key & kNoBuckets) != 0;
        if (lane < cur.cnt && !nobk) L.tab[cur.tb] = (uint8_t)lane;
        L.pres[lane] = 0;
        wave_sync();
        int32_t tprev = -1;             // the last record's order key (2 rank + 1; new: 2 below)
        uint32_t done = 0, nnew = 0;    // new tokens of the element so far
        u64 np = 0, nr = 0;             // their slot bits (present, removed)
        if (d.tok_max > 8 && !nobk) {
            // many records per element: locate them byte-parallel (the chain below only
            // when that does not validate)
            const uint32_t want = min(m_tok * (RL + 8u) + 8u, w.end - pc);
            if (pc + want > w.hi && w.hi < w.end) pc = refill(w, pc);
            if (locate_records(w, pc, m_tok, cur, e, kw, ksh, L, d, lane)) done = m_tok;
        }
        while (done < m_tok) {
            // room for the batch in the window
            {
                const uint32_t want = min((m_tok - done) * (RL + 8u) + 8u, w.end - pc);
                if (pc + want > w.hi && w.hi < w.end) pc = refill(w, pc);
            }
            // the chain, in window offsets: a record at x is complete before the
            // payload end when x <= tlim, inside the window when x <= wlim
            const int32_t tlim = (int32_t)w.end - (int32_t)RL - 6;
            const int32_t wlim = w.hi >= w.end ? 0x7FFFFFFF : (int32_t)w.hi - (int32_t)RL - 8;
            const int32_t lim = min(tlim, wlim);
            const uint32_t t0 = pc + RL < w.hi ? ub(w, pc + RL) : 0u;
            const uint32_t h = t0 == 119 ? 2u : 3u;     // the batch's atom header
            const uint32_t L0 = RL + h + 4u;              // a `true` record
            uint32_t nb = 0, x = pc, myx = 0;
            bool trunc = false;
            while (nb < 64 && done + nb < m_tok) {
                const uint32_t J = min(10u, min(64u - nb, m_tok - done - nb));
                // lane (lj, lf): the flag header of record lj after lf falses
                uint32_t code = 0;
                if (lcase && lj < J) {
                    const uint32_t q = x + lj * L0 + lf + RL;
                    if (q + 3 <= w.hi) {
                        code = flag_code(word_at(w.buf, q), h);
                        if (q + h + 4 + (code >> 1) > w.end) code = 0;
                    }
                }
                uint32_t f = 0, jr = 0, idx = 0;
                u64 fz = 0;
                bool stop_walk = false;
                for (; jr < J; ++jr) {
                    const int32_t xj = (int32_t)(x + jr * L0 + f);
                    if (xj > lim) { trunc = xj > tlim; stop_walk = true; break; }
                    const uint32_t cj = rdlane(code, idx + f);
                    if (!(cj & 1u)) break;
                    fz |= (u64)(cj >> 1) << jr;
                    f += cj >> 1;
                    idx += jr + 1;
                }
                // lanes nb .. nb + jr - 1: starts of the walked records
                if (lane >= nb && lane < nb + jr) {
                    const uint32_t i = lane - nb;
                    myx = x + i * L0 + __popcll(fz & ((1ull << i) - 1ull));
                }
                x += jr * L0 + f;
                nb += jr;
                if (stop_walk || nb >= 64 || done + nb >= m_tok) break;
                if (jr == J) continue;
                // a record the walk did not take: one general step
                if (lane == nb) myx = x;
                const uint32_t a0 = ub(w, x + RL), a1 = ub(w, x + RL + 1), a2 = ub(w, x + RL + 2);
                uint32_t gh = 0, len = 0;
                if ((a0 == 100 || a0 == 118) && a1 == 0) { gh = 3; len = a2; }
                else if (a0 == 119) { gh = 2; len = a1; }
                ++nb;
                // a bad flag header ends the chain; lane nb - 1 reports it
                if ((len != 4 && len != 5) || x + RL + gh + len > w.end) break;
                x += RL + gh + len;
            }
            if (nb == 0 && !trunc) { st = LASPJ_DEC_MALFORMED; break; }   // no progress
            // lane j < nb: record j
            const bool mine = lane < nb;
            int32_t lst = LASPJ_DEC_OK;
            uint32_t rank = 0xFFu, fl = 0;
            bool unk = false, fok = false;
            int32_t key = -1;
            if (mine) {
                bool eq = false;
                if (nobk) {
                    // template by template
                    for (uint32_t j = 0; j < cur.cnt && !eq; ++j)
                        if (rec_match(w.buf, myx, RL, d.rec_pad + ((u64)e * RK + j) * RS)) {
                            rank = j;
                            eq = true;
                        }
                } else {
                    rank = L.tab[(word_at(w.buf, myx + kw) >> ksh) & (kBuckets - 1u)];
                    eq = rank < cur.cnt;
                    if (eq) {                       // exact compare
                        eq = rec_match(w.buf, myx, RL, d.rec_pad + ((u64)e * RK + rank) * RS);
                    }
                }
                if (eq) {
                    key = 2 * (int32_t)rank + 1;
                } else if (tabs.nt.out && new_tok_image(w.buf, myx, RL)) {
                    // a token the element's images lack: its place among them
                    const int32_t ip = new_tok_rank(w.buf, myx, RL,
                                                    d.rec_pad + (u64)e * RK * RS, RS, cur.cnt);
                    if (ip >= 0) {
                        unk = true;
                        key = 2 * ip;
                    }
                }
                // ATOM_EXT / ATOM_UTF8_EXT (2-byte length), SMALL_ATOM_UTF8_EXT
                // (1-byte length), then "true" / "false"
                const uint32_t fo = myx + RL;
                const uint32_t* f32 = reinterpret_cast<const uint32_t*>(w.buf + (fo & ~3u));
                const uint32_t v0 = __builtin_amdgcn_alignbyte(f32[1], f32[0], fo & 3u);
                const uint32_t v1 = __builtin_amdgcn_alignbyte(f32[2], f32[1], fo & 3u);
                uint32_t fn;
                const uint32_t fk = flag_atom(v0, v1, fn);
                const uint32_t fend = fo + fn;            // one past the flag
                const bool tr = fk == 1u && fend <= w.end;
                const bool fa = fk == 2u && fend <= w.end;
                fl = tr;
                fok = tr || fa;
            }
            // term order: after the previous record (two new tokens between the same two
            // known ones: by their images)
            const int32_t pk = __shfl(key, (lane + 63u) & 63u, 64);
            const uint32_t px = __shfl(myx, (lane + 63u) & 63u, 64);
            if (mine) {
                const int32_t before = lane ? pk : tprev;
                const bool asc = key > before ||
                                 (unk && key == before && lane && img_after(w.buf, myx, px, RL));
                lst = key < 0 || !asc ? LASPJ_DEC_UNKNOWN_TERM
                      : !fok                       ? LASPJ_DEC_MALFORMED
                                                   : LASPJ_DEC_OK;
            }
            u64 bad = __ballot(lst != LASPJ_DEC_OK);
            const u64 um = __ballot(mine && unk);
            if (!bad && um) {
                // new tokens: the element's next free slots, in payload order; an entry each
                const uint32_t nu = (uint32_t)__popcll(um);
                if (cur.cnt + nnew + nu > 64u) {
                    bad = 1;
                    lst = LASPJ_DEC_UNKNOWN_TERM;
                } else {
                    const uint32_t slot =
                        cur.cnt + nnew + (uint32_t)__popcll(um & ((1ull << lane) - 1ull));
                    bool over = false;
                    if (mine && unk) {
                        const uint32_t idx = atomicAdd(tabs.nt.cnt, 1u);
                        over = idx >= tabs.nt.cap;
                        if (!over)
                            tabs.nt.out[idx] = NewTok{tabs.nt.seq, e, slot,
                                                      (uint32_t)(w.lo + myx + 2u)};
                    }
                    if (__ballot(over)) {
                        bad = 1;
                        lst = LASPJ_DEC_UNKNOWN_TERM;
                    } else {
                        const u64 tm = __ballot(mine && unk && fl);
                        u64 mm = um;
                        for (uint32_t k = 0; mm; ++k, mm &= mm - 1ull) {
                            const uint32_t f = (uint32_t)__ffsll((long long)mm) - 1u;
                            np |= 1ull << (cur.cnt + nnew + k);
                            if ((tm >> f) & 1ull) nr |= 1ull << (cur.cnt + nnew + k);
                        }
                        nnew += nu;
                    }
                }
            }
            if (bad) {
                st = (int32_t)rdlane((uint32_t)lst, (uint32_t)__ffsll((long long)bad) - 1u);
                break;
            }
            if (trunc) { st = LASPJ_DEC_MALFORMED; break; }
            if (mine && !unk) L.pres[rank] = (uint8_t)(1u | (fl << 1));
            tprev = (int32_t)rdlane((uint32_t)key, nb - 1u);
            done += nb;
            pc = x;
        }
        if (st != LASPJ_DEC_OK) break;
        if (pc + 1 > w.end) { st = LASPJ_DEC_MALFORMED; break; }
        pc = need(w, pc, 1);
        if (ub(w, pc) != 106) { st = LASPJ_DEC_MALFORMED; break; }
        pc += 1;
        // presence by rank -> slot bits: lane s reads its slot's rank
        wave_sync();
        const uint32_t v = cur.ros < 64u ? L.pres[cur.ros] : 0u;
        const u64 pb = __ballot(v & 1u), rb = __ballot(v & 2u);
        if (lane == 0) c[e] = u64x2{pb | np, rb | nr};
        ++k;
    }
    return k;
}

// One replica's payload decoded by one wave, from its head to its end (cells cleared
// first when `clear`): the reference's status.
template <bool SMALL>
__device__ int32_t decode_replica(const uint8_t* payload, u64 total, const u64* offs,
                                  uint64_t rep, uint32_t E, const DictView& d,
                                  const ReadTabs& tabs, const HdrHash& hh, int tag, int vers,
                                  u64x2* c, bool clear, ReadLds& L, ReadLdsX* X,
                                  uint32_t lane, Cases cs) {
    const uint32_t RK = d.tok_max;
    const u64 base = ufl(offs[rep]), aend = ufl(offs[rep + 1]);
    if (clear)
        for (uint32_t e = lane; e < E; e += 64) c[e] = u64x2{0, 0};
    PWin w{L.win, payload, total, aend, base, 0, (uint32_t)min(aend - base, (u64)0x7FFFFFFF)};
    uint32_t pc = 0, n = 0;
    bool list = false;
    int32_t st = parse_head(w, pc, tag, vers, n, list);
    if (st == LASPJ_DEC_OK) {
        int64_t prev = -1;                    // term rank of the previous element
        RankPre nx = load_rank(tabs, RK, 0, E, lane);   // the predicted next rank
        bool tail = false;
        decode_elems<SMALL>(w, pc, prev, nx, n, ~0ull, tail, st, tabs, d, hh, E, L, X, c, lane,
                            cs);
    }
    if (st == LASPJ_DEC_OK && list) {
        if (pc + 1 > w.end) st = LASPJ_DEC_MALFORMED;
        else {
            pc = need(w, pc, 1);
            if (ub(w, pc) != 106) st = LASPJ_DEC_MALFORMED;
            pc += 1;
        }
    }
    if (st == LASPJ_DEC_OK && w.lo + pc != aend) st = LASPJ_DEC_MALFORMED;   // trailing bytes
    return st;
}

// One wave per replica.  With `redo` (segment mode's fallback) the wave takes the
// replicas listed there (redo[0] of them) and clears their cells first.
// (element batches: 5 waves per SIMD give 96 VGPRs, 6 spilled instead of 20 at 6 waves,
// t3 1.05-1.09 -> 1.03-1.04 ms, profiles/r03k_decoder_occ5_ab.log; many-token
// dictionaries: the element batches' LDS leaves 4)
template <bool SMALL>
__global__ __launch_bounds__(kBlock, SMALL ? 5 : 4) void k_orset_etf_read(const uint8_t* payload, u64 total,
                                                           const u64* offs, uint64_t R,
                                                           uint32_t E, DictView d,
                                                           ReadTabs tabs, HdrHash hh, int tag,
                                                           int vers, u64x2* cells,
                                                           int32_t* status,
                                                           const uint32_t* redo) {
    __shared__ __attribute__((aligned(16))) ReadLds lds[kBlock / 64];
    __shared__ __attribute__((aligned(16))) ReadLdsX ldx[SMALL ? 1 : kBlock / 64];
    // the wave index as a scalar: everything per replica then stays wave-uniform
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint64_t nwaves = (uint64_t)gridDim.x * (kBlock / 64);
    ReadLdsX* X = SMALL ? nullptr : &ldx[wave];
    const Cases cs = lane_cases(lane);
    ReadLds& L = lds[wave];
    const uint64_t count = redo ? (uint64_t)ufl32(redo[0]) : R;
    for (uint64_t i = (uint64_t)blockIdx.x * (kBlock / 64) + wave; i < count; i += nwaves) {
        const uint64_t rep = redo ? (uint64_t)ufl32(redo[1 + i]) : i;
        const int32_t st = decode_replica<SMALL>(payload, total, offs, rep, E, d, tabs, hh, tag,
                                                 vers, cells + rep * E, redo != nullptr, L, X,
                                                 lane, cs);
        if (lane == 0) status[rep] = st;
    }
}

// ---- long payloads split between waves (segment mode)
//
// A payload of len bytes is cut into segments of S bytes; segment s of a replica is
// decoded by its own wave.  Segment 0 parses the list header; segment s > 0 first
// looks for an element header 106 104 2 <elem image> 108 at or after s S (the byte
// before an element is the previous element's closing 106) whose image is in the
// dictionary (hash of the header bytes -> rank, then an exact compare), then decodes
// every element that starts inside the segment.  A token image may contain such a
// byte run, so nothing is trusted yet: k_etf_read_chain checks per replica that each
// segment starts exactly where the previous one ended, ranks ascend across segments,
// the element count matches the header and the list closes at the payload end.  A
// replica that fails any of this (or any segment status) is decoded again from the
// start by k_orset_etf_read over the redo list, which gives the reference's status.
struct SegRes {
    int32_t st;
    uint32_t start, end, cnt;    // first element / cursor at the end (relative), elements
    int32_t rfirst, rlast;       // rank of the first / last element decoded
    uint32_t n, flags;           // segment 0: the header's count; kSeg* bits
};
constexpr uint32_t kSegNone = 0xFFFFFFFFu;
constexpr uint32_t kSegEmptyList = 1u;

// the rank of the element whose header template is at window offset x, or -1
__device__ int64_t resolve_hdr(const PWin& w, uint32_t x, const HdrHash& hh,
                               const ReadTabs& t, uint32_t E, uint32_t lane) {
    const uint32_t hl = lane + 1u;
    const uint32_t lim = min(w.hi, w.end);
    const bool on = ((hh.lens >> lane) & 1ull) && x + hl <= lim;
    uint32_t h = hl * 0x85EBCA6Bu;
    uint32_t q[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int rem = (int)hl - 4 * i;
        const uint32_t v = word_at(w.buf, min(x + 4u * i, kBWin + 56u));
        q[i] = rem >= 4 ? v : rem <= 0 ? 0u : v & ((1u << (8 * rem)) - 1u);
        if (rem > 0) h = hdr_mix(h, q[i]);            // ceil(hl / 4) words
    }
    int64_t rank = -1;
    if (on) {
        for (uint32_t i = h & hh.mask;; i = (i + 1) & hh.mask) {
            const uint32_t v = hh.tab[i];
            if (!v || v > E) break;
            const uint32_t rk = v - 1u;
            if (t.desc[rk].y != hl) continue;
            const u32x4* tp = reinterpret_cast<const u32x4*>(t.hdr + 64ull * rk);
            bool eq = true;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const u32x4 a = tp[j];
                eq &= a.x == q[4 * j] && a.y == q[4 * j + 1] && a.z == q[4 * j + 2] &&
                      a.w == q[4 * j + 3];
            }
            if (eq) { rank = rk; break; }
        }
    }
    const u64 m = __ballot(rank >= 0);
    // images are self-delimiting and distinct: at most one header length matches
    return m ? (int64_t)rdlane((uint32_t)rank, (uint32_t)__ffsll((long long)m) - 1u) : -1;
}

// Is replica's segment chain one well-formed orddict (segments g0 .. g0 + ns of res)?
// One wave, lanes over the segments 64 at a time: segment s's predecessor is the latest
// earlier segment that found an element start (a max-scan of indices over the lanes,
// carried between groups of 64), and every segment checks itself against it — a start
// that found nothing is fine only where no element starts, a found one must begin exactly
// at its predecessor's end with a higher first rank — then one ballot and one sum of
// element counts decide (the chain's checks, evaluated in parallel: the answer is whether
// any of them fails).
__device__ bool chain_ok(const uint8_t* payload, u64 base, u64 len, uint32_t g0, uint32_t ns,
                         uint32_t S, const SegRes* res, uint32_t lane) {
    const SegRes a = res[g0];
    bool ok = a.st == LASPJ_DEC_OK;
    if (ok && (a.flags & kSegEmptyList)) return a.end == len;
    if (!ok) return false;
    uint32_t q = a.end, cnt = 0;
    int32_t rl = a.rlast;
    bool bad = false;
    for (uint32_t s0 = 1; s0 < ns; s0 += 64) {
        const uint32_t s = s0 + lane;
        SegRes b{LASPJ_DEC_OK, kSegNone, 0, 0, -1, -1, 0, 0};
        if (s < ns) b = res[g0 + s];
        const bool valid = s < ns && b.start != kSegNone;
        int32_t li = valid ? (int32_t)lane : -1;      // latest valid lane <= this one
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int32_t v = __shfl_up(li, off, 64);
            if ((int)lane >= off) li = max(li, v);
        }
        int32_t lp = __shfl_up(li, 1, 64);             // ... strictly before it
        if (lane == 0) lp = -1;
        const uint32_t e_at = __shfl(b.end, lp < 0 ? 0 : lp, 64);
        const int32_t r_at = __shfl(b.rlast, lp < 0 ? 0 : lp, 64);
        const uint32_t pq = lp >= 0 ? e_at : q;
        const int32_t prl = lp >= 0 ? r_at : rl;
        if (s < ns) {
            if (!valid) {
                // no header found: fine only if none starts here (the predecessor's end
                // past the segment, or on the list's closing 106)
                const u64 send = (u64)(s + 1) * S;
                if (pq < send && pq < len && payload[base + pq] != 106) bad = true;
            } else if (b.start != pq || b.st != LASPJ_DEC_OK || b.rfirst <= prl) {
                bad = true;
            } else {
                cnt += b.cnt;
            }
        }
        const int32_t last = __shfl(li, 63, 64);
        if (last >= 0) {
            q = __shfl(b.end, last, 64);
            rl = __shfl(b.rlast, last, 64);
        }
    }
    uint32_t tot = cnt;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) tot += __shfl_xor(tot, off, 64);
    return !__ballot(bad) && a.cnt + tot == a.n && (u64)q + 1 == len && payload[base + q] == 106;
}

// The chain check as a status, for callers that cannot decode a failed payload again on
// the spot (the NIF merge checks chains beside the join, laspj_nif.hip): OK; a failing
// segment's own status when every segment before it chains (it then started where the
// serial decoder would be, so the serial decoder stops at the same element with the same
// status); kDecRedo when the chain breaks first (a false header match, a malformed
// payload): only a serial decode tells.  The same per-segment checks as chain_ok, the
// first offending segment in stream order deciding.
__device__ void chain_publish(const ChainArgs& cj, uint32_t r, int32_t st, uint32_t lane) {
    if (!cj.hres || st == LASPJ_DEC_OK) return;
    static_assert(sizeof(SegRes) == 32, "four words a segment");
    const uint32_t g0 = cj.segbase[r], n = 4u * (cj.segbase[r + 1] - g0);
    const u64* src = reinterpret_cast<const u64*>(cj.res + g0);
    u64* dst = reinterpret_cast<u64*>(cj.hres + g0);
    for (uint32_t k = lane; k < n; k += 64) dst[k] = src[k];
}

__device__ int32_t chain_verdict(const uint8_t* payload, u64 base, u64 len, uint32_t g0,
                                 uint32_t ns, uint32_t S, const SegRes* res, uint32_t lane) {
    // segment 0 and the first 256 segments' results loaded together (one memory round
    // trip for a payload of up to 257 segments, instead of one per 64)
    constexpr int kPre = 4;
    SegRes pre[kPre];
#pragma unroll
    for (int t = 0; t < kPre; ++t) {
        const uint32_t s = 1u + 64u * t + lane;
        pre[t] = s < ns ? res[g0 + s] : SegRes{LASPJ_DEC_OK, kSegNone, 0, 0, -1, -1, 0, 0};
    }
    const SegRes a = res[g0];
    if (a.st != LASPJ_DEC_OK) return a.st;                 // segment 0 starts at the head
    if (a.flags & kSegEmptyList) return a.end == len ? LASPJ_DEC_OK : kDecRedo;
    uint32_t q = a.end, cnt = 0;
    int32_t rl = a.rlast;
    for (uint32_t s0 = 1; s0 < ns; s0 += 64) {
        const uint32_t s = s0 + lane;
        SegRes b{LASPJ_DEC_OK, kSegNone, 0, 0, -1, -1, 0, 0};
        const uint32_t grp = (s0 - 1u) / 64u;
        if (grp < (uint32_t)kPre) {
#pragma unroll
            for (int t = 0; t < kPre; ++t)
                if ((uint32_t)t == grp) b = pre[t];
        } else if (s < ns) {
            b = res[g0 + s];
        }
        const bool valid = s < ns && b.start != kSegNone;
        int32_t li = valid ? (int32_t)lane : -1;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int32_t v = __shfl_up(li, off, 64);
            if ((int)lane >= off) li = max(li, v);
        }
        int32_t lp = __shfl_up(li, 1, 64);
        if (lane == 0) lp = -1;
        const uint32_t e_at = __shfl(b.end, lp < 0 ? 0 : lp, 64);
        const int32_t r_at = __shfl(b.rlast, lp < 0 ? 0 : lp, 64);
        const uint32_t pq = lp >= 0 ? e_at : q;
        const int32_t prl = lp >= 0 ? r_at : rl;
        bool brk = false, bad = false;
        if (s < ns) {
            if (!valid) {
                const u64 send = (u64)(s + 1) * S;
                brk = pq < send && pq < len && payload[base + pq] != 106;
            } else if (b.start != pq || b.rfirst <= prl) {
                brk = true;
            } else if (b.st != LASPJ_DEC_OK) {
                bad = true;
            }
        }
        const u64 ev = __ballot(brk || bad);
        if (ev) {
            const uint32_t f = (uint32_t)__ffsll((long long)ev) - 1u;
            const int32_t fst = __shfl(b.st, f, 64);
            const bool fbrk = __shfl((int)brk, f, 64) != 0;
            return fbrk ? kDecRedo : fst;
        }
        cnt += valid ? b.cnt : 0u;
        const int32_t last = __shfl(li, 63, 64);
        if (last >= 0) {
            q = __shfl(b.end, last, 64);
            rl = __shfl(b.rlast, last, 64);
        }
    }
    uint32_t tot = cnt;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) tot += __shfl_xor(tot, off, 64);
    return a.cnt + tot == a.n && (u64)q + 1 == len && payload[base + q] == 106 ? LASPJ_DEC_OK
                                                                              : kDecRedo;
}

// segment s of replica rep's payload (cells c: the replica's) decoded by one wave: its
// SegRes into *out
template <bool SMALL>
__device__ __forceinline__ void seg_decode(const uint8_t* payload, u64 total, const u64* offs,
                                           uint64_t rep, uint32_t s, uint32_t E,
                                           const DictView& d, const ReadTabs& tabs,
                                           const HdrHash& hh, int tag, int vers, u64x2* c,
                                           uint32_t S, SegRes* res_out, ReadLds& L,
                                           uint32_t lane, const Cases& cs) {
    const uint32_t RK = d.tok_max;
    {
        const u64 base = ufl(offs[rep]), aend = ufl(offs[rep + 1]);
        const uint32_t len = (uint32_t)min(aend - base, (u64)0x7FFFFFFF);
        PWin w{L.win, payload, total, aend, base, 0, len};
        SegRes out{LASPJ_DEC_OK, kSegNone, kSegNone, 0, -1, -1, 0, 0};
        const uint32_t send = (uint32_t)min((u64)(s + 1) * S, (u64)len);
        const u64 stop = base + (u64)(s + 1) * S;
        uint32_t pc = 0;
        int64_t prev = -1;
        RankPre nx;
        bool go = true;
        if (s == 0) {
            uint32_t n = 0;
            bool list = false;
            out.st = parse_head(w, pc, tag, vers, n, list);
            out.n = n;
            if (out.st != LASPJ_DEC_OK || !list) {
                if (out.st == LASPJ_DEC_OK) out.flags = kSegEmptyList;     // 131 106
                out.end = (uint32_t)(w.lo + pc - base);
                go = false;
            } else {
                out.start = (uint32_t)(w.lo + pc - base);
                nx = load_rank(tabs, RK, 0, E, lane);
            }
        } else {
            // the first element header at or after s S: 106 104 2 <elem image> 108
            pc = s * S - 1u;
            int64_t found = -1;
            while (w.lo + pc + 1u < base + send) {
                pc = need(w, pc, min(w.end - pc, 136u));
                const uint32_t lim = min(w.hi, w.end);
                const uint32_t x = pc + 1u + lane;
                const bool hit = w.lo + x < base + send && x + 1u < lim &&
                                 w.buf[min(x - 1u, kBWin + 63u)] == 106 &&
                                 w.buf[min(x, kBWin + 63u)] == 104 &&
                                 w.buf[min(x + 1u, kBWin + 63u)] == 2;
                u64 m = __ballot(hit);
                while (m && found < 0) {
                    const uint32_t f = (uint32_t)__ffsll((long long)m) - 1u;
                    m &= m - 1ull;
                    found = resolve_hdr(w, pc + 1u + f, hh, tabs, E, lane);
                    if (found >= 0) pc = pc + 1u + f;
                }
                if (found >= 0) break;
                pc += 64u;
            }
            if (found < 0) {
                go = false;                       // no element starts in this segment
            } else {
                out.start = (uint32_t)(w.lo + pc - base);
                out.rfirst = (int32_t)found;
                prev = found - 1;
                nx = load_rank(tabs, RK, found, E, lane);
            }
        }
        if (go) {
            bool tail = false;
            int32_t st = LASPJ_DEC_OK;
            out.cnt = decode_elems<SMALL>(w, pc, prev, nx, 0xFFFFFFFFu, stop, tail, st, tabs, d,
                                          hh, E, L, nullptr, c, lane, cs);
            out.st = st;
            out.end = (uint32_t)(w.lo + pc - base);
            out.rlast = (int32_t)prev;
        }
        if (lane == 0) *res_out = out;
    }
}

// the replica whose segments hold global segment g: the last r with segbase[r] <= g
__device__ __forceinline__ uint64_t seg_replica(const uint32_t* segbase, uint64_t R, uint64_t g) {
    uint64_t lo = 0, hi = R;
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (ufl32(segbase[mid]) <= g) lo = mid;
        else hi = mid;
    }
    return lo;
}

template <bool SMALL>
__global__ __launch_bounds__(kBlock, 6) void k_orset_etf_read_seg(
    const uint8_t* payload, u64 total, const u64* offs, uint64_t R, uint32_t E, DictView d,
    ReadTabs tabs, int tag, int vers, u64x2* cells, const uint32_t* segbase, uint64_t nseg,
    uint32_t S, HdrHash hh, SegRes* res, SegList only) {
    __shared__ __attribute__((aligned(16))) ReadLds lds[kBlock / 64];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint64_t nwaves = (uint64_t)gridDim.x * (kBlock / 64);
    const Cases cs = lane_cases(lane);
    ReadLds& L = lds[wave];
    const uint64_t count = only.n ? only.n : nseg;
    for (uint64_t j = (uint64_t)blockIdx.x * (kBlock / 64) + wave; j < count; j += nwaves) {
        const uint64_t g = only.n ? only.g[j] : j;
        const uint64_t rep = seg_replica(segbase, R, g);
        const uint32_t s = (uint32_t)(g - ufl32(segbase[rep]));
        seg_decode<SMALL>(payload, total, offs, rep, s, E, d, tabs, hh, tag, vers,
                          cells + rep * E, S, res + g, L, lane, cs);
    }
}

// per replica: is the segment chain one well-formed orddict?  Yes: status OK.  No:
// onto the redo list (decoded again serially, which gives the reference's status).
// One wave per replica, lanes over its segments 64 at a time: segment s's predecessor
// is the latest earlier segment that found an element start (a max-scan of indices
// over the lanes, carried between groups of 64), and every segment checks itself
// against it — a start that found nothing is fine only where no element starts, a
// found one must begin exactly at its predecessor's end with a higher first rank —
// then one ballot and one sum of element counts decide (the chain's checks, evaluated
// in parallel: the answer is whether any of them fails).
// With `cells` (the default), a replica whose chain fails is decoded again right here by
// this wave from its head, its cells cleared first (the redo pass's work, the reference's
// status): one launch fewer.  Without, it goes onto the redo list for k_orset_etf_read.
template <bool SMALL>
__global__ __launch_bounds__(64) void k_etf_read_chain(const uint8_t* payload, u64 total,
                                                       const u64* offs, uint64_t R,
                                                       const uint32_t* segbase, uint32_t S,
                                                       const SegRes* res, int32_t* status,
                                                       uint32_t* redo, uint32_t E, DictView d,
                                                       ReadTabs tabs, HdrHash hh, int tag,
                                                       int vers, u64x2* cells) {
    __shared__ __attribute__((aligned(16))) ReadLds L;
    const uint32_t lane = threadIdx.x;
    const Cases cs = lane_cases(lane);
    for (uint64_t r = blockIdx.x; r < R; r += gridDim.x) {
        const u64 base = offs[r];
        const bool ok = chain_ok(payload, base, offs[r + 1] - base, segbase[r],
                                 segbase[r + 1] - segbase[r], S, res, lane);
        if (ok) {
            if (lane == 0) status[r] = LASPJ_DEC_OK;
        } else if (cells) {
            const int32_t st = decode_replica<SMALL>(payload, total, offs, r, E, d, tabs, hh, tag,
                                                     vers, cells + r * E, true, L, nullptr, lane,
                                                     cs);
            if (lane == 0) status[r] = st;
        } else if (lane == 0) {
            status[r] = LASPJ_DEC_MALFORMED;           // rewritten by the redo pass
            const uint32_t i = atomicAdd(redo, 1u);
            redo[1 + i] = (uint32_t)r;
        }
    }
}

// ---- payloads over several dictionaries in one launch: the NIF binds many resident
// variables per call (lasp_vnode.erl:213-237), each variable in a token namespace — a
// dictionary — of its own.  A table holds every dictionary's decode views; a wave loads
// the views of the payload it takes (the index is wave-uniform: scalar loads) and decodes
// exactly as the one-dictionary kernels do.  Dictionaries with many tokens per element and
// the SMALL ones take separate launches of the same grid (each skips the other's payloads).
struct DecTabs {
    DictView d;
    ReadTabs tabs;
    HdrHash hh;          // header search (segment starts)
    HdrHash hh_small;    // element batches
    u64x2* cells;        // the cells of the group's first payload
    uint64_t rep0;       // the group's first payload
    uint32_t E;
    uint32_t small;      // d.tok_max <= kSmallTok
};

template <bool SMALL>
__global__ __launch_bounds__(kBlock, 6) void k_orset_etf_read_seg_multi(
    const uint8_t* payload, u64 total, const u64* offs, uint64_t R, const DecTabs* dts,
    const uint32_t* pay_dt, int tag, int vers, const uint32_t* segbase, uint64_t nseg,
    uint32_t S, SegRes* res, SegList only) {
    __shared__ __attribute__((aligned(16))) ReadLds lds[kBlock / 64];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint64_t nwaves = (uint64_t)gridDim.x * (kBlock / 64);
    const Cases cs = lane_cases(lane);
    ReadLds& L = lds[wave];
    const uint64_t count = only.n ? only.n : nseg;
    for (uint64_t j = (uint64_t)blockIdx.x * (kBlock / 64) + wave; j < count; j += nwaves) {
        const uint64_t g = only.n ? only.g[j] : j;
        const uint64_t rep = seg_replica(segbase, R, g);
        const uint32_t k = ufl32(pay_dt[rep]);
        if ((dts[k].small != 0) != SMALL) continue;
        const DecTabs D = dts[k];
        const uint32_t s = (uint32_t)(g - ufl32(segbase[rep]));
        seg_decode<SMALL>(payload, total, offs, rep, s, D.E, D.d, D.tabs, D.hh, tag, vers,
                          D.cells + (rep - D.rep0) * D.E, S, res + g, L, lane, cs);
    }
}

template <bool SMALL>
__global__ __launch_bounds__(64) void k_etf_read_chain_multi(const uint8_t* payload, u64 total,
                                                             const u64* offs, uint64_t R,
                                                             const uint32_t* segbase, uint32_t S,
                                                             const SegRes* res, int32_t* status,
                                                             const DecTabs* dts,
                                                             const uint32_t* pay_dt, int tag,
                                                             int vers) {
    __shared__ __attribute__((aligned(16))) ReadLds L;
    const uint32_t lane = threadIdx.x;
    const Cases cs = lane_cases(lane);
    for (uint64_t r = blockIdx.x; r < R; r += gridDim.x) {
        const uint32_t k = ufl32(pay_dt[r]);
        if ((dts[k].small != 0) != SMALL) continue;
        const u64 base = offs[r];
        const bool ok = chain_ok(payload, base, offs[r + 1] - base, segbase[r],
                                 segbase[r + 1] - segbase[r], S, res, lane);
        if (ok) {
            if (lane == 0) status[r] = LASPJ_DEC_OK;
            continue;
        }
        const DecTabs D = dts[k];
        const int32_t st = decode_replica<SMALL>(payload, total, offs, r, D.E, D.d, D.tabs,
                                                 D.hh_small, tag, vers,
                                                 D.cells + (r - D.rep0) * D.E, true, L, nullptr,
                                                 lane, cs);
        if (lane == 0) status[r] = st;
    }
}

template <bool SMALL>
__global__ __launch_bounds__(kBlock, SMALL ? 5 : 4) void k_orset_etf_read_multi(
    const uint8_t* payload, u64 total, const u64* offs, uint64_t R, const DecTabs* dts,
    const uint32_t* pay_dt, int tag, int vers, int32_t* status) {
    __shared__ __attribute__((aligned(16))) ReadLds lds[kBlock / 64];
    __shared__ __attribute__((aligned(16))) ReadLdsX ldx[SMALL ? 1 : kBlock / 64];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint64_t nwaves = (uint64_t)gridDim.x * (kBlock / 64);
    ReadLdsX* X = SMALL ? nullptr : &ldx[wave];
    const Cases cs = lane_cases(lane);
    ReadLds& L = lds[wave];
    for (uint64_t i = (uint64_t)blockIdx.x * (kBlock / 64) + wave; i < R; i += nwaves) {
        const uint32_t k = ufl32(pay_dt[i]);
        if ((dts[k].small != 0) != SMALL) continue;
        const DecTabs D = dts[k];
        const int32_t st = decode_replica<SMALL>(payload, total, offs, i, D.E, D.d, D.tabs,
                                                 D.hh_small, tag, vers,
                                                 D.cells + (i - D.rep0) * D.E, false, L, X, lane,
                                                 cs);
        if (lane == 0) status[i] = st;
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
    if (laspj::dev_malloc(ctx, &ctx->scratch, need) != hipSuccess) {
        hipGetLastError();
        return fail(ctx, LASPJ_E_NOMEM, "etf: scratch allocation of %llu bytes",
                    (unsigned long long)need);
    }
    ctx->scratch_bytes = need;
    return LASPJ_OK;
}

// ------------------------------------------------------------------ G-Set from_binary/1
// lasp_gset:from_binary/1 (lasp_gset.erl:122-128; riak_dt:from_binary = binary_to_term):
// <<Tag, Vers>> ++ the external term image of an ordset — [] (NIL_EXT), a LIST_EXT of
// element images with a NIL tail, or STRING_EXT when every element is an integer 0..255
// (term_to_binary's own choice).  One wave per payload: lane 0 checks the whole term is
// well-formed (binary_to_term fails first: MALFORMED wins over every later status) and
// lists element extents into LDS a chunk at a time; lanes then find each element's slot
// through the image hash, check ranks strictly ascend (an ordset) and set its bit.

__device__ __forceinline__ uint32_t be32(const uint8_t* p) {
    return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}

__device__ __host__ __forceinline__ uint32_t fnv1a(const uint8_t* p, uint32_t n) {
    uint32_t h = 2166136261u;
    for (uint32_t i = 0; i < n; ++i) h = (h ^ p[i]) * 16777619u;
    return h;
}

// extent of the external term at p within n bytes: its length; 0 when it runs past n or
// is not well-formed; kTermOther when it holds a tag no dictionary term has (pids, refs,
// funs, maps, bit strings, ...).  Terms are prefix-ordered, so one counter of pending
// sub-terms replaces a stack.
constexpr u64 kTermOther = ~0ull;

// well-formed UTF-8 (RFC 3629: no overlong forms, surrogates or code points past
// U+10FFFF) — binary_to_term/1 rejects ATOM_UTF8_EXT / SMALL_ATOM_UTF8_EXT names that
// are not
__device__ bool utf8_ok(const uint8_t* p, u64 n) {
    u64 i = 0;
    while (i < n) {
        const uint8_t c = p[i];
        if (c < 0x80) {
            ++i;
            continue;
        }
        uint32_t k;
        uint8_t lo = 0x80, hi = 0xBF;
        if (c >= 0xC2 && c <= 0xDF) k = 1;
        else if (c >= 0xE0 && c <= 0xEF) {
            k = 2;
            if (c == 0xE0) lo = 0xA0;
            if (c == 0xED) hi = 0x9F;
        } else if (c >= 0xF0 && c <= 0xF4) {
            k = 3;
            if (c == 0xF0) lo = 0x90;
            if (c == 0xF4) hi = 0x8F;
        } else {
            return false;
        }
        if (i + k >= n) return false;                 // continuation bytes run past n
        if (p[i + 1] < lo || p[i + 1] > hi) return false;
        for (uint32_t j = 2; j <= k; ++j)
            if (p[i + j] < 0x80 || p[i + j] > 0xBF) return false;
        i += 1 + k;
    }
    return true;
}

__device__ u64 etf_term_len(const uint8_t* p, u64 n) {
    u64 off = 0, pending = 1;
    while (pending) {
        if (off >= n) return 0;
        const uint8_t t = p[off];
        --pending;
        switch (t) {
        case 97: off += 2; break;                                   // SMALL_INTEGER
        case 98: off += 5; break;                                   // INTEGER
        case 70: off += 9; break;                                   // NEW_FLOAT
        case 99: off += 32; break;                                  // FLOAT
        case 106: off += 1; break;                                  // NIL
        case 100: case 118: case 107: {                             // ATOM(_UTF8), STRING
            if (off + 3 > n) return 0;
            const u64 len = (u64)p[off + 1] << 8 | p[off + 2];
            if (t == 118 && (off + 3 + len > n || !utf8_ok(p + off + 3, len))) return 0;
            off += 3 + len;
            break;
        }
        case 115: case 119: {                                       // SMALL_ATOM(_UTF8)
            if (off + 2 > n) return 0;
            const u64 len = p[off + 1];
            if (t == 119 && (off + 2 + len > n || !utf8_ok(p + off + 2, len))) return 0;
            off += 2 + len;
            break;
        }
        case 110:                                                   // SMALL_BIG
            if (off + 2 > n) return 0;
            off += 3 + (u64)p[off + 1];
            break;
        case 104:                                                   // SMALL_TUPLE
            if (off + 2 > n) return 0;
            pending += p[off + 1];
            off += 2;
            break;
        case 105:                                                   // LARGE_TUPLE
            if (off + 5 > n) return 0;
            pending += be32(p + off + 1);
            off += 5;
            break;
        case 108:                                                   // LIST: elements + tail
            if (off + 5 > n) return 0;
            pending += (u64)be32(p + off + 1) + 1;
            off += 5;
            break;
        case 109:                                                   // BINARY
            if (off + 5 > n) return 0;
            off += 5 + (u64)be32(p + off + 1);
            break;
        case 111:                                                   // LARGE_BIG
            if (off + 6 > n) return 0;
            off += 6 + (u64)be32(p + off + 1);
            break;
        default:
            return kTermOther;
        }
    }
    return off <= n ? off : 0;
}

struct GsTabs {
    const uint8_t* blob;
    const uint32_t* off;
    const uint32_t* htab;
    uint32_t hmask;
    const uint32_t* rank;
    const uint32_t* byte_slot;
    uint32_t E;
    const u64* itab;       // integer elements by value (see laspj_etf_dict::gs_itab)
    int64_t ilo;
    uint32_t in;
};


// the slot whose image is p[0, n), or kNoSlot
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;
__device__ __forceinline__ uint32_t gs_slot(const GsTabs& g, const uint8_t* p, uint32_t n) {
    for (uint32_t i = fnv1a(p, n) & g.hmask;; i = (i + 1) & g.hmask) {
        const uint32_t v = g.htab[i];
        if (!v) return kNoSlot;
        const uint32_t e = v - 1, o = g.off[e];
        if (g.off[e + 1] - o != n) continue;
        bool same = true;
        for (uint32_t k = 0; k < n && same; ++k) same = g.blob[o + k] == p[k];
        if (same) return e;
    }
}

// slot and rank of the element image p[0, n): integers through the value table (an image
// that is not the minimal encoding of its value is no dictionary image: not found, as in
// the hash), every other term through the image hash
__device__ __forceinline__ void gs_lookup(const GsTabs& g, const uint8_t* p, uint32_t n,
                                          uint32_t* slot, uint32_t* rk) {
    if (g.itab && (n == 2 || n == 5) && (p[0] == 97 || p[0] == 98)) {
        bool ok = false;
        int64_t v = 0;
        if (n == 2 && p[0] == 97) {
            v = p[1];
            ok = true;
        } else if (n == 5 && p[0] == 98) {
            v = (int32_t)((uint32_t)p[1] << 24 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 8 | p[4]);
            ok = v < 0 || v > 255;
        }
        if (ok) {
            const int64_t x = v - g.ilo;
            const u64 t = x >= 0 && x < (int64_t)g.in ? g.itab[x] : 0ull;
            *slot = (uint32_t)t ? (uint32_t)t - 1u : kNoSlot;
            *rk = (uint32_t)(t >> 32);
            return;
        }
    }
    *slot = gs_slot(g, p, n);
    *rk = *slot != kNoSlot ? g.rank[*slot] : 0;
}

constexpr uint32_t kGWin = 4096;          // LDS window over the payload (LIST_EXT walk)
constexpr uint32_t kGWords = 256;         // replicas of <= 256 words collect their bits in LDS

// extent of the element term at buf[o] within the window's bytes [0, lim) when its
// tag gives it directly (etf_term_len's rules for those tags); 0: not decidable here
__device__ __forceinline__ u64 gs_elem_len(const uint8_t* buf, uint32_t o, uint32_t lim) {
    const uint32_t t = buf[o];
    switch (t) {
    case 97: return 2;                                            // SMALL_INTEGER
    case 98: return 5;                                            // INTEGER
    case 70: return 9;                                            // NEW_FLOAT
    case 100:                                                     // ATOM_EXT (latin-1)
        return o + 3 <= lim ? 3u + ((uint32_t)buf[o + 1] << 8 | buf[o + 2]) : 0;
    case 115:                                                     // SMALL_ATOM_EXT
        return o + 2 <= lim ? 2u + buf[o + 1] : 0;
    case 110:                                                     // SMALL_BIG
        return o + 2 <= lim ? 3u + buf[o + 1] : 0;
    case 109:                                                     // BINARY
        return o + 5 <= lim ? 5ull + be32(buf + o + 1) : 0;
    default: return 0;                   // UTF-8 atoms, tuples, lists, ...: the general walk
    }
}

// a run's candidate test: with T0 (the run's tag when its images have a fixed length:
// SMALL_INTEGER_EXT 2, INTEGER_EXT 5, NEW_FLOAT_EXT 9 bytes) one byte compare, else the
// image sized by its header (gs_elem_len's branch tree costs ~100 instructions a lane; a
// candidate of another tag just ends the run early, the walk's next step takes it)
__device__ __forceinline__ bool gs_same_len(const uint8_t* buf, uint32_t q, uint32_t lim,
                                            uint32_t L0, uint32_t T0) {
    return T0 ? buf[q] == T0 : gs_elem_len(buf, q, lim) == L0;
}

__device__ __forceinline__ uint32_t gs_fixed_tag(uint32_t t) {
    return t == 97 || t == 98 || t == 70 ? t : 0u;
}

// One wave per replica.  LIST_EXT payloads are walked once: the payload is staged into
// LDS 4 KiB at a time, lane 0 finds the next <= CH element extents in the window
// (common tags by their headers, anything else by etf_term_len), then every lane takes
// ILP elements: dictionary slot by the integer table or by hash and exact compare (the
// table loads of all ILP elements in flight together), term order against the element
// before it, the bit set.  The statuses are those of the upfront whole-term validation
// this walk replaces: the first structural failure in stream order decides (truncation
// -> MALFORMED, a tag no dictionary term has -> UNKNOWN_TERM), then an improper tail or
// trailing bytes (MALFORMED), then an element outside the dictionary or out of order
// (UNKNOWN_TERM).
template <uint32_t CH, uint32_t ILP, bool KEEP, bool TAIL>
__global__ __launch_bounds__(64) void k_gset_etf_read(const uint8_t* payload, const u64* offs,
                                                      uint64_t R, GsTabs g, int tag, int vers,
                                                      u64* words, uint64_t W, int32_t* status) {
    __shared__ uint32_t s_o[CH], s_l[CH];
    __shared__ u64 s_h[4];
    __shared__ __attribute__((aligned(16))) uint8_t win[kGWin + 16];
    __shared__ u64 s_w[kGWords];
    const uint32_t lane = threadIdx.x;
    // the element bits: OR-ed into LDS and stored once per replica when the replica's
    // words fit (64 lanes setting bits of the same word would serialise on one global
    // atomic; every word is stored, so the batch needs no clearing first), else straight
    // into the (cleared) batch with global atomics
    const bool lw = W <= kGWords;
    for (uint64_t rep = blockIdx.x; rep < R; rep += gridDim.x) {
        const u64 ob = offs[rep], aend = offs[rep + 1];
        const uint8_t* p = payload + ob;
        const u64 n = aend - ob;
        u64* w = words + rep * W;
        if (lw)
            for (uint32_t x = lane; x < W; x += 64) s_w[x] = 0;
        // the LDS window [a0, a0 + wl) over the payload buffer: stage [at & ~15, + 4 KiB)
        // (absolute offsets stay 16-B aligned in the buffer: payload offsets are
        // arbitrary, so bytes go one by one into place through 16-byte loads of the
        // aligned span)
        u64 a0 = 0;
        uint32_t wl = 0;
        auto stage = [&](u64 at0) {
            a0 = at0 & ~15ull;
            wl = (uint32_t)min((u64)kGWin, aend - a0);
            const uint32_t nfull = wl >> 4;
            wave_copy16<2>(win, payload + a0, nfull, lane);
            for (uint32_t k = 16 * nfull + lane; k < wl; k += 64) win[k] = payload[a0 + k];
            __syncthreads();
        };
        // KEEP: the first window is staged at once and the header read from it (one
        // round trip instead of the header's dependent byte loads), and a window that
        // still holds the rest of the payload (or 2 KiB of it) is walked on, not restaged
        if (KEEP) stage(ob);
        const uint8_t* hp = KEEP ? win + (ob - a0) : p;
        if (lane == 0) {
            // s_h: {status, list tag, element count, first element offset}
            int st = LASPJ_DEC_OK;
            u64 h = 0;
            if (tag >= 0) {
                if (n < 2 || hp[0] != (uint8_t)tag) st = LASPJ_DEC_INVALID_BINARY;
                else if (hp[1] != (uint8_t)vers) st = LASPJ_DEC_UNSUPPORTED_VERSION;
                h = 2;
            }
            if (st == LASPJ_DEC_OK && (n < h + 2 || hp[h] != 131)) st = LASPJ_DEC_MALFORMED;
            u64 lt = 0, cnt = 0, first = 0;
            if (st == LASPJ_DEC_OK) {
                lt = hp[h + 1];
                if (lt == 108) {
                    // validated by the element walk below (one pass over the payload)
                    if (n - h - 1 < 5) st = LASPJ_DEC_MALFORMED;
                    else cnt = be32(hp + h + 2), first = h + 6;
                } else {
                    const u64 L = etf_term_len(p + h + 1, n - h - 1);
                    if (L == kTermOther) st = LASPJ_DEC_UNKNOWN_TERM;
                    else if (L == 0 || L != n - h - 1) st = LASPJ_DEC_MALFORMED;
                    else if (lt == 107) cnt = (u64)p[h + 2] << 8 | p[h + 3], first = h + 4;
                    else if (lt != 106) st = LASPJ_DEC_MALFORMED;      // not a list
                }
            }
            s_h[0] = (u64)st;
            s_h[1] = lt;
            s_h[2] = cnt;
            s_h[3] = first;
        }
        __syncthreads();
        int st = (int)s_h[0];
        const uint32_t lt = (uint32_t)s_h[1];
        const u64 cnt = s_h[2];
        u64 pos = s_h[3];
        bool unknown = false;
        uint32_t prev_rank = 0;
        bool have_prev = false;
        if (st == LASPJ_DEC_OK && lt == 107) {
            // STRING_EXT: every byte is the integer element of that value
            for (u64 c0 = 0; c0 < cnt; c0 += 64) {
                const u64 i = c0 + lane;
                uint32_t slot = kNoSlot, rk = 0;
                if (i < cnt) {
                    const uint32_t v = g.byte_slot[p[pos + i]];
                    slot = v ? v - 1 : kNoSlot;
                    rk = slot != kNoSlot ? g.rank[slot] : 0;
                }
                const uint32_t before = __shfl_up(rk, 1, 64);
                bool bad = i < cnt && (slot == kNoSlot ||
                                       (lane ? rk <= before : (have_prev && rk <= prev_rank)));
                if (i < cnt && !bad) {
                    if (lw) atomicOr(s_w + (slot >> 6), 1ull << (slot & 63));
                    else atomicOr(w + (slot >> 6), 1ull << (slot & 63));
                }
                unknown |= __ballot(bad) != 0;
                const uint32_t last = (uint32_t)((cnt - c0 < 64 ? cnt - c0 : 64) - 1);
                prev_rank = __shfl(rk, last, 64);
                have_prev = true;
            }
        } else if (st == LASPJ_DEC_OK && lt == 108) {
            u64 left = cnt;
            while (left > 0 && st == LASPJ_DEC_OK) {
                const u64 apos = ob + pos;
                if (!KEEP || !(apos >= a0 && apos <= a0 + wl &&
                               (aend <= a0 + wl || a0 + wl - apos >= 2048)))
                    stage(apos);
                const uint32_t base = (uint32_t)(apos - a0);                // pos in win
                {
                    // element extents inside the window, the whole wave walking together:
                    // lanes test whether the next 64 elements all have the length L0 of the
                    // one before (lane k: the element at o + k L0 has that length -- true
                    // for all k below the first failure, element by element), a run of
                    // equal-length images (small integers, then larger ones) at once;
                    // otherwise one element from its header, or the general walk (global
                    // bytes) for other tags and for an element the window does not hold
                    const uint32_t mx = (uint32_t)min(left, (u64)CH);
                    uint32_t k = 0, o = base, L0 = 0, T0 = 0;
                    int est = LASPJ_DEC_OK;
                    while (k < mx) {
                        const u64 rel = pos + (o - base);                  // payload offset
                        if (rel >= n) { est = LASPJ_DEC_MALFORMED; break; }
                        uint32_t run = 0;
                        // (gs_elem_len bounds its own reads: TAIL takes elements up to the
                        // window's last byte, so a payload's last elements, which sit
                        // within 16 bytes of its end, need no restage each)
                        if (L0) {
                            const uint32_t q = o + lane * L0;
                            const bool ok = lane < mx - k &&
                                            (TAIL ? q + L0 <= wl : q + 16 <= wl) &&
                                            gs_same_len(win, q, wl, L0, T0) &&
                                            rel + (u64)(lane + 1) * L0 <= n;
                            const u64 msk = __ballot(ok);
                            run = ~msk ? (uint32_t)__ffsll((long long)~msk) - 1u : 64u;
                        }
                        if (run) {
                            if (lane < run) {
                                s_o[k + lane] = (uint32_t)(rel + (u64)lane * L0);
                                s_l[k + lane] = L0;
                            }
                            o += run * L0;
                            k += run;
                            continue;
                        }
                        u64 L = (TAIL ? o < wl : o + 16 <= wl) ? gs_elem_len(win, o, wl) : 0;
                        L0 = (L && o + L <= wl && L <= 64) ? (uint32_t)L : 0u;
                        T0 = L0 ? gs_fixed_tag(win[o]) : 0u;
                        if (L == 0 || o + L > wl) {
                            // a tag the window cannot size (or a window that ends at the
                            // payload's end): the general walk over global bytes
                            if (o + 16 <= wl || k == 0 || (TAIL && a0 + wl >= aend)) {
                                L = etf_term_len(p + rel, n - rel);
                                if (L == kTermOther) { est = LASPJ_DEC_UNKNOWN_TERM; break; }
                                if (L == 0) { est = LASPJ_DEC_MALFORMED; break; }
                            } else {
                                break;                     // restage at this element
                            }
                        }
                        if (rel + L > n) { est = LASPJ_DEC_MALFORMED; break; }
                        if (lane == 0) {
                            s_o[k] = (uint32_t)rel;
                            s_l[k] = L <= 0xFFFFFFull ? (uint32_t)L : 0xFFFFFFFFu;
                        }
                        o += (uint32_t)min(L, (u64)0x7FFFFFFF);
                        ++k;
                        if (o > wl) break;                 // the next element starts past it
                    }
                    if (lane == 0) {
                        s_h[0] = (u64)est;
                        s_h[2] = k;
                        s_h[3] = pos + (o - base);
                    }
                }
                __syncthreads();
                st = (int)s_h[0];
                const uint32_t m = (uint32_t)s_h[2];
                for (uint32_t k0 = 0; k0 < m; k0 += 64 * ILP) {
                    // every element's integer-table load first (gs_lookup's integer case),
                    // then the hash probes of the rest, then the order checks in sequence
                    uint32_t slot[ILP], rk[ILP];
                    u64 t[ILP];
                    uint32_t how[ILP];             // 0 nothing, 1 integer table, 2 hash
#pragma unroll
                    for (uint32_t j = 0; j < ILP; ++j) {
                        const uint32_t k = k0 + 64 * j + lane;
                        how[j] = 0;
                        t[j] = 0;
                        if (k < m && s_l[k] <= 0xFFFFFFu) {
                            const uint32_t o = (uint32_t)(offs[rep] + s_o[k] - a0), L = s_l[k];
                            const uint8_t* q = o + L <= wl ? win + o : p + s_o[k];
                            how[j] = 2;
                            if (g.itab && (L == 2 || L == 5) && (q[0] == 97 || q[0] == 98)) {
                                bool ok = false;
                                int64_t v = 0;
                                if (L == 2 && q[0] == 97) {
                                    v = q[1];
                                    ok = true;
                                } else if (L == 5 && q[0] == 98) {
                                    v = (int32_t)((uint32_t)q[1] << 24 | (uint32_t)q[2] << 16 |
                                                  (uint32_t)q[3] << 8 | q[4]);
                                    ok = v < 0 || v > 255;
                                }
                                if (ok) {
                                    how[j] = 1;
                                    const int64_t x = v - g.ilo;
                                    if (x >= 0 && x < (int64_t)g.in) t[j] = g.itab[x];
                                }
                            }
                        }
                    }
#pragma unroll
                    for (uint32_t j = 0; j < ILP; ++j) {
                        slot[j] = kNoSlot;
                        rk[j] = 0;
                        if (how[j] == 1) {
                            slot[j] = (uint32_t)t[j] ? (uint32_t)t[j] - 1u : kNoSlot;
                            rk[j] = (uint32_t)(t[j] >> 32);
                        } else if (how[j] == 2) {
                            const uint32_t k = k0 + 64 * j + lane;
                            const uint32_t o = (uint32_t)(offs[rep] + s_o[k] - a0), L = s_l[k];
                            gs_lookup(g, o + L <= wl ? win + o : p + s_o[k], L, &slot[j], &rk[j]);
                        }
                    }
#pragma unroll
                    for (uint32_t j = 0; j < ILP; ++j) {
                        const uint32_t c0 = k0 + 64 * j;
                        if (c0 >= m) break;
                        const bool valid = c0 + lane < m;
                        const uint32_t before = __shfl_up(rk[j], 1, 64);
                        const bool bad = valid && (slot[j] == kNoSlot ||
                                                   (lane ? rk[j] <= before
                                                         : (have_prev && rk[j] <= prev_rank)));
                        if (valid && !bad) {
                            if (lw) atomicOr(s_w + (slot[j] >> 6), 1ull << (slot[j] & 63));
                            else atomicOr(w + (slot[j] >> 6), 1ull << (slot[j] & 63));
                        }
                        unknown |= __ballot(bad) != 0;
                        const uint32_t last = (m - c0 < 64 ? m - c0 : 64) - 1;
                        prev_rank = __shfl(rk[j], last, 64);
                        have_prev = true;
                    }
                }
                left -= m;
                pos = s_h[3];
                __syncthreads();
            }
            if (st == LASPJ_DEC_OK) {
                // the tail: [] closing the list at the payload end (an improper tail, a
                // tag no term has, or bytes after it are what the whole-term check saw)
                if (pos >= n) {
                    st = LASPJ_DEC_MALFORMED;
                } else if (p[pos] != 106) {
                    const u64 L = etf_term_len(p + pos, n - pos);
                    st = L == kTermOther ? LASPJ_DEC_UNKNOWN_TERM : LASPJ_DEC_MALFORMED;
                } else if (pos + 1 != n) {
                    st = LASPJ_DEC_MALFORMED;
                }
            }
        }
        if (st == LASPJ_DEC_OK && unknown) st = LASPJ_DEC_UNKNOWN_TERM;
        if (lane == 0) status[rep] = st;
        __syncthreads();
        if (lw)
            for (uint32_t x = lane; x < W; x += 64) w[x] = s_w[x];
    }
}

// the G-Set decoder's form: 256-element chunks, one element per lane per round, the
// header read from the first window and windows kept while they hold the rest, the
// payload's tail taken from the window (LASPJ_TUNE_ETF_READ 11: the round-4 form, 12:
// that with the tail from the window, 13: 4 elements per lane, 14: 512-element chunks;
// profiles/r05_gset_read_forms.log.  Tried and dropped: the bits of a word run of lanes
// OR-ed together before one atomic, 0.389 -> 0.42 ms)
using GsRead = void (*)(const uint8_t*, const u64*, uint64_t, GsTabs, int, int, u64*, uint64_t,
                        int32_t*);
GsRead gset_reader(const laspj_ctx* ctx) {
    switch (ctx->tune_etf_read) {
    case 11: return k_gset_etf_read<256, 1, false, false>;
    case 12: return k_gset_etf_read<256, 1, false, true>;
    case 13: return k_gset_etf_read<256, 4, true, true>;
    case 14: return k_gset_etf_read<512, 1, true, true>;
    default: return k_gset_etf_read<256, 1, true, true>;
    }
}

// Split G-Set decoder (few long payloads: the NIF's merge operands, one 10k-element
// ordset each, which one wave resolving 64 elements per round decoded in ~300 us).
// Pass 1 (k_gset_read_walk): one block per payload walks the element extents only -- the
// header from the first window, runs of equal-length images 256 at a time in a 32 KiB LDS
// window (staged by the block's four waves at once), the general walk for other tags, the
// tail -- and writes every element's offset
// relative to its payload to eo[offs[r] + r + k] (entry n: the tail's), the element count
// to en[r] and the walk's status to status[r] (the structural statuses of
// k_gset_etf_read; a STRING_EXT payload, at most 65535 bytes, is decoded here whole).
// Pass 2 (k_gset_read_lookup): waves over the chip take 64 elements each: slot and rank by
// gs_lookup, strictly ascending ranks (lane 0 resolves the element before its chunk too),
// the bit set with a global atomic (the words are zero on entry); a failure turns an OK
// status into UNKNOWN_TERM.  Statuses and bits are k_gset_etf_read's.
constexpr uint32_t kGWinL = 32768;

__global__ __launch_bounds__(kBlock) void k_gset_read_walk(const uint8_t* payload, const u64* offs,
                                                       uint64_t R, GsTabs g, int tag, int vers,
                                                       u64* words, uint64_t W, int32_t* status,
                                                       uint32_t* eo, uint32_t* en) {
    __shared__ __attribute__((aligned(16))) uint8_t win[kGWinL + 16];
    __shared__ u64 s_h[4];
    // the block's four waves stage each window together (32 KiB in one round of loads);
    // all four then walk it alike (uniform control, the same ballots) and wave 0 stores
    const uint32_t lane = threadIdx.x & 63u;
    const bool w0 = threadIdx.x < 64;
    for (uint64_t rep = blockIdx.x; rep < R; rep += gridDim.x) {
        const u64 ob = offs[rep], aend = offs[rep + 1];
        const uint8_t* p = payload + ob;
        const u64 n = aend - ob;
        u64* w = words + rep * W;
        uint32_t* e = eo + ob + rep;
        u64 a0 = 0;
        uint32_t wl = 0;
        auto stage = [&](u64 at0) {
            a0 = at0 & ~15ull;
            wl = (uint32_t)min((u64)kGWinL, aend - a0);
            const uint32_t nfull = wl >> 4;
            __syncthreads();                 // every wave is done with the last window
            {
                u32x4* dv = reinterpret_cast<u32x4*>(win);
                const u32x4* sv = reinterpret_cast<const u32x4*>(payload + a0);
                for (uint32_t v0 = 0; v0 < nfull; v0 += 8 * kBlock) {
                    u32x4 t[8];
#pragma unroll
                    for (uint32_t j = 0; j < 8; ++j) {
                        const uint32_t v = v0 + j * kBlock + threadIdx.x;
                        if (v < nfull) t[j] = sv[v];
                    }
#pragma unroll
                    for (uint32_t j = 0; j < 8; ++j) {
                        const uint32_t v = v0 + j * kBlock + threadIdx.x;
                        if (v < nfull) dv[v] = t[j];
                    }
                }
            }
            for (uint32_t k = 16 * nfull + threadIdx.x; k < wl; k += kBlock) win[k] = payload[a0 + k];
            __syncthreads();
        };
        stage(ob);
        const uint8_t* hp = win + (ob - a0);
        if (threadIdx.x == 0) {
            int st = LASPJ_DEC_OK;
            u64 h = 0;
            if (tag >= 0) {
                if (n < 2 || hp[0] != (uint8_t)tag) st = LASPJ_DEC_INVALID_BINARY;
                else if (hp[1] != (uint8_t)vers) st = LASPJ_DEC_UNSUPPORTED_VERSION;
                h = 2;
            }
            if (st == LASPJ_DEC_OK && (n < h + 2 || hp[h] != 131)) st = LASPJ_DEC_MALFORMED;
            u64 lt = 0, cnt = 0, first = 0;
            if (st == LASPJ_DEC_OK) {
                lt = hp[h + 1];
                if (lt == 108) {
                    if (n - h - 1 < 5) st = LASPJ_DEC_MALFORMED;
                    else cnt = be32(hp + h + 2), first = h + 6;
                } else {
                    const u64 L = etf_term_len(p + h + 1, n - h - 1);
                    if (L == kTermOther) st = LASPJ_DEC_UNKNOWN_TERM;
                    else if (L == 0 || L != n - h - 1) st = LASPJ_DEC_MALFORMED;
                    else if (lt == 107) cnt = (u64)p[h + 2] << 8 | p[h + 3], first = h + 4;
                    else if (lt != 106) st = LASPJ_DEC_MALFORMED;
                }
            }
            s_h[0] = (u64)st;
            s_h[1] = lt;
            s_h[2] = cnt;
            s_h[3] = first;
        }
        __syncthreads();
        int st = (int)s_h[0];
        const uint32_t lt = (uint32_t)s_h[1];
        const u64 cnt = s_h[2];
        u64 pos = s_h[3];
        __syncthreads();
        u64 found = 0;
        if (st == LASPJ_DEC_OK && lt == 107) {
            // STRING_EXT: every byte is the integer element of that value
            bool unknown = false, have_prev = false;
            uint32_t prev_rank = 0;
            for (u64 c0 = 0; c0 < cnt; c0 += 64) {
                const u64 i = c0 + lane;
                uint32_t slot = kNoSlot, rk = 0;
                if (i < cnt) {
                    const uint32_t v = g.byte_slot[p[pos + i]];
                    slot = v ? v - 1 : kNoSlot;
                    rk = slot != kNoSlot ? g.rank[slot] : 0;
                }
                const uint32_t before = __shfl_up(rk, 1, 64);
                const bool bad = i < cnt && (slot == kNoSlot ||
                                             (lane ? rk <= before : (have_prev && rk <= prev_rank)));
                if (w0 && i < cnt && !bad) atomicOr(w + (slot >> 6), 1ull << (slot & 63));
                unknown |= __ballot(bad) != 0;
                const uint32_t last = (uint32_t)((cnt - c0 < 64 ? cnt - c0 : 64) - 1);
                prev_rank = __shfl(rk, last, 64);
                have_prev = true;
            }
            if (unknown) st = LASPJ_DEC_UNKNOWN_TERM;
        } else if (st == LASPJ_DEC_OK && lt == 108) {
            u64 left = cnt;
            while (left > 0 && st == LASPJ_DEC_OK) {
                const u64 apos = ob + pos;
                if (!(apos >= a0 && apos <= a0 + wl &&
                      (aend <= a0 + wl || a0 + wl - apos >= kGWinL / 2)))
                    stage(apos);
                uint32_t o = (uint32_t)(apos - a0), L0 = 0, T0 = 0;
                u64 k = 0;
                int est = LASPJ_DEC_OK;
                while (k < left) {
                    const u64 rel = a0 + o - ob;                   // payload offset
                    if (rel >= n) { est = LASPJ_DEC_MALFORMED; break; }
                    uint32_t run = 0;
                    if (L0) {
                        // candidate j * 64 + lane at o + (j * 64 + lane) L0: the run is the
                        // first candidate whose image is not L0 long
                        bool go = true;
#pragma unroll
                        for (uint32_t j = 0; j < 4; ++j) {
                            if (!go) break;
                            const uint32_t idx = j * 64 + lane, q = o + idx * L0;
                            const bool ok = idx < left - k && q + L0 <= wl &&
                                            gs_same_len(win, q, wl, L0, T0) &&
                                            rel + (u64)(idx + 1) * L0 <= n;
                            const u64 msk = __ballot(ok);
                            const uint32_t r = ~msk ? (uint32_t)__ffsll((long long)~msk) - 1u : 64u;
                            run += r;
                            go = r == 64;
                        }
                    }
                    if (run) {
                        if (w0)
                            for (uint32_t idx = lane; idx < run; idx += 64)
                                e[found + k + idx] = (uint32_t)(rel + (u64)idx * L0);
                        o += run * L0;
                        k += run;
                        continue;
                    }
                    u64 L = o < wl ? gs_elem_len(win, o, wl) : 0;
                    L0 = (L && o + L <= wl && L <= 64) ? (uint32_t)L : 0u;
                    T0 = L0 ? gs_fixed_tag(win[o]) : 0u;
                    if (L == 0 || o + L > wl) {
                        if (o + 16 <= wl || k == 0 || a0 + wl >= aend) {
                            L = etf_term_len(p + rel, n - rel);
                            if (L == kTermOther) { est = LASPJ_DEC_UNKNOWN_TERM; break; }
                            if (L == 0) { est = LASPJ_DEC_MALFORMED; break; }
                        } else {
                            break;                     // restage at this element
                        }
                    }
                    if (rel + L > n) { est = LASPJ_DEC_MALFORMED; break; }
                    if (threadIdx.x == 0) e[found + k] = (uint32_t)rel;
                    o += (uint32_t)min(L, (u64)0x7FFFFFFF);
                    ++k;
                    if (o > wl) break;                 // the next element starts past it
                }
                found += k;
                left -= k;
                pos = a0 + o - ob;
                st = est;
            }
            if (st == LASPJ_DEC_OK) {
                if (pos >= n) {
                    st = LASPJ_DEC_MALFORMED;
                } else if (p[pos] != 106) {
                    const u64 L = etf_term_len(p + pos, n - pos);
                    st = L == kTermOther ? LASPJ_DEC_UNKNOWN_TERM : LASPJ_DEC_MALFORMED;
                } else if (pos + 1 != n) {
                    st = LASPJ_DEC_MALFORMED;
                }
            }
        }
        if (threadIdx.x == 0) {
            status[rep] = st;
            const bool list = st == LASPJ_DEC_OK && lt == 108;
            en[rep] = list ? (uint32_t)found : 0u;
            if (list) e[found] = (uint32_t)pos;
        }
        __syncthreads();
    }
}

// one wave resolves elements [64 c, 64 c + 64) of payload rep (k_gset_read_lookup)
__device__ __forceinline__ void gs_lookup_chunk(const uint8_t* payload, const u64* offs,
                                                const GsTabs& g, u64* words, uint64_t W,
                                                int32_t* status, const uint32_t* eo,
                                                const uint32_t* en, uint64_t rep, uint64_t c,
                                                uint32_t lane) {
    const uint32_t n = en[rep];
    const u64 ob = offs[rep];
    const uint8_t* p = payload + ob;
    const uint32_t* e = eo + ob + rep;
    u64* w = words + rep * W;
    const uint64_t k = c * 64 + lane;
    const bool valid = k < n;
    uint32_t slot = kNoSlot, rk = 0, prk = 0;
    if (valid) {
        const uint32_t o = e[k], L = e[k + 1] - o;
        if (L <= 0xFFFFFFu) gs_lookup(g, p + o, L, &slot, &rk);
    }
    const bool have_prev = lane == 0 && k > 0;
    if (have_prev) {
        const uint32_t o = e[k - 1], L = e[k] - o;
        uint32_t ps = kNoSlot;
        if (L <= 0xFFFFFFu) gs_lookup(g, p + o, L, &ps, &prk);
    }
    const uint32_t before = __shfl_up(rk, 1, 64);
    const bool bad = valid && (slot == kNoSlot ||
                               (lane ? rk <= before : (have_prev && rk <= prk)));
    if (valid && !bad) atomicOr(w + (slot >> 6), 1ull << (slot & 63));
    if (__ballot(bad) && lane == 0)
        atomicCAS(status + rep, (int32_t)LASPJ_DEC_OK, (int32_t)LASPJ_DEC_UNKNOWN_TERM);
}

__global__ __launch_bounds__(kBlock) void k_gset_read_lookup(const uint8_t* payload,
                                                             const u64* offs, uint64_t R, GsTabs g,
                                                             u64* words, uint64_t W,
                                                             int32_t* status, const uint32_t* eo,
                                                             const uint32_t* en) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t wave = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const uint64_t nwaves = (uint64_t)gridDim.x * (kBlock / 64);
    // chunks of 64 elements numbered across the payloads, 64 payloads at a time (lane r's
    // inclusive sum of their chunk counts), so no wave resolves payloads one after another
    uint64_t cbase = 0;
    for (uint64_t r0 = 0; r0 < R; r0 += 64) {
        const uint64_t r = r0 + lane;
        uint64_t x = r < R ? (en[r] + 63ull) / 64ull : 0ull;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint64_t y = __shfl_up(x, off, 64);
            if ((int)lane >= off) x += y;
        }
        const uint64_t upto = cbase + __shfl(x, 63, 64);
        // this wave's first chunk at or after cbase
        uint64_t c = cbase + (wave + nwaves - cbase % nwaves) % nwaves;
        for (; c < upto; c += nwaves) {
            const uint64_t rel = c - cbase;
            const uint32_t lr = (uint32_t)__ffsll((long long)__ballot(x > rel)) - 1u;
            const uint64_t first = __shfl(x, lr ? lr - 1 : 0, 64);
            gs_lookup_chunk(payload, offs, g, words, W, status, eo, en, r0 + lr,
                            rel - (lr ? first : 0ull), lane);
        }
        cbase = upto;
    }
}

// ------------------------------------------------------------------ exclusive scans
// out[i] = in[0] + ... + in[i-1] for i <= n (out[n] = the total): the payload offsets from
// the per-replica sizes.  Up to kScanOne values one block walks tiles of 256 with a carry
// (one launch: the NIF path's few payloads); beyond, tile sums -> one-block scan of the
// sums -> tiles re-scanned with their carry.
constexpr uint64_t kScanTile = 4096;                  // 256 threads x 16 values
constexpr uint64_t kScanOne = 8192;

__global__ __launch_bounds__(kBlock) void k_scan_one(const u64* in, u64* out, uint64_t n) {
    __shared__ u64 lds4[kBlock / 64];
    u64 carry = 0;
    for (uint64_t t0 = 0; t0 < n; t0 += kBlock) {
        const uint64_t t = t0 + threadIdx.x;
        const u64 v = t < n ? in[t] : 0;
        u64 tot;
        const u64 ex = block_excl_scan64(v, lds4, &tot);
        if (t < n) out[t] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) out[n] = carry;
}

__global__ __launch_bounds__(kBlock) void k_scan_tile_sums(const u64* in, uint64_t n, u64* sums) {
    __shared__ u64 lds4[kBlock / 64];
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
    u64 v = 0;
    for (uint32_t k = 0; k < kScanTile / kBlock; ++k) {
        const uint64_t i = base + (uint64_t)k * kBlock + threadIdx.x;
        if (i < n) v += in[i];
    }
    u64 tot;
    block_excl_scan64(v, lds4, &tot);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kBlock) void k_scan_tiles(const u64* in, u64* out, uint64_t n,
                                                       const u64* carries) {
    __shared__ u64 lds4[kBlock / 64];
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
    u64 carry = carries[blockIdx.x];
    for (uint32_t k = 0; k < kScanTile / kBlock; ++k) {
        const uint64_t i = base + (uint64_t)k * kBlock + threadIdx.x;
        const u64 v = i < n ? in[i] : 0;
        u64 tot;
        const u64 ex = block_excl_scan64(v, lds4, &tot);
        if (i < n) out[i] = carry + ex;
        carry += tot;
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) out[n] = carry;
}

// bytes of device scratch launch_scan needs for n values
uint64_t scan_tmp_bytes(uint64_t n) {
    return n <= kScanOne ? 0 : 8ull * ((n + kScanTile - 1) / kScanTile + 1);
}

hipError_t launch_scan(laspj_ctx* ctx, const u64* in, u64* out, uint64_t n, u64* tmp) {
    if (n <= kScanOne) {
        hipLaunchKernelGGL(k_scan_one, dim3(1), dim3(kBlock), 0, ctx->stream, in, out, n);
        return hipGetLastError();
    }
    const uint64_t tiles = (n + kScanTile - 1) / kScanTile;
    hipLaunchKernelGGL(k_scan_tile_sums, dim3((unsigned)tiles), dim3(kBlock), 0, ctx->stream, in,
                       n, tmp);
    // the carries in place: tmp[0..tiles] := exclusive scan of the tile sums
    hipLaunchKernelGGL(k_scan_one, dim3(1), dim3(kBlock), 0, ctx->stream, tmp, tmp, tiles);
    hipLaunchKernelGGL(k_scan_tiles, dim3((unsigned)tiles), dim3(kBlock), 0, ctx->stream, in, out,
                       n, tmp);
    return hipGetLastError();
}

// few payloads in split mode: sizes from the chunk totals (k_etf_sizes_from_chunks) and
// their exclusive scan in one launch
__global__ __launch_bounds__(kBlock) void k_etf_offsets_from_chunks(const u64* coff, uint64_t R,
                                                                    uint32_t nch, uint32_t hdr,
                                                                    u64* offs) {
    __shared__ u64 lds4[kBlock / 64];
    u64 carry = 0;
    for (uint64_t t0 = 0; t0 < R; t0 += kBlock) {
        const uint64_t rep = t0 + threadIdx.x;
        u64 v = 0;
        if (rep < R) {
            const u64 t = coff[rep * (nch + 1ull) + nch];
            const u64 n = t / kChunkCnt, sum = t & (kChunkCnt - 1);
            v = hdr + 1u + (n ? 5u + sum + 1u : 1u);
        }
        u64 tot;
        const u64 ex = block_excl_scan64(v, lds4, &tot);
        if (rep < R) offs[rep] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) offs[R] = carry;
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
    const uint64_t R = b->replicas;
    LJ_HIP(ctx, hipMemsetAsync(ctx->flag, 0, 4, ctx->stream));
    if (int s = etf_size_enqueue(ctx, b, d, kind, tag, static_cast<u64*>(offsets->dev), ctx->flag,
                                 nullptr))
        return s;
    uint32_t flag = 0;
    const laspj::ReadPiece rp[2] = {{&flag, ctx->flag, 4},
                                    {total, static_cast<u64*>(offsets->dev) + R, 8}};
    LJ_HIP(ctx, laspj::readback(ctx, rp, 2));
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
    LJ_HIP(ctx, laspj::readback(ctx, &total, static_cast<u64*>(offsets->dev) + R, 8));
    if (out->bytes < total)
        return fail(ctx, LASPJ_E_RANGE, "%s: output holds %llu bytes, payloads need %llu", what,
                    (unsigned long long)out->bytes, (unsigned long long)total);
    return etf_write_enqueue(ctx, b, d, kind, tag, vers, static_cast<const u64*>(offsets->dev),
                             static_cast<uint8_t*>(out->dev), out->bytes, nullptr);
}

int etf_read(laspj_ctx* ctx, laspj_batch* b, const laspj_etf_dict* d, int tag, int vers,
             const laspj_buf* payload, const laspj_buf* offsets, laspj_buf* status) {
    const char* what = "orset_etf_read";
    if (int s = check_args(ctx, b, d, LASPJ_KIND_ORSET, what)) return s;
    if (!d->rec_len)
        return fail(ctx, LASPJ_E_UNSUPPORTED, "%s: token images of different lengths", what);
    if (!payload || payload->ctx != ctx || !offsets || offsets->ctx != ctx || !status ||
        status->ctx != ctx)
        return fail(ctx, LASPJ_E_INVAL, "%s: bad buffer", what);
    if (offsets->bytes < 8ull * (b->replicas + 1) || status->bytes < 4ull * b->replicas)
        return fail(ctx, LASPJ_E_RANGE, "%s: offsets must hold R + 1 uint64, status R int32",
                    what);
    if (tag > 255 || vers < 0 || vers > 255)
        return fail(ctx, LASPJ_E_INVAL, "%s: tag and version are bytes", what);
    Guard g(ctx);
    const uint64_t R = b->replicas;
    std::vector<u64> off(R + 1);
    LJ_HIP(ctx, laspj::readback(ctx, off.data(), offsets->dev, 8ull * (R + 1)));
    for (uint64_t i = 0; i < R; ++i)
        if (off[i] > off[i + 1])
            return fail(ctx, LASPJ_E_RANGE, "%s: offsets decrease at replica %llu", what,
                        (unsigned long long)i);
    if (off[R] > payload->bytes)
        return fail(ctx, LASPJ_E_RANGE, "%s: offsets run past the payload buffer", what);
    EtfReadPlan plan;
    etf_read_plan(ctx, d, R, off.data(), &plan);
    return etf_read_enqueue(ctx, b, d, tag, vers, static_cast<const uint8_t*>(payload->dev),
                            payload->bytes, static_cast<const u64*>(offsets->dev), plan, nullptr,
                            static_cast<int32_t*>(status->dev), true, nullptr);
}

// few long G-Set payloads: the split decoder (knobs LASPJ_TUNE_ETF_READ 11..15: one wave
// per payload always)
static bool gset_read_split(const laspj_ctx* ctx, uint64_t R, const u64* off) {
    if ((ctx->tune_etf_read >= 11 && ctx->tune_etf_read <= 15) || R > (uint64_t)ctx->cus ||
        R == 0)
        return false;
    u64 longest = 0;
    for (uint64_t i = 0; i < R; ++i) longest = std::max<u64>(longest, off[i + 1] - off[i]);
    return longest >= 4096 && longest < (1ull << 31) && off[R] < (1ull << 40);
}

// pass 1 one wave per payload, pass 2 over the chip; the element offsets at the scratch's
// start (4 bytes per payload byte and per payload, + 4); the words are zero on entry
static int gset_read_split_enqueue(laspj_ctx* ctx, laspj_batch* b, const GsTabs& tabs, int tag,
                                   int vers, const uint8_t* payload, const u64* offs,
                                   u64 payload_end, int32_t* status) {
    const uint64_t R = b->replicas;
    const uint64_t eo_bytes = (4ull * (payload_end + R + 1) + 255ull) & ~255ull;
    if (int s = reserve_scratch(ctx, eo_bytes + 4ull * R)) return s;
    uint32_t* eo = static_cast<uint32_t*>(ctx->scratch);
    uint32_t* en = reinterpret_cast<uint32_t*>(static_cast<char*>(ctx->scratch) + eo_bytes);
    hipLaunchKernelGGL(k_gset_read_walk, dim3((unsigned)R), dim3(kBlock), 0, ctx->stream, payload,
                       offs, R, tabs, tag, vers, reinterpret_cast<u64*>(b->dev),
                       b->words_per_replica, status, eo, en);
    hipLaunchKernelGGL(k_gset_read_lookup, dim3((unsigned)ctx->cus * 2), dim3(kBlock), 0,
                       ctx->stream, payload, offs, R, tabs, reinterpret_cast<u64*>(b->dev),
                       b->words_per_replica, status, (const uint32_t*)eo, (const uint32_t*)en);
    LJ_LAUNCHED(ctx);
    return LASPJ_OK;
}

int gset_etf_read(laspj_ctx* ctx, laspj_batch* b, const laspj_etf_dict* d, int tag, int vers,
                  const laspj_buf* payload, const laspj_buf* offsets, laspj_buf* status) {
    const char* what = "gset_etf_read";
    if (int s = check_args(ctx, b, d, LASPJ_KIND_GSET, what)) return s;
    if (!payload || payload->ctx != ctx || !offsets || offsets->ctx != ctx || !status ||
        status->ctx != ctx)
        return fail(ctx, LASPJ_E_INVAL, "%s: bad buffer", what);
    if (offsets->bytes < 8ull * (b->replicas + 1) || status->bytes < 4ull * b->replicas)
        return fail(ctx, LASPJ_E_RANGE, "%s: offsets must hold R + 1 uint64, status R int32",
                    what);
    if (tag > 255 || vers < 0 || vers > 255)
        return fail(ctx, LASPJ_E_INVAL, "%s: tag and version are bytes", what);
    Guard g(ctx);
    const uint64_t R = b->replicas;
    std::vector<u64> off(R + 1);
    LJ_HIP(ctx, laspj::readback(ctx, off.data(), offsets->dev, 8ull * (R + 1)));
    for (uint64_t i = 0; i < R; ++i)
        if (off[i] > off[i + 1])
            return fail(ctx, LASPJ_E_RANGE, "%s: offsets decrease at replica %llu", what,
                        (unsigned long long)i);
    if (off[R] > payload->bytes)
        return fail(ctx, LASPJ_E_RANGE, "%s: offsets run past the payload buffer", what);
    if (!d->gs_htab)
        return fail(ctx, LASPJ_E_UNSUPPORTED, "gset read: a dictionary built without G-Set tables");
    const GsTabs tabs{d->elem_blob, d->elem_off, d->gs_htab, d->gs_hmask, d->gs_rank, d->gs_byte,
                      d->elements, reinterpret_cast<const u64*>(d->gs_itab), d->gs_ilo, d->gs_in};
    const uint64_t cap = (uint64_t)ctx->cus * 64;
    const uint8_t* pay = static_cast<const uint8_t*>(payload->dev);
    const u64* offs = static_cast<const u64*>(offsets->dev);
    if (gset_read_split(ctx, R, off.data())) {
        LJ_HIP(ctx, hipMemsetAsync(b->dev, 0, b->replicas * b->words_per_replica * 8ull,
                                   ctx->stream));
        return gset_read_split_enqueue(ctx, b, tabs, tag, vers, pay, offs, off[R],
                                       static_cast<int32_t*>(status->dev));
    }
    if (b->words_per_replica > kGWords)
        LJ_HIP(ctx, hipMemsetAsync(b->dev, 0, b->replicas * b->words_per_replica * 8ull,
                                   ctx->stream));
    // one wave per replica and a latency-bound extent walk: as many waves as LDS allows
    hipLaunchKernelGGL(gset_reader(ctx), dim3((unsigned)std::max<uint64_t>(1, std::min(R, cap))),
                       dim3(64), 0, ctx->stream, pay, offs, R, tabs, tag, vers,
                       reinterpret_cast<u64*>(b->dev), b->words_per_replica,
                       static_cast<int32_t*>(status->dev));
    LJ_LAUNCHED(ctx);
    return LASPJ_OK;
}

// lasp_core:bind/3 (lasp_core.erl:291-312) for n resident variables at once (the NIF's
// device-resident `#dv.value`, laspj_nif.hip): variable i's cells cur[i] and the decoded
// incoming value in[i] (wpr words each).  `case Value0 of Value` is word equality (the
// host dictionary holds one image per `==` class, so equal cells are equal terms);
// otherwise cur := merge(cur, in) — the slot-wise OR of two canonical orddicts / ordsets,
// which always inflates cur, so the reference writes it (:300-304).  WRITE (write/4,
// :839-844) replaces the cells instead.  A value whose decode failed leaves its variable
// untouched.  The decode status comes from dstat[i] or, with the chain check deferred
// here (cj.status set: the segment decoder ran without its chain launch), from
// chain_verdict, which every block of a variable evaluates for itself (deterministic, so
// all agree without a grid-wide wait; block 0 of the variable stores it in dstat[i]).
// in[] is left zero behind (the next call's decoders need clean cells).  The block that
// finishes last publishes per variable the status byte (0 no-op, 1 written) and the
// decode status into the pinned answer, and leaves the difference words and the ticket
// zero.
constexpr uint32_t kVarWords = 1024;     // words per block (4 per thread)
template <bool WRITE>
__global__ __launch_bounds__(kBlock) void k_var_bind(u64* const* __restrict__ curs,
                                                     u64* const* __restrict__ ins,
                                                     const uint64_t* __restrict__ wprs,
                                                     uint32_t nch, uint32_t n,
                                                     int32_t* __restrict__ dstat,
                                                     uint32_t* __restrict__ diff,
                                                     uint32_t* __restrict__ ticket,
                                                     uint8_t* __restrict__ out_res,
                                                     int32_t* __restrict__ out_st, ChainArgs cj) {
    __shared__ int32_t s_st;
    __shared__ bool s_last;
    const uint32_t i = blockIdx.x / nch, ch = blockIdx.x % nch;
    // (variables of different namespaces have different widths: the blocks past a
    // narrower one's words only take part in the ticket)
    u64* cur = curs[i];
    u64* src = ins[i];
    const uint64_t wpr = wprs[i];
    const uint64_t w0 = (uint64_t)ch * kVarWords;
    // both operands' words loaded first: they do not depend on the verdict, so their
    // loads overlap its dependent chain of loads (wave 0's)
    constexpr uint32_t kPer = kVarWords / kBlock;
    u64 av[kPer], bv[kPer];
#pragma unroll
    for (uint32_t t = 0; t < kPer; ++t) {
        const uint64_t w = w0 + threadIdx.x + t * kBlock;
        av[t] = bv[t] = 0;
        if (w < wpr) {
            bv[t] = src[w];
            av[t] = cur[w];
        }
    }
    if (cj.status) {
        if (threadIdx.x < 64) {
            const u64 base = cj.offs[i];
            const int32_t st = chain_verdict(cj.payload, base, cj.offs[i + 1] - base,
                                             cj.segbase[i], cj.segbase[i + 1] - cj.segbase[i],
                                             cj.S, cj.res, threadIdx.x);
            if (threadIdx.x == 0) {
                s_st = st;
                if (ch == 0) dstat[i] = st;
            }
            if (ch == 0) chain_publish(cj, i, st, threadIdx.x);
        }
    } else if (threadIdx.x == 0) {
        s_st = dstat[i];
    }
    __syncthreads();
    const bool ok = s_st == LASPJ_DEC_OK;
    u64 d = 0;
#pragma unroll
    for (uint32_t t = 0; t < kPer; ++t) {
        const uint64_t w = w0 + threadIdx.x + t * kBlock;
        if (w >= wpr || !ok) continue;
        // (an operand that did not decode keeps its cells: a redo pass of its failed
        // segments completes them, laspj_nif.hip)
        const u64 a = av[t], b = bv[t];
        d |= a ^ b;
        const u64 v = WRITE ? b : (a | b);
        if (v != a) cur[w] = v;
        if (b) src[w] = 0;
    }
    const bool any = __syncthreads_or(d != 0);
    if (threadIdx.x == 0) {
        if (any) atomicOr(diff + i, 1u);
        __threadfence();
        s_last = atomicAdd(ticket, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!s_last) return;
    __threadfence();
    for (uint32_t j = threadIdx.x; j < n; j += kBlock) {
        const uint32_t dj = atomicExch(diff + j, 0u);
        const int32_t st = __atomic_load_n(dstat + j, __ATOMIC_RELAXED);
        out_res[j] = st == LASPJ_DEC_OK ? (uint8_t)(dj ? 1 : 0) : (uint8_t)0;
        out_st[j] = st;
    }
    if (threadIdx.x == 0) *ticket = 0;
}

}  // namespace
}  // namespace laspj

// ------------------------------------------------------------------ enqueue-only forms
// (laspj_internal.h): the public entry points above validate, read back what they need and
// call these; the NIF-level entry points (laspj_nif.hip) call them directly with the
// offsets they staged themselves, so a whole decode -> join -> encode chain runs with one
// host synchronisation.
namespace laspj {

bool etf_dict_decodable(const laspj_etf_dict* d) { return d && d->rec_len != 0; }
bool etf_dict_bin_tokens(const laspj_etf_dict* d) { return d && d->bin_tokens; }
uint32_t etf_dict_tok_len(const laspj_etf_dict* d) { return d ? d->tok_uniform : 0; }
uint32_t etf_dict_elements(const laspj_etf_dict* d) { return d ? d->elements : 0; }

void etf_read_plan(const laspj_ctx* ctx, const laspj_etf_dict* d, uint64_t R, const u64* off,
                   EtfReadPlan* plan) {
    // Segment mode when there are too few payloads to fill the chip with one wave each
    // (fewer than 8 per CU) and they are long: segments of S bytes, S sized for ~48 waves
    // per CU (6 resident per SIMD, the rest queued behind them for balance), at least
    // 2 KiB.  Knob 4 splits every payload longer than 256 bytes into 256-byte segments
    // (what the tests use to stress the chain), 5 always splits with the sized S.
    plan->S = plan->nseg = 0;
    plan->segbase.clear();
    const bool batched = d->rd_desc && ctx->tune_etf_read != 1;
    if (!(batched && d->rd_htab && ctx->tune_etf_read != 3)) return;
    const uint64_t bytes_in = off[R] - off[0];
    const uint64_t want = (uint64_t)ctx->cus * 48;
    uint64_t longest = 0;
    for (uint64_t i = 0; i < R; ++i) longest = std::max<uint64_t>(longest, off[i + 1] - off[i]);
    uint64_t S = std::max<uint64_t>(2048, ((bytes_in / want) + 255) & ~255ull);
    if (ctx->tune_etf_read == 4) S = 256;
    if (ctx->tune_etf_seg) S = (uint64_t)ctx->tune_etf_seg;
    const bool split = (ctx->tune_etf_read >= 4 && ctx->tune_etf_read <= 6) ||
                       ctx->tune_etf_seg || R < (uint64_t)ctx->cus * 8;
    if (!(longest < (1ull << 31) && split && longest > S)) return;
    uint64_t acc = 0;
    plan->segbase.resize(R + 1);
    for (uint64_t i = 0; i < R; ++i) {
        plan->segbase[i] = (uint32_t)acc;
        acc += std::max<uint64_t>(1, (off[i + 1] - off[i] + S - 1) / S);
        if (acc >= (1ull << 32)) {
            plan->segbase.clear();
            return;
        }
    }
    plan->segbase[R] = (uint32_t)acc;
    plan->S = S;
    plan->nseg = acc;
}

int etf_read_enqueue(laspj_ctx* ctx, laspj_batch* b, const laspj_etf_dict* d, int tag, int vers,
                     const uint8_t* payload, uint64_t payload_bytes, const u64* offs,
                     const EtfReadPlan& plan, const uint32_t* segbase, int32_t* status,
                     bool clear, uint32_t* redo_zeroed, ChainJob* defer, const SegList* only,
                     const NewTokArgs* nt) {
    const uint64_t R = b->replicas;
    if (clear)
        LJ_HIP(ctx, hipMemsetAsync(b->dev, 0, b->replicas * b->words_per_replica * 8ull,
                                   ctx->stream));
    const bool batched = d->rd_desc && ctx->tune_etf_read != 1;
    auto kread = small_dict(d) && (ctx->tune_etf_read == 0 || ctx->tune_etf_read == 6 ||
                                              ctx->tune_etf_read >= 8)
                     ? k_orset_etf_read<true> : k_orset_etf_read<false>;
    ReadTabs tabs{static_cast<const uint4*>(d->rd_desc), d->rd_hdr, d->rd_tb, d->rd_ros};
    if (nt && nt->out && d->bin_tokens) tabs.nt = *nt;
    // the header hash (segment search; element batches without the scalar walk — knob 6
    // keeps the walking element batches)
    const HdrHash hh{d->rd_htab, d->rd_hmask, d->rd_hlens};
    // (knob 7: many-token dictionaries decode one element at a time)
    const HdrHash hh_small{ctx->tune_etf_read == 6 ? nullptr : d->rd_htab, d->rd_hmask,
                           d->rd_hlens, ctx->tune_etf_read == 7 ? 0u : 1u};
    if (plan.nseg) {
        const uint64_t nseg = plan.nseg;
        auto al = [](uint64_t x) { return (x + 255ull) & ~255ull; };
        const uint64_t o_res = al(4ull * (R + 1)), o_redo = o_res + al(sizeof(SegRes) * nseg);
        if (int s2 = reserve_scratch(ctx, o_redo + 4ull * (R + 1))) return s2;
        char* sc = static_cast<char*>(ctx->scratch);
        const uint32_t* dsegbase = segbase;
        if (!dsegbase) {
            uint32_t* up = reinterpret_cast<uint32_t*>(sc);
            LJ_HIP(ctx, hipMemcpyAsync(up, plan.segbase.data(), 4ull * (R + 1),
                                       hipMemcpyHostToDevice, ctx->stream));
            dsegbase = up;
        }
        static_assert(sizeof(SegRes) == kSegResBytes, "ChainJob::res sizing");
        const bool deferred = defer && defer->res;
        SegRes* dres = deferred ? static_cast<SegRes*>(defer->res)
                                : reinterpret_cast<SegRes*>(sc + o_res);
        const uint64_t sblocks = (nseg + 3) / 4, scap = (uint64_t)ctx->cus * 64;
        const bool small = small_dict(d) && ctx->tune_etf_read != 2;
        hipLaunchKernelGGL(small ? k_orset_etf_read_seg<true> : k_orset_etf_read_seg<false>,
                           dim3((unsigned)std::min(sblocks, scap)), dim3(kBlock), 0, ctx->stream,
                           payload, (u64)payload_bytes, offs, R, b->elements, view(d), tabs, tag,
                           vers, reinterpret_cast<u64x2*>(b->dev), dsegbase, nseg,
                           (uint32_t)plan.S, hh, dres, only ? *only : SegList{});
        LJ_LAUNCHED(ctx);
        if (deferred) {
            defer->payload = payload;
            defer->offs = offs;
            defer->segbase = dsegbase;
            defer->status = status;
            defer->nrep = (uint32_t)R;
            defer->S = (uint32_t)plan.S;
            defer->armed = true;
            return LASPJ_OK;
        }
        // the chain check, whose wave decodes a failed replica again itself (knob 10: the
        // redo list and a launch of the wave decoder over it, as before)
        const bool inline_redo = ctx->tune_etf_read != 10;
        uint32_t* redo = redo_zeroed;
        if (!redo && !inline_redo) {
            redo = reinterpret_cast<uint32_t*>(sc + o_redo);
            LJ_HIP(ctx, hipMemsetAsync(redo, 0, 4, ctx->stream));
        }
        const bool csmall = small_dict(d) &&
                            (ctx->tune_etf_read == 0 || ctx->tune_etf_read == 6 ||
                             ctx->tune_etf_read >= 8);
        hipLaunchKernelGGL(csmall ? k_etf_read_chain<true> : k_etf_read_chain<false>,
                           dim3((unsigned)std::min<uint64_t>(R, (uint64_t)ctx->cus * 32)), dim3(64), 0,
                           ctx->stream, payload, (u64)payload_bytes, offs, R, dsegbase,
                           (uint32_t)plan.S, dres, status, redo, b->elements, view(d), tabs,
                           hh_small, tag, vers,
                           inline_redo ? reinterpret_cast<u64x2*>(b->dev) : (u64x2*)nullptr);
        LJ_LAUNCHED(ctx);
        if (inline_redo) return LASPJ_OK;
        // the redo pass: usually an empty list (the kernel exits at once)
        const uint64_t rblocks = (R + 3) / 4, rcap = (uint64_t)ctx->cus * 4;
        hipLaunchKernelGGL(kread, dim3((unsigned)std::min(rblocks, rcap)), dim3(kBlock), 0,
                           ctx->stream, payload, (u64)payload_bytes, offs, R, b->elements,
                           view(d), tabs, hh_small, tag, vers, reinterpret_cast<u64x2*>(b->dev),
                           status, (const uint32_t*)redo);
        LJ_LAUNCHED(ctx);
        return LASPJ_OK;
    }
    // one replica per wave up to 64 blocks per CU: short blocks keep every CU busy to the
    // end (a grid-stride over a few resident waves left a 20 % tail at 65536 replicas)
    uint64_t blocks = (R + 3) / 4, cap = (uint64_t)ctx->cus * 64;
    const int grid = (int)(blocks < cap ? (blocks ? blocks : 1) : cap);
    if (batched)
        // 0: element batches when elements hold <= 8 token slots; 2: records batched only
        hipLaunchKernelGGL(kread, dim3(grid), dim3(kBlock), 0, ctx->stream, payload,
                           (u64)payload_bytes, offs, R, b->elements, view(d), tabs, hh_small, tag,
                           vers, reinterpret_cast<u64x2*>(b->dev), status,
                           (const uint32_t*)nullptr);
    else
        hipLaunchKernelGGL(k_orset_etf_read_serial, dim3(grid), dim3(kBlock), 0, ctx->stream,
                           payload, (u64)payload_bytes, offs, R, b->elements, view(d), tag, vers,
                           reinterpret_cast<u64x2*>(b->dev), status);
    LJ_LAUNCHED(ctx);
    return LASPJ_OK;
}

uint64_t etf_multi_bytes(uint32_t ngroups, uint32_t npay) {
    return ((sizeof(DecTabs) * ngroups + 15ull) & ~15ull) + 4ull * npay;
}

bool etf_multi_fill(const laspj_ctx* ctx, const EtfGroup* g, uint32_t ngroups, uint32_t npay,
                    void* host) {
    // the default decoders only (knobs select one-dictionary forms), every dictionary with
    // the batched tables and the header hash (what segment mode needs)
    if (ctx->tune_etf_read != 0) return false;
    for (uint32_t k = 0; k < ngroups; ++k) {
        const laspj_etf_dict* d = g[k].d;
        if (!d || !d->rd_desc || !d->rd_htab || !d->rec_len) return false;
    }
    if (!host) return true;                       // (the check alone)
    auto* dt = static_cast<DecTabs*>(host);
    auto* pd = reinterpret_cast<uint32_t*>(static_cast<char*>(host) +
                                           ((sizeof(DecTabs) * ngroups + 15ull) & ~15ull));
    for (uint32_t k = 0; k < ngroups; ++k) {
        const laspj_etf_dict* d = g[k].d;
        DecTabs t;
        std::memset(&t, 0, sizeof(t));
        t.d = view(d);
        t.tabs = ReadTabs{static_cast<const uint4*>(d->rd_desc), d->rd_hdr, d->rd_tb, d->rd_ros};
        t.hh = HdrHash{d->rd_htab, d->rd_hmask, d->rd_hlens};
        t.hh_small = HdrHash{d->rd_htab, d->rd_hmask, d->rd_hlens, 1u};
        t.cells = reinterpret_cast<u64x2*>(g[k].cells);
        t.rep0 = g[k].p0;
        t.E = g[k].E;
        t.small = small_dict(d) ? 1u : 0u;
        std::memcpy(dt + k, &t, sizeof(t));
        for (uint32_t i = g[k].p0; i < g[k].p1 && i < npay; ++i) pd[i] = k;
    }
    return true;
}

int etf_read_multi_enqueue(laspj_ctx* ctx, const EtfGroup* g, uint32_t ngroups,
                           const void* dev_tabs, uint32_t npay, const uint8_t* payload,
                           uint64_t payload_bytes, const u64* offs, const EtfReadPlan& plan,
                           const uint32_t* segbase, int32_t* status, ChainJob* defer,
                           const SegList* only) {
    const DecTabs* dts = static_cast<const DecTabs*>(dev_tabs);
    const uint32_t* pd = reinterpret_cast<const uint32_t*>(
        static_cast<const char*>(dev_tabs) + ((sizeof(DecTabs) * ngroups + 15ull) & ~15ull));
    bool any[2] = {false, false};                 // [SMALL]
    for (uint32_t k = 0; k < ngroups; ++k) any[small_dict(g[k].d) ? 1 : 0] = true;
    const uint64_t R = npay;
    if (plan.nseg) {
        const uint64_t nseg = plan.nseg;
        const bool deferred = defer && defer->res;
        SegRes* dres;
        if (deferred) {
            dres = static_cast<SegRes*>(defer->res);
        } else {
            if (int s2 = reserve_scratch(ctx, sizeof(SegRes) * nseg)) return s2;
            dres = static_cast<SegRes*>(ctx->scratch);
        }
        const uint64_t sblocks = (nseg + 3) / 4, scap = (uint64_t)ctx->cus * 64;
        for (int sm = 1; sm >= 0; --sm) {
            if (!any[sm]) continue;
            hipLaunchKernelGGL(sm ? k_orset_etf_read_seg_multi<true> : k_orset_etf_read_seg_multi<false>,
                               dim3((unsigned)std::min(sblocks, scap)), dim3(kBlock), 0, ctx->stream,
                               payload, (u64)payload_bytes, offs, R, dts, pd, -1, 1, segbase, nseg,
                               (uint32_t)plan.S, dres, only ? *only : SegList{});
            LJ_LAUNCHED(ctx);
        }
        if (deferred) {
            defer->payload = payload;
            defer->offs = offs;
            defer->segbase = segbase;
            defer->status = status;
            defer->nrep = (uint32_t)R;
            defer->S = (uint32_t)plan.S;
            defer->armed = true;
            return LASPJ_OK;
        }
        for (int sm = 1; sm >= 0; --sm) {
            if (!any[sm]) continue;
            hipLaunchKernelGGL(sm ? k_etf_read_chain_multi<true> : k_etf_read_chain_multi<false>,
                               dim3((unsigned)std::min<uint64_t>(R, (uint64_t)ctx->cus * 32)),
                               dim3(64), 0, ctx->stream, payload, (u64)payload_bytes, offs, R,
                               segbase, (uint32_t)plan.S, dres, status, dts, pd, -1, 1);
            LJ_LAUNCHED(ctx);
        }
        return LASPJ_OK;
    }
    const uint64_t blocks = (R + 3) / 4, cap = (uint64_t)ctx->cus * 64;
    for (int sm = 1; sm >= 0; --sm) {
        if (!any[sm]) continue;
        hipLaunchKernelGGL(sm ? k_orset_etf_read_multi<true> : k_orset_etf_read_multi<false>,
                           dim3((unsigned)std::max<uint64_t>(1, std::min(blocks, cap))),
                           dim3(kBlock), 0, ctx->stream, payload, (u64)payload_bytes, offs, R, dts,
                           pd, -1, 1, status);
        LJ_LAUNCHED(ctx);
    }
    return LASPJ_OK;
}

int gset_read_enqueue(laspj_ctx* ctx, laspj_batch* b, const laspj_etf_dict* d, int tag, int vers,
                      const uint8_t* payload, const u64* offs, int32_t* status, bool clear,
                      const u64* hoffs) {
    const uint64_t R = b->replicas;
    if (!d->gs_htab)
        return fail(ctx, LASPJ_E_UNSUPPORTED, "gset read: a dictionary built without G-Set tables");
    const GsTabs tabs{d->elem_blob, d->elem_off, d->gs_htab, d->gs_hmask, d->gs_rank, d->gs_byte,
                      d->elements, reinterpret_cast<const u64*>(d->gs_itab), d->gs_ilo, d->gs_in};
    if (hoffs && gset_read_split(ctx, R, hoffs)) {
        if (clear)
            LJ_HIP(ctx, hipMemsetAsync(b->dev, 0, R * b->words_per_replica * 8ull, ctx->stream));
        return gset_read_split_enqueue(ctx, b, tabs, tag, vers, payload, offs, hoffs[R], status);
    }
    if (clear && b->words_per_replica > kGWords)
        LJ_HIP(ctx, hipMemsetAsync(b->dev, 0, R * b->words_per_replica * 8ull, ctx->stream));
    hipLaunchKernelGGL(gset_reader(ctx),
                       dim3((unsigned)std::max<uint64_t>(1, std::min(R, (uint64_t)ctx->cus * 64))),
                       dim3(64), 0, ctx->stream, payload, offs, R, tabs, tag, vers,
                       reinterpret_cast<u64*>(b->dev), b->words_per_replica, status);
    LJ_LAUNCHED(ctx);
    return LASPJ_OK;
}

// few long G-Set payloads: chunks of 256 term-order slots spread over the chip for the
// size pass and the writer (LASPJ_TUNE_ETF_KERNEL 6: one wave per payload always)
static bool gset_split(const laspj_ctx* ctx, uint64_t R, uint32_t E) {
    return ctx->tune_etf != 6 && R <= (uint64_t)ctx->cus && (E + kBlock - 1) / kBlock >= 4;
}

// the split G-Set size pass: chunk sums and their scan (with `offsets`: the payload
// offsets too); the chunk table at the scratch's start
static int gset_chunks_enqueue(laspj_ctx* ctx, const laspj_batch* b, const laspj_etf_dict* d,
                               uint32_t hdr, u64* offsets, uint32_t* flag, const u64** chunks,
                               int src = 0, const u64* words2 = nullptr,
                               const ChainJob* chain = nullptr) {
    const ChainArgs cj = chain_args(chain);
    const uint64_t R = b->replicas;
    const uint32_t nch = (b->elements + kBlock - 1) / kBlock;
    if (int s = reserve_scratch(ctx, 16ull * R * (nch + 1ull))) return s;
    u64x2* co = static_cast<u64x2*>(ctx->scratch);
    const uint64_t sg = std::min<uint64_t>(R * nch, (uint64_t)ctx->cus * 16);
    auto ks = src == 1 ? k_gset_chunk_sizes<1> : src == 2 ? k_gset_chunk_sizes<2>
                                                          : k_gset_chunk_sizes<0>;
    hipLaunchKernelGGL(ks, dim3((unsigned)sg), dim3(kBlock), 0, ctx->stream, (const u64*)b->dev,
                       words2, R, b->elements, (uint32_t)b->words_per_replica, view(d), nch, co,
                       flag, cj);
    hipLaunchKernelGGL(k_gset_chunk_scan, dim3(1), dim3(kBlock), 0, ctx->stream, co, R, nch, hdr,
                       offsets);
    LJ_LAUNCHED(ctx);
    *chunks = reinterpret_cast<const u64*>(co);
    return LASPJ_OK;
}

int etf_size_enqueue(laspj_ctx* ctx, const laspj_batch* b, const laspj_etf_dict* d, int32_t kind,
                     int tag, u64* offsets, uint32_t* flag, const u64** chunks) {
    const uint64_t R = b->replicas;
    const uint32_t nch = (b->elements + kBlock - 1) / kBlock;
    const uint32_t hdr = tag >= 0 ? 2u : 0u;
    if (kind == LASPJ_KIND_GSET && gset_split(ctx, R, b->elements)) {
        const u64* co = nullptr;
        if (int s = gset_chunks_enqueue(ctx, b, d, hdr, offsets, flag, &co)) return s;
        if (chunks) *chunks = co;
        return LASPJ_OK;
    }
    // few long OR-Set payloads: sizes from per-chunk sums spread over the chip (as the
    // writer's split mode) instead of one wave walking each payload
    const bool split = kind == LASPJ_KIND_ORSET && R <= (uint64_t)ctx->cus && nch >= 4;
    if (chunks) *chunks = nullptr;
    if (split) {
        if (int s = reserve_scratch(ctx, 8ull * R * (nch + 1ull))) return s;
        u64* co = static_cast<u64*>(ctx->scratch);
        const uint64_t sg = std::min<uint64_t>(R * nch, (uint64_t)ctx->cus * 16);
        hipLaunchKernelGGL(k_etf_chunk_sizes, dim3((unsigned)sg), dim3(kBlock), 0, ctx->stream,
                           reinterpret_cast<const u64x2*>(b->dev), R, b->elements, view(d), nch,
                           co, flag);
        hipLaunchKernelGGL(k_etf_chunk_scan, dim3((unsigned)std::min<uint64_t>(R, 65535)),
                           dim3(kBlock), 0, ctx->stream, co, R, nch);
        hipLaunchKernelGGL(k_etf_offsets_from_chunks, dim3(1), dim3(kBlock), 0, ctx->stream, co,
                           R, nch, hdr, offsets);
        LJ_LAUNCHED(ctx);
        if (chunks) *chunks = co;
        return LASPJ_OK;
    }
    const uint64_t sizes_bytes = (8ull * R + 255ull) & ~255ull;
    if (int s = reserve_scratch(ctx, sizes_bytes + scan_tmp_bytes(R))) return s;
    u64* sizes = static_cast<u64*>(ctx->scratch);
    u64* tmp = reinterpret_cast<u64*>(static_cast<char*>(ctx->scratch) + sizes_bytes);
    uint64_t blocks = (R + 3) / 4, cap = (uint64_t)ctx->cus * 16;
    int grid = (int)(blocks < cap ? (blocks ? blocks : 1) : cap);
    if (kind == LASPJ_KIND_ORSET)
        hipLaunchKernelGGL(k_orset_etf_size, dim3(grid), dim3(kBlock), 0, ctx->stream,
                           reinterpret_cast<const u64x2*>(b->dev), R, b->elements, view(d), hdr,
                           sizes, flag);
    else
        hipLaunchKernelGGL(k_gset_etf_size, dim3(grid), dim3(kBlock), 0, ctx->stream,
                           (const u64*)b->dev, R, b->elements,
                           (uint32_t)b->words_per_replica, view(d), hdr, sizes, flag);
    LJ_LAUNCHED(ctx);
    LJ_HIP(ctx, launch_scan(ctx, sizes, offsets, R, tmp));
    return LASPJ_OK;
}

bool etf_merge_fused(const laspj_ctx* ctx, uint64_t R, uint32_t E) {
    const uint32_t nch = (E + kBlock - 1) / kBlock;
    return R <= (uint64_t)ctx->cus && nch >= 4;      // etf_size_enqueue's split mode
}

int etf_merge_size_enqueue(laspj_ctx* ctx, uint64_t* a, uint64_t* b, const laspj_batch* z,
                           const laspj_etf_dict* d, int tag, u64* offsets, uint32_t* flag,
                           uint32_t* ticket, const u64** chunks, const ChainJob* chain) {
    const uint64_t R = z->replicas;
    const uint32_t nch = (z->elements + kBlock - 1) / kBlock;
    const uint32_t hdr = tag >= 0 ? 2u : 0u;
    if (int s = reserve_scratch(ctx, 8ull * R * (nch + 1ull))) return s;
    u64* co = static_cast<u64*>(ctx->scratch);
    const uint64_t sg = std::min<uint64_t>(R * nch, (uint64_t)ctx->cus * 16);
    // up to 4 replicas the last block scans them all (one launch); more go to the
    // per-replica scan kernel
    const bool one = R <= 4;
    const ChainArgs cj = chain_args(chain);
    const uint64_t cblocks = cj.status ? (cj.nrep + 3u) / 4u : 0u;
    hipLaunchKernelGGL(k_etf_join_chunk_sizes, dim3((unsigned)(sg + cblocks)), dim3(kBlock), 0,
                       ctx->stream, reinterpret_cast<u64x2*>(a), reinterpret_cast<u64x2*>(b),
                       reinterpret_cast<u64x2*>(z->dev), R, z->elements, view(d), nch, co, flag,
                       one ? ticket : nullptr, hdr, offsets, cj);
    if (!one)
        hipLaunchKernelGGL(k_etf_chunk_scan_offsets, dim3((unsigned)std::min<uint64_t>(R, 65535)),
                           dim3(kBlock), 0, ctx->stream, co, R, nch, hdr, offsets, ticket);
    LJ_LAUNCHED(ctx);
    *chunks = co;
    return LASPJ_OK;
}

bool etf_merge_write_one(const laspj_ctx* ctx, const laspj_etf_dict* d, uint64_t R, uint32_t E) {
    return R == 1 && etf_merge_fused(ctx, R, E) && d->rec_len && ctx->tune_etf == 0 &&
           E < (1u << 22);
}

int etf_merge_write_enqueue(laspj_ctx* ctx, uint64_t* a, uint64_t* b, uint32_t E,
                            const laspj_etf_dict* d, int tag, int vers, u64* offs_out,
                            uint8_t* out, uint64_t cap_bytes, u64* lbst, uint32_t* ticket,
                            const ChainJob* chain, const uint32_t* skip) {
    const uint32_t nch = (E + kBlock - 1) / kBlock;
    LBJoin lb{reinterpret_cast<u64x2*>(a), reinterpret_cast<u64x2*>(b), lbst, ticket, offs_out,
              chain_args(chain), skip};
    const uint32_t cblocks = lb.cj.status ? (lb.cj.nrep + 3u) / 4u : 0u;
    auto k = d->tok_max <= 8 ? k_orset_etf_write_rec<24576, true, true>
                             : k_orset_etf_write_rec<24576, false, true>;
    hipLaunchKernelGGL(k, dim3(nch + cblocks), dim3(kBlock), 0, ctx->stream, (const u64x2*)nullptr,
                       (uint64_t)1, E, view(d), tag, vers, (const u64*)nullptr, out,
                       (const u64*)nullptr, 1u, (u64)cap_bytes, lb);
    LJ_LAUNCHED(ctx);
    return LASPJ_OK;
}

int var_bind_enqueue(laspj_ctx* ctx, uint64_t* const* curs, uint64_t* const* ins,
                     const uint64_t* wprs, uint64_t maxw, uint32_t n, int32_t* dstat,
                     uint32_t* diff, uint32_t* ticket, uint8_t* out_res, int32_t* out_st,
                     bool write, const ChainJob* chain) {
    const uint32_t nch = (uint32_t)std::max<uint64_t>(1, (maxw + kVarWords - 1) / kVarWords);
    const ChainArgs cj = chain_args(chain);
    hipLaunchKernelGGL(write ? k_var_bind<true> : k_var_bind<false>, dim3(nch * n), dim3(kBlock),
                       0, ctx->stream, reinterpret_cast<u64* const*>(curs),
                       reinterpret_cast<u64* const*>(ins), wprs, nch, n, dstat, diff, ticket,
                       out_res, out_st, cj);
    LJ_LAUNCHED(ctx);
    return LASPJ_OK;
}

bool etf_value_direct(const laspj_ctx* ctx, uint64_t R, uint32_t E) {
    return gset_split(ctx, R, E) && ctx->tune_etf != 1;
}

// value/1 of an OR-Set batch as G-Set images, straight from its cells (no value bits in
// between): the split G-Set size pass and writer reading {p, r}; zero_cells: the cells are
// cleared behind the writer's reads
int etf_value_write_enqueue(laspj_ctx* ctx, const laspj_batch* cells, const laspj_etf_dict* d,
                            int tag, int vers, u64* offsets, uint32_t* flag, uint8_t* out,
                            uint64_t cap_bytes, bool zero_cells, const ChainJob* chain) {
    const uint64_t R = cells->replicas;
    const uint32_t hdr = tag >= 0 ? 2u : 0u;
    const u64* co = nullptr;
    if (int s = gset_chunks_enqueue(ctx, cells, d, hdr, offsets, flag, &co, 1, nullptr, chain))
        return s;
    const uint32_t nch = (cells->elements + kBlock - 1) / kBlock;
    auto kw = zero_cells ? k_gset_write_chunks<1, true> : k_gset_write_chunks<1, false>;
    hipLaunchKernelGGL(kw,
                       dim3((unsigned)std::min<uint64_t>(R * nch, (uint64_t)ctx->cus * 16)),
                       dim3(kBlock), 0, ctx->stream, (const u64*)cells->dev, (const u64*)nullptr,
                       R, cells->elements,
                       (uint32_t)cells->words_per_replica, view(d), tag, vers, offsets, out,
                       (u64)cap_bytes, reinterpret_cast<const u64x2*>(co), nch);
    LJ_LAUNCHED(ctx);
    return LASPJ_OK;
}

// lasp_gset:merge/2 of few long operand pairs written as images straight from both
// operands' bits (their OR, never stored): the split size pass and writer
int etf_gset_merge_write_enqueue(laspj_ctx* ctx, const laspj_batch* lhs, const laspj_batch* rhs,
                                 const laspj_etf_dict* d, int tag, int vers, u64* offsets,
                                 uint32_t* flag, uint8_t* out, uint64_t cap_bytes) {
    const uint64_t R = lhs->replicas;
    const uint32_t hdr = tag >= 0 ? 2u : 0u;
    const u64* co = nullptr;
    if (int s = gset_chunks_enqueue(ctx, lhs, d, hdr, offsets, flag, &co, 2,
                                    (const u64*)rhs->dev))
        return s;
    const uint32_t nch = (lhs->elements + kBlock - 1) / kBlock;
    hipLaunchKernelGGL((k_gset_write_chunks<2, false>),
                       dim3((unsigned)std::min<uint64_t>(R * nch, (uint64_t)ctx->cus * 16)),
                       dim3(kBlock), 0, ctx->stream, (const u64*)lhs->dev, (const u64*)rhs->dev,
                       R, lhs->elements, (uint32_t)lhs->words_per_replica, view(d), tag, vers,
                       offsets, out, (u64)cap_bytes, reinterpret_cast<const u64x2*>(co), nch);
    LJ_LAUNCHED(ctx);
    return LASPJ_OK;
}

int etf_write_enqueue(laspj_ctx* ctx, const laspj_batch* b, const laspj_etf_dict* d,
                      int32_t kind, int tag, int vers, const u64* offsets, uint8_t* out,
                      uint64_t cap_bytes, const u64* chunks) {
    const uint64_t R = b->replicas;
    uint64_t cap = (uint64_t)ctx->cus * 8;
    int grid = (int)(R < cap ? R : cap);
    if (kind == LASPJ_KIND_ORSET && d->rec_len && ctx->tune_etf != 1) {
        // 0: 24 KiB window (profiles/r01_suite_etf_windows.log), records staged by their
        // element's thread when elements hold <= 8 token slots, spread over lanes otherwise;
        // 2, 3: 16 / 20 KiB windows, 4: 24 KiB, always spread over lanes
        auto k = d->tok_max <= 8 ? k_orset_etf_write_rec<24576, true>
                                 : k_orset_etf_write_rec<24576, false>;
        if (ctx->tune_etf == 2) k = k_orset_etf_write_rec<16384, false>;
        if (ctx->tune_etf == 3) k = k_orset_etf_write_rec<20480, false>;
        if (ctx->tune_etf == 4) k = k_orset_etf_write_rec<24576, false>;
        if (ctx->tune_etf == 5) k = k_orset_etf_write_rec<24576, true>;
        // one resident wave of blocks, each with a contiguous run of replicas (the
        // occupancy query is asked once per kernel variant: it costs host microseconds the
        // NIF path's single-merge calls would pay every time)
        static std::atomic<int> occ_cache[4];       // <24K, EPAR>, <24K>, <16K>, <20K>
        int variant = d->tok_max <= 8 ? 0 : 1;
        if (ctx->tune_etf == 2) variant = 2;
        if (ctx->tune_etf == 3) variant = 3;
        if (ctx->tune_etf == 4) variant = 1;
        if (ctx->tune_etf == 5) variant = 0;
        int occ = occ_cache[variant].load(std::memory_order_relaxed);
        if (occ <= 0) {
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, kBlock, 0) != hipSuccess ||
                occ < 1) {
                hipGetLastError();
                occ = 4;
            }
            occ_cache[variant].store(occ, std::memory_order_relaxed);
        }
        const uint64_t resident = (uint64_t)ctx->cus * (uint64_t)occ;
        grid = (int)(R < resident ? R : resident);
        const uint32_t nch = (b->elements + kBlock - 1) / kBlock;
        const u64* coff = nullptr;
        uint32_t cper = 0;
        if (4 * R <= resident && nch >= 4) {
            // split mode: few long payloads, their chunks spread over blocks (the chunk
            // offsets come from the size pass when it ran in split mode too)
            cper = (uint32_t)std::max<uint64_t>(1, (R * nch + resident - 1) / resident);
            const uint64_t groups = (nch + cper - 1) / cper;
            if (chunks) {
                coff = chunks;
            } else {
                if (int s = reserve_scratch(ctx, 8ull * R * (nch + 1ull))) return s;
                u64* co = static_cast<u64*>(ctx->scratch);
                const uint64_t sg = std::min<uint64_t>(R * nch, (uint64_t)ctx->cus * 16);
                hipLaunchKernelGGL(k_etf_chunk_sizes, dim3((unsigned)sg), dim3(kBlock), 0,
                                   ctx->stream, reinterpret_cast<const u64x2*>(b->dev), R,
                                   b->elements, view(d), nch, co, (uint32_t*)nullptr);
                hipLaunchKernelGGL(k_etf_chunk_scan, dim3((unsigned)std::min<uint64_t>(R, 65535)),
                                   dim3(kBlock), 0, ctx->stream, co, R, nch);
                coff = co;
            }
            grid = (int)(R * groups);
        }
        hipLaunchKernelGGL(k, dim3(grid ? grid : 1), dim3(kBlock), 0, ctx->stream,
                           reinterpret_cast<const u64x2*>(b->dev), R, b->elements, view(d), tag,
                           vers, offsets, out, coff, cper, (u64)cap_bytes, LBJoin{});
    } else if (kind == LASPJ_KIND_ORSET && d->tok_max > 8)
        hipLaunchKernelGGL(k_orset_etf_write_wave, dim3(grid ? grid : 1), dim3(kBlock), 0,
                           ctx->stream, reinterpret_cast<const u64x2*>(b->dev), R, b->elements,
                           view(d), tag, vers, offsets, out, (u64)cap_bytes);
    else if (kind == LASPJ_KIND_ORSET)
        hipLaunchKernelGGL(k_orset_etf_write, dim3(grid ? grid : 1), dim3(kBlock), 0, ctx->stream,
                           reinterpret_cast<const u64x2*>(b->dev), R, b->elements, view(d), tag,
                           vers, offsets, out, (u64)cap_bytes);
    else if (gset_split(ctx, R, b->elements) && ctx->tune_etf != 1) {
        // the chunk table from the size pass (or computed here when the caller's size
        // pass ran apart: the public size / write pair)
        const u64* co = chunks;
        if (!co)
            if (int s = gset_chunks_enqueue(ctx, b, d, tag >= 0 ? 2u : 0u, nullptr, nullptr, &co))
                return s;
        const uint32_t nch = (b->elements + kBlock - 1) / kBlock;
        hipLaunchKernelGGL((k_gset_write_chunks<0, false>),
                           dim3((unsigned)std::min<uint64_t>(R * nch, (uint64_t)ctx->cus * 16)),
                           dim3(kBlock), 0, ctx->stream, (const u64*)b->dev, (const u64*)nullptr,
                           R, b->elements,
                           (uint32_t)b->words_per_replica, view(d), tag, vers, offsets, out,
                           (u64)cap_bytes, reinterpret_cast<const u64x2*>(co), nch);
    } else
        // LASPJ_TUNE_ETF_KERNEL 1: the block-per-payload staging writer
        hipLaunchKernelGGL(ctx->tune_etf == 1 ? k_gset_etf_write : k_gset_etf_write_wave,
                           dim3(ctx->tune_etf == 1 ? (grid ? grid : 1)
                                                   : (int)std::max<uint64_t>(1, std::min<uint64_t>(
                                                         (R + 3) / 4, (uint64_t)ctx->cus * 32))),
                           dim3(kBlock), 0, ctx->stream,
                           (const u64*)b->dev, R, b->elements, (uint32_t)b->words_per_replica,
                           view(d), tag, vers, offsets, out, (u64)cap_bytes);
    LJ_LAUNCHED(ctx);
    return LASPJ_OK;
}

}  // namespace laspj

using laspj::fail;

extern "C" {

// tok_headroom: build the per-element token tables for up to that many more tokens per
// element than the widest element has (at most 8 while that stays <= 8, at most 64), keep
// the host state etf_dict_patch needs and room for appended token images
static int etf_dict_create_body(laspj_ctx* ctx, uint32_t E, const uint8_t* elem_blob,
                                const uint32_t* elem_off, const uint32_t* elem_order,
                                const uint8_t* tok_blob, const uint32_t* tok_off,
                                const uint8_t* tok_order, uint32_t tok_headroom,
                                laspj_etf_dict** out, bool trusted = false) {
    // (trusted: arrays the library exported itself from its host dictionary, where offsets
    // ascend, the order is a permutation and token orders name exactly the used slots by
    // construction — those checks, passes over every slot, are left out)
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
    {
        std::vector<uint8_t> ranked(trusted ? 0 : E, 0);    // (the order must be a permutation)
        for (uint32_t e = 0; e < E; ++e) {
            if (!trusted &&
                (elem_off[e + 1] < elem_off[e] || elem_order[e] >= E || ranked[elem_order[e]]++))
                return fail(ctx, LASPJ_E_RANGE, "etf_dict_create: element offsets / order invalid");
            ebyte[e] = elem_off[e + 1] - elem_off[e] == 2 && elem_blob[elem_off[e]] == 97;
        }
    }
    uint32_t uniform = 0;
    bool mixed = false, binall = true;
    // 16-byte-aligned copies of every image (the write kernels load them 16 B at a time);
    // an empty token slot keeps offset ~0u (the patch's "no image" mark)
    auto pad16 = [](uint64_t x) { return (x + 15ull) & ~15ull; };
    std::vector<uint32_t> epoff(E), tpoff;
    uint64_t epad_n = 0, tpad_n = 0;
    if (toks) {
        uint32_t bad = 0;                             // (branch-free: it vectorises)
        for (uint64_t t = 0; !trusted && t < 64ull * E; ++t) bad |= tok_off[t + 1] < tok_off[t];
        if (bad) return fail(ctx, LASPJ_E_RANGE, "etf_dict_create: token offsets decrease");
        tpoff.assign(64ull * E, 0xFFFFFFFFu);
        for (uint32_t e = 0; e < E; ++e) {
            const uint32_t* to = tok_off + 64ull * e;
            if (to[64] == to[0]) continue;            // no tokens: the common case, one test
            uint64_t m = 0;
            for (uint32_t k = 0; k < 64 && to[k] != to[64]; ++k) {   // (to the last token)
                const uint32_t len = to[k + 1] - to[k];
                if (!len) continue;
                m |= 1ull << k;
                if (!uniform) uniform = len;
                else if (uniform != len) mixed = true;
                if (binall) binall = tok_is_binary(tok_blob + to[k], len);
                tpoff[64ull * e + k] = (uint32_t)tpad_n;
                tpad_n += pad16(len);
            }
            tmask[e] = m;
        }
        for (uint32_t e = 0; e < E && !trusted; ++e) {
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
    uint32_t big = 0;
    for (uint32_t e = 0; e < E; ++e) big += __builtin_popcountll(tmask[e]) > 8 ? 1u : 0u;
    const bool bin = toks && !mixed && uniform >= 5u && binall;
    const uint64_t eblob = elem_off[E];
    for (uint32_t e = 0; e < E; ++e) {
        epoff[e] = (uint32_t)epad_n;
        epad_n += pad16(elem_off[e + 1] - elem_off[e]);
    }
    epad_n += 48;                 // a 48-byte load past the last image stays inside
    tpad_n += 48;
    if (epad_n >= (1ull << 32) || tpad_n >= (1ull << 32))
        return fail(ctx, LASPJ_E_RANGE, "etf_dict_create: images exceed 4 GiB");
    std::vector<uint8_t> epad(epad_n, 0), tpad(tpad_n, 0);
    for (uint32_t e = 0; e < E; ++e)
        std::copy(elem_blob + elem_off[e], elem_blob + elem_off[e + 1], epad.begin() + epoff[e]);
    uint32_t tok_max = 0;
    for (uint32_t x = 0; x < E; ++x)
        tok_max = std::max(tok_max, (uint32_t)__builtin_popcountll(tmask[x]));
    // (past 8 the head-room grows with the count: a hot element re-added again and again —
    // add_elem never collects a token — then rebuilds the images every count / 2 adds, not
    // every tok_headroom)
    if (tok_headroom && toks)
        tok_max = tok_max <= 8 ? std::min(8u, tok_max + tok_headroom)
                               : std::min(64u, tok_max + std::max(tok_headroom, tok_max / 2));
    // the writer's descriptors by (element, term rank), tok_max per element (not 64: a
    // rebuild then builds and uploads what the elements hold)
    std::vector<uint64_t> tdesc(toks ? (uint64_t)tok_max * E : 0, 0xFFull);
    for (uint64_t e = 0; toks && e < E; ++e)
        for (uint32_t j = 0; j < tok_max; ++j) {
            const uint64_t k = tok_order[64ull * e + j];
            if (k >= 64) break;
            const uint64_t t = 64ull * e + k, L = tok_off[t + 1] - tok_off[t];
            tdesc[e * tok_max + j] =
                k | (std::min<uint64_t>(L, 0xFFFFFFull) << 8) | ((uint64_t)tpoff[t] << 32);
        }
    // room for token images appended by etf_dict_patch
    const uint64_t tpad_cap = tpad_n + (tok_headroom && toks ? std::max<uint64_t>(tpad_n / 4, 1ull << 16) : 0);
    // record templates (uniform token images only): 104 2 <image> per (element, term rank),
    // and 104 2 <elem image> 108 per element
    const uint32_t rec_len = (toks && !mixed && uniform && uniform + 2u <= 48u) ? uniform + 2u : 0u;
    const uint64_t rec_stride = pad16(rec_len);
    uint64_t ehdr_max = 0;
    std::vector<uint8_t> rpad, hpad;
    std::vector<uint32_t> hpoff;
    std::vector<uint8_t> rd;
    bool hashed = rec_len != 0;
    if (rec_len) {
        rpad.assign((uint64_t)E * tok_max * rec_stride + 48, 0);
        for (uint64_t e = 0; e < E; ++e)
            for (uint32_t j = 0; j < tok_max; ++j) {
                const uint8_t k = tok_order[64ull * e + j];
                if (k >= 64) break;
                const uint64_t t = 64ull * e + k;
                uint8_t* r = rpad.data() + (e * tok_max + j) * rec_stride;
                r[0] = 104;
                r[1] = 2;
                std::copy(tok_blob + tok_off[t], tok_blob + tok_off[t + 1], r + 2);
            }
        hpoff.resize(E);
        uint64_t hn = 0;
        for (uint32_t e = 0; e < E; ++e) {
            hpoff[e] = (uint32_t)hn;
            hn += pad16(elem_off[e + 1] - elem_off[e] + 3ull);
            ehdr_max = std::max<uint64_t>(ehdr_max, elem_off[e + 1] - elem_off[e] + 3ull);
        }
        if (hn + 48 >= (1ull << 32) || rpad.size() >= (1ull << 40))
            return fail(ctx, LASPJ_E_RANGE, "etf_dict_create: record templates too large");
        hpad.assign(hn + 48, 0);
        for (uint32_t e = 0; e < E; ++e) {
            uint8_t* h = hpad.data() + hpoff[e];
            h[0] = 104;
            h[1] = 2;
            std::copy(elem_blob + elem_off[e], elem_blob + elem_off[e + 1], h + 2);
            h[2 + elem_off[e + 1] - elem_off[e]] = 108;
        }
        // from_binary tables by element rank: per element a template word and shift
        // that put its tokens in distinct buckets (none found: serial decode)
        rd.assign(laspj::rd_bytes(E, tok_max), 0);
        uint32_t* desc = reinterpret_cast<uint32_t*>(rd.data());
        uint8_t* hdr = rd.data() + 16ull * E;
        uint16_t* tbk = reinterpret_cast<uint16_t*>(hdr + 64ull * E);
        uint8_t* ros = reinterpret_cast<uint8_t*>(tbk + (uint64_t)E * tok_max);
        std::memset(ros, 0xFF, 64ull * E);
        const uint32_t nwords = rec_len / 4;     // whole words of the template
        std::vector<uint32_t> keys;
        // (by slot, each slot's rank looked up: the slot-indexed sources read in order)
        std::vector<uint32_t> rank_of(E);
        for (uint32_t r = 0; r < E; ++r) rank_of[elem_order[r]] = r;
        for (uint32_t e = 0; e < E && hashed; ++e) {
            const uint64_t r = rank_of[e];
            const uint32_t hl = elem_off[e + 1] - elem_off[e] + 3u;
            uint32_t cnt = 0;
            while (cnt < tok_max && tok_order[64ull * e + cnt] < 64) ++cnt;
            desc[4 * r] = e;
            desc[4 * r + 1] = hl;
            desc[4 * r + 3] = cnt;
            std::copy(hpad.data() + hpoff[e], hpad.data() + hpoff[e] + std::min(hl, 64u),
                      hdr + 64 * r);
            for (uint32_t j = 0; j < cnt; ++j) ros[64 * r + tok_order[64ull * e + j]] = (uint8_t)j;
            if (cnt == 0) continue;
            bool placed = false;
            for (uint32_t wi = nwords; wi-- > 0 && !placed;) {
                keys.resize(cnt);
                uint32_t diff = 0;                // the bits where some token differs
                for (uint32_t j = 0; j < cnt; ++j) {
                    std::memcpy(&keys[j], rpad.data() + ((uint64_t)e * tok_max + j) * rec_stride +
                                               4 * wi, 4);
                    diff |= keys[j] ^ keys[0];
                }
                if (cnt > 1 && !diff) continue;     // one word for all: no window parts them
                for (uint32_t sh = 0; sh + 10 <= 32 && !placed; ++sh) {
                    // (a window without a differing bit puts every token in one bucket)
                    if (cnt > 1 && !((diff >> sh) & (laspj::kBuckets - 1u))) continue;
                    bool ok = true;
                    if (cnt <= 16) {
                        for (uint32_t j = 1; j < cnt && ok; ++j) {
                            const uint32_t bj = (keys[j] >> sh) & (laspj::kBuckets - 1u);
                            for (uint32_t i = 0; i < j && ok; ++i)
                                ok = ((keys[i] >> sh) & (laspj::kBuckets - 1u)) != bj;
                        }
                    } else {
                        uint64_t seen[laspj::kBuckets / 64] = {};
                        for (uint32_t j = 0; j < cnt && ok; ++j) {
                            const uint32_t bk = (keys[j] >> sh) & (laspj::kBuckets - 1u);
                            ok = !((seen[bk / 64] >> (bk % 64)) & 1ull);
                            seen[bk / 64] |= 1ull << (bk % 64);
                        }
                    }
                    if (!ok) continue;
                    placed = true;
                    desc[4 * r + 2] = wi | (sh << 8);
                    for (uint32_t j = 0; j < cnt; ++j)
                        tbk[r * tok_max + j] = (uint16_t)((keys[j] >> sh) & (laspj::kBuckets - 1u));
                }
            }
            if (!placed) {
                // no one 10-bit window tells this element's tokens apart (tokens that agree
                // everywhere but where others also agree): its records are matched against
                // each of its templates instead (kNoBuckets; rare, and only this element)
                desc[4 * r + 2] = laspj::kNoBuckets;
                for (uint32_t j = 0; j < cnt; ++j) tbk[r * tok_max + j] = 0xFFFFu;
            }
        }
        if (!hashed) rd.clear();
    }
    // segment mode: header template (<= 64 bytes) -> rank, hashed as the device hashes
    std::vector<uint32_t> htab;
    uint64_t hlens = 0;
    if (hashed) {
        uint64_t cap = 64;
        while (cap < 2ull * E) cap <<= 1;
        htab.assign(cap, 0);
        const uint8_t* hdr = rd.data() + 16ull * E;
        const uint32_t* desc = reinterpret_cast<const uint32_t*>(rd.data());
        for (uint64_t r = 0; r < E; ++r) {
            const uint32_t hl = desc[4 * r + 1];
            if (hl < 4 || hl > 64) continue;
            uint32_t h = hl * 0x85EBCA6Bu;
            for (uint32_t i = 0; 4 * i < hl; ++i) {         // ceil(hl / 4) words
                uint32_t v;
                std::memcpy(&v, hdr + 64 * r + 4 * i, 4);   // zero past hl
                h = laspj::hdr_mix(h, v);
            }
            uint64_t i = h & (cap - 1);
            while (htab[i]) i = (i + 1) & (cap - 1);
            htab[i] = (uint32_t)r + 1u;
            hlens |= 1ull << (hl - 1);
        }
    }
    for (uint64_t e = 0; toks && e < E; ++e)
        for (uint64_t m = tmask[e]; m; m &= m - 1) {          // the slots holding a token
            const uint64_t t = 64ull * e + __builtin_ctzll(m);
            std::copy(tok_blob + tok_off[t], tok_blob + tok_off[t + 1], tpad.begin() + tpoff[t]);
        }
    // G-Set from_binary tables: ranks (equal terms share one), image hash, byte values.
    // Not for the library's own OR-Set namespaces (trusted, with tokens): their payloads
    // are OR-Set images only, and the tables cost a term comparison per slot per rebuild
    const bool gs = !(trusted && toks);
    uint64_t gs_cap = 64;
    while (gs && gs_cap < 2ull * E) gs_cap <<= 1;
    auto al = [](uint64_t x) { return (x + 255ull) & ~255ull; };
    std::vector<uint32_t> gs_rank(gs ? E : 0, 0), gs_byte(256, 0), gs_htab;
    if (gs) {
        uint32_t rk = 0;
        for (uint32_t k = 0; k < E; ++k) {
            const uint32_t e = elem_order[k];
            if (k) {
                const uint32_t p = elem_order[k - 1];
                int c = 1;
                const bool both = elem_off[e + 1] > elem_off[e] && elem_off[p + 1] > elem_off[p];
                if (!both || laspj_term_compare(elem_blob + elem_off[p], elem_off[p + 1] - elem_off[p],
                                                elem_blob + elem_off[e], elem_off[e + 1] - elem_off[e],
                                                &c) != LASPJ_OK)
                    c = 1;
                if (c != 0) ++rk;
            }
            gs_rank[e] = rk;
        }
        const uint64_t cap = gs_cap;
        gs_htab.assign(cap, 0);
        for (uint32_t e = 0; e < E; ++e) {
            const uint32_t n = elem_off[e + 1] - elem_off[e];
            if (!n) continue;
            const uint8_t* img = elem_blob + elem_off[e];
            if (n == 2 && img[0] == 97 && !gs_byte[img[1]]) gs_byte[img[1]] = e + 1;
            uint64_t i = laspj::fnv1a(img, n) & (cap - 1);
            bool dup = false;
            while (gs_htab[i]) {
                const uint32_t o = gs_htab[i] - 1;
                if (elem_off[o + 1] - elem_off[o] == n &&
                    std::memcmp(elem_blob + elem_off[o], img, n) == 0)
                    dup = true;                  // an image twice: the first slot keeps it
                if (dup) break;
                i = (i + 1) & (cap - 1);
            }
            if (!dup) gs_htab[i] = e + 1;
        }
    }
    // integer elements by value (minimal images: SMALL_INTEGER for 0..255, INTEGER past it)
    std::vector<uint64_t> gs_itab;
    int64_t ilo = 0;
    if (gs) {
        int64_t lo = INT64_MAX, hi = INT64_MIN;
        uint64_t cnt = 0;
        auto int_of = [&](uint32_t e, int64_t* v) {
            const uint32_t n = elem_off[e + 1] - elem_off[e];
            const uint8_t* img = elem_blob + elem_off[e];
            if (n == 2 && img[0] == 97) {
                *v = img[1];
                return true;
            }
            if (n == 5 && img[0] == 98) {
                *v = (int32_t)((uint32_t)img[1] << 24 | (uint32_t)img[2] << 16 |
                               (uint32_t)img[3] << 8 | img[4]);
                return *v < 0 || *v > 255;
            }
            return false;
        };
        for (uint32_t e = 0; e < E; ++e) {
            int64_t v;
            if (int_of(e, &v)) lo = std::min(lo, v), hi = std::max(hi, v), ++cnt;
        }
        if (cnt && (uint64_t)(hi - lo) < std::max<uint64_t>(4 * cnt, 1ull << 16)) {
            ilo = lo;
            gs_itab.assign((uint64_t)(hi - lo) + 1, 0);
            for (uint32_t e = 0; e < E; ++e) {
                int64_t v;
                if (int_of(e, &v) && !gs_itab[v - lo])      // one value twice: the first slot
                    gs_itab[v - lo] = (e + 1ull) | ((uint64_t)gs_rank[e] << 32);
            }
        }
    }
    // on the device: the token offsets only for mixed image lengths (the size pass reads
    // them then); the token images themselves and their padded offsets never (the kernels
    // read the padded copies through tok_desc) — 64 E-slot arrays the NIF path's rebuilds
    // would otherwise stage and copy every time
    const bool dev_toff = toks && mixed;
    const uint64_t o_eoff = 0, o_eord = o_eoff + al(4ull * (E + 1)), o_eb = o_eord + al(4ull * E),
                   o_mask = o_eb + al(E), o_toff = o_mask + al(8ull * E),
                   o_tord = o_toff + (dev_toff ? al(4ull * (64ull * E + 1)) : 0),
                   o_eblob = o_tord + (toks ? al(64ull * E) : 0), o_tblob = o_eblob + al(eblob + 1),
                   o_epoff = o_tblob, o_tpoff = o_epoff + al(4ull * E),
                   o_epad = o_tpoff, o_tpad = o_epad + al(epad_n),
                   o_tdesc = o_tpad + al(tpad_cap), o_rpad = o_tdesc + al(8ull * tdesc.size() + 8),
                   o_hpad = o_rpad + al(rpad.size()), o_hpoff = o_hpad + al(hpad.size()),
                   o_rd = o_hpoff + al(4ull * hpoff.size() + 4),
                   o_htab = o_rd + al(rd.size() + 8), o_gsh = o_htab + al(4ull * htab.size() + 4),
                   o_gsr = o_gsh + al(4ull * gs_cap), o_gsb = o_gsr + al(4ull * (gs ? E : 0)),
                   o_gsi = o_gsb + al(4ull * (gs ? 256 : 0)), bytes = o_gsi + al(8ull * gs_itab.size() + 8);
    auto* d = new (std::nothrow) laspj_etf_dict;
    if (!d) return fail(ctx, LASPJ_E_NOMEM, "etf_dict_create: host allocation");
    std::lock_guard<std::mutex> lk(ctx->mu);
    hipSetDevice(ctx->device);
    // a block from the context's cache (a rebuilt dictionary of the same size class takes
    // the block its predecessor gave back: no hipMalloc / hipFree per rebuild)
    if (laspj::dev_alloc(ctx, bytes, &d->block) != hipSuccess) {
        hipGetLastError();
        delete d;
        return fail(ctx, LASPJ_E_NOMEM, "etf_dict_create: hipMalloc(%llu)", (unsigned long long)bytes);
    }
    d->block_bytes = bytes;
    char* base = static_cast<char*>(d->block);
    // every array staged into one pinned host image of the block (the context's, grow-only;
    // the previous image's copy has finished before it is rewritten), then one async copy
    hipStreamSynchronize(ctx->stream);
    if (ctx->dstage_bytes < bytes) {
        if (ctx->dstage) hipHostFree(ctx->dstage);
        ctx->dstage = nullptr;
        ctx->dstage_bytes = 0;
        const uint64_t want = std::max<uint64_t>(bytes, 1ull << 20) + bytes / 4;
        if (hipHostMalloc(&ctx->dstage, want, hipHostMallocDefault) != hipSuccess) {
            hipGetLastError();
            ctx->dstage = nullptr;
            laspj::dev_release(ctx, d->block, bytes);
            delete d;
            return fail(ctx, LASPJ_E_NOMEM, "etf_dict_create: pinned staging");
        }
        ctx->dstage_bytes = want;
    }
    char* img = static_cast<char*>(ctx->dstage);
    // the arrays, then zeros in the alignment gaps between them (nothing reads them; kept
    // deterministic) — no zero fill of the whole image first
    std::vector<std::pair<uint64_t, uint64_t>> spans;
    auto up = [&](uint64_t off, const void* src, uint64_t n) {
        if (n) std::memcpy(img + off, src, n);
        spans.emplace_back(off, n);
        return hipSuccess;
    };
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = up(o_eoff, elem_off, 4ull * (E + 1));
    if (e == hipSuccess) e = up(o_eord, elem_order, 4ull * E);
    if (e == hipSuccess) e = up(o_eb, ebyte.data(), E);
    if (e == hipSuccess) e = up(o_mask, tmask.data(), 8ull * E);
    if (e == hipSuccess && dev_toff) e = up(o_toff, tok_off, 4ull * (64ull * E + 1));
    if (e == hipSuccess && toks) e = up(o_tord, tok_order, 64ull * E);
    if (e == hipSuccess) e = up(o_eblob, elem_blob, eblob);

    if (e == hipSuccess) e = up(o_epoff, epoff.data(), 4ull * E);

    if (e == hipSuccess) e = up(o_epad, epad.data(), epad_n);
    if (e == hipSuccess && toks) e = up(o_tpad, tpad.data(), tpad_n);
    if (e == hipSuccess && toks) e = up(o_tdesc, tdesc.data(), 8ull * tdesc.size());
    if (e == hipSuccess && rec_len) e = up(o_rpad, rpad.data(), rpad.size());
    if (e == hipSuccess && rec_len) e = up(o_hpad, hpad.data(), hpad.size());
    if (e == hipSuccess && rec_len) e = up(o_hpoff, hpoff.data(), 4ull * hpoff.size());
    if (e == hipSuccess && hashed) e = up(o_rd, rd.data(), rd.size());
    if (e == hipSuccess && hashed) e = up(o_htab, htab.data(), 4ull * htab.size());
    if (e == hipSuccess && gs) e = up(o_gsh, gs_htab.data(), 4ull * gs_htab.size());
    if (e == hipSuccess && gs) e = up(o_gsr, gs_rank.data(), 4ull * E);
    if (e == hipSuccess && gs) e = up(o_gsb, gs_byte.data(), 4ull * 256);
    if (e == hipSuccess && !gs_itab.empty()) e = up(o_gsi, gs_itab.data(), 8ull * gs_itab.size());
    if (e == hipSuccess) {
        std::sort(spans.begin(), spans.end());
        uint64_t at = 0;
        for (const auto& sp : spans) {
            if (sp.first > at) std::memset(img + at, 0, sp.first - at);
            at = std::max(at, sp.first + sp.second);
        }
        if (bytes > at) std::memset(img + at, 0, bytes - at);
        e = hipMemcpyAsync(base, img, bytes, hipMemcpyHostToDevice, ctx->stream);
    }
    if (e != hipSuccess) {
        laspj::dev_release(ctx, d->block, bytes);
        delete d;
        return fail(ctx, LASPJ_E_DEVICE, "etf_dict_create: upload: %s", hipGetErrorString(e));
    }
    d->ctx = ctx;
    d->elements = E;
    d->has_tokens = toks;
    d->tok_uniform = mixed ? 0u : uniform;
    d->tok_max = tok_max;
    d->rec_len = rec_len;
    d->bin_tokens = bin && rec_len != 0;
    d->big_elems = big;
    d->ehdr_max = (uint32_t)std::min<uint64_t>(ehdr_max, 0xFFFFFFFFull);
    d->rec_stride = (uint32_t)rec_stride;
    d->rec_pad = rec_len ? reinterpret_cast<const uint8_t*>(base + o_rpad) : nullptr;
    d->ehdr_pad = rec_len ? reinterpret_cast<const uint8_t*>(base + o_hpad) : nullptr;
    d->ehdr_poff = rec_len ? reinterpret_cast<const uint32_t*>(base + o_hpoff) : nullptr;
    if (hashed) {
        const uint8_t* t = reinterpret_cast<const uint8_t*>(base + o_rd);
        d->rd_desc = t;
        d->rd_hdr = t + 16ull * E;
        d->rd_tb = reinterpret_cast<const uint16_t*>(t + 16ull * E + 64ull * E);
        d->rd_ros = reinterpret_cast<const uint8_t*>(d->rd_tb + (uint64_t)E * tok_max);
        d->rd_htab = reinterpret_cast<const uint32_t*>(base + o_htab);
        d->rd_hmask = (uint32_t)(htab.size() - 1);
        d->rd_hlens = hlens;
    }
    d->gs_htab = gs ? reinterpret_cast<const uint32_t*>(base + o_gsh) : nullptr;
    d->gs_hmask = (uint32_t)(gs_cap - 1);
    d->gs_rank = gs ? reinterpret_cast<const uint32_t*>(base + o_gsr) : nullptr;
    d->gs_byte = gs ? reinterpret_cast<const uint32_t*>(base + o_gsb) : nullptr;
    d->gs_itab = gs_itab.empty() ? nullptr : reinterpret_cast<const uint64_t*>(base + o_gsi);
    d->gs_ilo = ilo;
    d->gs_in = (uint32_t)gs_itab.size();
    d->elem_off = reinterpret_cast<const uint32_t*>(base + o_eoff);
    d->elem_order = reinterpret_cast<const uint32_t*>(base + o_eord);
    d->elem_byte = reinterpret_cast<const uint8_t*>(base + o_eb);
    d->tok_mask = reinterpret_cast<const uint64_t*>(base + o_mask);
    d->tok_off = dev_toff ? reinterpret_cast<const uint32_t*>(base + o_toff) : nullptr;
    d->tok_order = toks ? reinterpret_cast<const uint8_t*>(base + o_tord) : nullptr;
    d->elem_blob = reinterpret_cast<const uint8_t*>(base + o_eblob);
    d->tok_blob = nullptr;                 // (host-side arrays only, see above)
    d->elem_poff = reinterpret_cast<const uint32_t*>(base + o_epoff);
    d->tok_poff = nullptr;
    d->elem_pad = reinterpret_cast<const uint8_t*>(base + o_epad);
    d->tok_pad = toks ? reinterpret_cast<const uint8_t*>(base + o_tpad) : nullptr;
    d->tok_desc = toks ? reinterpret_cast<const uint64_t*>(base + o_tdesc) : nullptr;
    if (tok_headroom && toks && rec_len && hashed) {
        d->patchable = true;
        d->h_rank.assign(E, 0);
        for (uint32_t r = 0; r < E; ++r) d->h_rank[elem_order[r]] = r;
        d->h_tpoff = std::move(tpoff);         // (~0u marks the empty slots already)
        d->o_mask = o_mask;
        d->o_tord = o_tord;
        d->o_tpad = o_tpad;
        d->o_tdesc = o_tdesc;
        d->o_rpad = o_rpad;
        d->o_rd = o_rd;
        d->tpad_used = tpad_n - 48;
        d->tpad_cap = tpad_cap;
    }
    *out = d;
    return LASPJ_OK;
}

int laspj_etf_dict_create(laspj_ctx* ctx, uint32_t E, const uint8_t* elem_blob,
                          const uint32_t* elem_off, const uint32_t* elem_order,
                          const uint8_t* tok_blob, const uint32_t* tok_off,
                          const uint8_t* tok_order, laspj_etf_dict** out) {
    return etf_dict_create_body(ctx, E, elem_blob, elem_off, elem_order, tok_blob, tok_off,
                                tok_order, 0, out);
}

int laspj_etf_dict_destroy(laspj_etf_dict* d) {
    if (!d) return LASPJ_E_INVAL;
    {
        std::lock_guard<std::mutex> lk(d->ctx->mu);
        hipSetDevice(d->ctx->device);
        // back to the context's cache: its next user is ordered after every kernel that
        // read this image (all on the context's stream)
        laspj::dev_release(d->ctx, d->block, d->block_bytes);
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

int laspj_orset_etf_read(laspj_ctx* ctx, laspj_batch* b, const laspj_etf_dict* d, int tag,
                         int vers, const laspj_buf* payload, const laspj_buf* offsets,
                         laspj_buf* status) {
    return laspj::etf_read(ctx, b, d, tag, vers, payload, offsets, status);
}

int laspj_gset_etf_read(laspj_ctx* ctx, laspj_batch* b, const laspj_etf_dict* d, int tag,
                        int vers, const laspj_buf* payload, const laspj_buf* offsets,
                        laspj_buf* status) {
    return laspj::gset_etf_read(ctx, b, d, tag, vers, payload, offsets, status);
}

}  // extern "C"

// ------------------------------------------------------------------ dictionary patches
namespace laspj {

namespace {

struct PatchRec {
    u64 dst;            // byte offset in the dictionary's block
    uint32_t src, len;  // bytes [src, src + len) of the staged patch data
};

// one block per record, bytes copied as they stand (records are a few hundred bytes)
__global__ __launch_bounds__(kBlock) void k_patch(const uint8_t* src, const PatchRec* recs,
                                                  uint32_t n, uint8_t* base) {
    for (uint32_t r = blockIdx.x; r < n; r += gridDim.x) {
        const PatchRec pr = recs[r];
        for (uint32_t i = threadIdx.x; i < pr.len; i += kBlock) base[pr.dst + i] = src[pr.src + i];
    }
}

}  // namespace

int etf_dict_create_ex(laspj_ctx* ctx, uint32_t E, const uint8_t* elem_blob,
                       const uint32_t* elem_off, const uint32_t* elem_order,
                       const uint8_t* tok_blob, const uint32_t* tok_off, const uint8_t* tok_order,
                       uint32_t tok_headroom, laspj_etf_dict** out) {
    return etf_dict_create_body(ctx, E, elem_blob, elem_off, elem_order, tok_blob, tok_off,
                                tok_order, tok_headroom, out, true);
}

// The device rows of element slots `dirty` (each gained tokens in the host dictionary `hd`
// since `d` was built or last patched) rewritten from the host dictionary, as a full
// rebuild would write them: token mask, term order, writer descriptors (a new token's
// padded image appended to the image area), record templates, the from_binary tables of
// its rank (bucket word and shift chosen again, bucket per term rank, slot -> rank).  One
// staged copy of the rows and one scatter launch, on the context's stream.  Returns
// LASPJ_E_UNSUPPORTED (nothing written) when only a rebuild will do: a dictionary built
// without headroom, an element past its token headroom, a token image of another length,
// no bucket choice that separates the element's tokens, the image area full.
int etf_dict_patch(laspj_ctx* ctx, laspj_etf_dict* d, const laspj_dict* hd,
                   const uint32_t* dirty, uint32_t n) {
    if (!d || !d->patchable) return LASPJ_E_UNSUPPORTED;
    if (n == 0) return LASPJ_OK;
    const uint32_t E = d->elements, RK = d->tok_max, RL = d->rec_len;
    const uint64_t RS = d->rec_stride;
    const uint32_t TL = d->tok_uniform;
    std::vector<uint8_t> data;
    std::vector<PatchRec> recs;
    auto put = [&](u64 dst, const void* p, uint32_t len) {
        const uint32_t at = (uint32_t)data.size();
        data.resize(data.size() + ((len + 15u) & ~15u), 0);
        std::memcpy(data.data() + at, p, len);
        recs.push_back(PatchRec{dst, at, len});
    };
    uint64_t tpad_used = d->tpad_used;
    uint32_t big_add = 0;
    std::vector<std::pair<uint64_t, uint32_t>> new_tpoff;     // (slot index, offset)
    std::vector<std::string_view> imgs;
    std::vector<uint8_t> order;
    const uint64_t o_desc = d->o_rd, o_tb = d->o_rd + 80ull * E,
                   o_ros = o_tb + 2ull * E * RK;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t e = dirty[i];
        if (e >= E || !dict_tokens(hd, e, &imgs, &order)) return LASPJ_E_UNSUPPORTED;
        const uint32_t cnt = (uint32_t)imgs.size();
        if (cnt > RK || cnt > 64 || cnt == 0) return LASPJ_E_UNSUPPORTED;
        {
            uint32_t had = 0;                  // (the element's count the images hold)
            for (uint32_t k = 0; k < 64; ++k) had += d->h_tpoff[64ull * e + k] != 0xFFFFFFFFu;
            if (had <= kSmallTok && cnt > kSmallTok) ++big_add;
        }
        for (const auto& im : imgs)
            if (im.size() != TL || TL + 2u != RL) return LASPJ_E_UNSUPPORTED;
        for (const auto& im : imgs)
            if (!tok_is_binary(reinterpret_cast<const uint8_t*>(im.data()), TL)) d->bin_tokens = false;
        // token mask and term order
        const u64 mask = cnt == 64 ? ~0ull : (1ull << cnt) - 1ull;
        put(d->o_mask + 8ull * e, &mask, 8);
        uint8_t ord[64];
        std::memset(ord, 0xFF, 64);
        std::memcpy(ord, order.data(), cnt);
        put(d->o_tord + 64ull * e, ord, 64);
        // padded images of the new slots, appended
        uint32_t tpo[64];
        for (uint32_t k = 0; k < 64; ++k) {
            uint32_t o = k < cnt ? d->h_tpoff[64ull * e + k] : 0xFFFFFFFFu;
            for (const auto& nt : new_tpoff)
                if (nt.first == 64ull * e + k) o = nt.second;
            if (k < cnt && o == 0xFFFFFFFFu) {
                const uint64_t need = (TL + 15u) & ~15u;
                if (tpad_used + need + 48 > d->tpad_cap) return LASPJ_E_UNSUPPORTED;
                o = (uint32_t)tpad_used;
                tpad_used += need;
                put(d->o_tpad + o, imgs[k].data(), TL);
                new_tpoff.emplace_back(64ull * e + k, o);
            }
            tpo[k] = o;
        }
        // writer descriptors by term rank: slot | length << 8 | padded offset << 32
        u64 td[64];
        for (uint32_t j = 0; j < RK; ++j)
            td[j] = j < cnt ? (u64)order[j] | ((u64)TL << 8) | ((u64)tpo[order[j]] << 32) : 0xFFull;
        put(d->o_tdesc + 8ull * RK * e, td, 8 * RK);
        // record templates by term rank
        std::vector<uint8_t> rows((size_t)RK * RS, 0);
        for (uint32_t j = 0; j < cnt; ++j) {
            uint8_t* r = rows.data() + j * RS;
            r[0] = 104;
            r[1] = 2;
            std::memcpy(r + 2, imgs[order[j]].data(), TL);
        }
        put(d->o_rpad + (u64)e * RK * RS, rows.data(), (uint32_t)rows.size());
        // from_binary tables of the element's rank
        const uint32_t r = d->h_rank[e];
        uint32_t key = 0;
        std::vector<uint16_t> tb(RK, 0);
        bool placed = false;
        std::vector<uint32_t> keys(cnt);
        for (uint32_t wi = RL / 4; wi-- > 0 && !placed;) {
            for (uint32_t j = 0; j < cnt; ++j) std::memcpy(&keys[j], rows.data() + j * RS + 4 * wi, 4);
            for (uint32_t sh = 0; sh + 10 <= 32 && !placed; ++sh) {
                uint64_t seen[kBuckets / 64] = {};
                bool ok = true;
                for (uint32_t j = 0; j < cnt && ok; ++j) {
                    const uint32_t bk = (keys[j] >> sh) & (kBuckets - 1u);
                    ok = !((seen[bk / 64] >> (bk % 64)) & 1ull);
                    seen[bk / 64] |= 1ull << (bk % 64);
                }
                if (!ok) continue;
                placed = true;
                key = wi | (sh << 8);
                for (uint32_t j = 0; j < cnt; ++j) tb[j] = (uint16_t)((keys[j] >> sh) & (kBuckets - 1u));
            }
        }
        if (!placed) {
            key = kNoBuckets;                  // (matched template by template, see create)
            for (uint32_t j = 0; j < cnt; ++j) tb[j] = 0xFFFFu;
        }
        // descriptor {slot, header length, key, tokens}: the first two do not change
        const uint32_t kc[2] = {key, cnt};
        put(o_desc + 16ull * r + 8, kc, 8);
        put(o_tb + 2ull * r * RK, tb.data(), 2 * RK);
        uint8_t ros[64];
        std::memset(ros, 0xFF, 64);
        for (uint32_t j = 0; j < cnt; ++j) ros[order[j]] = (uint8_t)j;
        put(o_ros + 64ull * r, ros, 64);
    }
    // stage and scatter
    std::lock_guard<std::mutex> lk(ctx->mu);
    hipSetDevice(ctx->device);
    const uint64_t rec_bytes = recs.size() * sizeof(PatchRec);
    const uint64_t total = data.size() + ((rec_bytes + 15) & ~15ull);
    if (total <= laspj_ctx::kUpSmall) {
        // a few elements' rows (an update's token, a bind's new tokens): through the pinned
        // upload ring, with no wait for the stream's earlier work
        data.resize(total, 0);
        std::memcpy(data.data() + (total - ((rec_bytes + 15) & ~15ull)), recs.data(), rec_bytes);
        const uint64_t dlen = total - ((rec_bytes + 15) & ~15ull);
        const void* staged = stage_small(ctx, data.data(), total);
        if (staged) {
            // k_patch reads the staged rows in place from pinned memory (a few KB: no copy
            // to launch first)
            const char* dev = static_cast<const char*>(staged_dev(ctx, staged));
            if (!dev) {
                if (int s = reserve_scratch(ctx, total)) return s;
                char* sc = static_cast<char*>(ctx->scratch);
                if (hipMemcpyAsync(sc, staged, total, hipMemcpyHostToDevice, ctx->stream) !=
                    hipSuccess)
                    return LASPJ_E_DEVICE;
                dev = sc;
            }
            hipLaunchKernelGGL(k_patch, dim3((unsigned)std::min<uint64_t>(recs.size(), 4096)),
                               dim3(kBlock), 0, ctx->stream, reinterpret_cast<const uint8_t*>(dev),
                               reinterpret_cast<const PatchRec*>(dev + dlen),
                               (uint32_t)recs.size(), static_cast<uint8_t*>(d->block));
            if (hipGetLastError() != hipSuccess) return LASPJ_E_DEVICE;
            for (const auto& nt : new_tpoff) d->h_tpoff[nt.first] = nt.second;
            d->tpad_used = tpad_used;
            d->big_elems += big_add;
            return LASPJ_OK;
        }
        data.resize(dlen);
    }
    hipStreamSynchronize(ctx->stream);                // the pinned staging is free
    if (ctx->dstage_bytes < total) {
        if (ctx->dstage) hipHostFree(ctx->dstage);
        ctx->dstage = nullptr;
        ctx->dstage_bytes = 0;
        if (hipHostMalloc(&ctx->dstage, std::max<uint64_t>(total, 1ull << 20), hipHostMallocDefault) != hipSuccess) {
            hipGetLastError();
            ctx->dstage = nullptr;
            return LASPJ_E_NOMEM;
        }
        ctx->dstage_bytes = std::max<uint64_t>(total, 1ull << 20);
    }
    char* st = static_cast<char*>(ctx->dstage);
    std::memcpy(st, data.data(), data.size());
    std::memcpy(st + data.size(), recs.data(), rec_bytes);
    if (int s = reserve_scratch(ctx, total)) return s;
    char* dev = static_cast<char*>(ctx->scratch);
    if (hipMemcpyAsync(dev, st, total, hipMemcpyHostToDevice, ctx->stream) != hipSuccess)
        return LASPJ_E_DEVICE;
    hipLaunchKernelGGL(k_patch, dim3((unsigned)std::min<uint64_t>(recs.size(), 4096)), dim3(kBlock),
                       0, ctx->stream, reinterpret_cast<const uint8_t*>(dev),
                       reinterpret_cast<const PatchRec*>(dev + data.size()), (uint32_t)recs.size(),
                       static_cast<uint8_t*>(d->block));
    if (hipGetLastError() != hipSuccess) return LASPJ_E_DEVICE;
    for (const auto& nt : new_tpoff) d->h_tpoff[nt.first] = nt.second;
    d->tpad_used = tpad_used;
    d->big_elems += big_add;
    return LASPJ_OK;
}

}  // namespace laspj


// ------------------------------------------------------------------ wide namespaces
// A resident variable whose element holds more than 64 tokens (add_elem mints a token per
// add and never collects one, lasp_orset.erl:222-241, 261-262) lives in cells of k {p, r}
// pairs per element (LASPJ_KIND_ORSET_WIDE's layout: token slot t in pair t / 64).  Its
// namespace's device tables hold, per element slot, its tokens in term order as ranks of
// a CSR array (slot of each rank, the record template 104 2 <token image> of each rank),
// and the decoder / writer below read and write images of such values.  The decoder is
// the serial one (one wave per payload, candidates ranked by lanes, LDS-staged payload
// windows); the size pass and writer assemble elements one thread each.  Token images of
// one length only (Lasp's 20-byte tokens), <= 46 bytes.
namespace laspj {

struct WideView {
    DictView d;                 // the element tables (images, term order, templates)
    const uint32_t* rb;         // E + 1: element slot e's ranks rb[e] .. rb[e + 1)
    const uint16_t* rslot;      // by rank: the token slot
    const uint8_t* rec;         // by rank: 104 2 <token image>, RS bytes each (RS = 16 k)
    uint32_t RL, RS, E, tw;     // template bytes, stride, element slots, pairs per cell
};

struct WideDict {
    laspj_ctx* ctx = nullptr;
    void* block = nullptr;
    uint64_t block_bytes = 0;
    WideView v;
    uint32_t max_cnt = 0;
};

namespace {


// bytes of one present element: 104 2 <elem> 108 <n:32> records 106; a record is
// 104 2 <token image> and the flag atom (false 8 bytes, true 7)
__device__ __forceinline__ uint32_t wide_elem_size(const WideView& W, uint32_t e,
                                                   const u64x2* c, uint32_t* npres, bool* bad) {
    uint32_t n = 0, nt = 0;
    const uint32_t cnt = W.rb[e + 1] - W.rb[e];
    for (uint32_t j = 0; j < W.tw; ++j) {
        const u64x2 v = c[j];
        n += (uint32_t)__popcll(v.x);
        nt += (uint32_t)__popcll(v.x & v.y);
        const uint32_t lo = 64u * j;
        const u64 valid = cnt >= lo + 64u ? ~0ull : (cnt > lo ? (1ull << (cnt - lo)) - 1ull : 0ull);
        *bad |= (v.x & ~valid) != 0;
    }
    *npres = n;
    const uint32_t el = W.d.elem_off[e + 1] - W.d.elem_off[e];
    return n ? 7u + el + n * (W.RL + 8u) - nt + 1u : 0u;
}

__global__ __launch_bounds__(kBlock) void k_wide_size(const u64x2* cells, uint64_t R, WideView W,
                                                      uint32_t hdr, u64* sizes, uint32_t* flag) {
    const int lane = threadIdx.x & 63;
    const uint64_t waves = (uint64_t)gridDim.x * (kBlock / 64);
    for (uint64_t rep = (uint64_t)blockIdx.x * (kBlock / 64) + threadIdx.x / 64; rep < R;
         rep += waves) {
        const u64x2* c = cells + rep * (u64)W.E * W.tw;
        u64 sum = 0, n = 0;
        bool bad = false;
        for (uint32_t e = lane; e < W.E; e += 64) {
            uint32_t np = 0;
            const uint32_t sz = wide_elem_size(W, e, c + (u64)e * W.tw, &np, &bad);
            if (np) {
                ++n;
                bad |= W.d.elem_off[e + 1] == W.d.elem_off[e];
                sum += sz;
            }
        }
        sum = wave_sum(sum);
        n = wave_sum(n);
        const bool any_bad = __ballot(bad) != 0;
        if (lane == 0) {
            sizes[rep] = hdr + 1u + (n ? 5u + sum + 1u : 1u);
            if (any_bad) atomicOr(flag, 1u);
        }
    }
}

__global__ __launch_bounds__(kBlock) void k_wide_write(const u64x2* cells, uint64_t R, WideView W,
                                                       int tag, int vers, const u64* offs,
                                                       uint8_t* out, u64 ocap) {
    if (offs[R] > ocap) return;              // the payloads do not fit: the host re-sizes
    __shared__ uint32_t lds4[kBlock / 64];
    __shared__ __attribute__((aligned(16))) uint8_t buf[kWin + 16];
    const uint32_t hdr = tag >= 0 ? 2u : 0u;
    const uint32_t E = W.E, tw = W.tw;
    for (uint64_t rep = blockIdx.x; rep < R; rep += gridDim.x) {
        const u64x2* c = cells + rep * (u64)E * tw;
        const u64 base = offs[rep], end = offs[rep + 1];
        u64 cursor = base + hdr + 6u;
        uint32_t n = 0;
        for (uint32_t c0 = 0; c0 < E; c0 += kBlock) {
            const uint32_t i = c0 + threadIdx.x;
            const uint32_t e = i < E ? W.d.elem_order[i] : 0u;
            uint32_t np = 0;
            bool bad = false;
            const uint32_t sz = i < E ? wide_elem_size(W, e, c + (u64)e * tw, &np, &bad) : 0u;
            uint32_t tot, cnt;
            const uint32_t pos = block_excl_scan(sz, lds4, &tot);
            block_excl_scan(np ? 1u : 0u, lds4, &cnt);
            if (cursor + tot + 1u > end) break;          // sizes disagree: never overrun
            for (uint32_t w0 = 0; w0 < tot; w0 += kWin) {
                const uint32_t wl = min(kWin, tot - w0);
                const u64 g = cursor + w0;
                const uint32_t sh = (uint32_t)(g & 15u);
                const Win win{buf + sh, w0, wl};
                if (np && win.hits(pos, sz)) {
                    stage_elem_header(win, W.d, e, np, pos);
                    uint32_t q = pos + 7u + (W.d.elem_off[e + 1] - W.d.elem_off[e]);
                    const uint32_t r0 = W.rb[e], rc = W.rb[e + 1] - r0;
                    for (uint32_t r = 0; r < rc; ++r) {
                        const uint32_t t = W.rslot[r0 + r];
                        const u64x2 v = c[(u64)e * tw + (t >> 6)];
                        if (!((v.x >> (t & 63u)) & 1ull)) continue;
                        const bool rm = (v.y >> (t & 63u)) & 1ull;
                        const uint32_t rl = W.RL + (rm ? 7u : 8u);
                        if (win.hits(q, rl)) {
                            win.span(q, W.rec + (u64)(r0 + r) * W.RS, W.RL);
                            if (rm) win.span(q + W.RL, kAtomTrue, 7);
                            else win.span(q + W.RL, kAtomFalse, 8);
                        }
                        q += rl;
                    }
                    win.put(q, 106);
                }
                __syncthreads();
                copy_out(buf, sh, wl, out, g);
                __syncthreads();
            }
            cursor += tot;
            n += cnt;
        }
        if (threadIdx.x == 0) {
            write_list_header(out, base, hdr, tag, vers, n ? 108 : 106, n);
            if (n && cursor < end) out[cursor] = 106;
        }
        __syncthreads();
    }
}

// cells re-laid: E_old x tw_old pairs -> E_new x tw_new (new element slots and pairs
// {0, 0}); a variable's cells when its namespace grows or goes wide
__global__ __launch_bounds__(kBlock) void k_relay(u64x2* dst, const u64x2* src, uint32_t eo,
                                                  uint32_t to, uint32_t en, uint32_t tn) {
    const u64 n = (u64)en * tn;
    for (u64 i = (u64)blockIdx.x * kBlock + threadIdx.x; i < n; i += (u64)gridDim.x * kBlock) {
        const uint32_t e = (uint32_t)(i / tn), j = (uint32_t)(i % tn);
        dst[i] = e < eo && j < to && src ? src[(u64)e * to + j] : u64x2{0, 0};
    }
}

}  // namespace

int wide_dict_create(laspj_ctx* ctx, const WideExport& x, uint32_t tw, WideDict** out) {
    *out = nullptr;
    const uint32_t K = (uint32_t)x.eorder.size();
    if (K == 0) return LASPJ_E_SHAPE;
    uint32_t TL = 0;
    for (size_t r = 0; r + 1 < x.toff.size(); ++r) {
        const uint32_t L = x.toff[r + 1] - x.toff[r];
        if (!TL) TL = L;
        else if (L != TL) return LASPJ_E_UNSUPPORTED;      // token images of several lengths
    }
    if (!TL) TL = 20;                                      // (no tokens yet)
    const uint32_t RL = TL + 2u;
    if (RL > 48) return LASPJ_E_UNSUPPORTED;
    const uint64_t RS = (RL + 15u) & ~15u;
    auto pad16 = [](uint64_t v) { return (v + 15ull) & ~15ull; };
    const uint64_t nr = x.rslot.size();
    // element tables as laspj_etf_dict_create lays them: images, offsets, order, padded
    // images, header templates 104 2 <elem image> 108
    std::vector<uint32_t> epoff(K), hpoff(K);
    uint64_t epn = 0, hpn = 0;
    for (uint32_t e = 0; e < K; ++e) {
        epoff[e] = (uint32_t)epn;
        epn += pad16(x.eoff[e + 1] - x.eoff[e]);
        hpoff[e] = (uint32_t)hpn;
        hpn += pad16(x.eoff[e + 1] - x.eoff[e] + 3ull);
    }
    epn += 48;
    hpn += 48;
    // the block: elem_blob | elem_off | elem_order | elem_pad | elem_poff | ehdr_pad |
    // ehdr_poff | rb | rslot | rec
    auto al = [](uint64_t v) { return (v + 255ull) & ~255ull; };
    const uint64_t o_eb = 0, o_eo = o_eb + al(x.eblob.size() + 1), o_ord = o_eo + al(4ull * (K + 1)),
                   o_ep = o_ord + al(4ull * K), o_epo = o_ep + al(epn), o_hp = o_epo + al(4ull * K),
                   o_hpo = o_hp + al(hpn), o_rb = o_hpo + al(4ull * K),
                   o_rs = o_rb + al(4ull * (K + 1)), o_rec = o_rs + al(2ull * nr + 2),
                   total = o_rec + al(nr * RS + 48);
    std::vector<uint8_t> h(total, 0);
    std::memcpy(h.data() + o_eb, x.eblob.data(), x.eblob.size());
    std::memcpy(h.data() + o_eo, x.eoff.data(), 4ull * (K + 1));
    std::memcpy(h.data() + o_ord, x.eorder.data(), 4ull * K);
    for (uint32_t e = 0; e < K; ++e) {
        const uint32_t l = x.eoff[e + 1] - x.eoff[e];
        std::memcpy(h.data() + o_ep + epoff[e], x.eblob.data() + x.eoff[e], l);
        uint8_t* hp = h.data() + o_hp + hpoff[e];
        hp[0] = 104;
        hp[1] = 2;
        std::memcpy(hp + 2, x.eblob.data() + x.eoff[e], l);
        hp[2 + l] = 108;
    }
    std::memcpy(h.data() + o_epo, epoff.data(), 4ull * K);
    std::memcpy(h.data() + o_hpo, hpoff.data(), 4ull * K);
    std::memcpy(h.data() + o_rb, x.rb.data(), 4ull * (K + 1));
    if (nr) std::memcpy(h.data() + o_rs, x.rslot.data(), 2ull * nr);
    for (uint64_t r = 0; r < nr; ++r) {
        uint8_t* t = h.data() + o_rec + r * RS;
        t[0] = 104;
        t[1] = 2;
        std::memcpy(t + 2, x.tblob.data() + x.toff[r], TL);
    }
    auto* w = new (std::nothrow) WideDict;
    if (!w) return LASPJ_E_NOMEM;
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        hipSetDevice(ctx->device);
        if (dev_alloc(ctx, total, &w->block) != hipSuccess) {
            hipGetLastError();
            delete w;
            return LASPJ_E_NOMEM;
        }
        w->block_bytes = total;
        if (hipMemcpyAsync(w->block, h.data(), total, hipMemcpyHostToDevice, ctx->stream) !=
                hipSuccess ||
            hipStreamSynchronize(ctx->stream) != hipSuccess) {
            dev_release(ctx, w->block, total);
            delete w;
            return LASPJ_E_DEVICE;
        }
    }
    const uint8_t* b = static_cast<const uint8_t*>(w->block);
    w->ctx = ctx;
    std::memset(&w->v, 0, sizeof(w->v));
    w->v.d.elem_blob = b + o_eb;
    w->v.d.elem_off = reinterpret_cast<const uint32_t*>(b + o_eo);
    w->v.d.elem_order = reinterpret_cast<const uint32_t*>(b + o_ord);
    w->v.d.elem_pad = b + o_ep;
    w->v.d.elem_poff = reinterpret_cast<const uint32_t*>(b + o_epo);
    w->v.d.ehdr_pad = b + o_hp;
    w->v.d.ehdr_poff = reinterpret_cast<const uint32_t*>(b + o_hpo);
    w->v.rb = reinterpret_cast<const uint32_t*>(b + o_rb);
    w->v.rslot = reinterpret_cast<const uint16_t*>(b + o_rs);
    w->v.rec = b + o_rec;
    w->v.RL = RL;
    w->v.RS = (uint32_t)RS;
    w->v.E = K;
    w->v.tw = tw;
    w->max_cnt = x.max_cnt;
    *out = w;
    return LASPJ_OK;
}

void wide_dict_destroy(WideDict* w) {
    if (!w) return;
    {
        std::lock_guard<std::mutex> lk(w->ctx->mu);
        hipSetDevice(w->ctx->device);
        dev_release(w->ctx, w->block, w->block_bytes);
    }
    delete w;
}

uint32_t wide_elements(const WideDict* w) { return w ? w->v.E : 0; }

int wide_size_enqueue(laspj_ctx* ctx, const WideDict* w, const uint64_t* cells, uint64_t R,
                      int tag, u64* offsets, uint32_t* flag) {
    const uint64_t sizes_bytes = (8ull * R + 255ull) & ~255ull;
    if (int s = reserve_scratch(ctx, sizes_bytes + scan_tmp_bytes(R))) return s;
    u64* sizes = static_cast<u64*>(ctx->scratch);
    u64* tmp = reinterpret_cast<u64*>(static_cast<char*>(ctx->scratch) + sizes_bytes);
    const uint64_t blocks = (R + 3) / 4, cap = (uint64_t)ctx->cus * 16;
    hipLaunchKernelGGL(k_wide_size, dim3((unsigned)std::max<uint64_t>(1, std::min(blocks, cap))),
                       dim3(kBlock), 0, ctx->stream, reinterpret_cast<const u64x2*>(cells), R, w->v,
                       tag >= 0 ? 2u : 0u, sizes, flag);
    LJ_LAUNCHED(ctx);
    LJ_HIP(ctx, launch_scan(ctx, sizes, offsets, R, tmp));
    return LASPJ_OK;
}

int wide_write_enqueue(laspj_ctx* ctx, const WideDict* w, const uint64_t* cells, uint64_t R,
                       int tag, int vers, const u64* offsets, uint8_t* out, uint64_t cap) {
    const uint64_t g = std::min<uint64_t>(R, (uint64_t)ctx->cus * 8);
    hipLaunchKernelGGL(k_wide_write, dim3((unsigned)std::max<uint64_t>(1, g)), dim3(kBlock), 0,
                       ctx->stream, reinterpret_cast<const u64x2*>(cells), R, w->v, tag, vers,
                       offsets, out, (u64)cap);
    LJ_LAUNCHED(ctx);
    return LASPJ_OK;
}

hipError_t launch_relay(laspj_ctx* ctx, uint64_t* dst, const uint64_t* src, uint32_t eo,
                        uint32_t to, uint32_t en, uint32_t tn) {
    const uint64_t n = (uint64_t)en * tn;
    const uint64_t g = std::max<uint64_t>(1, std::min<uint64_t>((n + kBlock - 1) / kBlock,
                                                                (uint64_t)ctx->cus * 8));
    hipLaunchKernelGGL(k_relay, dim3((unsigned)g), dim3(kBlock), 0, ctx->stream,
                       reinterpret_cast<u64x2*>(dst), reinterpret_cast<const u64x2*>(src), eo, to,
                       en, tn);
    return hipGetLastError();
}

}  // namespace laspj
