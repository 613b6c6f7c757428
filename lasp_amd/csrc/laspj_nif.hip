// NIF-level entry points (include/laspj.h "NIF entry points", "device-resident variables"):
// what a `laspj_nif` NIF function does between `enif_term_to_binary` and
// `enif_binary_to_term`, inside liblaspj so that it is compiled, tested and timed here
// rather than living as a listing.
//
// The reference's drop-in point is `Type:merge/2` and friends (lasp_orset.erl:32-36,
// 67-73, 128-138; lasp_gset.erl:39-43, 74-76, 99-105), called from lasp_core:bind/3
// (lasp_core.erl:291-312) on many BEAM schedulers at once (lasp_vnode.erl:213-237).
//
// Image calls (laspj_{orset,gset}_etf_*) take the operands as `term_to_binary/1` images and
//   1. stage them into the context's pinned memory; kernels on the context's stream pull
//      them to the device in pieces while the host stages the next (offsets and the
//      decoder's segment table ride along),
//   2. decode them on the device against the context's dictionary of that kind
//      (laspj_orset_etf_read's / laspj_gset_etf_read's kernels), join / test the cells,
//      encode the answer on the device straight into pinned memory — all enqueued on the
//      context's stream with ONE host synchronisation,
//   3. answer from pinned memory: the merged / value term's image (what the NIF hands to
//      enif_binary_to_term) or the boolean.
// Variable calls (laspj_var_*) keep `#dv.value` (include/lasp.hrl:60-63) on the device
// between calls: bind/3 ships only the incoming `Value`, decodes it, and one kernel decides
// `Value0 =:= Value`, joins it into the resident cells and answers the status; the value
// is encoded only when it is read.
//
// A token the dictionary has not seen (another node's unique/1) on a known element is
// taken by the decoder in the same pass when it is a binary of the namespace's token
// length (NewTok: the element's next free slot, registered after the pass; a merge's
// answer is then written by a second, write-only launch once the images know it).  Any
// other unseen term makes the decoder answer UNKNOWN_TERM: the call registers the
// operands' terms in the host dictionary (only the elements of the decoder segments that
// failed, when it decoded in segments; else the whole operands, laspj_dict_add), patches
// or rebuilds the device images and decodes again (only the failed segments, when it can).
// An element past 64 tokens widens its namespace (cells of k {p, r} pairs, the wide codec)
// — image calls start a fresh dictionary first.  An operand the columnar form does not
// take — not an orddict of {Elem, [{Token, Bool}]} (an ordset for G-Sets) in term order,
// an element with no tokens, a term `==` to a registered one under another image, a term
// kind no dictionary holds — gets verdict LASPJ_NIF_FALLBACK: the NIF then runs the
// reference's own Erlang clause, so the caller always gets the reference's answer (or its
// crash).  Scratch, dictionaries and staging are per context: one context per scheduler
// (or per vnode), or one per GPU with the binds of many schedulers committed in groups;
// no process globals.

#include <sys/random.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <new>
#include <unordered_set>
#include <vector>

#include "laspj_internal.h"

namespace laspj {

// One dictionary of one kind (OR-Set or G-Set) and its device images.  The image calls of a
// context share one per kind; every resident variable has one of its own — its token
// namespace — shared only with the replicas created beside it (laspj_var_create_replica),
// so a variable's dictionary holds the terms of its own value (and its replicas') and
// variables never compete for an element's token slots (include/lasp.hrl:60-63: each
// #dv.value is independent).
struct KindState {
    int32_t kind = LASPJ_KIND_ORSET;
    laspj_dict* dict = nullptr;     // term images -> slots (host, append-only)
    laspj_etf_dict* etf = nullptr;  // the device images of `dict` (rebuilt when it grows)
    uint32_t E = 0;                 // element slots of `etf` and of the batches
    bool stale = false;             // `dict` registered terms since `etf` was built
    uint64_t epoch = 1;             // bumped by every reset (variables' cells refer to one)
    // what `etf` was built (or last patched) from: host dictionary elements and each
    // one's token count, so registrations that only add tokens to known elements are
    // patched into the device images (etf_dict_patch) instead of rebuilding them
    uint32_t built_K = 0;
    std::vector<uint32_t> built_cnt;
    // the variables whose cells refer to this dictionary (none for the image calls')
    std::unordered_set<laspj_var*> vars;
    // a wide namespace: an element holds more than 64 tokens (add_elem never collects one,
    // lasp_orset.erl:222-241): cells of tw {p, r} pairs per element, the wide tables in wd
    // (etf then holds the element images only, for value/1's G-Set answer)
    bool wide = false;
    uint32_t tw = 1;
    WideDict* wd = nullptr;
};

}  // namespace laspj

// A device-resident variable's value (the `#dv.value` of lasp_core's store): cells over its
// namespace's dictionary, or — when its value is not representable, or between a dictionary
// reset and its next use — the value's image held on the host.
struct laspj_var {
    laspj_ctx* ctx = nullptr;        // null once the context is gone
    int32_t kind = LASPJ_KIND_ORSET;
    std::shared_ptr<laspj::KindState> ns;   // the token namespace (dictionary) of the cells
    uint64_t* cells = nullptr;       // one replica over `E` element slots (null: new())
    uint64_t cell_bytes = 0;         // the block's size (dev_alloc)
    uint32_t E = 0;
    uint32_t tw = 1;                 // {p, r} pairs per element slot (a wide namespace's)
    uint64_t epoch = 0;              // the dictionary generation the cells refer to
    bool resident = true;            // cells hold the value (else `image` does)
    bool held = false;               // `image` is a value write/4 could not represent
    std::vector<uint8_t> image;      // host-held value (term_to_binary image)
};

namespace laspj {

// a pinned host block a group-commit waiter stages its payload into while it waits
struct PinSlot {
    uint8_t* h = nullptr;           // host address
    const uint8_t* d = nullptr;     // its device address
    uint64_t cap = 0;
};

// a single bind waiting for a group-commit pass (laspj_var_etf_bind)
struct BindReq {
    laspj_var* var;
    const uint8_t* p;
    uint64_t n;
    // the payload's pinned copy (device address), valid once `staged` is set: made by the
    // waiter itself, so the leader's pass gathers it on the device instead of copying it
    const uint8_t* pre = nullptr;
    std::atomic<bool> staged{false};
    int32_t status = 0, verdict = LASPJ_NIF_FALLBACK;
    int rc = LASPJ_OK;
    // its own wake-up (no herd of waiters on one condition and one lock): done — answered;
    // lead — handed the leadership, its request still to serve
    std::mutex m;
    std::condition_variable cv;
    bool done = false, lead = false;
};

struct NifState {
    std::mutex mu;                  // one call at a time (ctx->mu is held per device phase)
    // single binds queued for the next group-commit pass, and whether a caller leads one
    std::mutex qmu;
    std::vector<BindReq*> queue;
    bool leading = false;
    // rebuild_etf's export arrays, kept between rebuilds (S->mu): fresh multi-MB blocks
    // would be paged in again by every rebuild
    std::vector<uint8_t> x_ebl, x_tbl, x_tord;
    std::vector<uint32_t> x_eoff, x_eord, x_toff;
    std::vector<PinSlot> pins;      // free waiters' staging blocks (qmu)
    uint32_t pins_live = 0;         // blocks allocated (qmu)
    KindState ks[2];                // the image calls' dictionaries: [0] OR-Set, [1] G-Set
    // device: [in region: offsets | segment table | zeroed words | variable cell pointers
    // | payloads or cells][segment results][variable calls' statuses]; cells: the batches
    void* dblk = nullptr;
    uint64_t dblk_bytes = 0;
    void* dcells = nullptr;
    uint64_t dcells_bytes = 0;
    // pinned host staging, coherent (kernels pull the operands from one and write the
    // answers into the other), and the device addresses of both
    void* hin = nullptr;
    uint64_t hin_bytes = 0;
    void* hout = nullptr;
    uint64_t hout_bytes = 0;
    uint8_t* hin_d = nullptr;
    uint8_t* hout_d = nullptr;
    const void* hin_dkey = nullptr;
    const void* hout_dkey = nullptr;
    uint64_t ocap = 1 << 20;        // bytes reserved for answer payloads
    // the operand cells known to be zero (the fused merge and the variable kernel clear
    // them behind them), so the next call's decoders need no memset
    uint64_t clean_words = 0;
    uint64_t stats[LASPJ_NIF_STATS] = {};
    uint32_t nt_seq = 0;            // device passes that took new tokens (their entries' tag)
    std::unordered_set<laspj_var*> vars;
    // laspj_var_etf_update's answers (valid until the context's next call): the tokens it
    // minted, the image of the element a failed precondition names
    std::vector<uint8_t> minted;
    std::string err_elem;
};

namespace {

enum class Op { MERGE, VALUE, EQUAL, INFLATION, BIND, WRITE, THRESHOLD, READ, VVALUE };

// The in region pulled from pinned host memory by a kernel on the context's stream: the
// decoder then starts right behind it instead of waiting for a copy engine's completion
// signal.  16-byte lanes, grid-stride.
typedef uint32_t pull16 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) k_nif_pull(const pull16* __restrict__ src,
                                                  pull16* __restrict__ dst, uint64_t n16) {
    // a wave moves 4 KiB per step: four 1 KiB loads in flight per instruction group
    const uint64_t lane = threadIdx.x & 63u;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t c = wave; c * 256 < n16; c += nw) {
        pull16 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint64_t i = c * 256 + k * 64 + lane;
            if (i < n16) v[k] = __builtin_nontemporal_load(src + i);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint64_t i = c * 256 + k * 64 + lane;
            if (i < n16) dst[i] = v[k];
        }
    }
}

// Payloads gathered into the in region at their (byte) offsets from pinned blocks: those
// group-commit waiters staged themselves, and the leader's own (copied into the staging
// at its offset).  8-byte lanes, four loads in flight per lane (2 KiB per wave step), a
// dst word composed of two source words (the neighbour lane's) when source and
// destination differ in alignment, partial words at a payload's ends written byte by
// byte (a neighbouring payload owns their other bytes).  blockIdx.y: the payload.
struct GatherDesc {
    const uint8_t* src;             // any alignment; readable 16 bytes past len
    uint64_t dst, len;              // offset in the region, bytes
};
constexpr uint32_t kGatherMax = 16;
constexpr uint32_t kGatherU = 4;
struct GatherArgs {
    GatherDesc d[kGatherMax];
};
__global__ void __launch_bounds__(256) k_nif_gather(GatherArgs g, uint8_t* __restrict__ dst) {
    const GatherDesc ds = g.d[blockIdx.y];
    const uint64_t d0 = ds.dst, d1 = ds.dst + ds.len;
    if (d1 == d0) return;
    const uint64_t w0 = d0 & ~7ull;
    const uint32_t sh = (uint32_t)(d0 - w0);
    const uint64_t nw = (d1 - w0 + 7) / 8;             // dst words touched
    const uint64_t sa = reinterpret_cast<uint64_t>(ds.src);
    const uint64_t* src = reinterpret_cast<const uint64_t*>(sa & ~7ull);
    // dst byte w0 + 8j + b is source word j's byte b + delta (of the aligned source)
    const int32_t delta = (int32_t)(sa & 7ull) - (int32_t)sh;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nwv = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t c = wave * 64 * kGatherU; c < nw; c += nwv * 64 * kGatherU) {
        uint64_t cur[kGatherU], edge[kGatherU];
#pragma unroll
        for (uint32_t u = 0; u < kGatherU; ++u) {
            const uint64_t j = c + 64 * u + lane;
            cur[u] = j < nw ? __builtin_nontemporal_load(src + j) : 0ull;
            // the one neighbour word no lane of this group loads
            edge[u] = 0;
            if (j < nw && delta < 0 && lane == 0 && j > 0) edge[u] = __builtin_nontemporal_load(src + j - 1);
            if (j < nw && delta > 0 && (lane == 63 || j + 1 == nw))
                edge[u] = __builtin_nontemporal_load(src + j + 1);
        }
#pragma unroll
        for (uint32_t u = 0; u < kGatherU; ++u) {
            const uint64_t up = __shfl_up(cur[u], 1, 64), dn = __shfl_down(cur[u], 1, 64);
            const uint64_t j = c + 64 * u + lane;
            if (j >= nw) continue;
            const uint64_t w = w0 + 8 * j;
            if (w >= d0 && w + 8 <= d1) {
                uint64_t v = cur[u];
                if (delta < 0) {
                    const uint64_t pv = lane ? up : edge[u];
                    v = (pv >> (8 * (8 + delta))) | (cur[u] << (8 * -delta));
                } else if (delta > 0) {
                    const uint64_t nx = (lane == 63 || j + 1 == nw) ? edge[u] : dn;
                    v = (cur[u] >> (8 * delta)) | (nx << (8 * (8 - delta)));
                }
                *reinterpret_cast<uint64_t*>(dst + w) = v;
            } else {
                for (uint32_t b = 0; b < 8; ++b)
                    if (w + b >= d0 && w + b < d1) dst[w + b] = ds.src[w + b - d0];
            }
        }
    }
}

// lasp_orset:update/3 / lasp_gset:update/3 (lasp_orset.erl:99-117, 222-259;
// lasp_gset.erl:84-88) of one call on a resident variable's cells: the ops in order, all or
// nothing.  A REMOVE whose element is absent — not in the cells and not added earlier in the
// call — fails the call ({error, {precondition, {not_present, E}}}, remove_elems / apply_ops
// stop there and the state is kept); element 0xFFFFFFFF is an element the dictionary has
// never held.  Few ops travel as kernel arguments (no upload on the update path); one lane
// walks them (a call is a handful of ops).  tw {p, r} pairs per element (a wide namespace:
// token slot t in pair t / 64, the slot's bits 8..15 in the op's pad byte).
constexpr uint32_t kUpdArgOps = 24;
struct UpdArgs {
    laspj_op op[kUpdArgOps];
};
constexpr uint32_t kNoElem = 0xFFFFFFFFu;

__device__ inline uint32_t op_slot(const laspj_op& o) { return o.slot | (uint32_t)o.pad << 8; }

__global__ void __launch_bounds__(64) k_var_update(uint64_t* __restrict__ cells, int32_t kind,
                                                   uint32_t tw, UpdArgs a,
                                                   const laspj_op* __restrict__ dops,
                                                   uint32_t nops, int32_t* __restrict__ status) {
    if (threadIdx.x != 0) return;
    auto op = [&](uint32_t k) -> laspj_op { return dops ? dops[k] : a.op[k]; };
    uint32_t bad = nops;
    if (kind == LASPJ_KIND_ORSET) {
        for (uint32_t k = 0; k < nops && bad == nops; ++k) {
            const laspj_op o = op(k);
            if (o.kind != LASPJ_OP_REMOVE) continue;
            bool present = false;
            if (o.element != kNoElem)
                for (uint32_t j = 0; j < tw && !present; ++j)
                    present = cells[2ull * ((uint64_t)o.element * tw + j)] != 0;
            for (uint32_t j = 0; j < k && !present; ++j) {
                const laspj_op q = op(j);
                present = q.kind == LASPJ_OP_ADD && q.element == o.element;
            }
            if (!present) bad = k;
        }
    }
    for (uint32_t k = 0; k < nops; ++k) {
        if (bad < nops) {
            if (status) status[k] = k == bad ? LASPJ_OPST_NOT_PRESENT : LASPJ_OPST_ROLLED_BACK;
            continue;
        }
        const laspj_op o = op(k);
        if (kind == LASPJ_KIND_ORSET) {
            uint64_t* c = cells + 2ull * (uint64_t)o.element * tw;
            if (o.kind == LASPJ_OP_ADD) {
                // orddict:store(Token, false, Tokens): present, flag false
                const uint32_t t = op_slot(o);
                c[2 * (t >> 6)] |= 1ull << (t & 63u);
                c[2 * (t >> 6) + 1] &= ~(1ull << (t & 63u));
            } else {
                for (uint32_t j = 0; j < tw; ++j)
                    c[2 * j + 1] = c[2 * j];           // every token of Elem := true
            }
        } else {
            cells[o.element >> 6] |= 1ull << (o.element & 63u);
        }
        if (status) status[k] = LASPJ_OPST_APPLIED;
    }
}

// the same for a call of ADDs only (add_all over many elements): commutative, one op per lane
__global__ void __launch_bounds__(256) k_var_adds(uint64_t* __restrict__ cells, int32_t kind,
                                                  uint32_t tw, const laspj_op* __restrict__ ops,
                                                  uint32_t nops) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nops) return;
    const laspj_op o = ops[k];
    if (kind == LASPJ_KIND_ORSET) {
        const uint32_t t = op_slot(o);
        unsigned long long* c = reinterpret_cast<unsigned long long*>(
            cells + 2ull * ((uint64_t)o.element * tw + (t >> 6)));
        atomicOr(c, 1ull << (t & 63u));
        atomicAnd(c + 1, ~(1ull << (t & 63u)));
    } else {
        atomicOr(reinterpret_cast<unsigned long long*>(cells + (o.element >> 6)),
                 1ull << (o.element & 63u));
    }
}

// lasp_core:union/7's body for OR-Sets (lasp_core.erl:602-627: orddict:merge keeping the
// left value of a key both hold) over resident l and r, bound into out (bind/3, :291-312:
// out := merge(out, AccValue), the OR of the cells): per element slot, l's cell where l
// holds the element (any pair's present word nonzero), else r's; *changed set when
// `Value0 =:= AccValue` fails (the bind's no-op test: canonical values of one namespace
// are equal exactly when their cells are; a wave's lanes agree on one atomic).  tw pairs
// per element.
// (out may be l or r: no restrict)
__global__ void __launch_bounds__(256) k_var_union(uint64_t* out, const uint64_t* l,
                                                   const uint64_t* r, uint32_t E, uint32_t tw,
                                                   uint32_t* __restrict__ changed) {
    const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
    bool ch = false;
    if (e < E) {
        const uint64_t base = 2ull * e * tw;
        bool inl = false;
        for (uint32_t j = 0; j < tw; ++j) inl |= l[base + 2 * j] != 0;
        const uint64_t* src = inl ? l : r;
        for (uint32_t j = 0; j < tw; ++j) {
            const uint64_t op = out[base + 2 * j], oq = out[base + 2 * j + 1];
            const uint64_t ap = src[base + 2 * j], aq = src[base + 2 * j + 1];
            ch |= op != ap || oq != aq;                    // Value0 =/= AccValue
            if ((op | ap) != op || (oq | aq) != oq) {
                out[base + 2 * j] = op | ap;
                out[base + 2 * j + 1] = oq | aq;
            }
        }
    }
    if (__ballot(ch) && (threadIdx.x & 63u) == 0) atomicOr(changed, 1u);
}

struct Guard {
    std::lock_guard<std::mutex> lk;
    explicit Guard(laspj_ctx* c) : lk(c->mu) { hipSetDevice(c->device); }
};

constexpr uint32_t kMaxDictElements = 1u << 20;   // a larger dictionary is reset
// a wide namespace (an element past 64 tokens): token slots per element, and the token
// image length its fixed-width templates hold
constexpr uint32_t kWideTokens = 1024, kWideTokenLen = 46;
// passes a group-commit leader runs back to back while binds keep queueing
constexpr int kLeadRounds = 8;
// waiters' staging blocks: payloads of at least kPinMin bytes, at most kPinSlots blocks
constexpr uint64_t kPinMin = 64ull << 10;
constexpr uint32_t kPinSlots = 64;

// a waiter's pinned block grown to `need` bytes (false: no pinned memory; the leader then
// copies that payload itself)
bool pin_grow(PinSlot* s, uint64_t need) {
    if (s->h) hipHostFree(s->h);
    *s = PinSlot{};
    const uint64_t cap = std::max<uint64_t>((need + (1ull << 20) - 1) & ~((1ull << 20) - 1), 1ull << 20);
    void* h = nullptr;
    if (hipHostMalloc(&h, cap, hipHostMallocCoherent) != hipSuccess) {
        hipGetLastError();
        return false;
    }
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
        hipGetLastError();
        hipHostFree(h);
        return false;
    }
    *s = PinSlot{static_cast<uint8_t*>(h), static_cast<const uint8_t*>(d), cap};
    return true;
}
// new tokens a single bind's decoder may take (NewTok entries; more: the two-pass path)
constexpr uint32_t kNewTokCap = 512;
// device passes per call: registration, a grown answer area and a serial re-decode each
// take one; a call still unresolved after this many answers FALLBACK (run's post-condition)
constexpr int kMaxPasses = 6;
// the in region is pulled by kernels in pieces of this many bytes: each piece's pull runs
// while the host stages the next (one copy-engine copy per call measured slower, and
// 512 KiB copy pieces hit a slow runtime path: profiles/r04i_nif_ab.log,
// r04pull_block_size_ab.log)
constexpr uint64_t kPullPiece = 512ull << 10;

uint64_t al(uint64_t x, uint64_t a) { return (x + a - 1) & ~(a - 1); }

uint64_t wpr_of(int32_t kind, uint32_t E, uint32_t tw = 1) {
    return kind == LASPJ_KIND_ORSET ? 2ull * E * tw : (E + 63ull) / 64ull;
}

// pairs per element slot of a namespace's cells
uint32_t ktw(const KindState& K) { return K.wide ? K.tw : 1u; }

// the payloads [p0, p1) of a call decoded against one dictionary (an image call: the
// context's; a variable call: one per namespace of its variables)
struct Group {
    KindState* K = nullptr;
    uint32_t p0 = 0, p1 = 0;
};

// one NIF-level call over m operand payloads giving n answers
struct Call {
    Op op = Op::MERGE;
    int32_t kind = LASPJ_KIND_ORSET;
    int strict = 0;
    uint32_t n = 0, m = 0;
    std::vector<Group> groups;      // >= 1; single-group ops (all but BIND / WRITE) use [0]
    std::vector<const uint8_t*> p;  // m payloads: MERGE / EQUAL / INFLATION: lhs[0..n) then rhs
    std::vector<uint64_t> len;
    std::vector<const uint8_t*> pre;   // (binds) a payload's pinned copy on the device, or null
    std::vector<laspj_var*> vars;   // variable calls: n variables (payload i -> variable i)
    std::vector<int32_t> st;        // m decode statuses
    std::vector<uint8_t> res;       // n answer bytes (EQUAL / INFLATION / BIND / THRESHOLD)
    std::vector<uint64_t> ooff;     // n + 1 answer payload offsets (MERGE / VALUE / READ)
    const uint8_t* obase = nullptr; // pinned answer payloads
    bool no_defer = false;          // a deferred chain check came back kDecRedo: decode serially
    // a redo pass: the last pass's payloads and cells stay on the device and only these
    // segments are decoded again (their terms registered since, patched into the images)
    SegList redo;
    // a deferred pass that met unknown terms: its segment results (SegRes records, 32 bytes
    // each: status, start, ...) and table, so only the failing segments are registered
    bool has_seg = false;
    std::vector<uint32_t> segres;   // 8 words per segment
    std::vector<uint32_t> segbase;
    uint64_t segS = 0;
    // a single bind / write whose decoder took tokens its namespace had not seen (NewTok):
    // the entries of a pass that decoded, registered by run(); `nt_met`: the pass met some
    // (its cells then hold slots nobody registered unless it decoded)
    std::vector<NewTok> newtoks;
    bool nt_met = false;
    bool no_newtok = false;         // (two payloads gave one slot to different tokens)
    // a merge whose decoders took new tokens: its operands' cells stay on the device and
    // the next pass only joins and writes (the images patched with the tokens first)
    bool write_only = false;
};

KindState& kstate(NifState* S, int32_t kind) {
    return S->ks[kind == LASPJ_KIND_GSET ? 1 : 0];
}

laspj_batch view(laspj_ctx* ctx, int32_t kind, uint64_t R, uint32_t E, uint64_t* dev,
                 uint32_t tw = 1) {
    laspj_batch b;
    b.ctx = ctx;
    b.kind = kind == LASPJ_KIND_ORSET && tw > 1 ? LASPJ_KIND_ORSET_WIDE : kind;
    b.elements = E;
    b.replicas = R;
    b.words_per_replica = wpr_of(kind, E, tw);
    b.cells = E;
    b.tok_words = kind == LASPJ_KIND_ORSET ? tw : 1;
    b.dev = dev;
    b.owns = false;
    return b;
}

int grow_dev(laspj_ctx* ctx, void** p, uint64_t* have, uint64_t need) {
    if (*have >= need) return LASPJ_OK;
    const uint64_t want = std::max<uint64_t>(need, *have + *have / 2);
    if (*p) {
        hipStreamSynchronize(ctx->stream);
        hipFree(*p);
        *p = nullptr;
        *have = 0;
    }
    if (dev_malloc(ctx, p, want) != hipSuccess) {
        hipGetLastError();
        *p = nullptr;
        return fail(ctx, LASPJ_E_NOMEM, "nif: device allocation of %llu bytes",
                    (unsigned long long)want);
    }
    *have = want;
    return LASPJ_OK;
}

int grow_host(laspj_ctx* ctx, void** p, uint64_t* have, uint64_t need) {
    if (*have >= need) return LASPJ_OK;
    const uint64_t want = std::max<uint64_t>(need, *have + *have / 2);
    if (*p) {
        hipStreamSynchronize(ctx->stream);
        hipHostFree(*p);
        *p = nullptr;
        *have = 0;
    }
    // coherent: kernels read the staging and write the answers themselves, and a device
    // L2 line of last call's operands must not outlive the host's rewrite
    if (hipHostMalloc(p, want, hipHostMallocCoherent) != hipSuccess) {
        hipGetLastError();
        *p = nullptr;
        return fail(ctx, LASPJ_E_NOMEM, "nif: pinned allocation of %llu bytes",
                    (unsigned long long)want);
    }
    *have = want;
    return LASPJ_OK;
}

void free_etf(KindState& K) {
    if (K.etf) laspj_etf_dict_destroy(K.etf);
    K.etf = nullptr;
    if (K.wd) wide_dict_destroy(K.wd);
    K.wd = nullptr;
    K.E = 0;
}

uint64_t now_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

// the device images of the dictionary (called without ctx->mu: etf_dict_create takes it)
// a wide namespace's tables (called as rebuild_etf): every element exactly (no headroom:
// any registration rebuilds — the wide path is the rare one), pairs per cell grown to hold
// the widest element; LASPJ_E_UNSUPPORTED: token images of several lengths
int rebuild_wide(laspj_ctx* ctx, NifState* S, KindState& K) {
    const uint64_t t0 = now_ns();
    WideExport x;
    if (int s = dict_export_wide(K.dict, &x)) return fail(ctx, s, "nif: wide export");
    const uint32_t n = (uint32_t)x.eorder.size();
    if (!n) return LASPJ_E_UNSUPPORTED;
    const uint32_t tw = std::max(K.tw, std::max(2u, (x.max_cnt + 63u) / 64u));
    WideDict* wd = nullptr;
    if (int s = wide_dict_create(ctx, x, tw, &wd)) return s;
    laspj_etf_dict* g = nullptr;
    if (int s = laspj_etf_dict_create(ctx, n, x.eblob.data(), x.eoff.data(), x.eorder.data(),
                                      nullptr, nullptr, nullptr, &g)) {
        wide_dict_destroy(wd);
        return s;
    }
    free_etf(K);
    K.wd = wd;
    K.etf = g;
    K.E = n;
    K.tw = tw;
    K.stale = false;
    K.built_K = n;
    {
        std::vector<uint32_t> gone;
        dict_take_dirty(K.dict, &gone);
    }
    ++S->stats[4];
    S->stats[13] += now_ns() - t0;
    return LASPJ_OK;
}

// the namespace takes elements of more than 64 tokens from now on (its cells widen on
// their next use; slots are unchanged, so nothing is written out)
// (false: the namespace stays narrow — its token images are not of one length, which the
// wide templates need)
bool go_wide(NifState* S, KindState& K) {
    if (K.wide) return true;
    if (K.kind != LASPJ_KIND_ORSET || !K.dict) return false;
    if (!dict_set_tok_cap(K.dict, kWideTokens, kWideTokenLen)) return false;
    K.wide = true;
    K.stale = true;
    ++S->stats[19];
    return true;
}

int rebuild_etf(laspj_ctx* ctx, NifState* S, KindState& K) {
    if (K.wide && dict_elements(K.dict) == 0) {
        // (every registration that widened it was refused: narrow again)
        dict_set_tok_cap(K.dict, 64, 0);
        K.wide = false;
        K.tw = 1;
    }
    if (K.wide) return rebuild_wide(ctx, S, K);
    const uint64_t t0 = now_ns();
    uint32_t n = 0;
    uint64_t eb = 0, tb = 0;
    if (laspj_dict_info(K.dict, &n, &eb, &tb) != LASPJ_OK)
        return fail(ctx, LASPJ_E_INVAL, "nif: dictionary info");
    // head-room: registrations are append-only, so a larger E holds the next terms
    uint32_t E = K.E;
    if (!K.etf || n > E) E = n + n / 4 + 64;
    const bool toks = K.kind == LASPJ_KIND_ORSET;
    // (the context's arrays, grown only: the export writes every entry it hands on)
    auto fit = [](auto& v, uint64_t n) {
        if (v.size() < n) v.resize(n + n / 4);
        return v.data();
    };
    uint8_t* ebl = fit(S->x_ebl, eb + 1);
    uint8_t* tbl = fit(S->x_tbl, toks ? tb + 1 : 1);
    uint8_t* tord = fit(S->x_tord, toks ? 64ull * E : 1);
    uint32_t* eoff = fit(S->x_eoff, E + 1ull);
    uint32_t* eord = fit(S->x_eord, E);
    uint32_t* toff = fit(S->x_toff, toks ? 64ull * E + 1 : 1);
    if (laspj_dict_export(K.dict, E, ebl, eoff, eord, toks ? tbl : nullptr,
                          toks ? toff : nullptr, toks ? tord : nullptr) != LASPJ_OK)
        return fail(ctx, LASPJ_E_INVAL, "nif: dictionary export");
    free_etf(K);
    laspj_etf_dict* d = nullptr;
    // OR-Sets: two tokens of headroom per element, so a call that only adds tokens to
    // known elements patches the images (patch_etf) instead of coming back here
    if (int s = toks ? etf_dict_create_ex(ctx, E, ebl, eoff, eord, tbl, toff, tord, 2, &d)
                     : laspj_etf_dict_create(ctx, E, ebl, eoff, eord, nullptr, nullptr,
                                             nullptr, &d))
        return s;
    K.etf = d;
    K.E = E;
    K.stale = false;
    K.built_K = n;
    {
        std::vector<uint32_t> gone;
        dict_take_dirty(K.dict, &gone);             // (the rebuild holds every token)
    }
    K.built_cnt.resize(n);
    for (uint32_t e = 0; e < n; ++e) K.built_cnt[e] = toks ? dict_token_count(K.dict, e) : 0;
    ++S->stats[4];
    S->stats[13] += now_ns() - t0;
    return LASPJ_OK;
}

// Registrations that only added tokens to elements the images already hold: their rows
// patched in place.  False: rebuild (new elements, an element past its headroom, ...).
bool patch_etf(laspj_ctx* ctx, NifState* S, KindState& K) {
    if (!K.etf || K.kind != LASPJ_KIND_ORSET || K.wide) return false;
    const uint64_t t0 = now_ns();
    const uint32_t n = dict_elements(K.dict);
    if (n != K.built_K || n > K.E) return false;
    // the slots the dictionary saw gain tokens (no scan over every element)
    std::vector<uint32_t> seen, dirty;
    dict_take_dirty(K.dict, &seen);
    std::sort(seen.begin(), seen.end());
    seen.erase(std::unique(seen.begin(), seen.end()), seen.end());
    for (uint32_t e : seen)
        if (e < n && dict_token_count(K.dict, e) != K.built_cnt[e]) dirty.push_back(e);
    if (!dirty.empty() &&
        etf_dict_patch(ctx, K.etf, K.dict, dirty.data(), (uint32_t)dirty.size()) != LASPJ_OK)
        return false;
    for (uint32_t e : dirty) K.built_cnt[e] = dict_token_count(K.dict, e);
    K.stale = false;
    ++S->stats[14];
    S->stats[13] += now_ns() - t0;
    return true;
}

void release_cells(laspj_ctx* ctx, laspj_var* v) {
    if (v->cells) dev_release(ctx, v->cells, v->cell_bytes);
    v->cells = nullptr;
    v->cell_bytes = 0;
    v->E = 0;
    v->tw = 1;
}

// a variable's cells widened to the dictionary's E (slots are append-only: the old cells
// stay where they are, the new slots start absent); call with ctx->mu held
int fit_var(laspj_ctx* ctx, laspj_var* v, uint32_t E, uint32_t tw = 1) {
    if (v->cells && v->E == E && v->tw == tw) return LASPJ_OK;
    const uint64_t wnew = wpr_of(v->kind, E, tw), wold = v->cells ? wpr_of(v->kind, v->E, v->tw) : 0;
    const uint64_t bytes = std::max<uint64_t>(8ull * wnew, 256);
    void* p = nullptr;
    if (dev_alloc(ctx, bytes, &p) != hipSuccess) {
        hipGetLastError();
        return fail(ctx, LASPJ_E_NOMEM, "nif: variable cells (%llu bytes)",
                    (unsigned long long)bytes);
    }
    uint64_t* c = static_cast<uint64_t*>(p);
    if (v->kind == LASPJ_KIND_ORSET && (tw != 1 || (v->cells && v->tw != 1))) {
        // pairs per element change (a namespace gone wide): re-laid, slot for slot
        LJ_HIP(ctx, launch_relay(ctx, c, v->cells, v->cells ? v->E : 0, v->cells ? v->tw : 1, E, tw));
    } else {
        const uint64_t keep = std::min(wold, wnew);
        if (keep) LJ_HIP(ctx, hipMemcpyAsync(c, v->cells, 8ull * keep, hipMemcpyDeviceToDevice,
                                             ctx->stream));
        if (wnew > keep)
            LJ_HIP(ctx, hipMemsetAsync(c + keep, 0, 8ull * (wnew - keep), ctx->stream));
    }
    release_cells(ctx, v);
    v->cells = c;
    v->cell_bytes = bytes;
    v->E = E;
    v->tw = tw;
    return LASPJ_OK;
}

// One device pass: stage, pull, decode (or upload host-encoded cells), answer, one
// synchronisation.  Fills c.st / c.res / c.ooff / c.obase.

int device_pass(laspj_ctx* ctx, NifState* S, Call& c) {
    const uint64_t t0 = now_ns();
    uint64_t t_copy = 0;
    const uint32_t m = c.m, n = c.n;
    const size_t G = c.groups.size();
    // single-group ops (every op but BIND / WRITE) answer over group 0's dictionary
    KindState& K = *c.groups[0].K;
    const uint32_t E = K.E, TW = ktw(K);
    const bool orset = c.kind == LASPJ_KIND_ORSET;
    const bool wide = orset && K.wide;            // (single-group ops: answers by the wide codec)
    bool dec = m != 0;
    // (a wide namespace's operands are encoded by the host dictionary: dict_encode_cells)
    for (const Group& g : c.groups)
        if (orset && g.p1 > g.p0 && (g.K->wide || !etf_dict_decodable(g.K->etf))) dec = false;
    const bool var_op = c.op == Op::BIND || c.op == Op::WRITE;
    const bool var_in = var_op || c.op == Op::THRESHOLD || c.op == Op::READ || c.op == Op::VVALUE;
    std::vector<unsigned long long> hoffs(m + 1ull, 0);
    for (uint32_t i = 0; i < m; ++i) hoffs[i + 1] = hoffs[i] + c.len[i];
    const uint64_t pay = hoffs[m];
    // per group: its operand cells (words into the cell area: its payloads' replicas at its
    // own width)
    std::vector<uint64_t> gseg(G, 0), gcell(G, 0);
    std::vector<EtfGroup> eg(G);
    uint64_t seg_area = 0, in_words = 0;
    for (size_t g = 0; g < G; ++g) {
        const Group& gr = c.groups[g];
        gcell[g] = in_words;
        in_words += (uint64_t)(gr.p1 - gr.p0) * wpr_of(c.kind, gr.K->E, ktw(*gr.K));
        eg[g] = EtfGroup{gr.K->etf, gr.p0, gr.p1, nullptr, gr.K->E};
    }
    // several namespaces' OR-Set payloads: one decode launch over all of them (a table of
    // the dictionaries rides in the in region) with one plan, else group by group, each
    // with its own plan and segment table
    bool any_wide = false;
    for (const Group& g : c.groups) any_wide |= orset && g.K->wide;
    const bool multi = G > 1 && dec && orset && !any_wide &&
                       etf_multi_fill(ctx, eg.data(), (uint32_t)G, m, nullptr);
    std::vector<EtfReadPlan> plans(multi ? 1 : G);
    for (size_t g = 0; g < plans.size(); ++g) {
        const Group& gr = c.groups[g];
        const uint32_t p0 = multi ? 0 : gr.p0, R = multi ? m : gr.p1 - gr.p0;
        if (dec && orset && R && !gr.K->wide)
            etf_read_plan(ctx, gr.K->etf, R, hoffs.data() + p0, &plans[g]);
        gseg[g] = seg_area;
        if (plans[g].nseg) seg_area += al(4ull * (R + 1), 16);
    }
    const EtfReadPlan& plan = plans[0];
    const uint64_t mtab_bytes = multi ? al(etf_multi_bytes((uint32_t)G, m), 256) : 0;
    const bool has_payload_out = c.op == Op::MERGE || c.op == Op::VALUE || c.op == Op::READ ||
                                 c.op == Op::VVALUE;
    const uint64_t W = wpr_of(c.kind, E, TW);        // words per replica (single-group ops)
    // in region (host -> device)
    // [offsets | segment tables | zeroed words: the size pass's ticket, the decoders' redo
    //  lists, the one-launch merge's look-back words, the variable kernel's difference words
    //  and ticket | variable cell pointers, operand cell pointers, widths | the decode
    //  table of several dictionaries | payloads]
    const uint64_t i_offs = 0, i_seg = al(8ull * (m + 1), 256),
                   i_zero = i_seg + al(seg_area, 256),
                   z_lb = al(4ull * (m + G + 2), 16), z_var = z_lb + 8ull * ((E + 255) / 256),
                   z_nt = z_var + 4ull * (n + 1), z_bytes = z_nt + 4,
                   i_vptr = i_zero + al(z_bytes, 256),
                   i_mtab = i_vptr + (var_op ? al(24ull * n, 256) : 0),
                   i_pay = i_mtab + mtab_bytes;
    const uint64_t cells_in = in_words * 8ull;
    const uint64_t in_bytes = i_pay + (dec ? al(pay + 64, 256) : al(cells_in, 256));
    // out region: written by kernels into the pinned staging
    const uint64_t o_st = 0, o_res = al(4ull * m, 16), o_ooff = o_res + al(n, 16),
                   o_seg = o_ooff + al(8ull * (n + 1), 16);
    uint64_t o_pay = o_seg;          // (after the segment results of a deferred decode)
    // answer payload bound: a merge's image is at most both operands' (flags may be
    // re-encoded one byte longer than a SMALL_ATOM_UTF8 input: the slack, and a second
    // pass when even that is short); value/1's at most its operand's; a variable's image
    // is bounded by nothing the call knows (a second pass when the area is short)
    uint64_t bound = 64ull * n + 64;
    for (uint32_t i = 0; i < m; ++i) bound += c.len[i];
    if (has_payload_out && S->ocap < bound + bound / 8) S->ocap = al(bound + bound / 8, 1 << 16);
    const uint64_t ocap = has_payload_out ? S->ocap : 0;
    // MERGE: the segment decoder's chain check rides on the join's launch (ChainJob), its
    // per-segment results in a device area of their own after the in region
    // (one plan only: the join / bind launch carries one chain check)
    const bool defer = (G == 1 || multi) && dec && orset && plan.nseg && !c.no_defer &&
                       !c.write_only &&
                       ((c.op == Op::MERGE && etf_merge_fused(ctx, n, E)) || var_op ||
                        (c.op == Op::VALUE && etf_value_direct(ctx, n, E)));
    const uint64_t seg_bytes = defer ? al(plan.nseg * kSegResBytes, 256) : 0;
    o_pay += seg_bytes;              // (a failed payload's results, written by its chain check)
    // one operand over binary tokens (a bind, write/4, a threshold, value/1 — no answer
    // carries token images): tokens the namespace has not seen are taken by the decoder
    // (NewTok entries into the answer area, registered by run())
    const bool nt_merge = c.op == Op::MERGE && n == 1 && m == 2 &&
                          etf_merge_write_one(ctx, K.etf, n, E);
    const bool nt_on = (((var_op || c.op == Op::THRESHOLD || c.op == Op::VALUE) && m == 1) ||
                        nt_merge) &&
                       G == 1 && orset && !K.wide && dec && !c.redo.n && !c.write_only &&
                       !c.no_newtok && etf_dict_bin_tokens(K.etf);
    const uint64_t o_nt = o_pay, nt_bytes = nt_on ? al(sizeof(NewTok) * kNewTokCap, 256) : 0;
    o_pay += nt_bytes;
    const uint64_t out_bytes = o_pay + ocap;
    // device statuses of the variable calls (their kernel reads them)
    const uint64_t vst_bytes = var_op ? al(4ull * m, 256) : 0;
    // cells: in batch m x W words; MERGE: answers n x W; VALUE / VVALUE: value words
    const uint64_t VW = (E + 63ull) / 64ull;
    const uint64_t cells_out = c.op == Op::MERGE ? (uint64_t)n * W * 8ull
                               : (c.op == Op::VALUE || c.op == Op::VVALUE) ? (uint64_t)n * VW * 8ull
                                                                            : 0;
    const uint64_t c_out = al(cells_in, 256);
    {
        Guard g(ctx);
        if (int s = grow_dev(ctx, &S->dblk, &S->dblk_bytes,
                             al(in_bytes, 256) + seg_bytes + vst_bytes))
            return s;
        const uint64_t had = S->dcells_bytes;
        if (int s = grow_dev(ctx, &S->dcells, &S->dcells_bytes, c_out + cells_out + 256)) return s;
        if (S->dcells_bytes != had) S->clean_words = 0;
        if (int s = grow_host(ctx, &S->hin, &S->hin_bytes, in_bytes)) return s;
        if (int s = grow_host(ctx, &S->hout, &S->hout_bytes, out_bytes)) return s;
        // the staging's device addresses (looked up once per allocation: the runtime's
        // lookup costs host microseconds)
        void* hd = nullptr;
        if (S->hin_dkey != S->hin) {
            LJ_HIP(ctx, hipHostGetDevicePointer(&hd, S->hin, 0));
            S->hin_d = static_cast<uint8_t*>(hd);
            S->hin_dkey = S->hin;
        }
        if (S->hout_dkey != S->hout) {
            LJ_HIP(ctx, hipHostGetDevicePointer(&hd, S->hout, 0));
            S->hout_d = static_cast<uint8_t*>(hd);
            S->hout_dkey = S->hout;
        }
        if (var_in)
            for (laspj_var* v : c.vars)
                if (int s = fit_var(ctx, v, v->ns->E, v->ns->wide ? v->ns->tw : 1)) return s;
    }
    uint8_t* hin = static_cast<uint8_t*>(S->hin);
    uint8_t* din = static_cast<uint8_t*>(S->dblk);
    // a group commit's waiters staged their payloads into pinned blocks of their own while
    // they waited: gathered to their offsets by the device (k_nif_gather), launched before
    // the host builds the rest of the pass
    const bool gathered = dec && !c.redo.n && !c.write_only &&
                          std::any_of(c.pre.begin(), c.pre.end(),
                                      [](const uint8_t* x) { return x != nullptr; });
    GatherArgs ga{};
    uint32_t ng = 0;
    uint64_t most = 0;
    auto gather = [&]() -> int {
        if (!ng) return LASPJ_OK;
        // (one wave step of 2 KiB per wave, 8 KiB per block)
        const uint64_t blocks = std::min<uint64_t>((most + 8191) / 8192, (uint64_t)ctx->cus);
        hipLaunchKernelGGL(k_nif_gather, dim3((unsigned)std::max<uint64_t>(blocks, 1), ng),
                           dim3(256), 0, ctx->stream, ga, din + i_pay);
        LJ_LAUNCHED(ctx);
        ng = 0;
        most = 0;
        return LASPJ_OK;
    };
    if (gathered) {
        Guard g(ctx);
        for (uint32_t i = 0; i < m; ++i) {
            if (!c.len[i] || !c.pre[i]) continue;
            ga.d[ng++] = GatherDesc{c.pre[i], hoffs[i], c.len[i]};
            most = std::max(most, c.len[i]);
            if (ng == kGatherMax)
                if (int s = gather()) return s;
        }
        if (int s = gather()) return s;
    }
    uint8_t* dseg = din + al(in_bytes, 256);          // deferred segment results
    int32_t* dvst = reinterpret_cast<int32_t*>(dseg + seg_bytes);   // variable calls' statuses
    uint8_t* rout = S->hout_d;                        // where kernels write the out region
    const uint8_t* hin_d = S->hin_d;
    uint64_t* cin = static_cast<uint64_t*>(S->dcells);
    uint64_t* cout = reinterpret_cast<uint64_t*>(static_cast<uint8_t*>(S->dcells) + c_out);
    std::memcpy(hin + i_offs, hoffs.data(), 8ull * (m + 1));
    for (size_t g = 0; g < plans.size(); ++g)
        if (plans[g].nseg)
            std::memcpy(hin + i_seg + gseg[g], plans[g].segbase.data(),
                        4ull * plans[g].segbase.size());
    if (multi) {
        for (size_t g = 0; g < G; ++g) eg[g].cells = static_cast<uint64_t*>(S->dcells) + gcell[g];
        etf_multi_fill(ctx, eg.data(), (uint32_t)G, m, hin + i_mtab);
    }
    std::memset(hin + i_zero, 0, z_bytes);
    uint64_t maxw = 0;                                // widest variable (the bind's chunks)
    if (var_op) {
        // per variable: its cells, its decoded operand's cells, their width
        for (size_t g = 0; g < G; ++g) {
            const Group& gr = c.groups[g];
            const uint64_t w = wpr_of(c.kind, gr.K->E, ktw(*gr.K));
            maxw = std::max(maxw, w);
            for (uint32_t i = gr.p0; i < gr.p1; ++i) {
                const uint64_t cur = reinterpret_cast<uint64_t>(c.vars[i]->cells);
                const uint64_t in = reinterpret_cast<uint64_t>(
                    static_cast<uint64_t*>(S->dcells) + gcell[g] + (uint64_t)(i - gr.p0) * w);
                std::memcpy(hin + i_vptr + 8ull * i, &cur, 8);
                std::memcpy(hin + i_vptr + 8ull * (n + i), &in, 8);
                std::memcpy(hin + i_vptr + 8ull * (2ull * n + i), &w, 8);
            }
        }
    }
    uint32_t* dticket = reinterpret_cast<uint32_t*>(din + i_zero);
    auto* dlb = reinterpret_cast<unsigned long long*>(din + i_zero + z_lb);
    uint32_t* dvdiff = reinterpret_cast<uint32_t*>(din + i_zero + z_var);
    const bool clean = S->clean_words >= in_words;
    std::vector<int32_t> hst;
    if (m && !dec) {
        // token images of several lengths (or no tokens yet): the host dictionaries encode
        // the cells (laspj_dict_encode), the device does the rest
        std::vector<uint8_t> blob(pay);
        for (uint32_t i = 0; i < m; ++i)
            if (c.len[i]) std::memcpy(blob.data() + hoffs[i], c.p[i], c.len[i]);
        hst.assign(m, 0);
        for (size_t g = 0; g < G; ++g) {
            const Group& gr = c.groups[g];
            if (gr.p1 == gr.p0) continue;
            if (int s = dict_encode_cells(gr.K->dict, c.kind, blob.data(),
                                          reinterpret_cast<const uint64_t*>(hoffs.data()) + gr.p0,
                                          gr.p1 - gr.p0, -1, gr.K->E, ktw(*gr.K),
                                          reinterpret_cast<uint64_t*>(hin + i_pay) + gcell[g],
                                          hst.data() + gr.p0))
                return fail(ctx, s, "nif: host encode failed (%d)", s);
        }
        ++S->stats[5];
    }
    {
        Guard g(ctx);
        // the head, then the payloads (or host-encoded cells) a piece at a time: each
        // piece's pull runs while the host stages the next
        uint64_t sent = 0;                   // region bytes already pulled
        auto send = [&](uint64_t upto) -> int {
            // 16-byte lanes: sent is a multiple of 16 (the head is 256-aligned, pieces
            // 4096-multiples), upto is rounded up inside the staged region
            const uint64_t n16 = (al(upto, 16) - sent) / 16;
            if (!n16) return LASPJ_OK;
            const uint64_t blocks = std::min<uint64_t>((n16 + 255) / 256, (uint64_t)ctx->cus * 4);
            hipLaunchKernelGGL(k_nif_pull, dim3((unsigned)std::max<uint64_t>(blocks, 1)),
                               dim3(256), 0, ctx->stream,
                               reinterpret_cast<const pull16*>(hin_d + sent),
                               reinterpret_cast<pull16*>(din + sent), n16);
            LJ_LAUNCHED(ctx);
            sent = al(upto, 16);
            return LASPJ_OK;
        };
        if (dec && (c.redo.n || c.write_only)) {
            // (a redo or write-only pass: the head and payloads the last pass pulled are
            // still there)
        } else if (gathered) {
            // the head, then the payloads not staged by their callers (the leader's own)
            // copied into the staging and gathered to their offsets (the staged ones are
            // on their way since the region was allocated)
            if (int s = send(i_pay)) return s;
            for (uint32_t i = 0; i < m; ++i) {
                if (!c.len[i] || c.pre[i]) continue;
                const uint64_t tc = now_ns();
                std::memcpy(hin + i_pay + hoffs[i], c.p[i], c.len[i]);
                t_copy += now_ns() - tc;
                ga.d[ng++] = GatherDesc{hin_d + i_pay + hoffs[i], hoffs[i], c.len[i]};
                most = std::max(most, c.len[i]);
                if (ng == kGatherMax)
                    if (int s = gather()) return s;
            }
            if (int s = gather()) return s;
        } else if (dec) {
            uint64_t at = 0;
            uint32_t i = 0;
            uint64_t io = 0;                     // offset inside payload i
            while (i < m && c.len[i] == 0) ++i;
            while (at < pay) {
                const uint64_t piece = std::min(kPullPiece, pay - at);
                uint64_t done = 0;
                const uint64_t tc = now_ns();
                while (done < piece) {
                    const uint64_t take = std::min(piece - done, c.len[i] - io);
                    std::memcpy(hin + i_pay + at + done, c.p[i] + io, take);
                    done += take;
                    io += take;
                    if (io == c.len[i]) {
                        ++i;
                        io = 0;
                        while (i < m && c.len[i] == 0) ++i;
                    }
                }
                t_copy += now_ns() - tc;
                at += piece;
                if (int s = send(i_pay + at)) return s;
            }
            if (pay == 0)
                if (int s = send(i_pay)) return s;
        } else {
            // the head and (when there are operands) the host-encoded cells
            if (int s = send(i_pay)) return s;
            if (m) LJ_HIP(ctx, hipMemcpyAsync(cin, hin + i_pay, cells_in, hipMemcpyHostToDevice,
                                              ctx->stream));
        }
        laspj_batch inb = view(ctx, c.kind, m, E, cin, TW);
        // statuses: straight into the pinned answer, or (variable calls) device memory their
        // kernel reads and publishes
        int32_t* dst = var_op ? dvst : reinterpret_cast<int32_t*>(rout + o_st);
        ChainJob cjob;
        if (defer) {
            cjob.res = dseg;
            cjob.hres = rout + o_seg;
        }
        if (c.write_only) {
            // (the operands' cells the last pass decoded are still there)
        } else if (dec && multi) {
            // every namespace's payloads in one launch (the cells zeroed first when the last
            // call left them dirty: the decoders only set what they decode)
            if (!clean && !c.redo.n) LJ_HIP(ctx, hipMemsetAsync(cin, 0, cells_in, ctx->stream));
            if (int s = etf_read_multi_enqueue(
                    ctx, eg.data(), (uint32_t)G, din + i_mtab, m, din + i_pay, pay,
                    reinterpret_cast<const unsigned long long*>(din + i_offs), plan,
                    plan.nseg ? reinterpret_cast<const uint32_t*>(din + i_seg) : nullptr, dst,
                    defer ? &cjob : nullptr, c.redo.n ? &c.redo : nullptr))
                return s;
        } else if (dec) {
            // each group's payloads against its own dictionary (offsets are absolute in the
            // payload area, so a group reads its slice of them in place)
            for (size_t g = 0; g < G; ++g) {
                const Group& gr = c.groups[g];
                const uint32_t R = gr.p1 - gr.p0;
                if (!R) continue;
                laspj_batch gb = view(ctx, c.kind, R, gr.K->E, cin + gcell[g]);
                const auto* doffs = reinterpret_cast<const unsigned long long*>(din + i_offs) + gr.p0;
                NewTokArgs nta;
                if (nt_on) {
                    if (!++S->nt_seq) ++S->nt_seq;           // (0 never tags an entry)
                    nta = NewTokArgs{reinterpret_cast<uint32_t*>(din + i_zero + z_nt),
                                     reinterpret_cast<NewTok*>(rout + o_nt), kNewTokCap,
                                     S->nt_seq};
                }
                if (orset) {
                    if (int s = etf_read_enqueue(
                            ctx, &gb, gr.K->etf, -1, 1, din + i_pay, pay, doffs, plans[g],
                            plans[g].nseg ? reinterpret_cast<const uint32_t*>(din + i_seg + gseg[g])
                                          : nullptr,
                            dst + gr.p0, !clean && !c.redo.n, dticket + 1 + gr.p0 + g,
                            defer ? &cjob : nullptr, c.redo.n ? &c.redo : nullptr,
                            nt_on ? &nta : nullptr))
                        return s;
                } else if (int s = gset_read_enqueue(ctx, &gb, gr.K->etf, -1, 1, din + i_pay, doffs,
                                                     dst + gr.p0, !clean, hoffs.data() + gr.p0)) {
                    return s;
                }
            }
        } else if (m && var_op) {
            LJ_HIP(ctx, hipMemcpyAsync(dvst, hst.data(), 4ull * m, hipMemcpyHostToDevice,
                                       ctx->stream));
        }
        laspj_batch lhs = view(ctx, c.kind, n, E, cin, TW);
        laspj_batch rhs = view(ctx, c.kind, n, E, cin + (uint64_t)n * W, TW);
        auto* dooff = reinterpret_cast<unsigned long long*>(rout + o_ooff);
        uint8_t* dopay = rout + o_pay;
        switch (c.op) {
        case Op::MERGE: {
            // lasp_orset:merge/2 (lasp_orset.erl:128-134): the nested orddict:merge of two
            // canonical orddicts is the slot-wise OR of their cells; lasp_gset:merge/2
            // (lasp_gset.erl:99-101): ordsets:union of two ordsets, the OR of their bits
            laspj_batch ob = view(ctx, c.kind, n, E, cout, TW);
            const unsigned long long* chunks = nullptr;
            if (wide) {
                // elements past 64 tokens: the OR, then the wide size pass and writer
                LJ_HIP(ctx, launch_or(ctx, cout, lhs.dev, rhs.dev, (uint64_t)n * W));
                if (int s = wide_size_enqueue(ctx, K.wd, cout, n, -1, dooff, ctx->flag)) return s;
                if (int s = wide_write_enqueue(ctx, K.wd, cout, n, -1, 1, dooff, dopay, ocap))
                    return s;
                S->clean_words = 0;
                break;
            }
            if (orset && etf_merge_write_one(ctx, K.etf, n, E)) {
                // one answer: join, size pass and writer in one launch (look-back), the
                // operands cleared behind it, the chain checks riding along
                if (int s = etf_merge_write_enqueue(
                        ctx, lhs.dev, rhs.dev, E, K.etf, -1, 1, dooff, dopay, ocap, dlb, dticket,
                        &cjob,
                        nt_on ? reinterpret_cast<const uint32_t*>(din + i_zero + z_nt) : nullptr))
                    return s;
                S->clean_words = in_words;
                break;
            }
            if (!orset && etf_value_direct(ctx, n, E)) {
                // few long G-Set answers: written from both operands' bits
                if (int s = etf_gset_merge_write_enqueue(ctx, &lhs, &rhs, K.etf, -1, 1, dooff,
                                                         ctx->flag, dopay, ocap))
                    return s;
                S->clean_words = 0;
                break;
            }
            if (orset && etf_merge_fused(ctx, n, E)) {
                // the OR fused with the answer's size pass, the operands cleared behind it
                if (int s = etf_merge_size_enqueue(ctx, lhs.dev, rhs.dev, &ob, K.etf, -1, dooff,
                                                   ctx->flag, dticket, &chunks, &cjob))
                    return s;
                S->clean_words = in_words;
            } else {
                LJ_HIP(ctx, launch_or(ctx, cout, lhs.dev, rhs.dev, (uint64_t)n * W));
                if (int s = etf_size_enqueue(ctx, &ob, K.etf, c.kind, -1, dooff, ctx->flag,
                                             &chunks))
                    return s;
                S->clean_words = 0;
            }
            if (int s = etf_write_enqueue(ctx, &ob, K.etf, c.kind, -1, 1, dooff, dopay, ocap,
                                          chunks))
                return s;
            break;
        }
        case Op::VALUE:
        case Op::VVALUE: {
            // value/1 (lasp_orset.erl:67-73): the elements with a {_, false} token, as the
            // ordset image the G-Set writer gives a bit row (term_to_binary of the keys)
            // (VVALUE has no operand cells: its value bits land where they would start)
            laspj_batch src = c.op == Op::VALUE ? inb : view(ctx, c.kind, 1, E, c.vars[0]->cells, TW);
            if (wide) {
                // the value bits of the wide cells, then the G-Set writer over the element images
                S->clean_words = 0;
                LJ_HIP(ctx, launch_wide_value(ctx, &src, cout, false));
                laspj_batch vb = view(ctx, LASPJ_KIND_GSET, n, E, cout);
                const unsigned long long* chunks = nullptr;
                if (int s = etf_size_enqueue(ctx, &vb, K.etf, LASPJ_KIND_GSET, -1, dooff, ctx->flag,
                                             &chunks))
                    return s;
                if (int s = etf_write_enqueue(ctx, &vb, K.etf, LASPJ_KIND_GSET, -1, 1, dooff, dopay,
                                              ocap, chunks))
                    return s;
                break;
            }
            if (c.kind == LASPJ_KIND_ORSET && etf_value_direct(ctx, n, E)) {
                // few long answers: written from the cells (no value bits in between), a
                // decoded operand's cells cleared behind the reads
                if (int s = etf_value_write_enqueue(ctx, &src, K.etf, -1, 1, dooff, ctx->flag,
                                                    dopay, ocap, c.op == Op::VALUE, &cjob))
                    return s;
                S->clean_words = c.op == Op::VALUE ? in_words : S->clean_words;
                break;
            }
            S->clean_words = 0;
            LJ_HIP(ctx, launch_orset_value(ctx, &src, cout, false));
            laspj_batch vb = view(ctx, LASPJ_KIND_GSET, n, E, cout);
            const unsigned long long* chunks = nullptr;
            if (int s = etf_size_enqueue(ctx, &vb, K.etf, LASPJ_KIND_GSET, -1, dooff, ctx->flag,
                                         &chunks))
                return s;
            if (int s = etf_write_enqueue(ctx, &vb, K.etf, LASPJ_KIND_GSET, -1, 1, dooff, dopay,
                                          ocap, chunks))
                return s;
            break;
        }
        case Op::READ: {
            // the variable's value as its term_to_binary image (#dv.value read back)
            laspj_batch vb = view(ctx, c.kind, 1, E, c.vars[0]->cells, TW);
            if (wide) {
                if (int s = wide_size_enqueue(ctx, K.wd, vb.dev, 1, -1, dooff, ctx->flag)) return s;
                if (int s = wide_write_enqueue(ctx, K.wd, vb.dev, 1, -1, 1, dooff, dopay, ocap))
                    return s;
                break;
            }
            const unsigned long long* chunks = nullptr;
            if (int s = etf_size_enqueue(ctx, &vb, K.etf, c.kind, -1, dooff, ctx->flag, &chunks))
                return s;
            if (int s = etf_write_enqueue(ctx, &vb, K.etf, c.kind, -1, 1, dooff, dopay, ocap,
                                          chunks))
                return s;
            break;
        }
        case Op::EQUAL:
            S->clean_words = 0;
            // equal/2 (lasp_orset.erl:136-138, lasp_gset.erl:103-105): A == B
            LJ_HIP(ctx, launch_equal(ctx, &lhs, &rhs, rout + o_res));
            break;
        case Op::INFLATION:
            S->clean_words = 0;
            // is_inflation / is_strict_inflation (lasp_lattice.erl:137-161, 212-253)
            LJ_HIP(ctx, wide ? launch_wide_inflation(ctx, &lhs, &rhs, c.strict != 0, rout + o_res)
                        : orset ? launch_orset_inflation(ctx, &lhs, &rhs, c.strict != 0, rout + o_res)
                              : launch_gset_inflation(ctx, &lhs, &rhs, c.strict != 0, rout + o_res));
            break;
        case Op::THRESHOLD: {
            // threshold_met(Type, Value, Threshold) (lasp_lattice.erl:62-75): is_(strict_)
            // inflation(Threshold, Value) with Value the resident cells
            S->clean_words = 0;
            laspj_batch cur = view(ctx, c.kind, 1, E, c.vars[0]->cells, TW);
            LJ_HIP(ctx, wide ? launch_wide_inflation(ctx, &lhs, &cur, c.strict != 0, rout + o_res)
                        : orset ? launch_orset_inflation(ctx, &lhs, &cur, c.strict != 0, rout + o_res)
                              : launch_gset_inflation(ctx, &lhs, &cur, c.strict != 0, rout + o_res));
            break;
        }
        case Op::BIND:
        case Op::WRITE: {
            // bind/3 (lasp_core.erl:291-312) / write/4 (:839-844) into the resident cells
            // (the segment decoder's chain check rides on this launch when deferred)
            if (int s = var_bind_enqueue(ctx, reinterpret_cast<uint64_t* const*>(din + i_vptr),
                                         reinterpret_cast<uint64_t* const*>(din + i_vptr + 8ull * n),
                                         reinterpret_cast<const uint64_t*>(din + i_vptr + 16ull * n),
                                         maxw, n, dvst, dvdiff, dvdiff + n, rout + o_res,
                                         reinterpret_cast<int32_t*>(rout + o_st),
                                         c.op == Op::WRITE, &cjob))
                return s;
            S->clean_words = in_words;
            break;
        }
        }
        const uint64_t t1 = now_ns();
        LJ_HIP(ctx, hipStreamSynchronize(ctx->stream));
        const uint64_t t2 = now_ns();
        ++S->stats[1];
        S->stats[8] += t1 - t0;
        S->stats[9] += t2 - t1;
        S->stats[11] += t_copy;
        const uint8_t* hout = static_cast<const uint8_t*>(S->hout);
        c.st.assign(m, 0);
        if (dec || var_op) std::memcpy(c.st.data(), hout + o_st, 4ull * m);
        else c.st = hst;
        c.newtoks.clear();
        c.nt_met = false;
        if (nt_on) {
            // the decoder's new tokens: the entries tagged with this pass, in the order the
            // device numbered them
            const NewTok* ents = reinterpret_cast<const NewTok*>(hout + o_nt);
            uint32_t k = 0;
            while (k < kNewTokCap && ents[k].seq == S->nt_seq) ++k;
            c.nt_met = k != 0;
            bool ok = true;
            for (uint32_t i = 0; i < m; ++i) ok &= c.st[i] == LASPJ_DEC_OK;
            if (k && ok) c.newtoks.assign(ents, ents + k);
            // (a merge's writer then wrote nothing and left the operands' cells)
            if (k && c.op == Op::MERGE) S->clean_words = 0;
        }
        if (var_op)
            for (int32_t x : c.st)
                if (x != LASPJ_DEC_OK) S->clean_words = 0;   // (its cells were kept)
        c.has_seg = false;
        if (defer && cjob.armed &&
            std::find(c.st.begin(), c.st.end(), (int32_t)LASPJ_DEC_UNKNOWN_TERM) != c.st.end()) {
            // (the chain checks copied the failed payloads' results into the answer area;
            // those of payloads that decoded are not read)
            c.segres.resize(8ull * plan.nseg);
            std::memcpy(c.segres.data(), hout + o_seg, kSegResBytes * plan.nseg);
            c.segbase = plan.segbase;
            c.segS = plan.S;
            c.has_seg = true;
        }
        c.res.assign(hout + o_res, hout + o_res + n);
        if (has_payload_out) {
            c.ooff.resize(n + 1ull);
            std::memcpy(c.ooff.data(), hout + o_ooff, 8ull * (n + 1));
            const uint64_t total = c.ooff[n];
            if (total > ocap) {
                // the writer wrote nothing: a larger answer area, the encode again
                S->ocap = al(total + total / 4, 1 << 16);
                return -1000;            // caller re-runs the pass
            }
            c.obase = hout + o_pay;
        }
        S->stats[10] += now_ns() - t2;
    }
    return LASPJ_OK;
}

int register_payloads(laspj_ctx* ctx, NifState* S, KindState& K,
                      const std::vector<const uint8_t*>& p, const std::vector<uint64_t>& len,
                      std::vector<int32_t>* st) {
    const uint64_t t0 = now_ns();
    const uint64_t k = p.size();
    std::vector<uint64_t> offs(k + 1, 0);
    for (uint64_t i = 0; i < k; ++i) offs[i + 1] = offs[i] + len[i];
    std::vector<uint8_t> blob(offs[k] + 1);
    for (uint64_t i = 0; i < k; ++i)
        if (len[i]) std::memcpy(blob.data() + offs[i], p[i], len[i]);
    st->assign(k, 0);
    if (int s = laspj_dict_add(K.dict, K.kind, blob.data(), offs.data(), k, -1, st->data()))
        return fail(ctx, s, "nif: dictionary registration failed (%d)", s);
    ++S->stats[2];
    S->stats[12] += now_ns() - t0;
    K.stale = true;
    return LASPJ_OK;
}

// A deferred pass's unknown terms: each failing segment of those operands (a status and a
// start: its first element, where the chain check found it) registers the elements that
// start in it — what the segment's decoder could not take; the segments that decoded hold
// known terms.  False: a range did not register (nothing is kept), the caller registers
// whole operands.
bool register_segments(NifState* S, const Call& c, const std::vector<uint32_t>& ops) {
    const uint64_t t0 = now_ns();
    struct Range {
        uint32_t i;
        uint64_t from, to;
    };
    std::vector<Range> rs;
    for (uint32_t i : ops) {
        if (i + 1 >= c.segbase.size()) return false;
        for (uint32_t g = c.segbase[i]; g < c.segbase[i + 1]; ++g) {
            const int32_t st = (int32_t)c.segres[8ull * g];
            const uint32_t start = c.segres[8ull * g + 1];
            if (st == LASPJ_DEC_OK) continue;
            if (start == 0xFFFFFFFFu) return false;
            const uint64_t s = g - c.segbase[i];
            rs.push_back({i, start, std::min<uint64_t>((s + 1) * c.segS, c.len[i])});
        }
    }
    if (rs.empty()) return false;
    for (const Range& r : rs) {
        // (the payload's group: its namespace's dictionary)
        size_t g = 0;
        while (g + 1 < c.groups.size() && r.i >= c.groups[g].p1) ++g;
        KindState& K = *c.groups[g].K;
        if (dict_add_elems(K.dict, c.p[r.i], c.len[r.i], r.from, r.to) != LASPJ_DEC_OK)
            return false;       // (ranges already added stay: they hold well-formed terms)
        K.stale = true;
    }
    ++S->stats[2];
    S->stats[12] += now_ns() - t0;
    return true;
}

int run(laspj_ctx* ctx, NifState* S, Call& c, std::vector<int32_t>* verdict);

// The tokens a pass's decoder took (NewTok): registered in the host dictionary at the
// slots the device gave them — each element's next free slots in payload order, which is
// the order the dictionary numbers them in; the device images learn them on the next call
// (patch_etf).  A slot the dictionary would number otherwise cannot happen by
// construction; it fails the call loudly (the cells already hold the device's slots).
int register_new_tokens(laspj_ctx* ctx, NifState* S, KindState& K, const Call& c,
                        bool* conflict) {
    const uint64_t t0 = now_ns();
    *conflict = false;
    std::vector<NewTok> ts = c.newtoks;
    std::sort(ts.begin(), ts.end(), [](const NewTok& a, const NewTok& b) {
        return a.e != b.e ? a.e < b.e : a.slot < b.slot;
    });
    const uint32_t TL = etf_dict_tok_len(K.etf);
    // an entry's image: offsets are into the call's payloads laid end to end
    auto image = [&](const NewTok& t) -> const uint8_t* {
        uint64_t at = 0;
        for (uint32_t i = 0; i < c.m; ++i) {
            if (t.off >= at && (uint64_t)t.off + TL <= at + c.len[i]) return c.p[i] + (t.off - at);
            at += c.len[i];
        }
        return nullptr;
    };
    // two operands of a merge may each take a token for one element: the same slot is
    // the same token (kept once) or a conflict (the caller decodes the usual way)
    std::vector<NewTok> uniq;
    for (size_t i = 0; i < ts.size(); ++i) {
        if (!uniq.empty() && uniq.back().e == ts[i].e && uniq.back().slot == ts[i].slot) {
            const uint8_t *x = image(uniq.back()), *y = image(ts[i]);
            if (!x || !y || std::memcmp(x, y, TL) != 0) {
                *conflict = true;
                return LASPJ_OK;
            }
            continue;
        }
        uniq.push_back(ts[i]);
    }
    dict_begin(K.dict);
    for (const NewTok& t : uniq) {
        uint32_t slot = 0;
        const uint8_t* img = image(t);
        const int st = img ? dict_reg_tok(K.dict, t.e, img, TL, &slot) : LASPJ_DEC_MALFORMED;
        if (st != LASPJ_DEC_OK || slot != t.slot) {
            dict_rollback(K.dict);
            return fail(ctx, LASPJ_E_DEVICE,
                        "nif: new token of element %u at slot %u registered as %u (%d)", t.e,
                        t.slot, slot, st);
        }
    }
    dict_begin(K.dict);                           // (the journal kept nothing)
    K.stale = true;                               // (patched on the next call)
    ++S->stats[2];
    S->stats[18] += uniq.size();
    S->stats[12] += now_ns() - t0;
    return LASPJ_OK;
}

// the call's payloads decoded against one dictionary
void one_group(Call& c, KindState* K) { c.groups.assign(1, Group{K, 0, c.m}); }

// the image of a resident variable (a READ pass; the caller holds S->mu)
int read_var(laspj_ctx* ctx, NifState* S, laspj_var* v, std::vector<uint8_t>* img) {
    Call c;
    c.op = Op::READ;
    c.kind = v->kind;
    c.n = 1;
    c.m = 0;
    c.vars.push_back(v);
    one_group(c, v->ns.get());
    std::vector<int32_t> vd;
    if (int s = run(ctx, S, c, &vd)) return s;
    if (vd[0] != LASPJ_NIF_OK) return fail(ctx, LASPJ_E_DEVICE, "nif: variable encode failed");
    img->assign(c.obase + c.ooff[0], c.obase + c.ooff[1]);
    return LASPJ_OK;
}

// Before a dictionary of this kind is dropped: every resident variable over it is written
// out to its image (encoded on the device with the dictionary its cells refer to) and its
// cells released; the next call that uses it decodes the image again (hydrate)
int spill_vars(laspj_ctx* ctx, NifState* S, KindState& K) {
    for (laspj_var* v : K.vars) {
        if (!v->resident || v->epoch != K.epoch) continue;
        if (!v->cells) {
            v->image.assign({131, 106});              // new() = []
        } else if (int s = read_var(ctx, S, v, &v->image)) {
            return s;
        }
        {
            Guard g(ctx);
            release_cells(ctx, v);
        }
        v->resident = false;
        ++S->stats[16];
    }
    return LASPJ_OK;
}

int reset_dict(laspj_ctx* ctx, NifState* S, KindState& K) {
    const bool had = K.dict != nullptr;       // (creating a namespace's first is no reset)
    if (had)
        if (int s = spill_vars(ctx, S, K)) return s;
    free_etf(K);
    if (K.dict) laspj_dict_destroy(K.dict);
    K.dict = nullptr;
    if (laspj_dict_create(&K.dict) != LASPJ_OK)
        return fail(ctx, LASPJ_E_NOMEM, "nif: dictionary allocation");
    K.stale = false;
    K.wide = false;                           // (a fresh dictionary starts narrow)
    K.tw = 1;
    ++K.epoch;
    if (had) ++S->stats[3];
    return LASPJ_OK;
}

// an operand met an element's 64 token slots all taken: the namespace goes wide (true: the
// caller registers the operands again)
bool widen(NifState* S, KindState& K, const std::vector<int32_t>& st) {
    if (K.wide || K.kind != LASPJ_KIND_ORSET) return false;
    for (int32_t x : st)
        if (x == LASPJ_DEC_UNREPRESENTABLE) return go_wide(S, K);
    return false;
}

// The call: device pass; operands with unknown terms registered and a second pass; every
// other undecodable operand -> FALLBACK.  verdict[j] per answer.
int run(laspj_ctx* ctx, NifState* S, Call& c, std::vector<int32_t>* verdict) {
    ++S->stats[0];
    const size_t G = c.groups.size();
    for (const Group& g : c.groups)
        if (!g.K->dict && reset_dict(ctx, S, *g.K)) return LASPJ_E_NOMEM;
    const uint32_t n = c.n, m = c.m;
    auto answer_of = [&](uint32_t i) { return i % n; };
    auto group_of = [&](uint32_t i) {
        size_t g = 0;
        while (g + 1 < G && i >= c.groups[g].p1) ++g;
        return g;
    };
    auto slice = [&](uint32_t p0, uint32_t p1, std::vector<const uint8_t*>* p,
                     std::vector<uint64_t>* l) {
        p->assign(c.p.begin() + p0, c.p.begin() + p1);
        l->assign(c.len.begin() + p0, c.len.begin() + p1);
    };
    // a variable call's operands are its own (payload i belongs to variable i): an element
    // past its 64 token slots widens the namespace's cells (k {p, r} pairs); only image
    // calls start a fresh dictionary for it, and only write/4 resets a dictionary grown past
    // its bound (bind / threshold answer FALLBACK there and the NIF runs the reference's
    // clause over the variable's read image)
    const bool may_reset = !(c.op == Op::BIND || c.op == Op::THRESHOLD);
    std::vector<uint8_t> fallback(n, 0);
    std::vector<uint8_t> registered(G, 0);
    bool partial = false;           // the last registration took the failing segments only
    bool resolved = false;          // the last pass's answers stand (statuses all final)
    const int passes = ctx->tune_nif_passes ? (int)ctx->tune_nif_passes : kMaxPasses;
    std::vector<const uint8_t*> rp;
    std::vector<uint64_t> rl;
    std::vector<int32_t> rst;
    std::vector<uint8_t> written;
    for (int pass = 0; pass < passes && !resolved; ++pass) {
        for (size_t g = 0; g < G; ++g) {
            KindState& K = *c.groups[g].K;
            if (K.etf && !K.stale) continue;
            const uint32_t p0 = c.groups[g].p0, p1 = c.groups[g].p1;
            if (!K.etf && p1 > p0) {
                // nothing registered yet: register this group's operands first
                slice(p0, p1, &rp, &rl);
                if (int s = register_payloads(ctx, S, K, rp, rl, &rst)) return s;
                if (widen(S, K, rst))
                    if (int s = register_payloads(ctx, S, K, rp, rl, &rst)) return s;
                registered[g] = 1;
                for (uint32_t i = p0; i < p1; ++i)
                    if (rst[i - p0] != LASPJ_DEC_OK) fallback[answer_of(i)] = 1;
            }
            // a wide namespace's operands are host-encoded: its device images serve the
            // answers' writers only, so a call that writes none keeps the stale ones
            // (while the cells' element slots and pairs still hold every term)
            if (K.wide && K.etf && dict_elements(K.dict) <= K.E &&
                dict_max_tokens(K.dict) <= 64u * K.tw && c.op != Op::MERGE &&
                c.op != Op::VALUE && c.op != Op::VVALUE && c.op != Op::READ)
                continue;
            if (!patch_etf(ctx, S, K)) {
                if (int s = rebuild_etf(ctx, S, K)) return s;
                c.redo.n = 0;         // (element ranks moved: the last pass's results stale)
            }
        }
        int s = device_pass(ctx, S, c);
        c.redo.n = 0;                 // (a redo pass is taken once)
        if (s == -1000) {
            // answer area grown: once more (a write-only pass's writer may have cleared
            // the operands: decode them again)
            if (c.write_only) {
                c.write_only = false;
                S->clean_words = 0;
            }
            continue;
        }
        if (s) return s;
        c.write_only = false;
        if (!c.newtoks.empty()) {
            KindState& K = *c.groups[0].K;
            bool conflict = false;
            if (int s2 = register_new_tokens(ctx, S, K, c, &conflict)) return s2;
            if (conflict) {
                // two operands gave one slot to different tokens: decode again the usual
                // way (registration, then a pass over the known terms)
                c.no_newtok = true;
                S->clean_words = 0;
                continue;
            }
            if (c.op == Op::MERGE) {
                // the answer needs the tokens' images: patch them in, then join and write
                // the cells the decoders left (a rebuild moves element slots: decode again)
                if (patch_etf(ctx, S, K)) {
                    c.write_only = true;
                } else {
                    if (int s2 = rebuild_etf(ctx, S, K)) return s2;
                    S->clean_words = 0;
                }
                continue;
            }
        }
        // a bind that decoded in this pass was merged in it: WRITTEN if this pass (or an
        // earlier one, for an operand whose call needed another pass) changed its value
        if (c.op == Op::BIND) {
            written.resize(n, 0);
            for (uint32_t i = 0; i < m; ++i)
                if (c.st[i] == LASPJ_DEC_OK) written[i] |= c.res[i];
        }
        bool redo = false;
        for (uint32_t i = 0; i < m; ++i) redo |= c.st[i] == kDecRedo;
        if (redo) {
            // a segment chain that only a serial decode can judge: once more, decoding
            // serially (the join's answer of this pass is not used)
            c.no_defer = true;
            ++S->stats[15];
            continue;
        }
        std::vector<uint32_t> unknown;
        for (uint32_t i = 0; i < m; ++i) {
            if (fallback[answer_of(i)]) continue;
            // (an element past a narrow namespace's 64 token slots: its registration widens
            // the namespace)
            const KindState& Ki = *c.groups[group_of(i)].K;
            const bool grow = c.st[i] == LASPJ_DEC_UNREPRESENTABLE &&
                              Ki.kind == LASPJ_KIND_ORSET && !Ki.wide;
            if ((c.st[i] == LASPJ_DEC_UNKNOWN_TERM || grow) &&
                (!registered[group_of(i)] || partial))
                unknown.push_back(i);
            else if (c.st[i] != LASPJ_DEC_OK)
                fallback[answer_of(i)] = 1;
        }
        if (unknown.empty()) {
            resolved = true;
            break;
        }
        bool fresh = true;            // no group of an unknown operand registered yet
        for (uint32_t i : unknown) fresh &= !registered[group_of(i)];
        if (fresh && c.has_seg && register_segments(S, c, unknown)) {
            // the failing segments' elements registered; if the next pass still meets an
            // unknown term, the whole operands are registered after all
            partial = true;
            for (uint32_t i : unknown) registered[group_of(i)] = 1;
            // a single bind: the next pass decodes only those segments again, over the
            // payload and cells this pass left (when the images are patched, not rebuilt)
            if (c.op == Op::BIND && n == 1 && !c.no_defer && !c.nt_met) {
                SegList sl;
                for (uint32_t i : unknown)
                    for (uint32_t g = c.segbase[i]; g < c.segbase[i + 1] && sl.n <= 31; ++g)
                        if ((int32_t)c.segres[8ull * g] != LASPJ_DEC_OK) {
                            if (sl.n < 31) sl.g[sl.n] = g;
                            ++sl.n;
                        }
                if (sl.n <= 31) c.redo = sl;
            }
            continue;
        }
        partial = false;
        // terms a dictionary has not seen (or operands that are not orddicts, which the
        // second pass tells apart): each group registers its operands that met them (an
        // operand that decoded holds only registered terms)
        for (size_t g = 0; g < G; ++g) {
            KindState& K = *c.groups[g].K;
            const uint32_t p0 = c.groups[g].p0, p1 = c.groups[g].p1;
            std::vector<uint32_t> ri;
            rp.clear();
            rl.clear();
            for (uint32_t i : unknown)
                if (i >= p0 && i < p1) {
                    rp.push_back(c.p[i]);
                    rl.push_back(c.len[i]);
                    ri.push_back(i);
                }
            if (ri.empty()) continue;
            uint32_t nd = 0;
            uint64_t eb, tb;
            if (int s2 = register_payloads(ctx, S, K, rp, rl, &rst)) return s2;
            bool full = false;
            for (int32_t x : rst) full |= x == LASPJ_DEC_UNREPRESENTABLE;
            laspj_dict_info(K.dict, &nd, &eb, &tb);
            // image calls own their namespace's terms for the call only: a wide one starts
            // over narrow when it meets new terms (the narrow codec is the fast one)
            const bool image_call = c.vars.empty();
            if (may_reset && ((image_call && ((full && nd) || K.wide)) || nd > kMaxDictElements)) {
                // an element's 64 token slots used up by earlier calls (or a dictionary grown
                // past its bound): start a fresh dictionary holding this group's terms only —
                // image calls are self-contained (images in, images out); the namespace's
                // resident variables are written out to their images first and decoded again
                // when next used
                if (int s2 = reset_dict(ctx, S, K)) return s2;
                slice(p0, p1, &rp, &rl);
                if (int s2 = register_payloads(ctx, S, K, rp, rl, &rst)) return s2;
                // (an operand of more than 64 tokens on an element even so: wide)
                if (widen(S, K, rst))
                    if (int s2 = register_payloads(ctx, S, K, rp, rl, &rst)) return s2;
                for (uint32_t i = p0; i < p1; ++i)
                    if (rst[i - p0] != LASPJ_DEC_OK) fallback[answer_of(i)] = 1;
                for (uint32_t i = p0; i < p1 && i < c.vars.size(); ++i) {
                    c.vars[i]->epoch = K.epoch;           // write/4's own variable: new cells
                    c.vars[i]->resident = true;
                }
            } else {
                // a variable's namespace (its replicas' cells hold its slots) goes wide
                // rather than start over
                if (widen(S, K, rst))
                    if (int s2 = register_payloads(ctx, S, K, rp, rl, &rst)) return s2;
                for (size_t k = 0; k < ri.size(); ++k)
                    if (rst[k] != LASPJ_DEC_OK) fallback[answer_of(ri[k])] = 1;
            }
            registered[g] = 1;
        }
    }
    // post-condition: an answer is OK only from a pass whose statuses were all final; a
    // call whose passes ran out (the answer area grown, a segment chain only a serial
    // decode judges, terms registered — each on the last pass) hands every operand to the
    // reference's clause rather than answer from a superseded pass
    if (c.op == Op::BIND && written.size() == n) c.res = written;
    verdict->assign(n, LASPJ_NIF_OK);
    for (uint32_t j = 0; j < n; ++j)
        if (fallback[j] || !resolved) {
            (*verdict)[j] = LASPJ_NIF_FALLBACK;
            ++S->stats[6];
        }
    return LASPJ_OK;
}

NifState* state(laspj_ctx* ctx) {
    // (without ctx->mu once it exists: a device phase holds that lock, and binds arriving
    // meanwhile must reach the group-commit queue, not wait behind it)
    if (NifState* s = __atomic_load_n(&ctx->nif, __ATOMIC_ACQUIRE)) return s;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (!ctx->nif) {
        NifState* s = new (std::nothrow) NifState;
        if (s) s->ks[1].kind = LASPJ_KIND_GSET;
        __atomic_store_n(&ctx->nif, s, __ATOMIC_RELEASE);
    }
    return ctx->nif;
}

// A variable whose value sits in its host image (written out by a dictionary reset) gets
// cells again: write/4 of that image.  *ok: the variable is resident over the current
// dictionary (false: it stays host-held; its calls answer FALLBACK)
int hydrate(laspj_ctx* ctx, NifState* S, laspj_var* v, bool* ok) {
    KindState& K = *v->ns;
    *ok = v->resident && v->epoch == K.epoch;
    // (a value write/4 could not represent stays an image until the next write)
    if (*ok || v->image.empty() || v->held) return LASPJ_OK;
    const std::vector<uint8_t> img = v->image;
    Call c;
    c.op = Op::WRITE;
    c.kind = v->kind;
    c.n = c.m = 1;
    c.p.push_back(img.data());
    c.len.push_back(img.size());
    c.vars.push_back(v);
    one_group(c, &K);
    {
        Guard g(ctx);
        release_cells(ctx, v);
    }
    v->resident = true;                   // (fit_var gives it zeroed cells)
    v->epoch = K.epoch;
    std::vector<int32_t> vd;
    const int s = run(ctx, S, c, &vd);
    if (s == LASPJ_OK && vd[0] == LASPJ_NIF_OK) {
        v->image.clear();
        v->image.shrink_to_fit();
        *ok = true;
        ++S->stats[17];
        return LASPJ_OK;
    }
    // (a reset inside the call may have written the empty cells out over the image)
    v->image = img;
    v->resident = false;
    v->held = s == LASPJ_OK;
    {
        Guard g(ctx);
        release_cells(ctx, v);
    }
    return s;
}

// a namespace's dictionary and device images dropped (the context still alive)
void free_ns(KindState& K) {
    free_etf(K);
    if (K.dict) laspj_dict_destroy(K.dict);
    K.dict = nullptr;
}

}  // namespace

void nif_destroy(laspj_ctx* ctx) {
    NifState* S = ctx->nif;
    if (!S) return;
    {
        std::lock_guard<std::mutex> lk(S->mu);
        {
            Guard g(ctx);
            for (laspj_var* v : S->vars) {
                // the variables' cells go with the context (the cache it frees next)
                release_cells(ctx, v);
                v->ctx = nullptr;
                v->resident = false;
            }
        }
        // their namespaces' device images too (a variable outliving its context keeps only
        // the host side, which its destroy frees)
        for (laspj_var* v : S->vars) {
            free_ns(*v->ns);
            v->ns->vars.clear();
        }
        S->vars.clear();
    }
    for (KindState& K : S->ks) free_ns(K);
    hipSetDevice(ctx->device);
    hipStreamSynchronize(ctx->stream);
    if (S->dblk) hipFree(S->dblk);
    if (S->dcells) hipFree(S->dcells);
    if (S->hin) hipHostFree(S->hin);
    if (S->hout) hipHostFree(S->hout);
    for (const PinSlot& p : S->pins) hipHostFree(p.h);
    delete S;
    ctx->nif = nullptr;
}

}  // namespace laspj

using laspj::fail;

namespace {

int pair_call(laspj_ctx* ctx, laspj::NifState* S, int32_t kind, laspj::Op op, int strict,
              uint32_t n, const uint8_t* const* a, const uint64_t* na, const uint8_t* const* b,
              const uint64_t* nb, laspj::Call* c, std::vector<int32_t>* verdict) {
    if (!n || !a || !na || (op != laspj::Op::VALUE && (!b || !nb)))
        return fail(ctx, LASPJ_E_INVAL, "nif: null operand array");
    const uint32_t per = op == laspj::Op::VALUE ? 1u : 2u;
    if ((uint64_t)n * per > (1ull << 31))
        return fail(ctx, LASPJ_E_RANGE, "nif: too many operands");
    c->op = op;
    c->kind = kind;
    c->strict = strict;
    c->n = n;
    c->m = n * per;
    c->p.resize(c->m);
    c->len.resize(c->m);
    for (uint32_t i = 0; i < n; ++i) {
        if ((!a[i] && na[i]) || (per == 2 && !b[i] && nb[i]))
            return fail(ctx, LASPJ_E_INVAL, "nif: null payload");
        c->p[i] = a[i];
        c->len[i] = na[i];
        if (per == 2) {
            c->p[n + i] = b[i];
            c->len[n + i] = nb[i];
        }
    }
    laspj::one_group(*c, &laspj::kstate(S, kind));
    return laspj::run(ctx, S, *c, verdict);
}

int merge_many(int32_t kind, laspj_ctx* ctx, uint32_t n, const uint8_t* const* a,
               const uint64_t* na, const uint8_t* const* b, const uint64_t* nb,
               const uint8_t** out, uint64_t* out_len, int32_t* verdict) {
    if (!ctx) return LASPJ_E_INVAL;
    if (!out || !out_len || !verdict) return fail(ctx, LASPJ_E_INVAL, "nif: null output array");
    laspj::NifState* S = laspj::state(ctx);
    if (!S) return fail(ctx, LASPJ_E_NOMEM, "nif: state allocation");
    std::lock_guard<std::mutex> lk(S->mu);
    laspj::Call c;
    std::vector<int32_t> v;
    if (int s = pair_call(ctx, S, kind, laspj::Op::MERGE, 0, n, a, na, b, nb, &c, &v)) return s;
    for (uint32_t i = 0; i < n; ++i) {
        verdict[i] = v[i];
        out[i] = v[i] == LASPJ_NIF_OK ? c.obase + c.ooff[i] : nullptr;
        out_len[i] = v[i] == LASPJ_NIF_OK ? c.ooff[i + 1] - c.ooff[i] : 0;
    }
    return LASPJ_OK;
}

int bool_call(int32_t kind, laspj_ctx* ctx, laspj::Op op, int strict, const uint8_t* a,
              uint64_t na, const uint8_t* b, uint64_t nb, int32_t* result, int32_t* verdict) {
    if (!ctx) return LASPJ_E_INVAL;
    if (!result || !verdict) return fail(ctx, LASPJ_E_INVAL, "nif: null output");
    laspj::NifState* S = laspj::state(ctx);
    if (!S) return fail(ctx, LASPJ_E_NOMEM, "nif: state allocation");
    std::lock_guard<std::mutex> lk(S->mu);
    laspj::Call c;
    std::vector<int32_t> v;
    if (int s = pair_call(ctx, S, kind, op, strict, 1, &a, &na, &b, &nb, &c, &v)) return s;
    *verdict = v[0];
    *result = v[0] == LASPJ_NIF_OK ? (int32_t)(c.res[0] != 0) : 0;
    return LASPJ_OK;
}

// the variable's context state (its S->mu is taken by the caller)
laspj::NifState* var_state(laspj_var* v) {
    if (!v || !v->ctx) return nullptr;
    return laspj::state(v->ctx);
}

int var_image_call(laspj_var* var, bool value, const uint8_t** out, uint64_t* out_len,
                   int32_t* verdict) {
    laspj::NifState* S = var_state(var);
    if (!S) return LASPJ_E_INVAL;
    laspj_ctx* ctx = var->ctx;
    if (!out || !out_len || !verdict) return fail(ctx, LASPJ_E_INVAL, "var: null output");
    std::lock_guard<std::mutex> lk(S->mu);
    if (!S->vars.count(var)) return fail(ctx, LASPJ_E_INVAL, "var: unknown variable");
    bool ok = false;
    if (int s = laspj::hydrate(ctx, S, var, &ok)) return s;
    if (!ok) {
        // host-held: read answers the image itself; value/1 is the reference's to compute
        *out = !value ? var->image.data() : nullptr;
        *out_len = !value ? var->image.size() : 0;
        *verdict = !value ? LASPJ_NIF_OK : LASPJ_NIF_FALLBACK;
        return LASPJ_OK;
    }
    laspj::Call c;
    // value/1 of a G-Set is its own term (ordsets:to_list, lasp_gset.erl:74-76)
    c.op = value && var->kind == LASPJ_KIND_ORSET ? laspj::Op::VVALUE : laspj::Op::READ;
    c.kind = var->kind;
    c.n = 1;
    c.m = 0;
    c.vars.push_back(var);
    laspj::one_group(c, var->ns.get());
    std::vector<int32_t> vd;
    if (int s = laspj::run(ctx, S, c, &vd)) return s;
    *verdict = vd[0];
    *out = vd[0] == LASPJ_NIF_OK ? c.obase + c.ooff[0] : nullptr;
    *out_len = vd[0] == LASPJ_NIF_OK ? c.ooff[1] - c.ooff[0] : 0;
    return LASPJ_OK;
}

}  // namespace

extern "C" {

int laspj_orset_etf_merge_many(laspj_ctx* ctx, uint32_t n, const uint8_t* const* a,
                               const uint64_t* na, const uint8_t* const* b, const uint64_t* nb,
                               const uint8_t** out, uint64_t* out_len, int32_t* verdict) {
    return merge_many(LASPJ_KIND_ORSET, ctx, n, a, na, b, nb, out, out_len, verdict);
}

int laspj_orset_etf_merge(laspj_ctx* ctx, const uint8_t* a, uint64_t na, const uint8_t* b,
                          uint64_t nb, const uint8_t** out, uint64_t* out_len, int32_t* verdict) {
    return laspj_orset_etf_merge_many(ctx, 1, &a, &na, &b, &nb, out, out_len, verdict);
}

int laspj_orset_etf_value(laspj_ctx* ctx, const uint8_t* s, uint64_t ns, const uint8_t** out,
                          uint64_t* out_len, int32_t* verdict) {
    if (!ctx) return LASPJ_E_INVAL;
    if (!out || !out_len || !verdict) return fail(ctx, LASPJ_E_INVAL, "nif: null output");
    laspj::NifState* S = laspj::state(ctx);
    if (!S) return fail(ctx, LASPJ_E_NOMEM, "nif: state allocation");
    std::lock_guard<std::mutex> lk(S->mu);
    laspj::Call c;
    std::vector<int32_t> v;
    if (int st = pair_call(ctx, S, LASPJ_KIND_ORSET, laspj::Op::VALUE, 0, 1, &s, &ns, nullptr,
                           nullptr, &c, &v))
        return st;
    *verdict = v[0];
    *out = v[0] == LASPJ_NIF_OK ? c.obase + c.ooff[0] : nullptr;
    *out_len = v[0] == LASPJ_NIF_OK ? c.ooff[1] - c.ooff[0] : 0;
    return LASPJ_OK;
}

int laspj_orset_etf_equal(laspj_ctx* ctx, const uint8_t* a, uint64_t na, const uint8_t* b,
                          uint64_t nb, int32_t* result, int32_t* verdict) {
    return bool_call(LASPJ_KIND_ORSET, ctx, laspj::Op::EQUAL, 0, a, na, b, nb, result, verdict);
}

int laspj_orset_etf_inflation(laspj_ctx* ctx, const uint8_t* prev, uint64_t np,
                              const uint8_t* cur, uint64_t nc, int strict, int32_t* result,
                              int32_t* verdict) {
    return bool_call(LASPJ_KIND_ORSET, ctx, laspj::Op::INFLATION, strict ? 1 : 0, prev, np, cur,
                     nc, result, verdict);
}

// ---------------------------------------------------------------- lasp_gset

int laspj_gset_etf_merge_many(laspj_ctx* ctx, uint32_t n, const uint8_t* const* a,
                              const uint64_t* na, const uint8_t* const* b, const uint64_t* nb,
                              const uint8_t** out, uint64_t* out_len, int32_t* verdict) {
    return merge_many(LASPJ_KIND_GSET, ctx, n, a, na, b, nb, out, out_len, verdict);
}

int laspj_gset_etf_merge(laspj_ctx* ctx, const uint8_t* a, uint64_t na, const uint8_t* b,
                         uint64_t nb, const uint8_t** out, uint64_t* out_len, int32_t* verdict) {
    return laspj_gset_etf_merge_many(ctx, 1, &a, &na, &b, &nb, out, out_len, verdict);
}

int laspj_gset_etf_value(laspj_ctx* ctx, const uint8_t* s, uint64_t ns, const uint8_t** out,
                         uint64_t* out_len, int32_t* verdict) {
    // value/1 = ordsets:to_list/1 (lasp_gset.erl:74-76), the identity on any term: the
    // answer is the operand's own image (no device work)
    if (!ctx) return LASPJ_E_INVAL;
    if (!out || !out_len || !verdict || (!s && ns))
        return fail(ctx, LASPJ_E_INVAL, "nif: null argument");
    *out = s;
    *out_len = ns;
    *verdict = LASPJ_NIF_OK;
    return LASPJ_OK;
}

int laspj_gset_etf_equal(laspj_ctx* ctx, const uint8_t* a, uint64_t na, const uint8_t* b,
                         uint64_t nb, int32_t* result, int32_t* verdict) {
    return bool_call(LASPJ_KIND_GSET, ctx, laspj::Op::EQUAL, 0, a, na, b, nb, result, verdict);
}

int laspj_gset_etf_inflation(laspj_ctx* ctx, const uint8_t* prev, uint64_t np,
                             const uint8_t* cur, uint64_t nc, int strict, int32_t* result,
                             int32_t* verdict) {
    return bool_call(LASPJ_KIND_GSET, ctx, laspj::Op::INFLATION, strict ? 1 : 0, prev, np, cur,
                     nc, result, verdict);
}

// ---------------------------------------------------------------- resident variables

}  // extern "C"

namespace {

// a variable in namespace `ns` (a fresh one when null); call with S->mu held
int var_new(laspj_ctx* ctx, laspj::NifState* S, int32_t kind,
            std::shared_ptr<laspj::KindState> ns, laspj_var** out) {
    auto* v = new (std::nothrow) laspj_var;
    if (!v) return fail(ctx, LASPJ_E_NOMEM, "var_create: host allocation");
    v->ctx = ctx;
    v->kind = kind;
    try {
        if (!ns) {
            ns = std::make_shared<laspj::KindState>();
            ns->kind = kind;
        }
        v->ns = ns;
        if (!ns->dict && laspj::reset_dict(ctx, S, *ns)) {
            delete v;
            return LASPJ_E_NOMEM;
        }
        v->epoch = ns->epoch;         // new(): no cells until the first call sizes them
        S->vars.insert(v);
        try {
            ns->vars.insert(v);
        } catch (const std::bad_alloc&) {
            S->vars.erase(v);
            throw;
        }
    } catch (const std::bad_alloc&) {
        delete v;
        return fail(ctx, LASPJ_E_NOMEM, "var_create: registry");
    }
    *out = v;
    return LASPJ_OK;
}

// the tokens unique/1 mints (lasp_orset.erl:261-262: crypto:strong_rand_bytes(20)), from the
// kernel's CSPRNG
bool strong_rand(uint8_t* p, size_t n) {
    while (n) {
        const ssize_t r = getrandom(p, n, 0);
        if (r < 0) {
            if (errno == EINTR) continue;
            return false;
        }
        p += r;
        n -= (size_t)r;
    }
    return true;
}

// bind_many with S->mu held (laspj_var_etf_bind_many's body)
int bind_many_locked(laspj_ctx* ctx, laspj::NifState* S, uint32_t n, laspj_var* const* vars,
                     const uint8_t* const* values, const uint64_t* lens, int32_t* status,
                     int32_t* verdict, const uint8_t* const* pre = nullptr) {
    const int32_t kind = vars[0] ? vars[0]->kind : 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (!vars[i] || vars[i]->ctx != ctx || !S->vars.count(vars[i]))
            return fail(ctx, LASPJ_E_INVAL, "var_bind: variable %u is not this context's", i);
        if (vars[i]->kind != kind)
            return fail(ctx, LASPJ_E_KIND, "var_bind: variables of one kind per call");
        if (!values[i] && lens[i]) return fail(ctx, LASPJ_E_INVAL, "var_bind: null payload");
    }
    {
        std::unordered_set<laspj_var*> seen;
        for (uint32_t i = 0; i < n; ++i)
            if (!seen.insert(vars[i]).second)
                return fail(ctx, LASPJ_E_INVAL, "var_bind: variable %u named twice", i);
    }
    // variables whose value sits in an image (after a dictionary reset) are decoded first;
    // one that stays host-held answers FALLBACK (the NIF binds its read image in Erlang)
    for (uint32_t i = 0; i < n; ++i) {
        bool ok = false;
        if (int s = laspj::hydrate(ctx, S, vars[i], &ok)) return s;
        verdict[i] = LASPJ_NIF_FALLBACK;
        status[i] = 0;
    }
    std::vector<uint32_t> live;
    for (uint32_t i = 0; i < n; ++i)
        if (vars[i]->resident && vars[i]->epoch == vars[i]->ns->epoch) live.push_back(i);
    if (live.empty()) return LASPJ_OK;
    // one decode per namespace (its own dictionary): the payloads grouped by namespace
    std::stable_sort(live.begin(), live.end(), [&](uint32_t x, uint32_t y) {
        return std::less<const laspj::KindState*>()(vars[x]->ns.get(), vars[y]->ns.get());
    });
    laspj::Call c;
    c.op = laspj::Op::BIND;
    c.kind = kind;
    c.n = c.m = (uint32_t)live.size();
    for (uint32_t k = 0; k < live.size(); ++k) {
        const uint32_t i = live[k];
        c.p.push_back(values[i]);
        c.len.push_back(lens[i]);
        c.pre.push_back(pre ? pre[i] : nullptr);
        c.vars.push_back(vars[i]);
        if (k == 0 || vars[live[k - 1]]->ns != vars[i]->ns)
            c.groups.push_back(laspj::Group{vars[i]->ns.get(), k, k + 1});
        else
            c.groups.back().p1 = k + 1;
    }
    std::vector<int32_t> vd;
    if (int s = laspj::run(ctx, S, c, &vd)) return s;
    for (size_t k = 0; k < live.size(); ++k) {
        verdict[live[k]] = vd[k];
        status[live[k]] = vd[k] == LASPJ_NIF_OK ? (int32_t)c.res[k] : 0;
    }
    return LASPJ_OK;
}

}  // namespace

namespace laspj {
namespace {

// one batch of queued single binds (laspj_var_etf_bind's group commit), S->mu held: the
// requests of each kind that name distinct variables go into one bind_many; a request
// whose variable is not this context's answers LASPJ_E_INVAL on its own; a variable named
// again waits for the next round of the same batch (the caller marks them done)
void serve_binds(laspj_ctx* ctx, NifState* S, std::vector<BindReq*>& batch) {
    std::vector<BindReq*> todo;
    for (BindReq* r : batch) {
        if (r->var->ctx != ctx || !S->vars.count(r->var)) {
            r->rc = fail(ctx, LASPJ_E_INVAL, "var_bind: unknown variable");
        } else {
            todo.push_back(r);
        }
    }
    while (!todo.empty()) {
        std::vector<BindReq*> now, later;
        std::unordered_set<laspj_var*> seen;
        const int32_t kind = todo[0]->var->kind;
        for (BindReq* r : todo)
            (r->var->kind == kind && seen.insert(r->var).second ? now : later).push_back(r);
        const uint32_t k = (uint32_t)now.size();
        std::vector<laspj_var*> vs(k);
        std::vector<const uint8_t*> ps(k), pre(k);
        std::vector<uint64_t> ls(k);
        std::vector<int32_t> st(k, 0), vd(k, LASPJ_NIF_FALLBACK);
        for (uint32_t i = 0; i < k; ++i) {
            vs[i] = now[i]->var;
            ps[i] = now[i]->p;
            ls[i] = now[i]->n;
            // (a waiter still copying: the leader copies the payload itself)
            pre[i] = now[i]->staged.load(std::memory_order_acquire) ? now[i]->pre : nullptr;
        }
        const int rc = bind_many_locked(ctx, S, k, vs.data(), ps.data(), ls.data(), st.data(),
                                        vd.data(), pre.data());
        for (uint32_t i = 0; i < k; ++i) {
            now[i]->rc = rc;
            now[i]->status = rc ? 0 : st[i];
            now[i]->verdict = rc ? LASPJ_NIF_FALLBACK : vd[i];
        }
        todo.swap(later);
    }
}

}  // namespace
}  // namespace laspj

extern "C" {

int laspj_var_create(laspj_ctx* ctx, int32_t kind, laspj_var** out) {
    if (!ctx || !out) return LASPJ_E_INVAL;
    *out = nullptr;
    if (kind != LASPJ_KIND_ORSET && kind != LASPJ_KIND_GSET)
        return fail(ctx, LASPJ_E_KIND, "var_create: OR-Set or G-Set variables");
    laspj::NifState* S = laspj::state(ctx);
    if (!S) return fail(ctx, LASPJ_E_NOMEM, "nif: state allocation");
    std::lock_guard<std::mutex> lk(S->mu);
    return var_new(ctx, S, kind, nullptr, out);
}

int laspj_var_create_replica(laspj_var* peer, laspj_var** out) {
    laspj::NifState* S = var_state(peer);
    if (!S || !out) return LASPJ_E_INVAL;
    *out = nullptr;
    laspj_ctx* ctx = peer->ctx;
    std::lock_guard<std::mutex> lk(S->mu);
    if (!S->vars.count(peer)) return fail(ctx, LASPJ_E_INVAL, "var_create_replica: unknown variable");
    return var_new(ctx, S, peer->kind, peer->ns, out);
}

int laspj_var_destroy(laspj_var* v) {
    if (!v) return LASPJ_E_INVAL;
    if (v->ctx) {
        laspj::NifState* S = laspj::state(v->ctx);
        if (S) {
            std::lock_guard<std::mutex> lk(S->mu);
            S->vars.erase(v);
            v->ns->vars.erase(v);
            {
                std::lock_guard<std::mutex> lk2(v->ctx->mu);
                hipSetDevice(v->ctx->device);
                laspj::release_cells(v->ctx, v);
            }
            // the namespace's last variable: its device images go too
            if (v->ns.use_count() == 1) laspj::free_ns(*v->ns);
        }
    } else if (v->ns && v->ns.use_count() == 1 && v->ns->dict) {
        laspj_dict_destroy(v->ns->dict);         // (its device images went with the context)
        v->ns->dict = nullptr;
    }
    delete v;
    return LASPJ_OK;
}

int laspj_var_etf_bind_many(laspj_ctx* ctx, uint32_t n, laspj_var* const* vars,
                            const uint8_t* const* values, const uint64_t* lens, int32_t* status,
                            int32_t* verdict) {
    if (!ctx) return LASPJ_E_INVAL;
    if (!n) return LASPJ_OK;
    if (!vars || !values || !lens || !status || !verdict)
        return fail(ctx, LASPJ_E_INVAL, "var_bind: null array");
    laspj::NifState* S = laspj::state(ctx);
    if (!S) return fail(ctx, LASPJ_E_NOMEM, "nif: state allocation");
    std::lock_guard<std::mutex> lk(S->mu);
    return bind_many_locked(ctx, S, n, vars, values, lens, status, verdict);
}

int laspj_var_etf_bind(laspj_var* var, const uint8_t* value, uint64_t n, int32_t* status,
                       int32_t* verdict) {
    if (!var || !var->ctx) return LASPJ_E_INVAL;
    laspj_ctx* ctx = var->ctx;
    if ((!value && n) || !status || !verdict) return fail(ctx, LASPJ_E_INVAL, "var_bind: null argument");
    laspj::NifState* S = laspj::state(ctx);
    if (!S) return fail(ctx, LASPJ_E_NOMEM, "nif: state allocation");
    // Group commit: schedulers binding through one context at once are served by one device
    // pass.  The caller that finds no pass running leads: it takes every queued bind (its
    // own first) and runs them as one bind_many, again while more arrive; the others wait
    // for their answers.  One context per GPU then batches many schedulers' binds
    // (lasp_vnode.erl:213-237) instead of one stream and pass per scheduler.
    laspj::BindReq r;
    r.var = var;
    r.p = value;
    r.n = n;
    laspj::PinSlot slot;
    bool want_slot = false;
    {
        std::lock_guard<std::mutex> q(S->qmu);
        if (S->leading) {
            S->queue.push_back(&r);
            // a waiter stages its own payload into a pinned block while the pass before
            // it runs (the leader then only gathers it on the device)
            if (n >= laspj::kPinMin) {
                if (!S->pins.empty()) {
                    slot = S->pins.back();
                    S->pins.pop_back();
                    want_slot = true;
                } else if (S->pins_live < laspj::kPinSlots) {
                    ++S->pins_live;
                    want_slot = true;
                }
            }
        } else {
            S->leading = true;
            r.lead = true;
        }
    }
    if (want_slot) {
        if (slot.cap < n + 16 && !laspj::pin_grow(&slot, n + 16)) {
            std::lock_guard<std::mutex> q(S->qmu);
            --S->pins_live;
            want_slot = false;
        }
        if (want_slot) {
            std::memcpy(slot.h, value, n);
            r.pre = slot.d;
            r.staged.store(true, std::memory_order_release);
        }
    }
    // (the block back to the pool once the pass that read it has answered)
    auto give_back = [&]() {
        if (!want_slot) return;
        std::lock_guard<std::mutex> q(S->qmu);
        S->pins.push_back(slot);
    };
    if (!r.lead) {
        std::unique_lock<std::mutex> lk(r.m);
        r.cv.wait(lk, [&] { return r.done || r.lead; });
        if (r.done) {
            lk.unlock();
            give_back();
            *status = r.status;
            *verdict = r.verdict;
            return r.rc;
        }
    }
    // the leader: its own request and every queued one per pass, again while binds keep
    // arriving (up to kLeadRounds), then it hands the leadership to the oldest waiter
    std::vector<laspj::BindReq*> batch;
    bool own = true;
    for (int round = 0; round < laspj::kLeadRounds; ++round) {
        batch.clear();
        {
            std::lock_guard<std::mutex> q(S->qmu);
            batch.swap(S->queue);
        }
        if (own) batch.insert(batch.begin(), &r);
        own = false;
        if (batch.empty()) break;
        {
            std::lock_guard<std::mutex> lk(S->mu);
            laspj::serve_binds(ctx, S, batch);
        }
        // (each answer published under its request's own lock; the waiter may return and
        // drop the request as soon as that lock is released)
        for (laspj::BindReq* b : batch) {
            if (b == &r) continue;
            std::lock_guard<std::mutex> lk(b->m);
            b->done = true;
            b->cv.notify_one();
        }
    }
    {
        std::lock_guard<std::mutex> q(S->qmu);
        if (S->queue.empty()) {
            S->leading = false;
        } else {
            laspj::BindReq* nx = S->queue.front();
            S->queue.erase(S->queue.begin());
            std::lock_guard<std::mutex> lk(nx->m);
            nx->lead = true;
            nx->cv.notify_one();
        }
    }
    give_back();
    *status = r.status;
    *verdict = r.verdict;
    return r.rc;
}

int laspj_var_etf_write(laspj_var* var, const uint8_t* value, uint64_t n, int32_t* verdict) {
    laspj::NifState* S = var_state(var);
    if (!S) return LASPJ_E_INVAL;
    laspj_ctx* ctx = var->ctx;
    if ((!value && n) || !verdict) return fail(ctx, LASPJ_E_INVAL, "var_write: null argument");
    std::lock_guard<std::mutex> lk(S->mu);
    if (!S->vars.count(var)) return fail(ctx, LASPJ_E_INVAL, "var_write: unknown variable");
    laspj::KindState& K = *var->ns;
    if (!K.dict && laspj::reset_dict(ctx, S, K)) return LASPJ_E_NOMEM;
    // write/4 replaces the value: the old cells (or image) are not read — but a write that
    // fails with an error status (no memory, a device error) leaves the variable as it was
    const bool was_resident = var->resident, was_held = var->held;
    const uint64_t was_epoch = var->epoch;
    std::vector<uint8_t> was_image;
    was_image.swap(var->image);
    const bool had_cells = was_resident && was_epoch == K.epoch;
    var->resident = true;
    var->held = false;
    var->epoch = K.epoch;
    laspj::Call c;
    c.op = laspj::Op::WRITE;
    c.kind = var->kind;
    c.n = c.m = 1;
    c.p.push_back(value);
    c.len.push_back(n);
    c.vars.push_back(var);
    laspj::one_group(c, &K);
    std::vector<int32_t> vd;
    const int s = laspj::run(ctx, S, c, &vd);
    auto drop_cells = [&] {
        std::lock_guard<std::mutex> lk2(ctx->mu);
        hipSetDevice(ctx->device);
        laspj::release_cells(ctx, var);
    };
    if (s) {
        // the write never answered (no memory, a device error): the old value stands
        if (!var->image.empty()) {
            // a reset inside the call wrote the old cells out: the image is the old value
            drop_cells();
            var->resident = false;
            var->held = false;
        } else if (had_cells) {
            var->epoch = was_epoch;   // the old cells (widened, perhaps): the old value
            var->held = was_held;
        } else {
            drop_cells();             // host-held before: cells the call sized are dropped
            var->resident = was_resident;
            var->epoch = was_epoch;
            var->held = was_held;
            var->image.swap(was_image);
        }
        return s;
    }
    *verdict = vd[0];
    if (vd[0] == LASPJ_NIF_OK) {
        var->image.clear();       // (a reset inside the call wrote the old cells out)
        return LASPJ_OK;
    }
    // not representable here: the variable holds the image on the host, and its calls
    // answer FALLBACK until a value the device takes is written
    try {
        var->image.assign(value, value + n);
    } catch (const std::bad_alloc&) {
        return fail(ctx, LASPJ_E_NOMEM, "var_write: host image");
    }
    var->resident = false;
    var->held = true;
    drop_cells();
    return LASPJ_OK;
}

int laspj_var_etf_read(laspj_var* var, const uint8_t** out, uint64_t* out_len, int32_t* verdict) {
    return var_image_call(var, false, out, out_len, verdict);
}

int laspj_var_etf_value(laspj_var* var, const uint8_t** out, uint64_t* out_len,
                        int32_t* verdict) {
    return var_image_call(var, true, out, out_len, verdict);
}

int laspj_var_etf_threshold(laspj_var* var, const uint8_t* threshold, uint64_t n, int strict,
                            int32_t* result, int32_t* verdict) {
    laspj::NifState* S = var_state(var);
    if (!S) return LASPJ_E_INVAL;
    laspj_ctx* ctx = var->ctx;
    if ((!threshold && n) || !result || !verdict)
        return fail(ctx, LASPJ_E_INVAL, "var_threshold: null argument");
    std::lock_guard<std::mutex> lk(S->mu);
    if (!S->vars.count(var)) return fail(ctx, LASPJ_E_INVAL, "var_threshold: unknown variable");
    bool ok = false;
    if (int s = laspj::hydrate(ctx, S, var, &ok)) return s;
    *result = 0;
    *verdict = LASPJ_NIF_FALLBACK;
    if (!ok) return LASPJ_OK;
    laspj::Call c;
    c.op = laspj::Op::THRESHOLD;
    c.kind = var->kind;
    c.strict = strict ? 1 : 0;
    c.n = c.m = 1;
    c.p.push_back(threshold);
    c.len.push_back(n);
    c.vars.push_back(var);
    laspj::one_group(c, var->ns.get());
    std::vector<int32_t> vd;
    if (int s = laspj::run(ctx, S, c, &vd)) return s;
    *verdict = vd[0];
    *result = vd[0] == LASPJ_NIF_OK ? (int32_t)(c.res[0] != 0) : 0;
    return LASPJ_OK;
}

int laspj_var_union(laspj_var* out, laspj_var* l, laspj_var* r, int32_t* status,
                    int32_t* verdict) {
    laspj::NifState* S = var_state(out);
    if (!S || !l || !r) return LASPJ_E_INVAL;
    laspj_ctx* ctx = out->ctx;
    if (!status || !verdict) return fail(ctx, LASPJ_E_INVAL, "var_union: null argument");
    if (l->ctx != ctx || r->ctx != ctx)
        return fail(ctx, LASPJ_E_INVAL, "var_union: variables of different contexts");
    std::lock_guard<std::mutex> lk(S->mu);
    if (!S->vars.count(out) || !S->vars.count(l) || !S->vars.count(r))
        return fail(ctx, LASPJ_E_INVAL, "var_union: unknown variable");
    ++S->stats[0];
    *status = LASPJ_BIND_NOOP;
    *verdict = LASPJ_NIF_FALLBACK;
    // OR-Sets of one namespace only: a G-Set's body is `LValue ++ RValue` (a list value),
    // and cells of two namespaces name different terms by one slot
    if (out->kind != LASPJ_KIND_ORSET || l->kind != LASPJ_KIND_ORSET ||
        r->kind != LASPJ_KIND_ORSET || l->ns != out->ns || r->ns != out->ns) {
        ++S->stats[6];
        return LASPJ_OK;
    }
    for (laspj_var* v : {out, l, r}) {
        bool ok = false;
        if (int s = laspj::hydrate(ctx, S, v, &ok)) return s;
        if (!ok) {
            ++S->stats[6];
            return LASPJ_OK;
        }
    }
    laspj::KindState& K = *out->ns;
    *verdict = LASPJ_NIF_OK;
    if (!K.dict || K.E == 0) return LASPJ_OK;             // three new() values
    laspj::Guard g(ctx);
    const uint32_t tw = laspj::ktw(K);
    for (laspj_var* v : {out, l, r})
        if (int s = laspj::fit_var(ctx, v, K.E, tw)) return s;
    void* word = nullptr;
    if (laspj::dev_alloc(ctx, 256, &word) != hipSuccess) {
        hipGetLastError();
        return fail(ctx, LASPJ_E_NOMEM, "var_union: flag word");
    }
    uint32_t changed = 0;                                 // (Value0 =/= AccValue)
    hipError_t e = hipMemsetAsync(word, 0, 4, ctx->stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(laspj::k_var_union, dim3((K.E + 255) / 256), dim3(256), 0,
                           ctx->stream, out->cells, l->cells, r->cells, K.E, tw,
                           static_cast<uint32_t*>(word));
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = laspj::readback(ctx, &changed, word, 4);
    laspj::dev_release(ctx, word, 256);
    if (e != hipSuccess) return fail(ctx, LASPJ_E_DEVICE, "var_union: %s", hipGetErrorString(e));
    *status = changed ? LASPJ_BIND_WRITTEN : LASPJ_BIND_NOOP;
    return LASPJ_OK;
}

int laspj_var_resident(const laspj_var* var, int32_t* resident) {
    if (!var || !resident) return LASPJ_E_INVAL;
    *resident = var->ctx && var->resident ? 1 : 0;
    return LASPJ_OK;
}

int laspj_var_etf_update(laspj_var* var, const uint8_t* op, uint64_t nop, int32_t* result,
                         const uint8_t** err_elem, uint64_t* err_len, const uint8_t** minted,
                         uint32_t* nminted, int32_t* verdict) {
    laspj::NifState* S = var_state(var);
    if (!S) return LASPJ_E_INVAL;
    laspj_ctx* ctx = var->ctx;
    if (!op || !nop || !result || !verdict)
        return fail(ctx, LASPJ_E_INVAL, "var_update: null argument");
    std::lock_guard<std::mutex> lk(S->mu);
    if (!S->vars.count(var)) return fail(ctx, LASPJ_E_INVAL, "var_update: unknown variable");
    ++S->stats[0];
    *result = LASPJ_UPDATE_OK;
    *verdict = LASPJ_NIF_FALLBACK;
    if (err_elem) *err_elem = nullptr;
    if (err_len) *err_len = 0;
    if (minted) *minted = nullptr;
    if (nminted) *nminted = 0;
    bool ok = false;
    if (int s = laspj::hydrate(ctx, S, var, &ok)) return s;
    auto fallback = [&] {
        ++S->stats[6];
        return LASPJ_OK;
    };
    if (!ok) return fallback();
    // Type:update(Op, Actor, Value0) (lasp_core.erl:283-287): the op's terms
    std::vector<laspj::UpdateOp> ops;
    const int ps = laspj::parse_update_op(var->kind, op, nop, &ops);
    if (ps == LASPJ_E_NOMEM) return fail(ctx, LASPJ_E_NOMEM, "var_update: host allocation");
    if (ps != LASPJ_DEC_OK || ops.size() > (1u << 24)) return fallback();
    if (ops.empty()) {
        // {add_all, []}, {remove_all, []}, {update, []}: {ok, Value0}
        *verdict = LASPJ_NIF_OK;
        return LASPJ_OK;
    }
    const bool orset = var->kind == LASPJ_KIND_ORSET;
    laspj::KindState& K = *var->ns;
    if (!K.dict && laspj::reset_dict(ctx, S, K)) return LASPJ_E_NOMEM;
    uint32_t nmint = 0;
    for (const auto& o : ops) nmint += o.mint ? 1u : 0u;
    S->minted.resize(20ull * nmint);
    if (nmint && !strong_rand(S->minted.data(), S->minted.size()))
        return fail(ctx, LASPJ_E_DEVICE, "var_update: getrandom failed (%d)", errno);
    // the terms registered in the variable's namespace (element slots, token slots); the
    // whole call's registrations undone when one is refused
    const uint64_t t0 = laspj::now_ns();
    const uint32_t nd0 = laspj::dict_elements(K.dict);
    std::vector<laspj_op> dops(ops.size());
    bool any_remove = false, registered = false;
    uint8_t timg[25] = {109, 0, 0, 0, 20};       // BINARY_EXT of 20 bytes
    laspj::dict_begin(K.dict);
    uint32_t mi = 0;
    for (size_t k = 0; k < ops.size(); ++k) {
        if (k == 0) {
            any_remove = registered = false;
            mi = 0;
        }
        const laspj::UpdateOp& o = ops[k];
        laspj_op& d = dops[k];
        d = laspj_op{};
        d.kind = o.kind;
        d.flags = k == 0 ? LASPJ_OP_FLAG_NEW_CALL : 0;
        const auto* eimg = reinterpret_cast<const uint8_t*>(o.elem.data());
        if (o.kind == LASPJ_OP_REMOVE) {
            // orddict:find/2 (lasp_orset.erl:233): absent unless the namespace holds it
            const int64_t e = laspj::dict_find_elem(K.dict, eimg, o.elem.size());
            if (e == -2) {
                laspj::dict_rollback(K.dict);
                return fallback();            // an `==`-equal key under another image
            }
            d.element = e < 0 ? laspj::kNoElem : (uint32_t)e;
            any_remove = true;
            continue;
        }
        uint32_t e = 0, t = 0;
        int st = laspj::dict_reg_elem(K.dict, eimg, o.elem.size(), &e);
        if (st == LASPJ_DEC_OK && orset) {
            const uint8_t* tp;
            size_t tl;
            if (o.mint) {
                std::memcpy(timg + 5, S->minted.data() + 20ull * mi++, 20);
                tp = timg;
                tl = sizeof(timg);
            } else {
                tp = reinterpret_cast<const uint8_t*>(o.tok.data());
                tl = o.tok.size();
            }
            const uint32_t had = laspj::dict_token_count(K.dict, e);
            st = laspj::dict_reg_tok(K.dict, e, tp, tl, &t);
            registered |= laspj::dict_token_count(K.dict, e) != had;
        }
        if (st == LASPJ_E_NOMEM) {
            laspj::dict_rollback(K.dict);
            return fail(ctx, LASPJ_E_NOMEM, "var_update: registration");
        }
        if (st == LASPJ_DEC_UNREPRESENTABLE && !K.wide) {
            // a 65th token on an element: the namespace goes wide and the call's
            // registrations start over
            laspj::dict_rollback(K.dict);
            if (laspj::go_wide(S, K)) {
                laspj::dict_begin(K.dict);
                k = (size_t)-1;
                continue;
            }
            return fallback();
        }
        if (st != LASPJ_DEC_OK) {
            // an `==`-equal term under another image, a token image a wide namespace cannot
            // hold: the reference's clause on the NIF side
            laspj::dict_rollback(K.dict);
            return fallback();
        }
        d.element = e;
        d.slot = (uint8_t)t;
        d.pad = (uint8_t)(t >> 8);
    }
    laspj::dict_begin(K.dict);                    // (the journal kept nothing)
    registered |= laspj::dict_elements(K.dict) != nd0;
    if (registered) {
        ++S->stats[2];
        K.stale = true;
    }
    S->stats[12] += laspj::now_ns() - t0;
    // the device images learn the new terms before the namespace's next device pass: a
    // token on a known element is patched in by that pass (run() patches a stale namespace
    // first — consecutive updates batch their patches); new elements or a new width need
    // the images now (the cells' element slots and pairs come from them)
    const bool lazy = orset && K.etf && laspj::dict_elements(K.dict) == K.built_K &&
                      (!K.wide || laspj::dict_max_tokens(K.dict) <= 64u * K.tw);
    if ((K.stale || !K.etf) && !lazy)
        if (!laspj::patch_etf(ctx, S, K))
            if (int s = laspj::rebuild_etf(ctx, S, K)) return s;
    const uint32_t nops = (uint32_t)dops.size();
    bool all_add = !any_remove;
    int32_t* dstat = nullptr;
    {
        laspj::Guard g(ctx);
        const uint32_t tw = laspj::ktw(K);
        if (int s = laspj::fit_var(ctx, var, K.E, tw)) return s;
        laspj::UpdArgs args;
        std::memset(&args, 0, sizeof(args));
        const laspj_op* dev_ops = nullptr;
        void* blk = nullptr;
        const uint64_t stat_bytes = any_remove ? 4ull * nops : 0;
        const uint64_t ops_bytes = nops > laspj::kUpdArgOps ? 16ull * nops : 0;
        if (stat_bytes + ops_bytes) {
            if (laspj::dev_alloc(ctx, ((stat_bytes + 255) & ~255ull) + ops_bytes, &blk) != hipSuccess) {
                hipGetLastError();
                return fail(ctx, LASPJ_E_NOMEM, "var_update: op buffer");
            }
            dstat = static_cast<int32_t*>(blk);
            if (ops_bytes) {
                auto* p = reinterpret_cast<laspj_op*>(static_cast<uint8_t*>(blk) +
                                                      ((stat_bytes + 255) & ~255ull));
                LJ_HIP(ctx, hipMemcpyAsync(p, dops.data(), ops_bytes, hipMemcpyHostToDevice,
                                           ctx->stream));
                dev_ops = p;
            }
        }
        if (!dev_ops) std::memcpy(args.op, dops.data(), 16ull * nops);
        if (all_add && dev_ops) {
            hipLaunchKernelGGL(laspj::k_var_adds, dim3((nops + 255) / 256), dim3(256), 0,
                               ctx->stream, var->cells, var->kind, tw, dev_ops, nops);
        } else {
            hipLaunchKernelGGL(laspj::k_var_update, dim3(1), dim3(64), 0, ctx->stream, var->cells,
                               var->kind, tw, args, dev_ops, nops, any_remove ? dstat : nullptr);
        }
        LJ_LAUNCHED(ctx);
        std::vector<int32_t> st;
        if (any_remove) {
            // a precondition may fail: its statuses back (one synchronisation)
            st.resize(nops);
            LJ_HIP(ctx, laspj::readback(ctx, st.data(), dstat, 4ull * nops));
        }
        if (blk) laspj::dev_release(ctx, blk, ((stat_bytes + 255) & ~255ull) + ops_bytes);
        for (uint32_t k = 0; k < st.size(); ++k)
            if (st[k] == LASPJ_OPST_NOT_PRESENT) {
                // {error, {precondition, {not_present, Elem}}} (lasp_orset.erl:239-240)
                *result = LASPJ_UPDATE_NOT_PRESENT;
                S->err_elem = ops[k].elem;
                if (err_elem) *err_elem = reinterpret_cast<const uint8_t*>(S->err_elem.data());
                if (err_len) *err_len = S->err_elem.size();
                break;
            }
    }
    if (minted) *minted = S->minted.empty() ? nullptr : S->minted.data();
    if (nminted) *nminted = nmint;
    *verdict = LASPJ_NIF_OK;
    return LASPJ_OK;
}

// ---------------------------------------------------------------- counters

int laspj_nif_stats(laspj_ctx* ctx, uint64_t* out, uint32_t n) {
    if (!ctx || (n && !out)) return LASPJ_E_INVAL;
    laspj::NifState* S = laspj::state(ctx);
    if (!S) return fail(ctx, LASPJ_E_NOMEM, "nif: state allocation");
    std::lock_guard<std::mutex> lk(S->mu);
    for (uint32_t i = 0; i < n && i < LASPJ_NIF_STATS; ++i) out[i] = S->stats[i];
    if (n > 7) {
        // [7] is the dictionaries' size, not a counter: the image calls' and every
        // namespace's
        uint64_t tot = 0;
        std::unordered_set<const laspj::KindState*> seen;
        auto add = [&](const laspj::KindState* K) {
            uint32_t e = 0;
            uint64_t eb, tb;
            if (K->dict && seen.insert(K).second) {
                laspj_dict_info(K->dict, &e, &eb, &tb);
                tot += e;
            }
        };
        for (const laspj::KindState& K : S->ks) add(&K);
        for (const laspj_var* v : S->vars) add(v->ns.get());
        out[7] = tot;
    }
    return LASPJ_OK;
}

int laspj_nif_reset(laspj_ctx* ctx) {
    if (!ctx) return LASPJ_E_INVAL;
    laspj::NifState* S = laspj::state(ctx);
    if (!S) return fail(ctx, LASPJ_E_NOMEM, "nif: state allocation");
    std::lock_guard<std::mutex> lk(S->mu);
    for (laspj::KindState& K : S->ks)
        if (int s = laspj::reset_dict(ctx, S, K)) return s;
    std::unordered_set<laspj::KindState*> seen;
    std::vector<std::shared_ptr<laspj::KindState>> nss;
    for (laspj_var* v : S->vars)
        if (seen.insert(v->ns.get()).second) nss.push_back(v->ns);
    for (auto& ns : nss)
        if (int s = laspj::reset_dict(ctx, S, *ns)) return s;
    return LASPJ_OK;
}

}  // extern "C"
