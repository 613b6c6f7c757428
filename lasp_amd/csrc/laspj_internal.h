// Internal definitions shared by the liblaspj translation units (not installed).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <map>
#include <mutex>
#include <string>
#include <string_view>
#include <vector>

#include "../../include/laspj.h"
#include "../../include/laspj_tune.h"

namespace laspj {
struct NifState;                       // laspj_nif.hip
struct ListEtfState;                   // laspj_list_etf.cpp
void nif_destroy(laspj_ctx* ctx);      // call without ctx->mu held
}  // namespace laspj

struct laspj_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;
    std::string err;
    int cus = 256;
    // tuning knobs (LASPJ_TUNE_*); 0 = default
    int64_t tune_grid = 0;
    int64_t tune_unroll = 0;
    int64_t tune_nt = -1;
    int64_t tune_etf = 0;
    int64_t tune_etf_read = 0;
    int64_t tune_etf_seg = 0;
    int64_t tune_reduce = 0;
    int64_t tune_product_rows = 0;
    int64_t tune_product_cols = 0;
    int64_t tune_list_walk = 0;
    int64_t tune_nif_passes = 0;     // NIF device passes per call (0: the default)
    int64_t tune_list_chunk = 0;     // rows per chunk of the chunked list walk (0: default)
    // device scratch for apply_ops (grown on demand)
    void* scratch = nullptr;
    uint64_t scratch_bytes = 0;
    // one device word for kernel-detected argument violations (product token slots)
    uint32_t* flag = nullptr;
    // per-replica partial records of segmented reductions (grown on demand)
    void* partials = nullptr;
    uint64_t partials_bytes = 0;
    // list kernels' scratch (merge plans, key-order arrays, hash tables, sizes)
    void* lscratch = nullptr;
    uint64_t lscratch_bytes = 0;
    // list_bind's keyfind tables, kept zeroed between calls (each call's last kernel zeroes
    // what it used), so a bind needs no memset of them; dirty: a call may have left them used
    void* ltab = nullptr;
    uint64_t ltab_bytes = 0;
    bool ltab_dirty = false;
    // list_bind's per-call words (device, kept zeroed between calls by the call's last
    // block, as ltab) and its answer (pinned, coherent: the last block writes it there)
    void* lbind = nullptr;
    uint64_t lbind_bytes = 0;
    bool lbind_dirty = false;
    void* lbind_h = nullptr;
    void* lbind_hd = nullptr;       // its device address
    uint64_t lbind_h_bytes = 0;
    // list_bind's rank-indexed path (both lists strictly ascending): per-call words and
    // look-back states (kept zeroed between calls as lbind), and the rank -> entry index
    // maps, tagged with the call's epoch so they are never cleared (0 never valid)
    void* lfz = nullptr;            // two halves: a call's words, the previous call's
    uint64_t lfz_bytes = 0;
    bool lfz_dirty = false;
    uint32_t lf_parity = 0;         // the half the last call used
    uint64_t lf_prev_use = 0;       // the bytes of it that call used (the next one zeroes them)
    void* lfi = nullptr;
    uint64_t lfi_bytes = 0;
    uint32_t lf_epoch = 0;
    // the list merges' chunked walk (k_merge_spec): per-replica round and chunk words,
    // kept zeroed between calls by the kernel's last block per replica
    void* lspec = nullptr;
    uint64_t lspec_bytes = 0;
    bool lspec_dirty = false;
    // laspj_batch_bind_many_host's statuses (pinned, coherent: the kernel writes them there)
    void* many_h = nullptr;
    void* many_hd = nullptr;
    uint64_t many_h_bytes = 0;
    // pinned host staging for the small readbacks (sizes, statuses, flags): a round trip
    // into pageable memory costs ~26 us, into pinned ~13 us (tools/readback_probe.py)
    void* pinned = nullptr;
    // pinned staging for device dictionary images (laspj_etf_dict_create), grow-only: the
    // NIF path rebuilds its image whenever a call registers new terms
    void* dstage = nullptr;
    uint64_t dstage_bytes = 0;
    // pinned ring for small laspj_buf_upload calls: the bytes copied in and the copy
    // enqueued without waiting (the stream orders every later use; the ring synchronises
    // the stream when it wraps)
    void* upring = nullptr;
    uint64_t upring_at = 0;
    const uint8_t* upring_dev = nullptr;   // the ring's device address (kernels read it)
    static constexpr uint64_t kUpRing = 1 << 20, kUpSmall = 64 * 1024;
    static constexpr uint64_t kPinned = 64 * 1024;
    // released device blocks by size class (laspj::dev_alloc / dev_release): every kernel
    // runs on `stream`, so a block released after its last enqueued use can serve the
    // next allocation without waiting — no hipFree (a device-wide synchronisation) and
    // no hipMalloc on the bind path's short-lived lists and buffers
    std::map<uint64_t, std::vector<void*>> cache;
    uint64_t cached_bytes = 0;
    // the NIF-level entry points' dictionary, staging and scratch (laspj_nif.hip)
    laspj::NifState* nif = nullptr;
    // the list-image entry points' dictionary and scratch (laspj_list_etf.cpp)
    laspj::ListEtfState* listetf = nullptr;
};

struct laspj_buf {
    laspj_ctx* ctx = nullptr;
    void* dev = nullptr;
    uint64_t bytes = 0;
    // the device address was handed out (laspj_buf_device_ptr): work on other streams may
    // still use the block, so its release synchronises the device first
    mutable bool exported = false;
};

struct laspj_batch {
    laspj_ctx* ctx = nullptr;
    int32_t kind = 0;
    uint32_t elements = 0;      // E
    uint64_t replicas = 0;      // R
    uint64_t words_per_replica = 0;  // u64 words: 2E (OR-Set) or ceil(E/64) (G-Set) ...
    uint32_t elements_r = 0;    // ER of product batches
    uint64_t cells = 0;         // cells per replica: E, or EL*ER for products
    uint32_t tok_words = 1;     // {p, r} pairs per cell (LASPJ_KIND_ORSET_WIDE), else 1
    uint64_t* dev = nullptr;
    bool owns = true;           // false for laspj_batch_wrap
    mutable bool exported = false;  // laspj_batch_device_ptr handed out the address
    // LASPJ_KIND_*_LIST: entry / token capacity per replica (laspj_lists.hip)
    uint32_t cap_e = 0;
    uint32_t cap_t = 0;
    // list batches: every replica holds at most known_e entries and known_t tokens (kept
    // on the host by the operations that write lists, so a merge can size its output
    // without reading the inputs' counts back)
    uint32_t known_e = 0;
    uint32_t known_t = 0;
    // list batches, a hint only: list_bind found some replica's keys not strictly ascending
    // (or product pairs) — its rank-indexed path is not tried again until the list is
    // rewritten (upload, or a merge / bind writing it)
    mutable bool not_asc = false;
    // (a hint too) a merge of this list's keys with another's took the one-wave walk after
    // the chunked walk's walks did not meet: the next merge goes to the one-wave walk
    mutable bool no_spec = false;
};

inline bool laspj_is_list(int32_t kind) {
    return kind == LASPJ_KIND_ORSET_LIST || kind == LASPJ_KIND_GSET_LIST;
}

struct laspj_event {
    laspj_ctx* ctx = nullptr;
    hipEvent_t ev = nullptr;
};

namespace laspj {

int fail(laspj_ctx* ctx, int code, const char* fmt, ...);

inline uint64_t bytes_of(const laspj_batch* b) { return b->replicas * b->words_per_replica * 8ull; }

// Device -> host copies of up to a few pieces in one synchronisation, staged through the
// context's pinned buffer when they fit (laspj_runtime.hip).  Returns a hipError_t.
struct ReadPiece {
    void* host;
    const void* dev;
    uint64_t bytes;
};
hipError_t readback(laspj_ctx* ctx, const ReadPiece* pieces, int n);

// Device blocks through the context's cache (laspj_runtime.hip).  Blocks up to
// kCacheMax are rounded to a power of two and reused in stream order; larger ones go to
// hipMalloc / hipFree directly.  Call with the context's mutex held.
constexpr uint64_t kCacheMax = 256ull << 20;      // largest cached block
constexpr uint64_t kCacheCap = 2ull << 30;        // bytes a context keeps cached
hipError_t dev_alloc(laspj_ctx* ctx, uint64_t bytes, void** out);
// src copied into the context's pinned ring for a stream-ordered host -> device copy with
// no wait (<= 64 KiB; null: not staged).  Call with ctx->mu held.
const void* stage_small(laspj_ctx* ctx, const void* src, uint64_t bytes);
// the device address of a stage_small slot (kernels read staged bytes in place), or null
const void* staged_dev(const laspj_ctx* ctx, const void* slot);
// hipMalloc that gives the context's cached blocks back and retries once when it fails
// (every long-lived scratch allocation goes through it)
hipError_t dev_malloc(laspj_ctx* ctx, void** out, uint64_t bytes);
void dev_release(laspj_ctx* ctx, void* p, uint64_t bytes);
void dev_cache_clear(laspj_ctx* ctx);
inline hipError_t readback(laspj_ctx* ctx, void* host, const void* dev, uint64_t bytes) {
    const ReadPiece p{host, dev, bytes};
    return readback(ctx, &p, 1);
}

#define LJ_HIP(ctx, call)                                                              \
    do {                                                                               \
        hipError_t e_ = (call);                                                        \
        if (e_ != hipSuccess)                                                          \
            return ::laspj::fail((ctx), LASPJ_E_DEVICE, "%s: %s (%s:%d)", #call,        \
                                 hipGetErrorString(e_), __FILE__, __LINE__);           \
    } while (0)

#define LJ_LAUNCHED(ctx)                                                               \
    do {                                                                               \
        hipError_t e_ = hipGetLastError();                                             \
        if (e_ != hipSuccess)                                                          \
            return ::laspj::fail((ctx), LASPJ_E_DEVICE, "kernel launch: %s (%s:%d)",   \
                                 hipGetErrorString(e_), __FILE__, __LINE__);           \
    } while (0)

// Launch wrappers implemented in laspj_kernels.hip.  All take validated shapes.
struct StreamTune {
    int grid;
    int unroll;
    bool nt;
};
StreamTune stream_tune(const laspj_ctx* ctx, uint64_t n16);

hipError_t launch_or(laspj_ctx* ctx, uint64_t* dst, const uint64_t* a, const uint64_t* b,
                     uint64_t words);
hipError_t launch_max(laspj_ctx* ctx, uint64_t* dst, const uint64_t* a, const uint64_t* b,
                      uint64_t words);
hipError_t launch_reduce_max(laspj_ctx* ctx, uint64_t* dst, const uint64_t* src,
                             uint64_t groups, uint32_t group, uint64_t wr);
hipError_t launch_gcounter_sums(laspj_ctx* ctx, const laspj_batch* b, uint64_t* sums);
hipError_t launch_gcounter_threshold(laspj_ctx* ctx, const laspj_batch* b, uint64_t t,
                                     bool strict, uint8_t* out);
hipError_t launch_gcounter_inflation(laspj_ctx* ctx, const laspj_batch* prev,
                                     const laspj_batch* cur, bool strict, uint8_t* out);
hipError_t launch_gcounter_incr(laspj_ctx* ctx, laspj_batch* b, const laspj_incr* incs,
                                uint64_t n);
// max_join: per-word unsigned max (G-Counter counts) instead of OR (set bitmaps)
hipError_t launch_reduce_chunks(laspj_ctx* ctx, uint64_t* dst, const uint64_t* src,
                                uint64_t words, uint32_t nchunks, bool max_join);
hipError_t launch_reduce_ptrs(laspj_ctx* ctx, uint64_t* dst, const uint64_t* const* srcs,
                              uint32_t nsrc, uint64_t words, bool max_join);
hipError_t launch_reduce_or(laspj_ctx* ctx, uint64_t* dst, const uint64_t* src,
                            uint64_t groups, uint32_t group, uint64_t words_per_replica);
hipError_t launch_fill_synthetic(laspj_ctx* ctx, laspj_batch* b, uint64_t seed,
                                 uint64_t replica_base, uint64_t tmask = ~0ull);
hipError_t launch_orset_fragment(laspj_ctx* ctx, const laspj_batch* b, uint32_t e, void* out);
hipError_t launch_orset_context(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src);
// head / next: the key chains of the KEYED form (laspj_orset_gather_inflation_keyed), or null
hipError_t launch_gather_inflation(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                                   const uint32_t* index, const uint32_t* head,
                                   const uint32_t* next, const laspj_batch* prev, bool strict,
                                   uint8_t* res);
hipError_t launch_orset_value(laspj_ctx* ctx, const laspj_batch* b, uint64_t* out,
                              bool removed);
hipError_t launch_orset_stats(laspj_ctx* ctx, const laspj_batch* b, uint64_t* out);
hipError_t launch_gset_stats(laspj_ctx* ctx, const laspj_batch* b, uint64_t* out);
hipError_t launch_equal(laspj_ctx* ctx, const laspj_batch* a, const laspj_batch* b,
                        uint8_t* out);
hipError_t launch_orset_inflation(laspj_ctx* ctx, const laspj_batch* prev,
                                  const laspj_batch* cur, bool strict, uint8_t* out);
hipError_t launch_gset_inflation(laspj_ctx* ctx, const laspj_batch* prev,
                                 const laspj_batch* cur, bool strict, uint8_t* out);
hipError_t launch_apply_ops(laspj_ctx* ctx, laspj_batch* b, const laspj_op* ops,
                            uint64_t nops, int32_t* status);
hipError_t launch_orset_union(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                              const laspj_batch* r);
hipError_t launch_orset_filter(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                               const uint64_t* keep);
hipError_t launch_orset_intersection(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                                     const laspj_batch* r);
hipError_t launch_orset_product(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                                const laspj_batch* r, uint32_t* flag);
hipError_t launch_orset_product_diag(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                                     const laspj_batch* r, uint32_t* flag);
hipError_t launch_orset_gather(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                               const uint32_t* index);
hipError_t launch_and(laspj_ctx* ctx, uint64_t* dst, const uint64_t* a, const uint64_t* b,
                      uint64_t words);
// LASPJ_KIND_ORSET_WIDE (laspj_wide.hip)
hipError_t launch_wide_value(laspj_ctx* ctx, const laspj_batch* b, uint64_t* out, bool removed);
hipError_t launch_wide_stats(laspj_ctx* ctx, const laspj_batch* b, uint64_t* out);
hipError_t launch_wide_inflation(laspj_ctx* ctx, const laspj_batch* prev, const laspj_batch* cur,
                                 bool strict, uint8_t* out);
hipError_t launch_wide_apply(laspj_ctx* ctx, laspj_batch* b, const laspj_op* ops, uint64_t nops,
                             int32_t* status);
hipError_t launch_wide_widen(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src);
hipError_t launch_gset_filter(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                              const uint64_t* keep);
hipError_t launch_gset_product(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                               const laspj_batch* r);
hipError_t launch_gset_gather(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                              const uint32_t* index);


// ---- wire codec, enqueue-only forms (laspj_codec.hip) -----------------------------------
// For callers that hold ctx->mu and know the payload offsets on the host (the NIF-level
// entry points, laspj_nif.hip): no readbacks, no synchronisation — a decode -> join ->
// encode chain then costs one host round trip.  Pointers are device addresses.
struct EtfReadPlan {
    uint64_t S = 0, nseg = 0;               // segment bytes / count (0: a wave per payload)
    std::vector<uint32_t> segbase;          // R + 1 when nseg
};
bool etf_dict_decodable(const laspj_etf_dict* d);     // from_binary runs on the device
uint32_t etf_dict_elements(const laspj_etf_dict* d);
void etf_read_plan(const laspj_ctx* ctx, const laspj_etf_dict* d, uint64_t R,
                   const unsigned long long* host_offsets, EtfReadPlan* plan);
// A segment-mode decode whose chain check is left to the join (etf_merge_size_enqueue):
// the caller gives `res` (device memory, kSegResBytes per segment: ctx->scratch is reused
// by the join); etf_read_enqueue fills the rest and sets `armed` when it decoded in
// segments.  The statuses then come from the join's launch; kDecRedo = the chain broke
// before any failing segment: decode that call again without deferring.
constexpr uint64_t kSegResBytes = 32;
// a redo pass's segments (global segment numbers; n = 0: every segment): the segments of a
// deferred pass that met terms since registered, decoded again over the cells they left
// A single payload's tokens its namespace has not seen, taken by the decoder on the spot
// (binary tokens of the dictionary's token length on known elements): each gets the next
// free slot of its element (the element's token count, then one up per new token in
// payload order — one wave decodes an element, so no two waves hand out its slots) and
// an entry {seq, element slot, token slot, image offset} in `out`, numbered by the device
// counter `cnt`; the host registers them in slot order after the call (the dictionary's
// own numbering: count, count + 1, ...).  An entry past `cap`, a slot past 63, or two new
// tokens whose order the decoder cannot tell answer UNKNOWN_TERM as before.
struct NewTok {
    uint32_t seq, e, slot, off;
};
struct NewTokArgs {
    uint32_t* cnt = nullptr;
    NewTok* out = nullptr;
    uint32_t cap = 0, seq = 0;
};

struct SegList {
    uint32_t n = 0;
    uint32_t g[31] = {};
};
constexpr int32_t kDecRedo = 64;
struct ChainJob {
    void* res = nullptr;
    const uint8_t* payload = nullptr;
    const unsigned long long* offs = nullptr;
    const uint32_t* segbase = nullptr;
    int32_t* status = nullptr;
    uint32_t nrep = 0, S = 0;
    bool armed = false;
    void* hres = nullptr;      // (or null) host-visible copy of a failed payload's results
};
// segbase: plan.segbase already on the device, or null (uploaded here); clear: zero the
// batch first (the decoders only set the cells they decode)
// redo_zeroed: R + 1 words the caller has zeroed (segment mode's redo list), or null
int etf_read_enqueue(laspj_ctx* ctx, laspj_batch* b, const laspj_etf_dict* d, int tag, int vers,
                     const uint8_t* payload, uint64_t payload_bytes,
                     const unsigned long long* offsets, const EtfReadPlan& plan,
                     const uint32_t* segbase, int32_t* status, bool clear,
                     uint32_t* redo_zeroed, ChainJob* defer = nullptr,
                     const SegList* only = nullptr, const NewTokArgs* nt = nullptr);
// every token template of the dictionary a BINARY_EXT of the record's length (the new-token
// decode compares such images bytewise, which is their term order)
bool etf_dict_bin_tokens(const laspj_etf_dict* d);
uint32_t etf_dict_tok_len(const laspj_etf_dict* d);      // the uniform token image length
// OR-Set payloads over several dictionaries decoded in one launch (the NIF's binds of many
// variables, one token namespace each): group k's payloads [p0, p1) against dictionary d
// into cells (its first payload's; E slots per replica, consecutive).  The caller stages
// etf_multi_bytes of tables (etf_multi_fill: false when some dictionary cannot take the
// shared launch — decode group by group then; host null: that check only) and hands their
// device copy to
// etf_read_multi_enqueue; offsets are every payload's (absolute), the plan and segbase
// are over all payloads (etf_read_plan with any of the dictionaries); cells are not
// cleared (the caller's are zero); defer as etf_read_enqueue's
struct EtfGroup {
    const laspj_etf_dict* d;
    uint32_t p0, p1;
    uint64_t* cells;
    uint32_t E;
};
uint64_t etf_multi_bytes(uint32_t ngroups, uint32_t npay);
bool etf_multi_fill(const laspj_ctx* ctx, const EtfGroup* g, uint32_t ngroups, uint32_t npay,
                    void* host);
int etf_read_multi_enqueue(laspj_ctx* ctx, const EtfGroup* g, uint32_t ngroups,
                           const void* dev_tabs, uint32_t npay, const uint8_t* payload,
                           uint64_t payload_bytes, const unsigned long long* offs,
                           const EtfReadPlan& plan, const uint32_t* segbase, int32_t* status,
                           ChainJob* defer, const SegList* only = nullptr);
// lasp_gset:from_binary/1's decoder (k_gset_etf_read: one wave per payload), enqueue only;
// offsets / status are device addresses; clear: zero the batch first
int gset_read_enqueue(laspj_ctx* ctx, laspj_batch* b, const laspj_etf_dict* d, int tag, int vers,
                      const uint8_t* payload, const unsigned long long* offsets, int32_t* status,
                      bool clear,
                      const unsigned long long* hoffs = nullptr);
// merge/2 of a[i] and b[i] into z fused with z's size pass (and a, b cleared behind it),
// when etf_merge_fused(ctx, R, E) holds; ticket: one zeroed word (left zero)
bool etf_merge_fused(const laspj_ctx* ctx, uint64_t R, uint32_t E);
int etf_merge_size_enqueue(laspj_ctx* ctx, uint64_t* a, uint64_t* b, const laspj_batch* z,
                           const laspj_etf_dict* d, int tag, unsigned long long* offsets,
                           uint32_t* flag, uint32_t* ticket, const unsigned long long** chunks,
                           const ChainJob* chain = nullptr);
// the NIF's single merge (R == 1): join, size pass and writer in ONE launch
// (k_orset_etf_write_rec's look-back form), when etf_merge_write_one holds; lbst: a zeroed
// word per 256-element chunk, ticket: a zeroed word (left zero), offs_out: {0, total}
// (total > cap: nothing written), chain: the deferred chain checks ride along; skip (or
// null): a device word the decoders set when they took unseen tokens (NewTok) — then
// nothing is written, {0, 0} answered and the operands kept
bool etf_merge_write_one(const laspj_ctx* ctx, const laspj_etf_dict* d, uint64_t R, uint32_t E);
int etf_merge_write_enqueue(laspj_ctx* ctx, uint64_t* a, uint64_t* b, uint32_t E,
                            const laspj_etf_dict* d, int tag, int vers,
                            unsigned long long* offs_out, uint8_t* out, uint64_t cap_bytes,
                            unsigned long long* lbst, uint32_t* ticket, const ChainJob* chain,
                            const uint32_t* skip = nullptr);
// lasp_core:bind/3 (write = false) / write/4 (write = true) of n resident variables: curs /
// ins / wprs (device arrays of n: the variable's cells, its decoded operand's cells — left
// zero — and their width in words; maxw the widest), dstat (n decode statuses: read, or —
// chain armed — written from the deferred chain check), diff (n zeroed words) and ticket
// (a zeroed word) left zero; out_res / out_st (n bytes / n int32, pinned) get the bind
// statuses and decode statuses
int var_bind_enqueue(laspj_ctx* ctx, uint64_t* const* curs, uint64_t* const* ins,
                     const uint64_t* wprs, uint64_t maxw, uint32_t n, int32_t* dstat,
                     uint32_t* diff, uint32_t* ticket, uint8_t* out_res, int32_t* out_st,
                     bool write, const ChainJob* chain);
// offsets: R + 1 (offsets[R] = total); flag: set when a present slot has no image (the
// caller zeroes it); *chunks: the split-mode chunk offsets etf_write_enqueue can reuse
// (valid until the context's scratch is next used), or null
int etf_size_enqueue(laspj_ctx* ctx, const laspj_batch* b, const laspj_etf_dict* d, int32_t kind,
                     int tag, unsigned long long* offsets, uint32_t* flag,
                     const unsigned long long** chunks);
// writes nothing when offsets[R] > cap (the caller reads offsets[R] back and re-sizes)
int etf_write_enqueue(laspj_ctx* ctx, const laspj_batch* b, const laspj_etf_dict* d,
                      int32_t kind, int tag, int vers, const unsigned long long* offsets,
                      uint8_t* out, uint64_t cap, const unsigned long long* chunks);
// value/1 of an OR-Set batch written as G-Set images straight from its cells (size pass,
// offsets and writer; few long payloads: etf_value_direct); zero_cells clears the cells
// behind the reads (even when the answer does not fit)
bool etf_value_direct(const laspj_ctx* ctx, uint64_t R, uint32_t E);
// lasp_gset:merge/2 of few long pairs written from both operands' bits (their OR never
// stored); the same condition as etf_value_direct
int etf_gset_merge_write_enqueue(laspj_ctx* ctx, const laspj_batch* lhs, const laspj_batch* rhs,
                                 const laspj_etf_dict* d, int tag, int vers,
                                 unsigned long long* offsets, uint32_t* flag, uint8_t* out,
                                 uint64_t cap);
// chain: the segment decoder's chain check deferred onto the size pass (as the merge's)
int etf_value_write_enqueue(laspj_ctx* ctx, const laspj_batch* cells, const laspj_etf_dict* d,
                            int tag, int vers, unsigned long long* offsets, uint32_t* flag,
                            uint8_t* out, uint64_t cap, bool zero_cells,
                            const ChainJob* chain = nullptr);

// laspj_etf_dict_create with per-element token headroom (up to tok_headroom more tokens
// per element than the widest has) and the host state etf_dict_patch needs, over arrays
// laspj_dict_export wrote (consistent by construction: the per-slot checks are skipped)
int etf_dict_create_ex(laspj_ctx* ctx, uint32_t E, const uint8_t* elem_blob,
                       const uint32_t* elem_off, const uint32_t* elem_order,
                       const uint8_t* tok_blob, const uint32_t* tok_off, const uint8_t* tok_order,
                       uint32_t tok_headroom, laspj_etf_dict** out);
// rewrite the device rows of element slots that gained tokens in the host dictionary
// (call without ctx->mu held); LASPJ_E_UNSUPPORTED: rebuild instead (nothing written)
int etf_dict_patch(laspj_ctx* ctx, laspj_etf_dict* d, const laspj_dict* hd,
                   const uint32_t* dirty, uint32_t n);
// host dictionary (laspj_host.cpp): element slots, tokens of a slot, its images and their
// term order (order[j] = slot of the j-th smallest)
uint32_t dict_elements(const laspj_dict* dict);
uint32_t dict_token_count(const laspj_dict* dict, uint32_t e);
uint32_t dict_max_tokens(const laspj_dict* dict);   // most tokens of one element (upper bound)
// laspj_dict_encode with tw {p, r} pairs per OR-Set element (a wide namespace's cells)
int dict_encode_cells(const laspj_dict* dict, int32_t kind, const uint8_t* blob,
                      const uint64_t* offsets, uint64_t n, int tag, uint32_t E, uint32_t tw,
                      uint64_t* out, int32_t* status);
// the element slots that gained tokens since the last call (repeats possible), cleared
void dict_take_dirty(laspj_dict* dict, std::vector<uint32_t>* out);
bool dict_tokens(const laspj_dict* dict, uint32_t e, std::vector<std::string_view>* imgs,
                 std::vector<uint8_t>* order);
// register the terms of the OR-Set payload elements that start in [from, to) (from: an
// element's first byte); a DEC status (the range's registrations undone on failure)
int dict_add_elems(laspj_dict* dict, const uint8_t* p, size_t n, size_t from, size_t to);
// update/3's Op (lasp_orset.erl:101-117, lasp_gset.erl:84-88) read from its image (131 +
// the term), flattened in application order: {add, E} / {add_all, Es} (one ADD per element,
// `mint` for an OR-Set: unique/1 mints its token), {add_by_token, T, E}, {remove, E},
// {remove_all, Es}, {update, Ops}.  LASPJ_DEC_MALFORMED: no clause of the reference's update
// takes it as written (the NIF runs the reference's, which raises)
struct UpdateOp {
    uint8_t kind = 0;            // LASPJ_OP_ADD / LASPJ_OP_REMOVE
    bool mint = false;
    std::string elem, tok;       // term images (no version byte); tok empty when minted
};
int parse_update_op(int32_t kind, const uint8_t* img, size_t n, std::vector<UpdateOp>* ops);
// the element slot of an image, -1 when absent, -2 when a term `==` to it holds a slot
// under another image (or the term is outside this path); single registrations inside a
// journal that
// dict_rollback undoes (LASPJ_DEC_* statuses as laspj_dict_add's)
int64_t dict_find_elem(const laspj_dict* dict, const uint8_t* img, size_t n);
void dict_begin(laspj_dict* dict);
void dict_rollback(laspj_dict* dict);
int dict_reg_elem(laspj_dict* dict, const uint8_t* img, size_t n, uint32_t* slot);
int dict_reg_tok(laspj_dict* dict, uint32_t e, const uint8_t* img, size_t n, uint32_t* slot);
// token slots per element (64 by default; a wide namespace's 64 k)
// token slots per element (64: the narrow cells); max_len > 0: from now on every token image
// has the length of the first (at most max_len) — false when those registered already differ
bool dict_set_tok_cap(laspj_dict* dict, uint32_t cap, uint32_t max_len = 0);
uint32_t dict_tok_cap(const laspj_dict* dict);
// a wide namespace's dictionary for its device tables: element images by slot (eblob /
// eoff) and slots in term order (eorder); per element slot e the tokens in term order,
// ranks rb[e] .. rb[e+1): rslot = the rank's token slot, its image tblob[toff[r] ..
// toff[r+1]); max_cnt = the most tokens any element holds
struct WideExport {
    std::vector<uint8_t> eblob, tblob;
    std::vector<uint32_t> eoff, eorder, rb, toff;
    std::vector<uint16_t> rslot;
    uint32_t max_cnt = 0;
};
int dict_export_wide(const laspj_dict* dict, WideExport* x);

// ---- wide namespaces (laspj_codec.hip): device tables of a dictionary whose elements may
// hold up to 64 tw tokens, cells of tw {p, r} pairs per element slot; LASPJ_E_UNSUPPORTED
// for token images of several lengths (or longer than 46 bytes)
struct WideDict;
int wide_dict_create(laspj_ctx* ctx, const WideExport& x, uint32_t tw, WideDict** out);
void wide_dict_destroy(WideDict* w);
uint32_t wide_elements(const WideDict* w);
// the answers' size pass and writer, enqueue only (offsets, out: device addresses); a wide
// namespace's operands are encoded on the host (dict_encode_cells)
int wide_size_enqueue(laspj_ctx* ctx, const WideDict* w, const uint64_t* cells, uint64_t R,
                      int tag, unsigned long long* offsets, uint32_t* flag);
int wide_write_enqueue(laspj_ctx* ctx, const WideDict* w, const uint64_t* cells, uint64_t R,
                       int tag, int vers, const unsigned long long* offsets, uint8_t* out,
                       uint64_t cap);
// dst (en x tn pairs) := src (eo x to pairs) re-laid, the rest {0, 0}; src may be null
hipError_t launch_relay(laspj_ctx* ctx, uint64_t* dst, const uint64_t* src, uint32_t eo,
                        uint32_t to, uint32_t en, uint32_t tn);


// ---- list values as images (laspj_host.cpp; used by laspj_list_etf.cpp) ---------------
// A list value as the list kernels take it (include/laspj.h "list values"): key items
// (element slot, or a pair {X, Y}: bit 62, x << 31 | y), each entry's token run
// toks[toff[i], toff[i+1]) (token g = 64 e + k, bit 63 the flag; bit 62: a pair [Tx, Ty])
struct ListItems {
    std::vector<uint64_t> keys;
    std::vector<uint32_t> toff;      // keys.size() + 1
    std::vector<uint64_t> toks;
};
// walk a term_to_binary image (131 + a list; OR-Set: of {Key, [{Token, Bool}]}, G-Set:
// of elements, in any order, duplicates kept) into items, registering its terms (the
// registrations undone when it fails); args (optional): per entry the slot of the fun's
// argument (the key; a G-Set 2-tuple element's first component).  A LASPJ_DEC_* status,
// or LASPJ_E_NOMEM
int list_walk(laspj_dict* dict, int32_t kind, const uint8_t* p, size_t n, ListItems* it,
              std::vector<uint32_t>* args);
// register one term image (no version byte) as an element; a LASPJ_DEC_* status
int list_register(laspj_dict* dict, const uint8_t* img, size_t n, uint32_t* slot);
std::string_view list_elem_image(const laspj_dict* dict, uint32_t e);
std::string_view list_tok_image(const laspj_dict* dict, uint64_t g);
size_t list_term_len(const uint8_t* p, size_t n);
uint32_t list_dict_elements(const laspj_dict* dict);
// dense term-order ranks: krank per element slot, grank per token g (64 per slot)
int list_ranks(const laspj_dict* dict, std::vector<uint32_t>* krank, std::vector<uint32_t>* grank);
// items -> 131 + the list as term_to_binary/1 writes it
int list_write(const laspj_dict* dict, int32_t kind, const ListItems& it, std::string* out);
void list_etf_destroy(laspj_ctx* ctx);     // laspj_list_etf.cpp; call without ctx->mu held

}  // namespace laspj
