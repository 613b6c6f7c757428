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
// A term the dictionary has not seen (a freshly minted token) makes the decoder answer
// UNKNOWN_TERM: the call registers the operands' terms in the host dictionary (only the
// elements of the decoder segments that failed, when it decoded in segments; else the
// whole operands, laspj_dict_add), patches or rebuilds the device images and runs the
// device pass again.  An operand the columnar form does not take — not an orddict of
// {Elem, [{Token, Bool}]} (an ordset for G-Sets) in term order, an element with no tokens
// or more than 64, a term `==` to a registered one under another image, a term kind no
// dictionary holds — gets verdict LASPJ_NIF_FALLBACK: the NIF then runs the reference's
// own Erlang clause, so the caller always gets the reference's answer (or its crash).
// Scratch, dictionaries and staging are per context: one context per scheduler (or per
// vnode), no process globals.

#include <algorithm>
#include <chrono>
#include <cstring>
#include <new>
#include <unordered_set>
#include <vector>

#include "laspj_internal.h"

// A device-resident variable's value (the `#dv.value` of lasp_core's store): cells over the
// dictionary of its kind in its context, or — when its value is not representable, or
// between a dictionary reset and its next use — the value's image held on the host.
struct laspj_var {
    laspj_ctx* ctx = nullptr;        // null once the context is gone
    int32_t kind = LASPJ_KIND_ORSET;
    uint64_t* cells = nullptr;       // one replica over `E` element slots (null: new())
    uint64_t cell_bytes = 0;         // the block's size (dev_alloc)
    uint32_t E = 0;
    uint64_t epoch = 0;              // the dictionary generation the cells refer to
    bool resident = true;            // cells hold the value (else `image` does)
    std::vector<uint8_t> image;      // host-held value (term_to_binary image)
};

namespace laspj {

// one dictionary of one kind (OR-Set or G-Set) and its device images
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
};

struct NifState {
    std::mutex mu;                  // one call at a time (ctx->mu is held per device phase)
    KindState ks[2];                // [0] OR-Set, [1] G-Set
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
    std::unordered_set<laspj_var*> vars;
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

struct Guard {
    std::lock_guard<std::mutex> lk;
    explicit Guard(laspj_ctx* c) : lk(c->mu) { hipSetDevice(c->device); }
};

constexpr uint32_t kMaxDictElements = 1u << 20;   // a larger dictionary is reset
// device passes per call: registration, a grown answer area and a serial re-decode each
// take one; a call still unresolved after this many answers FALLBACK (run's post-condition)
constexpr int kMaxPasses = 6;
// the in region is pulled by kernels in pieces of this many bytes: each piece's pull runs
// while the host stages the next (one copy-engine copy per call measured slower, and
// 512 KiB copy pieces hit a slow runtime path: profiles/r04i_nif_ab.log,
// r04pull_block_size_ab.log)
constexpr uint64_t kPullPiece = 512ull << 10;

uint64_t al(uint64_t x, uint64_t a) { return (x + a - 1) & ~(a - 1); }

uint64_t wpr_of(int32_t kind, uint32_t E) {
    return kind == LASPJ_KIND_ORSET ? 2ull * E : (E + 63ull) / 64ull;
}

// one NIF-level call over m operand payloads giving n answers
struct Call {
    Op op = Op::MERGE;
    int32_t kind = LASPJ_KIND_ORSET;
    int strict = 0;
    uint32_t n = 0, m = 0;
    std::vector<const uint8_t*> p;  // m payloads: MERGE / EQUAL / INFLATION: lhs[0..n) then rhs
    std::vector<uint64_t> len;
    std::vector<laspj_var*> vars;   // variable calls: n variables (payload i -> variable i)
    std::vector<int32_t> st;        // m decode statuses
    std::vector<uint8_t> res;       // n answer bytes (EQUAL / INFLATION / BIND / THRESHOLD)
    std::vector<uint64_t> ooff;     // n + 1 answer payload offsets (MERGE / VALUE / READ)
    const uint8_t* obase = nullptr; // pinned answer payloads
    bool no_defer = false;          // a deferred chain check came back kDecRedo: decode serially
    // a deferred pass that met unknown terms: its segment results (SegRes records, 32 bytes
    // each: status, start, ...) and table, so only the failing segments are registered
    bool has_seg = false;
    std::vector<uint32_t> segres;   // 8 words per segment
    std::vector<uint32_t> segbase;
    uint64_t segS = 0;
};

KindState& kstate(NifState* S, int32_t kind) {
    return S->ks[kind == LASPJ_KIND_GSET ? 1 : 0];
}

laspj_batch view(laspj_ctx* ctx, int32_t kind, uint64_t R, uint32_t E, uint64_t* dev) {
    laspj_batch b;
    b.ctx = ctx;
    b.kind = kind;
    b.elements = E;
    b.replicas = R;
    b.words_per_replica = wpr_of(kind, E);
    b.cells = E;
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
    K.E = 0;
}

uint64_t now_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

// the device images of the dictionary (called without ctx->mu: etf_dict_create takes it)
int rebuild_etf(laspj_ctx* ctx, NifState* S, KindState& K) {
    const uint64_t t0 = now_ns();
    uint32_t n = 0;
    uint64_t eb = 0, tb = 0;
    if (laspj_dict_info(K.dict, &n, &eb, &tb) != LASPJ_OK)
        return fail(ctx, LASPJ_E_INVAL, "nif: dictionary info");
    // head-room: registrations are append-only, so a larger E holds the next terms
    uint32_t E = K.E;
    if (!K.etf || n > E) E = n + n / 4 + 64;
    const bool toks = K.kind == LASPJ_KIND_ORSET;
    std::vector<uint8_t> ebl(eb + 1), tbl(toks ? tb + 1 : 0), tord(toks ? 64ull * E : 0);
    std::vector<uint32_t> eoff(E + 1ull), eord(E), toff(toks ? 64ull * E + 1 : 0);
    if (laspj_dict_export(K.dict, E, ebl.data(), eoff.data(), eord.data(),
                          toks ? tbl.data() : nullptr, toks ? toff.data() : nullptr,
                          toks ? tord.data() : nullptr) != LASPJ_OK)
        return fail(ctx, LASPJ_E_INVAL, "nif: dictionary export");
    free_etf(K);
    laspj_etf_dict* d = nullptr;
    // OR-Sets: two tokens of headroom per element, so a call that only adds tokens to
    // known elements patches the images (patch_etf) instead of coming back here
    if (int s = toks ? etf_dict_create_ex(ctx, E, ebl.data(), eoff.data(), eord.data(),
                                          tbl.data(), toff.data(), tord.data(), 2, &d)
                     : laspj_etf_dict_create(ctx, E, ebl.data(), eoff.data(), eord.data(),
                                             nullptr, nullptr, nullptr, &d))
        return s;
    K.etf = d;
    K.E = E;
    K.stale = false;
    K.built_K = n;
    K.built_cnt.resize(n);
    for (uint32_t e = 0; e < n; ++e) K.built_cnt[e] = toks ? dict_token_count(K.dict, e) : 0;
    ++S->stats[4];
    S->stats[13] += now_ns() - t0;
    return LASPJ_OK;
}

// Registrations that only added tokens to elements the images already hold: their rows
// patched in place.  False: rebuild (new elements, an element past its headroom, ...).
bool patch_etf(laspj_ctx* ctx, NifState* S, KindState& K) {
    if (!K.etf || K.kind != LASPJ_KIND_ORSET) return false;
    const uint64_t t0 = now_ns();
    const uint32_t n = dict_elements(K.dict);
    if (n != K.built_K || n > K.E) return false;
    std::vector<uint32_t> dirty;
    for (uint32_t e = 0; e < n; ++e)
        if (dict_token_count(K.dict, e) != K.built_cnt[e]) dirty.push_back(e);
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
}

// a variable's cells widened to the dictionary's E (slots are append-only: the old cells
// stay where they are, the new slots start absent); call with ctx->mu held
int fit_var(laspj_ctx* ctx, laspj_var* v, uint32_t E) {
    if (v->cells && v->E == E) return LASPJ_OK;
    const uint64_t wnew = wpr_of(v->kind, E), wold = v->cells ? wpr_of(v->kind, v->E) : 0;
    const uint64_t bytes = std::max<uint64_t>(8ull * wnew, 256);
    void* p = nullptr;
    if (dev_alloc(ctx, bytes, &p) != hipSuccess) {
        hipGetLastError();
        return fail(ctx, LASPJ_E_NOMEM, "nif: variable cells (%llu bytes)",
                    (unsigned long long)bytes);
    }
    uint64_t* c = static_cast<uint64_t*>(p);
    const uint64_t keep = std::min(wold, wnew);
    if (keep) LJ_HIP(ctx, hipMemcpyAsync(c, v->cells, 8ull * keep, hipMemcpyDeviceToDevice,
                                         ctx->stream));
    if (wnew > keep)
        LJ_HIP(ctx, hipMemsetAsync(c + keep, 0, 8ull * (wnew - keep), ctx->stream));
    release_cells(ctx, v);
    v->cells = c;
    v->cell_bytes = bytes;
    v->E = E;
    return LASPJ_OK;
}

// One device pass: stage, pull, decode (or upload host-encoded cells), answer, one
// synchronisation.  Fills c.st / c.res / c.ooff / c.obase.

int device_pass(laspj_ctx* ctx, NifState* S, KindState& K, Call& c) {
    const uint64_t t0 = now_ns();
    uint64_t t_copy = 0;
    const uint32_t m = c.m, n = c.n, E = K.E;
    const bool orset = c.kind == LASPJ_KIND_ORSET;
    const bool dec = m && (orset ? etf_dict_decodable(K.etf) : true);
    const bool var_op = c.op == Op::BIND || c.op == Op::WRITE;
    const bool var_in = var_op || c.op == Op::THRESHOLD || c.op == Op::READ || c.op == Op::VVALUE;
    std::vector<unsigned long long> hoffs(m + 1ull, 0);
    for (uint32_t i = 0; i < m; ++i) hoffs[i + 1] = hoffs[i] + c.len[i];
    const uint64_t pay = hoffs[m];
    EtfReadPlan plan;
    if (dec && orset) etf_read_plan(ctx, K.etf, m, hoffs.data(), &plan);
    const bool has_payload_out = c.op == Op::MERGE || c.op == Op::VALUE || c.op == Op::READ ||
                                 c.op == Op::VVALUE;
    const uint64_t W = wpr_of(c.kind, E);            // words per replica
    // in region (host -> device)
    // [offsets | segment table | zeroed words: the size pass's ticket, the decoder's redo
    //  list, the one-launch merge's look-back words, the variable kernel's difference words
    //  and ticket | variable cell pointers | payloads]
    const uint64_t i_offs = 0, i_seg = al(8ull * (m + 1), 256),
                   i_zero = i_seg + (plan.nseg ? al(4ull * (m + 1), 256) : 0),
                   z_lb = al(4ull * (m + 2), 16), z_var = z_lb + 8ull * ((E + 255) / 256),
                   z_bytes = z_var + 4ull * (n + 1),
                   i_vptr = i_zero + al(z_bytes, 256),
                   i_pay = i_vptr + (var_op ? al(8ull * n, 256) : 0);
    const uint64_t cells_in = (uint64_t)m * W * 8ull;
    const uint64_t in_bytes = i_pay + (dec ? al(pay + 64, 256) : al(cells_in, 256));
    // out region: written by kernels into the pinned staging
    const uint64_t o_st = 0, o_res = al(4ull * m, 16), o_ooff = o_res + al(n, 16),
                   o_pay = o_ooff + al(8ull * (n + 1), 16);
    // answer payload bound: a merge's image is at most both operands' (flags may be
    // re-encoded one byte longer than a SMALL_ATOM_UTF8 input: the slack, and a second
    // pass when even that is short); value/1's at most its operand's; a variable's image
    // is bounded by nothing the call knows (a second pass when the area is short)
    uint64_t bound = 64ull * n + 64;
    for (uint32_t i = 0; i < m; ++i) bound += c.len[i];
    if (has_payload_out && S->ocap < bound + bound / 8) S->ocap = al(bound + bound / 8, 1 << 16);
    const uint64_t ocap = has_payload_out ? S->ocap : 0;
    const uint64_t out_bytes = o_pay + ocap;
    // MERGE: the segment decoder's chain check rides on the join's launch (ChainJob), its
    // per-segment results in a device area of their own after the in region
    const bool defer = dec && orset && plan.nseg && !c.no_defer &&
                       ((c.op == Op::MERGE && etf_merge_fused(ctx, n, E)) || var_op ||
                        (c.op == Op::VALUE && etf_value_direct(ctx, n, E)));
    const uint64_t seg_bytes = defer ? al(plan.nseg * kSegResBytes, 256) : 0;
    // device statuses of the variable calls (their kernel reads them)
    const uint64_t vst_bytes = var_op ? al(4ull * m, 256) : 0;
    // cells: in batch m x W words; MERGE: answers n x W; VALUE / VVALUE: value words
    const uint64_t VW = (E + 63ull) / 64ull;
    const uint64_t cells_out = c.op == Op::MERGE ? (uint64_t)n * W * 8ull
                               : (c.op == Op::VALUE || c.op == Op::VVALUE) ? (uint64_t)n * VW * 8ull
                                                                            : 0;
    const uint64_t c_out = al(cells_in, 256);
    const uint64_t in_words = (uint64_t)m * W;
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
                if (int s = fit_var(ctx, v, E)) return s;
    }
    uint8_t* hin = static_cast<uint8_t*>(S->hin);
    uint8_t* din = static_cast<uint8_t*>(S->dblk);
    uint8_t* dseg = din + al(in_bytes, 256);          // deferred segment results
    int32_t* dvst = reinterpret_cast<int32_t*>(dseg + seg_bytes);   // variable calls' statuses
    uint8_t* rout = S->hout_d;                        // where kernels write the out region
    const uint8_t* hin_d = S->hin_d;
    uint64_t* cin = static_cast<uint64_t*>(S->dcells);
    uint64_t* cout = reinterpret_cast<uint64_t*>(static_cast<uint8_t*>(S->dcells) + c_out);
    std::memcpy(hin + i_offs, hoffs.data(), 8ull * (m + 1));
    if (plan.nseg) std::memcpy(hin + i_seg, plan.segbase.data(), 4ull * (m + 1));
    std::memset(hin + i_zero, 0, z_bytes);
    if (var_op)
        for (uint32_t i = 0; i < n; ++i) {
            const uint64_t p = reinterpret_cast<uint64_t>(c.vars[i]->cells);
            std::memcpy(hin + i_vptr + 8ull * i, &p, 8);
        }
    uint32_t* dticket = reinterpret_cast<uint32_t*>(din + i_zero);
    auto* dlb = reinterpret_cast<unsigned long long*>(din + i_zero + z_lb);
    uint32_t* dvdiff = reinterpret_cast<uint32_t*>(din + i_zero + z_var);
    const bool clean = S->clean_words >= in_words;
    std::vector<int32_t> hst;
    if (m && !dec) {
        // token images of several lengths (or no tokens yet): the host dictionary encodes
        // the cells (laspj_dict_encode), the device does the rest
        std::vector<uint8_t> blob(pay);
        for (uint32_t i = 0; i < m; ++i)
            if (c.len[i]) std::memcpy(blob.data() + hoffs[i], c.p[i], c.len[i]);
        hst.assign(m, 0);
        if (int s = laspj_dict_encode(K.dict, c.kind, blob.data(),
                                      reinterpret_cast<const uint64_t*>(hoffs.data()), m, -1, E,
                                      reinterpret_cast<uint64_t*>(hin + i_pay), hst.data()))
            return fail(ctx, s, "nif: host encode failed (%d)", s);
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
        if (dec) {
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
        laspj_batch inb = view(ctx, c.kind, m, E, cin);
        // statuses: straight into the pinned answer, or (variable calls) device memory their
        // kernel reads and publishes
        int32_t* dst = var_op ? dvst : reinterpret_cast<int32_t*>(rout + o_st);
        ChainJob cjob;
        if (defer) cjob.res = dseg;
        if (dec) {
            if (orset) {
                if (int s = etf_read_enqueue(ctx, &inb, K.etf, -1, 1, din + i_pay, pay,
                                             reinterpret_cast<const unsigned long long*>(din + i_offs),
                                             plan,
                                             plan.nseg ? reinterpret_cast<const uint32_t*>(din + i_seg)
                                                       : nullptr,
                                             dst, !clean, dticket + 1, defer ? &cjob : nullptr))
                    return s;
            } else if (int s = gset_read_enqueue(ctx, &inb, K.etf, -1, 1, din + i_pay,
                                                 reinterpret_cast<const unsigned long long*>(din + i_offs),
                                                 dst, !clean, hoffs.data())) {
                return s;
            }
        } else if (m && var_op) {
            LJ_HIP(ctx, hipMemcpyAsync(dvst, hst.data(), 4ull * m, hipMemcpyHostToDevice,
                                       ctx->stream));
        }
        laspj_batch lhs = view(ctx, c.kind, n, E, cin);
        laspj_batch rhs = view(ctx, c.kind, n, E, cin + (uint64_t)n * W);
        auto* dooff = reinterpret_cast<unsigned long long*>(rout + o_ooff);
        uint8_t* dopay = rout + o_pay;
        switch (c.op) {
        case Op::MERGE: {
            // lasp_orset:merge/2 (lasp_orset.erl:128-134): the nested orddict:merge of two
            // canonical orddicts is the slot-wise OR of their cells; lasp_gset:merge/2
            // (lasp_gset.erl:99-101): ordsets:union of two ordsets, the OR of their bits
            laspj_batch ob = view(ctx, c.kind, n, E, cout);
            const unsigned long long* chunks = nullptr;
            if (orset && etf_merge_write_one(ctx, K.etf, n, E)) {
                // one answer: join, size pass and writer in one launch (look-back), the
                // operands cleared behind it, the chain checks riding along
                if (int s = etf_merge_write_enqueue(ctx, lhs.dev, rhs.dev, E, K.etf, -1, 1, dooff,
                                                    dopay, ocap, dlb, dticket, &cjob))
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
            laspj_batch src = c.op == Op::VALUE ? inb : view(ctx, c.kind, 1, E, c.vars[0]->cells);
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
            laspj_batch vb = view(ctx, c.kind, 1, E, c.vars[0]->cells);
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
            LJ_HIP(ctx, orset ? launch_orset_inflation(ctx, &lhs, &rhs, c.strict != 0, rout + o_res)
                              : launch_gset_inflation(ctx, &lhs, &rhs, c.strict != 0, rout + o_res));
            break;
        case Op::THRESHOLD: {
            // threshold_met(Type, Value, Threshold) (lasp_lattice.erl:62-75): is_(strict_)
            // inflation(Threshold, Value) with Value the resident cells
            S->clean_words = 0;
            laspj_batch cur = view(ctx, c.kind, 1, E, c.vars[0]->cells);
            LJ_HIP(ctx, orset ? launch_orset_inflation(ctx, &lhs, &cur, c.strict != 0, rout + o_res)
                              : launch_gset_inflation(ctx, &lhs, &cur, c.strict != 0, rout + o_res));
            break;
        }
        case Op::BIND:
        case Op::WRITE: {
            // bind/3 (lasp_core.erl:291-312) / write/4 (:839-844) into the resident cells
            // (the segment decoder's chain check rides on this launch when deferred)
            if (int s = var_bind_enqueue(ctx, reinterpret_cast<uint64_t* const*>(din + i_vptr),
                                         cin, W, n, dvst, dvdiff, dvdiff + n, rout + o_res,
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
        c.has_seg = false;
        if (defer && cjob.armed &&
            std::find(c.st.begin(), c.st.end(), (int32_t)LASPJ_DEC_UNKNOWN_TERM) != c.st.end()) {
            c.segres.resize(8ull * plan.nseg);
            LJ_HIP(ctx, hipMemcpyAsync(c.segres.data(), cjob.res, kSegResBytes * plan.nseg,
                                       hipMemcpyDeviceToHost, ctx->stream));
            LJ_HIP(ctx, hipStreamSynchronize(ctx->stream));
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
bool register_segments(NifState* S, KindState& K, const Call& c, const std::vector<uint32_t>& ops) {
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
    for (const Range& r : rs)
        if (dict_add_elems(K.dict, c.p[r.i], c.len[r.i], r.from, r.to) != LASPJ_DEC_OK)
            return false;       // (ranges already added stay: they hold well-formed terms)
    ++S->stats[2];
    S->stats[12] += now_ns() - t0;
    K.stale = true;
    return true;
}

int run(laspj_ctx* ctx, NifState* S, Call& c, std::vector<int32_t>* verdict);

// the image of a resident variable (a READ pass; the caller holds S->mu)
int read_var(laspj_ctx* ctx, NifState* S, laspj_var* v, std::vector<uint8_t>* img) {
    Call c;
    c.op = Op::READ;
    c.kind = v->kind;
    c.n = 1;
    c.m = 0;
    c.vars.push_back(v);
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
    for (laspj_var* v : S->vars) {
        if (v->kind != K.kind || !v->resident || v->epoch != K.epoch) continue;
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
    if (K.dict)
        if (int s = spill_vars(ctx, S, K)) return s;
    free_etf(K);
    if (K.dict) laspj_dict_destroy(K.dict);
    K.dict = nullptr;
    if (laspj_dict_create(&K.dict) != LASPJ_OK)
        return fail(ctx, LASPJ_E_NOMEM, "nif: dictionary allocation");
    K.stale = false;
    ++K.epoch;
    ++S->stats[3];
    return LASPJ_OK;
}

// The call: device pass; operands with unknown terms registered and a second pass; every
// other undecodable operand -> FALLBACK.  verdict[j] per answer.
int run(laspj_ctx* ctx, NifState* S, Call& c, std::vector<int32_t>* verdict) {
    ++S->stats[0];
    KindState& K = kstate(S, c.kind);
    if (!K.dict && reset_dict(ctx, S, K)) return LASPJ_E_NOMEM;
    const uint32_t n = c.n, m = c.m;
    auto answer_of = [&](uint32_t i) { return i % n; };
    // a variable call's operands are its own (payload i belongs to variable i): one whose
    // value needs a fresh dictionary (an element's 64 token slots used up) would write out
    // every other variable's cells, so only write/4 resets; bind / threshold answer
    // FALLBACK and the NIF runs the reference's clause over the variable's read image
    const bool may_reset = !(c.op == Op::BIND || c.op == Op::THRESHOLD);
    std::vector<uint8_t> fallback(n, 0);
    bool registered = false;
    bool partial = false;           // the last registration took the failing segments only
    bool resolved = false;          // the last pass's answers stand (statuses all final)
    const int passes = ctx->tune_nif_passes ? (int)ctx->tune_nif_passes : kMaxPasses;
    for (int pass = 0; pass < passes && !resolved; ++pass) {
        if (!K.etf || K.stale) {
            if (!K.etf && m) {
                // nothing registered yet: register this call's operands first
                std::vector<int32_t> rst;
                if (int s = register_payloads(ctx, S, K, c.p, c.len, &rst)) return s;
                registered = true;
                for (uint32_t i = 0; i < m; ++i)
                    if (rst[i] != LASPJ_DEC_OK) fallback[answer_of(i)] = 1;
            }
            if (!patch_etf(ctx, S, K))
                if (int s = rebuild_etf(ctx, S, K)) return s;
        }
        int s = device_pass(ctx, S, K, c);
        if (s == -1000) continue;                // answer area grown: once more
        if (s) return s;
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
            if (c.st[i] == LASPJ_DEC_UNKNOWN_TERM && (!registered || partial)) unknown.push_back(i);
            else if (c.st[i] != LASPJ_DEC_OK) fallback[answer_of(i)] = 1;
        }
        if (unknown.empty()) {
            resolved = true;
            break;
        }
        if (!registered && c.has_seg && register_segments(S, K, c, unknown)) {
            // the failing segments' elements registered; if the next pass still meets an
            // unknown term, the whole operands are registered after all
            partial = true;
            registered = true;
            continue;
        }
        partial = false;
        // terms the dictionary has not seen (or operands that are not orddicts, which the
        // second pass tells apart): register the operands that met them (an operand that
        // decoded holds only registered terms)
        std::vector<const uint8_t*> rp;
        std::vector<uint64_t> rl;
        std::vector<uint32_t> ri;
        for (uint32_t i : unknown) {
            rp.push_back(c.p[i]);
            rl.push_back(c.len[i]);
            ri.push_back(i);
        }
        uint32_t nd = 0;
        uint64_t eb, tb;
        std::vector<int32_t> rst;
        if (int s2 = register_payloads(ctx, S, K, rp, rl, &rst)) return s2;
        bool full = false;
        for (int32_t x : rst) full |= x == LASPJ_DEC_UNREPRESENTABLE;
        laspj_dict_info(K.dict, &nd, &eb, &tb);
        if (may_reset && ((full && nd) || nd > kMaxDictElements)) {
            // an element's 64 token slots used up by earlier calls (or a dictionary grown
            // past its bound): start a fresh dictionary holding this call's terms only —
            // image calls are self-contained (images in, images out); resident variables
            // are written out to their images first and decoded again when next used
            if (int s2 = reset_dict(ctx, S, K)) return s2;
            if (int s2 = register_payloads(ctx, S, K, c.p, c.len, &rst)) return s2;
            for (uint32_t i = 0; i < m; ++i)
                if (rst[i] != LASPJ_DEC_OK) fallback[answer_of(i)] = 1;
            for (laspj_var* v : c.vars) {             // write/4's own variable: new cells
                v->epoch = K.epoch;
                v->resident = true;
            }
        } else {
            for (size_t k = 0; k < ri.size(); ++k)
                if (rst[k] != LASPJ_DEC_OK) fallback[answer_of(ri[k])] = 1;
        }
        registered = true;
    }
    // post-condition: an answer is OK only from a pass whose statuses were all final; a
    // call whose passes ran out (the answer area grown, a segment chain only a serial
    // decode judges, terms registered — each on the last pass) hands every operand to the
    // reference's clause rather than answer from a superseded pass
    verdict->assign(n, LASPJ_NIF_OK);
    for (uint32_t j = 0; j < n; ++j)
        if (fallback[j] || !resolved) {
            (*verdict)[j] = LASPJ_NIF_FALLBACK;
            ++S->stats[6];
        }
    return LASPJ_OK;
}

NifState* state(laspj_ctx* ctx) {
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (!ctx->nif) {
        ctx->nif = new (std::nothrow) NifState;
        if (ctx->nif) ctx->nif->ks[1].kind = LASPJ_KIND_GSET;
    }
    return ctx->nif;
}

// A variable whose value sits in its host image (written out by a dictionary reset) gets
// cells again: write/4 of that image.  *ok: the variable is resident over the current
// dictionary (false: it stays host-held; its calls answer FALLBACK)
int hydrate(laspj_ctx* ctx, NifState* S, laspj_var* v, bool* ok) {
    KindState& K = kstate(S, v->kind);
    *ok = v->resident && v->epoch == K.epoch;
    if (*ok || v->image.empty()) return LASPJ_OK;
    const std::vector<uint8_t> img = v->image;
    Call c;
    c.op = Op::WRITE;
    c.kind = v->kind;
    c.n = c.m = 1;
    c.p.push_back(img.data());
    c.len.push_back(img.size());
    c.vars.push_back(v);
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
    {
        Guard g(ctx);
        release_cells(ctx, v);
    }
    return s;
}

}  // namespace

void nif_destroy(laspj_ctx* ctx) {
    NifState* S = ctx->nif;
    if (!S) return;
    {
        std::lock_guard<std::mutex> lk(S->mu);
        Guard g(ctx);
        for (laspj_var* v : S->vars) {
            // the variables' cells go with the context (the cache it frees next)
            release_cells(ctx, v);
            v->ctx = nullptr;
            v->resident = false;
        }
        S->vars.clear();
    }
    for (KindState& K : S->ks) {
        if (K.etf) laspj_etf_dict_destroy(K.etf);
        if (K.dict) laspj_dict_destroy(K.dict);
    }
    hipSetDevice(ctx->device);
    hipStreamSynchronize(ctx->stream);
    if (S->dblk) hipFree(S->dblk);
    if (S->dcells) hipFree(S->dcells);
    if (S->hin) hipHostFree(S->hin);
    if (S->hout) hipHostFree(S->hout);
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

int laspj_var_create(laspj_ctx* ctx, int32_t kind, laspj_var** out) {
    if (!ctx || !out) return LASPJ_E_INVAL;
    *out = nullptr;
    if (kind != LASPJ_KIND_ORSET && kind != LASPJ_KIND_GSET)
        return fail(ctx, LASPJ_E_KIND, "var_create: OR-Set or G-Set variables");
    laspj::NifState* S = laspj::state(ctx);
    if (!S) return fail(ctx, LASPJ_E_NOMEM, "nif: state allocation");
    auto* v = new (std::nothrow) laspj_var;
    if (!v) return fail(ctx, LASPJ_E_NOMEM, "var_create: host allocation");
    v->ctx = ctx;
    v->kind = kind;
    std::lock_guard<std::mutex> lk(S->mu);
    laspj::KindState& K = laspj::kstate(S, kind);
    if (!K.dict && laspj::reset_dict(ctx, S, K)) {
        delete v;
        return LASPJ_E_NOMEM;
    }
    v->epoch = K.epoch;               // new(): no cells until the first call sizes them
    try {
        S->vars.insert(v);
    } catch (const std::bad_alloc&) {
        delete v;
        return fail(ctx, LASPJ_E_NOMEM, "var_create: registry");
    }
    *out = v;
    return LASPJ_OK;
}

int laspj_var_destroy(laspj_var* v) {
    if (!v) return LASPJ_E_INVAL;
    if (v->ctx) {
        laspj::NifState* S = laspj::state(v->ctx);
        if (S) {
            std::lock_guard<std::mutex> lk(S->mu);
            S->vars.erase(v);
            std::lock_guard<std::mutex> lk2(v->ctx->mu);
            hipSetDevice(v->ctx->device);
            laspj::release_cells(v->ctx, v);
        }
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
    const laspj::KindState& K = laspj::kstate(S, kind);
    std::vector<uint32_t> live;
    for (uint32_t i = 0; i < n; ++i)
        if (vars[i]->resident && vars[i]->epoch == K.epoch) live.push_back(i);
    if (live.empty()) return LASPJ_OK;
    laspj::Call c;
    c.op = laspj::Op::BIND;
    c.kind = kind;
    c.n = c.m = (uint32_t)live.size();
    for (uint32_t i : live) {
        c.p.push_back(values[i]);
        c.len.push_back(lens[i]);
        c.vars.push_back(vars[i]);
    }
    std::vector<int32_t> vd;
    if (int s = laspj::run(ctx, S, c, &vd)) return s;
    for (size_t k = 0; k < live.size(); ++k) {
        verdict[live[k]] = vd[k];
        status[live[k]] = vd[k] == LASPJ_NIF_OK ? (int32_t)c.res[k] : 0;
    }
    return LASPJ_OK;
}

int laspj_var_etf_bind(laspj_var* var, const uint8_t* value, uint64_t n, int32_t* status,
                       int32_t* verdict) {
    if (!var || !var->ctx) return LASPJ_E_INVAL;
    return laspj_var_etf_bind_many(var->ctx, 1, &var, &value, &n, status, verdict);
}

int laspj_var_etf_write(laspj_var* var, const uint8_t* value, uint64_t n, int32_t* verdict) {
    laspj::NifState* S = var_state(var);
    if (!S) return LASPJ_E_INVAL;
    laspj_ctx* ctx = var->ctx;
    if ((!value && n) || !verdict) return fail(ctx, LASPJ_E_INVAL, "var_write: null argument");
    std::lock_guard<std::mutex> lk(S->mu);
    if (!S->vars.count(var)) return fail(ctx, LASPJ_E_INVAL, "var_write: unknown variable");
    laspj::KindState& K = laspj::kstate(S, var->kind);
    if (!K.dict && laspj::reset_dict(ctx, S, K)) return LASPJ_E_NOMEM;
    // write/4 replaces the value: the old cells (or image) are not read
    var->resident = true;
    var->epoch = K.epoch;
    var->image.clear();
    laspj::Call c;
    c.op = laspj::Op::WRITE;
    c.kind = var->kind;
    c.n = c.m = 1;
    c.p.push_back(value);
    c.len.push_back(n);
    c.vars.push_back(var);
    std::vector<int32_t> vd;
    if (int s = laspj::run(ctx, S, c, &vd)) return s;
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
    std::lock_guard<std::mutex> lk2(ctx->mu);
    hipSetDevice(ctx->device);
    laspj::release_cells(ctx, var);
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
    std::vector<int32_t> vd;
    if (int s = laspj::run(ctx, S, c, &vd)) return s;
    *verdict = vd[0];
    *result = vd[0] == LASPJ_NIF_OK ? (int32_t)(c.res[0] != 0) : 0;
    return LASPJ_OK;
}

int laspj_var_resident(const laspj_var* var, int32_t* resident) {
    if (!var || !resident) return LASPJ_E_INVAL;
    *resident = var->ctx && var->resident ? 1 : 0;
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
        uint32_t e = 0, g = 0;  // [7] is the dictionaries' size, not a counter
        uint64_t eb, tb;
        if (S->ks[0].dict) laspj_dict_info(S->ks[0].dict, &e, &eb, &tb);
        if (S->ks[1].dict) laspj_dict_info(S->ks[1].dict, &g, &eb, &tb);
        out[7] = (uint64_t)e + g;
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
    return LASPJ_OK;
}

}  // extern "C"
