// NIF-level entry points (include/laspj.h "NIF entry points"): what a `laspj_nif` NIF
// function does between `enif_term_to_binary` and `enif_binary_to_term`, inside liblaspj
// so that it is compiled, tested and timed here rather than living as a listing.
//
// The reference's drop-in point is `Type:merge/2` and friends (lasp_orset.erl:32-36,
// 67-73, 128-138), called from lasp_core:bind/3 (lasp_core.erl:291-312) on many BEAM
// schedulers at once (lasp_vnode.erl:213-237).  A call here takes the operands as
// `term_to_binary/1` images and
//   1. stages them into the context's pinned memory, and kernels on the context's stream
//      pull them to the device in pieces while the host stages the next (offsets and the
//      decoder's segment table ride along; LASPJ_TUNE_NIF_DIRECT 0: copy-engine copies),
//   2. decodes them on the device against the context's dictionary (laspj_orset_etf_read's
//      kernels), joins / tests / filters the cells, encodes the answer on the device
//      (laspj_orset_etf_write's kernels) straight into pinned memory — all enqueued on the
//      context's stream with ONE host synchronisation,
//   3. answers from pinned memory: the merged / value term's image (what the NIF hands to
//      enif_binary_to_term) or the boolean.
// A term the dictionary has not seen (a freshly minted token) makes the decoder answer
// UNKNOWN_TERM: the call registers the operands' terms in the host dictionary (only the
// elements of the decoder segments that failed, when it decoded in segments; else the
// whole operands, laspj_dict_add), patches or rebuilds the device images and runs the
// device pass again.  An
// operand the columnar form does not take — not an orddict of {Elem, [{Token, Bool}]} in
// term order, an element with no tokens or more than 64, a term kind no dictionary holds —
// gets verdict LASPJ_NIF_FALLBACK: the NIF then runs the reference's own Erlang clause,
// so the caller always gets the reference's answer (or its crash).  Scratch, dictionary
// and staging are per context: one context per scheduler, no process globals.

#include <algorithm>
#include <chrono>
#include <cstring>
#include <new>
#include <vector>

#include "laspj_internal.h"

namespace laspj {

struct NifState {
    std::mutex mu;                  // one call at a time (ctx->mu is held per device phase)
    laspj_dict* dict = nullptr;     // term images -> slots (host, append-only)
    laspj_etf_dict* etf = nullptr;  // the device images of `dict` (rebuilt when it grows)
    uint32_t E = 0;                 // element slots of `etf` and of the batches
    bool stale = false;             // `dict` registered terms since `etf` was built
    // device: [in region: offsets | segment table | payloads or cells][out region: statuses
    // | answer bytes | payload offsets | payloads]; cells: the batches
    void* dblk = nullptr;
    uint64_t dblk_bytes = 0;
    void* dcells = nullptr;
    uint64_t dcells_bytes = 0;
    // pinned host staging for the two copies
    void* hin = nullptr;
    uint64_t hin_bytes = 0;
    void* hout = nullptr;
    uint64_t hout_bytes = 0;
    bool h_coherent = false;        // both allocated coherent (LASPJ_TUNE_NIF_DIRECT)
    uint8_t* hin_d = nullptr;       // their device addresses, for the allocations hin_dkey /
    uint8_t* hout_d = nullptr;      // hout_dkey
    const void* hin_dkey = nullptr;
    const void* hout_dkey = nullptr;
    uint64_t ocap = 1 << 20;        // device bytes reserved for answer payloads
    // the operand cells known to be new() (the fused merge clears them behind it), so the
    // next call's decoders need no memset: words [0, clean_words) at element slots clean_E
    uint64_t clean_words = 0;
    uint32_t clean_E = 0;
    uint64_t stats[LASPJ_NIF_STATS] = {};
    // what `etf` was built (or last patched) from: host dictionary elements and each
    // one's token count, so registrations that only add tokens to known elements are
    // patched into the device images (etf_dict_patch) instead of rebuilding them
    uint32_t built_K = 0;
    std::vector<uint32_t> built_cnt;
};

namespace {

// The in region pulled from pinned host memory by a kernel on the context's stream
// (LASPJ_TUNE_NIF_DIRECT bit 2): the decoder then starts right behind it instead of
// waiting for a copy engine's completion signal.  16-byte lanes, grid-stride.
typedef uint32_t pull16 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) k_nif_pull(const pull16* __restrict__ src,
                                                  pull16* __restrict__ dst, uint64_t n16) {
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += step)
        dst[i] = __builtin_nontemporal_load(src + i);
}

struct Guard {
    std::lock_guard<std::mutex> lk;
    explicit Guard(laspj_ctx* c) : lk(c->mu) { hipSetDevice(c->device); }
};

constexpr uint32_t kMaxDictElements = 1u << 20;   // a larger dictionary is reset
// host -> pinned staging granule: one copy per call up to 64 MiB (a single ~1 MiB copy
// beat 256 KiB pieces, 135 vs 154 us per config-1 merge, and 512 KiB pieces hit a slow
// runtime path, 475 us: profiles/r04i_nif_ab.log)
constexpr uint64_t kStagePiece = 64ull << 20;
// ... but pulled by kernels (LASPJ_TUNE_NIF_DIRECT bit 2) in pieces of this many bytes:
// each piece's pull runs while the host stages the next
constexpr uint64_t kPullPiece = 512ull << 10;

uint64_t al(uint64_t x, uint64_t a) { return (x + a - 1) & ~(a - 1); }

enum class Op { MERGE, VALUE, EQUAL, INFLATION };

// one NIF-level call over m operand payloads giving n answers
struct Call {
    Op op = Op::MERGE;
    int strict = 0;
    uint32_t n = 0, m = 0;
    std::vector<const uint8_t*> p;  // m payloads: MERGE / EQUAL / INFLATION: lhs[0..n) then rhs
    std::vector<uint64_t> len;
    std::vector<int32_t> st;        // m decode statuses
    std::vector<uint8_t> res;       // n answer bytes (EQUAL / INFLATION)
    std::vector<uint64_t> ooff;     // n + 1 answer payload offsets (MERGE / VALUE)
    const uint8_t* obase = nullptr; // pinned answer payloads
    bool no_defer = false;          // a deferred chain check came back kDecRedo: decode serially
    // a deferred pass that met unknown terms: its segment results (SegRes records, 32 bytes
    // each: status, start, ...) and table, so only the failing segments are registered
    bool has_seg = false;
    std::vector<uint32_t> segres;   // 8 words per segment
    std::vector<uint32_t> segbase;
    uint64_t segS = 0;
};

laspj_batch view(laspj_ctx* ctx, int32_t kind, uint64_t R, uint32_t E, uint64_t* dev) {
    laspj_batch b;
    b.ctx = ctx;
    b.kind = kind;
    b.elements = E;
    b.replicas = R;
    b.words_per_replica = kind == LASPJ_KIND_ORSET ? 2ull * E : (E + 63ull) / 64ull;
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

int grow_host(laspj_ctx* ctx, void** p, uint64_t* have, uint64_t need, bool coherent) {
    if (*have >= need) return LASPJ_OK;
    const uint64_t want = std::max<uint64_t>(need, *have + *have / 2);
    if (*p) {
        hipStreamSynchronize(ctx->stream);
        hipHostFree(*p);
        *p = nullptr;
        *have = 0;
    }
    // kernels that read or write the staging themselves need it coherent: a device L2
    // line of last call's operands must not outlive the host's rewrite
    const unsigned flags = coherent || ctx->tune_nif_host == 2 ? hipHostMallocCoherent
                           : ctx->tune_nif_host == 1           ? hipHostMallocNonCoherent
                                                               : hipHostMallocDefault;
    if (hipHostMalloc(p, want, flags) != hipSuccess) {
        hipGetLastError();
        *p = nullptr;
        return fail(ctx, LASPJ_E_NOMEM, "nif: pinned allocation of %llu bytes",
                    (unsigned long long)want);
    }
    *have = want;
    return LASPJ_OK;
}

void free_etf(NifState* S) {
    if (S->etf) laspj_etf_dict_destroy(S->etf);
    S->etf = nullptr;
    S->E = 0;
}

int reset_dict(laspj_ctx* ctx, NifState* S) {
    free_etf(S);
    if (S->dict) laspj_dict_destroy(S->dict);
    S->dict = nullptr;
    if (laspj_dict_create(&S->dict) != LASPJ_OK)
        return fail(ctx, LASPJ_E_NOMEM, "nif: dictionary allocation");
    S->stale = false;
    ++S->stats[3];
    return LASPJ_OK;
}

uint64_t now_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

// the device images of the dictionary (called without ctx->mu: etf_dict_create takes it)
int rebuild_etf(laspj_ctx* ctx, NifState* S) {
    const uint64_t t0 = now_ns();
    uint32_t n = 0;
    uint64_t eb = 0, tb = 0;
    if (laspj_dict_info(S->dict, &n, &eb, &tb) != LASPJ_OK)
        return fail(ctx, LASPJ_E_INVAL, "nif: dictionary info");
    // head-room: registrations are append-only, so a larger E holds the next terms
    uint32_t E = S->E;
    if (!S->etf || n > E) E = n + n / 4 + 64;
    std::vector<uint8_t> ebl(eb + 1), tbl(tb + 1), tord(64ull * E);
    std::vector<uint32_t> eoff(E + 1ull), eord(E), toff(64ull * E + 1);
    if (laspj_dict_export(S->dict, E, ebl.data(), eoff.data(), eord.data(), tbl.data(),
                          toff.data(), tord.data()) != LASPJ_OK)
        return fail(ctx, LASPJ_E_INVAL, "nif: dictionary export");
    free_etf(S);
    laspj_etf_dict* d = nullptr;
    // two tokens of headroom per element: a call that only adds tokens to known elements
    // patches the images (patch_etf) instead of coming back here
    if (int s = etf_dict_create_ex(ctx, E, ebl.data(), eoff.data(), eord.data(), tbl.data(),
                                   toff.data(), tord.data(), 2, &d))
        return s;
    S->etf = d;
    S->E = E;
    S->stale = false;
    S->built_K = n;
    S->built_cnt.resize(n);
    for (uint32_t e = 0; e < n; ++e) S->built_cnt[e] = dict_token_count(S->dict, e);
    ++S->stats[4];
    S->stats[13] += now_ns() - t0;
    return LASPJ_OK;
}

// Registrations that only added tokens to elements the images already hold: their rows
// patched in place.  False: rebuild (new elements, an element past its headroom, ...).
bool patch_etf(laspj_ctx* ctx, NifState* S) {
    if (!S->etf) return false;
    const uint64_t t0 = now_ns();
    const uint32_t n = dict_elements(S->dict);
    if (n != S->built_K || n > S->E) return false;
    std::vector<uint32_t> dirty;
    for (uint32_t e = 0; e < n; ++e)
        if (dict_token_count(S->dict, e) != S->built_cnt[e]) dirty.push_back(e);
    if (!dirty.empty() &&
        etf_dict_patch(ctx, S->etf, S->dict, dirty.data(), (uint32_t)dirty.size()) != LASPJ_OK)
        return false;
    for (uint32_t e : dirty) S->built_cnt[e] = dict_token_count(S->dict, e);
    S->stale = false;
    ++S->stats[14];
    S->stats[13] += now_ns() - t0;
    return true;
}

// One device pass: stage, copy, decode (or upload host-encoded cells), answer, copy back,
// one synchronisation.  Fills c.st / c.res / c.ooff / c.obase.

int device_pass(laspj_ctx* ctx, NifState* S, Call& c) {
    const uint64_t t0 = now_ns();
    uint64_t t_copy = 0;
    const uint32_t m = c.m, n = c.n, E = S->E;
    const bool dec = etf_dict_decodable(S->etf);
    std::vector<unsigned long long> hoffs(m + 1ull, 0);
    for (uint32_t i = 0; i < m; ++i) hoffs[i + 1] = hoffs[i] + c.len[i];
    const uint64_t pay = hoffs[m];
    EtfReadPlan plan;
    if (dec) etf_read_plan(ctx, S->etf, m, hoffs.data(), &plan);
    const bool has_payload_out = c.op == Op::MERGE || c.op == Op::VALUE;
    // in region (host -> device)
    // [offsets | segment table | zeroed words: the size pass's ticket, the decoder's redo
    //  list | payloads]
    const uint64_t i_offs = 0, i_seg = al(8ull * (m + 1), 256),
                   i_zero = i_seg + (plan.nseg ? al(4ull * (m + 1), 256) : 0),
                   // [ticket | redo list m + 1 | one-launch merge's look-back words]
                   z_lb = al(4ull * (m + 2), 16), z_bytes = z_lb + 8ull * ((E + 255) / 256),
                   i_pay = i_zero + al(z_bytes, 256);
    const uint64_t cells_in = (uint64_t)m * E * 16ull;
    const uint64_t in_bytes = i_pay + (dec ? al(pay + 64, 256) : al(cells_in, 256));
    // out region (device -> host)
    const uint64_t o_st = 0, o_res = al(4ull * m, 16), o_ooff = o_res + al(n, 16),
                   o_pay = o_ooff + al(8ull * (n + 1), 16);
    // answer payload bound: a merge's image is at most both operands' (flags may be
    // re-encoded one byte longer than a SMALL_ATOM_UTF8 input: the slack, and a second
    // copy when even that is short); value/1's at most its operand's
    uint64_t bound = 64ull * n + 64;
    for (uint32_t i = 0; i < m; ++i) bound += c.len[i];
    if (has_payload_out) {
        if (S->ocap < bound + bound / 8) S->ocap = al(bound + bound / 8, 1 << 16);
    }
    const uint64_t ocap = has_payload_out ? S->ocap : 0;
    const uint64_t out_bytes = o_pay + ocap;
    // MERGE: the segment decoder's chain check rides on the join's launch (ChainJob), its
    // per-segment results in a device area of their own after the out region
    const bool defer = dec && plan.nseg && c.op == Op::MERGE && !c.no_defer &&
                       etf_merge_fused(ctx, n, E);
    const uint64_t seg_bytes = defer ? al(plan.nseg * kSegResBytes, 256) : 0;
    // cells: in batch m x E; MERGE: answers n x E; VALUE: value words n x ceil(E/64)
    const uint64_t W = (E + 63ull) / 64ull;
    const uint64_t cells_out = c.op == Op::MERGE ? (uint64_t)n * E * 16ull
                               : c.op == Op::VALUE ? (uint64_t)n * W * 8ull : 0;
    const uint64_t c_out = al(cells_in, 256);
    std::vector<uint8_t> blob;      // the host-encode path's contiguous payloads
    {
        Guard g(ctx);
        if (int s = grow_dev(ctx, &S->dblk, &S->dblk_bytes,
                             al(in_bytes, 256) + al(out_bytes, 256) + seg_bytes))
            return s;
        const uint64_t had = S->dcells_bytes;
        if (int s = grow_dev(ctx, &S->dcells, &S->dcells_bytes, c_out + cells_out + 256)) return s;
        if (S->dcells_bytes != had) S->clean_words = 0;
        if (ctx->tune_nif_direct && !S->h_coherent) {
            // the staging reallocated coherent (once: it stays so)
            hipStreamSynchronize(ctx->stream);
            if (S->hin) hipHostFree(S->hin);
            if (S->hout) hipHostFree(S->hout);
            S->hin = S->hout = nullptr;
            S->hin_bytes = S->hout_bytes = 0;
            S->h_coherent = true;
        }
        if (int s = grow_host(ctx, &S->hin, &S->hin_bytes, in_bytes, S->h_coherent)) return s;
        if (int s = grow_host(ctx, &S->hout, &S->hout_bytes, out_bytes, S->h_coherent)) return s;
    }
    uint8_t* hin = static_cast<uint8_t*>(S->hin);
    uint8_t* din = static_cast<uint8_t*>(S->dblk);
    uint8_t* dout = din + al(in_bytes, 256);
    // LASPJ_TUNE_NIF_DIRECT: the decoder reads the in region where the host staged it (the
    // zeroed words stay on the device), the answer's kernels write the out region where
    // the host reads it
    // (bit 2: a kernel pulls the in region to the device instead)
    const bool pull_in = dec && (ctx->tune_nif_direct & 4);
    const bool direct_in = dec && (ctx->tune_nif_direct & 1) && !pull_in;
    const bool direct_out = (ctx->tune_nif_direct & 2) != 0;
    uint8_t* rin = din;                  // where the kernels read the in region
    uint8_t* rout = dout;                // where they write the out region
    const uint8_t* hin_d = nullptr;      // the staging as the device addresses it
    if (direct_in || pull_in || direct_out) {
        // (looked up once per allocation: the runtime's lookup costs host microseconds)
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
        if (direct_in || pull_in) {
            hin_d = S->hin_d;
            if (direct_in) rin = S->hin_d;
        }
        if (direct_out) rout = S->hout_d;
    }
    uint64_t* cin = static_cast<uint64_t*>(S->dcells);
    uint64_t* cout = reinterpret_cast<uint64_t*>(static_cast<uint8_t*>(S->dcells) + c_out);
    std::memcpy(hin + i_offs, hoffs.data(), 8ull * (m + 1));
    if (plan.nseg) std::memcpy(hin + i_seg, plan.segbase.data(), 4ull * (m + 1));
    std::memset(hin + i_zero, 0, z_bytes);
    uint32_t* dticket = reinterpret_cast<uint32_t*>(din + i_zero);
    auto* dlb = reinterpret_cast<unsigned long long*>(din + i_zero + z_lb);
    const uint64_t in_words = (uint64_t)m * 2ull * E;
    const bool clean = S->clean_E == E && S->clean_words >= in_words;
    std::vector<int32_t> hst;
    if (!dec) {
        // token images of several lengths (or no tokens yet): the host dictionary encodes
        // the cells (laspj_dict_encode), the device does the rest
        blob.resize(pay);
        for (uint32_t i = 0; i < m; ++i)
            if (c.len[i]) std::memcpy(blob.data() + hoffs[i], c.p[i], c.len[i]);
        hst.assign(m, 0);
        if (int s = laspj_dict_encode(S->dict, LASPJ_KIND_ORSET, blob.data(),
                                      reinterpret_cast<const uint64_t*>(hoffs.data()), m, -1, E,
                                      reinterpret_cast<uint64_t*>(hin + i_pay), hst.data()))
            return fail(ctx, s, "nif: host encode failed (%d)", s);
        ++S->stats[5];
    }
    {
        Guard g(ctx);
        // the offsets (and segment table), then the payloads a piece at a time: each
        // piece's copy starts while the next one is staged
        if (direct_in) {
            // staged whole; only the zeroed words go to the device
            uint64_t at = 0;
            const uint64_t tc = now_ns();
            for (uint32_t i = 0; i < m; ++i) {
                if (c.len[i]) std::memcpy(hin + i_pay + at, c.p[i], c.len[i]);
                at += c.len[i];
            }
            t_copy += now_ns() - tc;
            LJ_HIP(ctx, hipMemsetAsync(din + i_zero, 0, z_bytes, ctx->stream));
        } else if (dec) {
            uint64_t at = 0;
            uint32_t i = 0;
            uint64_t io = 0;                     // offset inside payload i
            uint64_t sent = 0;                   // region bytes already copied
            const uint64_t head = i_pay;
            while (i < m && c.len[i] == 0) ++i;
            // (a kernel pulls each piece: while it runs the host stages the next)
            const uint64_t dflt = pull_in ? kPullPiece : kStagePiece;
            auto send = [&](uint64_t upto) -> int {
                if (!pull_in) {
                    LJ_HIP(ctx, hipMemcpyAsync(din + sent, hin + sent, upto - sent,
                                               hipMemcpyHostToDevice, ctx->stream));
                    return LASPJ_OK;
                }
                // 16-byte lanes: sent is a multiple of 16 (the head is 256-aligned, pieces
                // 4096-multiples), upto is rounded up inside the staged region
                const uint64_t n16 = (al(upto, 16) - sent) / 16;
                const uint64_t blocks = std::min<uint64_t>((n16 + 255) / 256,
                                                           (uint64_t)ctx->cus * 4);
                hipLaunchKernelGGL(k_nif_pull, dim3((unsigned)std::max<uint64_t>(blocks, 1)),
                                   dim3(256), 0, ctx->stream,
                                   reinterpret_cast<const pull16*>(hin_d + sent),
                                   reinterpret_cast<pull16*>(din + sent), n16);
                LJ_LAUNCHED(ctx);
                return LASPJ_OK;
            };
            while (at < pay) {
                uint64_t piece = ctx->tune_nif_piece ? (uint64_t)ctx->tune_nif_piece : dflt;
                piece = std::min(piece, pay - at);
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
                const uint64_t upto = head + at;
                if (int s = send(upto)) return s;
                sent = upto;
            }
            if (pay == 0)
                if (int s = send(head)) return s;
        } else {
            LJ_HIP(ctx, hipMemcpyAsync(din, hin, i_pay, hipMemcpyHostToDevice, ctx->stream));
            LJ_HIP(ctx, hipMemcpyAsync(cin, hin + i_pay, cells_in, hipMemcpyHostToDevice,
                                       ctx->stream));
        }
        laspj_batch inb = view(ctx, LASPJ_KIND_ORSET, m, E, cin);
        int32_t* dst = reinterpret_cast<int32_t*>(rout + o_st);
        ChainJob cjob;
        if (defer) cjob.res = din + al(in_bytes, 256) + al(out_bytes, 256);
        if (dec) {
            if (int s = etf_read_enqueue(ctx, &inb, S->etf, -1, 1, rin + i_pay, pay,
                                         reinterpret_cast<const unsigned long long*>(rin + i_offs),
                                         plan,
                                         plan.nseg ? reinterpret_cast<const uint32_t*>(rin + i_seg)
                                                   : nullptr,
                                         dst, !clean, dticket + 1, defer ? &cjob : nullptr))
                return s;
        }
        laspj_batch lhs = view(ctx, LASPJ_KIND_ORSET, n, E, cin);
        laspj_batch rhs = view(ctx, LASPJ_KIND_ORSET, n, E, cin + (uint64_t)n * 2ull * E);
        auto* dooff = reinterpret_cast<unsigned long long*>(rout + o_ooff);
        uint8_t* dopay = rout + o_pay;
        switch (c.op) {
        case Op::MERGE: {
            // lasp_orset:merge/2 (lasp_orset.erl:128-134): the nested orddict:merge of two
            // canonical orddicts is the slot-wise OR of their cells
            laspj_batch ob = view(ctx, LASPJ_KIND_ORSET, n, E, cout);
            const unsigned long long* chunks = nullptr;
            if (etf_merge_write_one(ctx, S->etf, n, E)) {
                // one answer: join, size pass and writer in one launch (look-back), the
                // operands cleared behind it, the chain checks riding along
                if (int s = etf_merge_write_enqueue(ctx, lhs.dev, rhs.dev, E, S->etf, -1, 1, dooff,
                                                    dopay, ocap, dlb, dticket, &cjob))
                    return s;
                S->clean_words = in_words;
                S->clean_E = E;
                break;
            }
            if (etf_merge_fused(ctx, n, E)) {
                // the OR fused with the answer's size pass, the operands cleared behind it
                if (int s = etf_merge_size_enqueue(ctx, lhs.dev, rhs.dev, &ob, S->etf, -1, dooff,
                                                   ctx->flag, dticket, &chunks, &cjob))
                    return s;
                S->clean_words = in_words;
                S->clean_E = E;
            } else {
                LJ_HIP(ctx, launch_or(ctx, cout, lhs.dev, rhs.dev, (uint64_t)n * 2ull * E));
                if (int s = etf_size_enqueue(ctx, &ob, S->etf, LASPJ_KIND_ORSET, -1, dooff,
                                             ctx->flag, &chunks))
                    return s;
                S->clean_words = 0;
            }
            if (int s = etf_write_enqueue(ctx, &ob, S->etf, LASPJ_KIND_ORSET, -1, 1, dooff, dopay,
                                          ocap, chunks))
                return s;
            break;
        }
        case Op::VALUE: {
            S->clean_words = 0;
            // value/1 (lasp_orset.erl:67-73): the elements with a {_, false} token, as the
            // ordset image the G-Set writer gives a bit row (term_to_binary of the keys)
            LJ_HIP(ctx, launch_orset_value(ctx, &inb, cout, false));
            laspj_batch vb = view(ctx, LASPJ_KIND_GSET, n, E, cout);
            if (int s = etf_size_enqueue(ctx, &vb, S->etf, LASPJ_KIND_GSET, -1, dooff, ctx->flag,
                                         nullptr))
                return s;
            if (int s = etf_write_enqueue(ctx, &vb, S->etf, LASPJ_KIND_GSET, -1, 1, dooff, dopay,
                                          ocap, nullptr))
                return s;
            break;
        }
        case Op::EQUAL:
            S->clean_words = 0;
            // equal/2 (lasp_orset.erl:136-138): ORDictA == ORDictB
            LJ_HIP(ctx, launch_equal(ctx, &lhs, &rhs, rout + o_res));
            break;
        case Op::INFLATION:
            S->clean_words = 0;
            // is_inflation / is_strict_inflation (lasp_lattice.erl:153-161, 235-253)
            LJ_HIP(ctx, launch_orset_inflation(ctx, &lhs, &rhs, c.strict != 0, rout + o_res));
            break;
        }
        const uint64_t first = o_pay + (has_payload_out ? std::min(ocap, bound) : 0);
        if (!direct_out)
            LJ_HIP(ctx, hipMemcpyAsync(S->hout, dout, first, hipMemcpyDeviceToHost, ctx->stream));
        const uint64_t t1 = now_ns();
        LJ_HIP(ctx, hipStreamSynchronize(ctx->stream));
        const uint64_t t2 = now_ns();
        ++S->stats[1];
        S->stats[8] += t1 - t0;
        S->stats[9] += t2 - t1;
        S->stats[11] += t_copy;
        const uint8_t* hout = static_cast<const uint8_t*>(S->hout);
        c.st.assign(m, 0);
        if (dec) std::memcpy(c.st.data(), hout + o_st, 4ull * m);
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
                // the writer wrote nothing: a larger answer area, the encode again (the
                // cells are still in place)
                S->ocap = al(total + total / 4, 1 << 16);
                return -1000;            // caller re-runs the pass (rare)
            }
            if (!direct_out && total > first - o_pay) {
                LJ_HIP(ctx, hipMemcpyAsync(static_cast<uint8_t*>(S->hout) + first, dout + first,
                                           o_pay + total - first, hipMemcpyDeviceToHost,
                                           ctx->stream));
                LJ_HIP(ctx, hipStreamSynchronize(ctx->stream));
            }
            c.obase = hout + o_pay;
        }
        S->stats[10] += now_ns() - t2;
    }
    return LASPJ_OK;
}

int register_payloads(laspj_ctx* ctx, NifState* S, const std::vector<const uint8_t*>& p,
                      const std::vector<uint64_t>& len, std::vector<int32_t>* st) {
    const uint64_t t0 = now_ns();
    const uint64_t k = p.size();
    std::vector<uint64_t> offs(k + 1, 0);
    for (uint64_t i = 0; i < k; ++i) offs[i + 1] = offs[i] + len[i];
    std::vector<uint8_t> blob(offs[k] + 1);
    for (uint64_t i = 0; i < k; ++i)
        if (len[i]) std::memcpy(blob.data() + offs[i], p[i], len[i]);
    st->assign(k, 0);
    if (int s = laspj_dict_add(S->dict, LASPJ_KIND_ORSET, blob.data(), offs.data(), k, -1,
                               st->data()))
        return fail(ctx, s, "nif: dictionary registration failed (%d)", s);
    ++S->stats[2];
    S->stats[12] += now_ns() - t0;
    S->stale = true;
    return LASPJ_OK;
}

// A deferred pass's unknown terms: each failing segment of those operands (a status and a
// start: its first element, where the chain check found it) registers the elements that
// start in it — what the segment's decoder could not take; the segments that decoded hold
// known terms.  False: a range did not register (nothing is kept), the caller registers
// whole operands.
bool register_segments(laspj_ctx* ctx, NifState* S, const Call& c,
                       const std::vector<uint32_t>& ops) {
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
        if (dict_add_elems(S->dict, c.p[r.i], c.len[r.i], r.from, r.to) != LASPJ_DEC_OK)
            return false;       // (ranges already added stay: they hold well-formed terms)
    ++S->stats[2];
    S->stats[12] += now_ns() - t0;
    S->stale = true;
    return true;
}

// The call: device pass; operands with unknown terms registered and a second pass; every
// other undecodable operand -> FALLBACK.  verdict[j] per answer.
int run(laspj_ctx* ctx, NifState* S, Call& c, std::vector<int32_t>* verdict) {
    ++S->stats[0];
    if (!S->dict && reset_dict(ctx, S)) return LASPJ_E_NOMEM;
    const uint32_t n = c.n, m = c.m;
    auto answer_of = [&](uint32_t i) { return i % n; };
    std::vector<uint8_t> fallback(n, 0);
    bool registered = false;
    bool partial = false;           // the last registration took the failing segments only
    for (int pass = 0; pass < 4; ++pass) {
        if (!S->etf || S->stale) {
            if (!S->etf) {
                // nothing registered yet: register this call's operands first
                std::vector<int32_t> rst;
                if (int s = register_payloads(ctx, S, c.p, c.len, &rst)) return s;
                registered = true;
                for (uint32_t i = 0; i < m; ++i)
                    if (rst[i] != LASPJ_DEC_OK) fallback[answer_of(i)] = 1;
            }
            if (!patch_etf(ctx, S))
                if (int s = rebuild_etf(ctx, S)) return s;
        }
        int s = device_pass(ctx, S, c);
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
        if (unknown.empty()) break;
        if (!registered && c.has_seg && register_segments(ctx, S, c, unknown)) {
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
        laspj_dict_info(S->dict, &nd, &eb, &tb);
        std::vector<int32_t> rst;
        if (int s2 = register_payloads(ctx, S, rp, rl, &rst)) return s2;
        bool full = false;
        for (int32_t x : rst) full |= x == LASPJ_DEC_UNREPRESENTABLE;
        laspj_dict_info(S->dict, &nd, &eb, &tb);
        if ((full && nd) || nd > kMaxDictElements) {
            // an element's 64 token slots used up by earlier calls (or a dictionary grown
            // past its bound): start a fresh dictionary holding this call's terms only —
            // calls are self-contained (images in, images out), so nothing else refers to
            // the old slots
            if (int s2 = reset_dict(ctx, S)) return s2;
            if (int s2 = register_payloads(ctx, S, c.p, c.len, &rst)) return s2;
            for (uint32_t i = 0; i < m; ++i)
                if (rst[i] != LASPJ_DEC_OK) fallback[answer_of(i)] = 1;
        } else {
            for (size_t k = 0; k < ri.size(); ++k)
                if (rst[k] != LASPJ_DEC_OK) fallback[answer_of(ri[k])] = 1;
        }
        registered = true;
    }
    verdict->assign(n, LASPJ_NIF_OK);
    for (uint32_t j = 0; j < n; ++j)
        if (fallback[j]) {
            (*verdict)[j] = LASPJ_NIF_FALLBACK;
            ++S->stats[6];
        }
    return LASPJ_OK;
}

NifState* state(laspj_ctx* ctx) {
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (!ctx->nif) ctx->nif = new (std::nothrow) NifState;
    return ctx->nif;
}

}  // namespace

void nif_destroy(laspj_ctx* ctx) {
    NifState* S = ctx->nif;
    if (!S) return;
    if (S->etf) laspj_etf_dict_destroy(S->etf);
    if (S->dict) laspj_dict_destroy(S->dict);
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

int pair_call(laspj_ctx* ctx, laspj::NifState* S, laspj::Op op, int strict, uint32_t n,
              const uint8_t* const* a, const uint64_t* na, const uint8_t* const* b,
              const uint64_t* nb, laspj::Call* c, std::vector<int32_t>* verdict) {
    if (!n || !a || !na || (op != laspj::Op::VALUE && (!b || !nb)))
        return fail(ctx, LASPJ_E_INVAL, "nif: null operand array");
    const uint32_t per = op == laspj::Op::VALUE ? 1u : 2u;
    if ((uint64_t)n * per > (1ull << 31))
        return fail(ctx, LASPJ_E_RANGE, "nif: too many operands");
    c->op = op;
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

}  // namespace

extern "C" {

int laspj_orset_etf_merge_many(laspj_ctx* ctx, uint32_t n, const uint8_t* const* a,
                               const uint64_t* na, const uint8_t* const* b, const uint64_t* nb,
                               const uint8_t** out, uint64_t* out_len, int32_t* verdict) {
    if (!ctx) return LASPJ_E_INVAL;
    if (!out || !out_len || !verdict) return fail(ctx, LASPJ_E_INVAL, "nif: null output array");
    laspj::NifState* S = laspj::state(ctx);
    if (!S) return fail(ctx, LASPJ_E_NOMEM, "nif: state allocation");
    std::lock_guard<std::mutex> lk(S->mu);
    laspj::Call c;
    std::vector<int32_t> v;
    if (int s = pair_call(ctx, S, laspj::Op::MERGE, 0, n, a, na, b, nb, &c, &v)) return s;
    for (uint32_t i = 0; i < n; ++i) {
        verdict[i] = v[i];
        out[i] = v[i] == LASPJ_NIF_OK ? c.obase + c.ooff[i] : nullptr;
        out_len[i] = v[i] == LASPJ_NIF_OK ? c.ooff[i + 1] - c.ooff[i] : 0;
    }
    return LASPJ_OK;
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
    if (int st = pair_call(ctx, S, laspj::Op::VALUE, 0, 1, &s, &ns, nullptr, nullptr, &c, &v))
        return st;
    *verdict = v[0];
    *out = v[0] == LASPJ_NIF_OK ? c.obase + c.ooff[0] : nullptr;
    *out_len = v[0] == LASPJ_NIF_OK ? c.ooff[1] - c.ooff[0] : 0;
    return LASPJ_OK;
}

static int bool_call(laspj_ctx* ctx, laspj::Op op, int strict, const uint8_t* a, uint64_t na,
                     const uint8_t* b, uint64_t nb, int32_t* result, int32_t* verdict) {
    if (!ctx) return LASPJ_E_INVAL;
    if (!result || !verdict) return fail(ctx, LASPJ_E_INVAL, "nif: null output");
    laspj::NifState* S = laspj::state(ctx);
    if (!S) return fail(ctx, LASPJ_E_NOMEM, "nif: state allocation");
    std::lock_guard<std::mutex> lk(S->mu);
    laspj::Call c;
    std::vector<int32_t> v;
    if (int s = pair_call(ctx, S, op, strict, 1, &a, &na, &b, &nb, &c, &v)) return s;
    *verdict = v[0];
    *result = v[0] == LASPJ_NIF_OK ? (int32_t)(c.res[0] != 0) : 0;
    return LASPJ_OK;
}

int laspj_orset_etf_equal(laspj_ctx* ctx, const uint8_t* a, uint64_t na, const uint8_t* b,
                          uint64_t nb, int32_t* result, int32_t* verdict) {
    return bool_call(ctx, laspj::Op::EQUAL, 0, a, na, b, nb, result, verdict);
}

int laspj_orset_etf_inflation(laspj_ctx* ctx, const uint8_t* prev, uint64_t np,
                              const uint8_t* cur, uint64_t nc, int strict, int32_t* result,
                              int32_t* verdict) {
    return bool_call(ctx, laspj::Op::INFLATION, strict ? 1 : 0, prev, np, cur, nc, result,
                     verdict);
}

int laspj_nif_stats(laspj_ctx* ctx, uint64_t* out, uint32_t n) {
    if (!ctx || (n && !out)) return LASPJ_E_INVAL;
    laspj::NifState* S = laspj::state(ctx);
    if (!S) return fail(ctx, LASPJ_E_NOMEM, "nif: state allocation");
    std::lock_guard<std::mutex> lk(S->mu);
    for (uint32_t i = 0; i < n && i < LASPJ_NIF_STATS; ++i) out[i] = S->stats[i];
    if (n > 7) {
        uint32_t e = 0;  // [7] is the dictionary's size, not a counter
        uint64_t eb, tb;
        out[7] = S->dict && laspj_dict_info(S->dict, &e, &eb, &tb) == LASPJ_OK ? e : 0;
    }
    return LASPJ_OK;
}

int laspj_nif_reset(laspj_ctx* ctx) {
    if (!ctx) return LASPJ_E_INVAL;
    laspj::NifState* S = laspj::state(ctx);
    if (!S) return fail(ctx, LASPJ_E_NOMEM, "nif: state allocation");
    std::lock_guard<std::mutex> lk(S->mu);
    return laspj::reset_dict(ctx, S);
}

}  // extern "C"
