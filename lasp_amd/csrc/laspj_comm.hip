// Anti-entropy across GPUs behind the C ABI (BASELINE config 3).
//
// The reference's fan-out -> N-way fold-merge -> read-repair (lasp_update_fsm.erl:174-216,
// lasp_bind_fsm.erl:170-212, coverage reduce lasp_execute_coverage_fsm.erl:59-62) is an
// all-reduce whose operator is the lattice join.  Every rank holds one replica of each
// object; a round leaves every rank with the join of all ranks' replicas:
//   * bitmap kinds (OR-Set, G-Set): RCCL has no bitwise-OR reduction and max on packed
//     masks is not a join, so a round is a grouped ncclSend/ncclRecv all-to-all (rank j
//     receives every rank's copy of object chunk j: the reduce-scatter layout, driving
//     all n-1 xGMI links at once), the HIP reduce kernel (one OR over the n copies, in
//     place), and an all-gather of the joined chunks made of the same grouped
//     ncclSend/ncclRecv pieces (1 GiB each: one p2p call moves at most 4 GiB);
//   * G-Counters: the join IS the per-actor max, so a round is one ncclAllReduce(ncclMax)
//     on ncclUint64 counts (the unsigned max the device join uses).
// All phases are enqueued on the engine context's stream: RCCL, the reduce kernel and the
// next round are ordered by the stream, with no host synchronisation.
//
// RCCL is loaded at run time (dlopen): the copy already in the process (torch's bundled
// librccl.so.1) if there is one, else ROCm's.  A library without RCCL still loads; the
// comm entry points then return LASPJ_E_UNSUPPORTED.

#include <dlfcn.h>

#include <cstring>
#include <memory>
#include <new>
#include <vector>

#include <rccl/rccl.h>

#include "laspj_internal.h"

struct laspj_comm {
    laspj_ctx* ctx = nullptr;
    ncclComm_t comm = nullptr;
    int rank = 0;
    int nranks = 1;
};

namespace {

using laspj::fail;

struct Rccl {
    bool tried = false, ok = false;
    std::string why;
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t,
                              ncclComm_t, hipStream_t) = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

std::mutex g_rccl_mu;
Rccl g_rccl;

template <class F>
bool sym(void* h, const char* name, F* out) {
    *out = reinterpret_cast<F>(dlsym(h, name));
    return *out != nullptr;
}

const Rccl* rccl() {
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    Rccl& r = g_rccl;
    if (r.tried) return r.ok ? &r : nullptr;
    r.tried = true;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        const char* e = dlerror();
        r.why = e ? e : "dlopen(librccl.so.1) failed";
        return nullptr;
    }
    r.ok = sym(h, "ncclGetUniqueId", &r.GetUniqueId) && sym(h, "ncclCommInitRank", &r.CommInitRank) &&
           sym(h, "ncclCommInitAll", &r.CommInitAll) && sym(h, "ncclCommDestroy", &r.CommDestroy) &&
           sym(h, "ncclGroupStart", &r.GroupStart) && sym(h, "ncclGroupEnd", &r.GroupEnd) &&
           sym(h, "ncclSend", &r.Send) && sym(h, "ncclRecv", &r.Recv) &&
           sym(h, "ncclAllReduce", &r.AllReduce) &&
           sym(h, "ncclGetErrorString", &r.GetErrorString);
    if (!r.ok) r.why = "librccl lacks a required symbol";
    return r.ok ? &r : nullptr;
}

#define LJ_NCCL(ctx, R, call)                                                               \
    do {                                                                                    \
        ncclResult_t e_ = (call);                                                           \
        if (e_ != ncclSuccess)                                                              \
            return fail((ctx), LASPJ_E_COMM, "%s: %s", #call, (R)->GetErrorString(e_));     \
    } while (0)

struct CGuard {
    std::lock_guard<std::mutex> lk;
    explicit CGuard(laspj_ctx* c) : lk(c->mu) { hipSetDevice(c->device); }
};

bool set_kind(int32_t k) {
    return k == LASPJ_KIND_ORSET || k == LASPJ_KIND_GSET || k == LASPJ_KIND_GCOUNTER;
}

// shapes of one rank's round: state R objects (R % n == 0), recv >= (n-1) R / n objects
// (may be NULL when n == 1), chunk (optional, unused) R / n objects
int round_checks(const laspj_comm* c, const laspj_batch* state, const laspj_batch* recv,
                 const laspj_batch* chunk, const char* what) {
    laspj_ctx* ctx = c->ctx;
    if (!state || state->ctx != ctx || !set_kind(state->kind))
        return fail(ctx, LASPJ_E_INVAL, "%s: state must be an OR-Set, G-Set or G-Counter batch of "
                    "the communicator's context", what);
    if (state->kind == LASPJ_KIND_GCOUNTER) return LASPJ_OK;   // in place, no scratch
    const uint64_t n = (uint64_t)c->nranks;
    if (n > 8)
        return fail(ctx, LASPJ_E_UNSUPPORTED, "%s: more than 8 ranks (one node's GPUs)", what);
    if (!recv && n > 1) return fail(ctx, LASPJ_E_INVAL, "%s: recv batch missing", what);
    if (recv && recv->ctx != ctx) return fail(ctx, LASPJ_E_INVAL, "%s: recv of another context", what);
    if ((recv && recv->kind != state->kind) || (chunk && chunk->kind != state->kind))
        return fail(ctx, LASPJ_E_KIND, "%s: kinds differ", what);
    if (state->replicas % n ||
        (recv && (recv->replicas < state->replicas / n * (n - 1) ||
                  recv->elements != state->elements)) ||
        (chunk && (chunk->replicas * n != state->replicas || chunk->elements != state->elements)))
        return fail(ctx, LASPJ_E_SHAPE, "%s: need objects %% ranks == 0, recv >= (ranks-1) / "
                    "ranks x objects (chunk, when given = objects / ranks)", what);
    if (recv) {
        const uint64_t sb = laspj::bytes_of(state), rb = laspj::bytes_of(recv);
        const uintptr_t s0 = (uintptr_t)state->dev, r0 = (uintptr_t)recv->dev;
        if (s0 < r0 + rb && r0 < s0 + sb)
            return fail(ctx, LASPJ_E_INVAL, "%s: state and recv must not overlap", what);
    }
    if ((state->words_per_replica * (state->replicas / n)) & 1)
        return fail(ctx, LASPJ_E_SHAPE, "%s: a chunk must hold an even word count", what);
    return LASPJ_OK;
}

// RCCL point-to-point calls move at most 4 GiB each (measured: a 64 GiB ncclSend/Recv
// pair delivered only the first 2^32 bytes, tools/ae_probe.py), so every transfer goes
// in pieces of 2^27 words (1 GiB).
constexpr uint64_t kPiece = 1ull << 27;

// The schedule (laspj_antientropy_plan).  Bitmap kinds:
//   all-to-all: piece k of every peer's chunk is one group -- SEND this rank's copy of
//     chunk p (state words [p cw + k P, ...)) to p, RECV p's copy of this rank's chunk into
//     recv slot p - (p > rank);
//   reduce: the rank's own chunk joined in place with the n-1 received copies;
//   all-gather: piece k of the joined chunk to every peer, and every peer's joined chunk
//     into its place in state.
// Per round this rank moves (n-1)/n S over xGMI each way and reads S + writes S/n of HBM
// for the join.  G-Counters: all-reduce(max) of each piece of the state.
struct Plan {
    laspj_ae_step* out;
    uint64_t cap, n = 0;
    void put(const laspj_ae_step& s) {
        if (out && n < cap) out[n] = s;
        ++n;
    }
};

void plan_steps(Plan& P, int32_t kind, int rank, int nranks, uint64_t words, uint64_t piece) {
    uint32_t group = 0;
    if (kind == LASPJ_KIND_GCOUNTER) {
        if (nranks == 1) return;
        for (uint64_t off = 0; off < words; off += piece)
            P.put({group++, LASPJ_AE_ALLREDUCE_MAX, -1, LASPJ_AE_BUF_STATE, off,
                   words - off < piece ? words - off : piece, 0, 0, 0});
        return;
    }
    if (nranks == 1) return;                       // the join of one copy: nothing to do
    const uint64_t cw = words / (uint64_t)nranks;
    const uint64_t pieces = (cw + piece - 1) / piece;
    auto slot = [&](int p) { return (uint64_t)(p - (p > rank ? 1 : 0)); };
    for (uint64_t k = 0; k < pieces; ++k, ++group) {
        const uint64_t off = k * piece, len = cw - off < piece ? cw - off : piece;
        for (int d = 1; d < nranks; ++d) {
            const int to = (rank + d) % nranks, from = (rank - d + nranks) % nranks;
            P.put({group, LASPJ_AE_SEND, to, LASPJ_AE_BUF_STATE, (uint64_t)to * cw + off, len,
                   0, 0, (uint32_t)k});
            P.put({group, LASPJ_AE_RECV, from, LASPJ_AE_BUF_RECV, slot(from) * cw + off, len,
                   0, 0, (uint32_t)k});
        }
    }
    P.put({group++, LASPJ_AE_REDUCE, -1, LASPJ_AE_BUF_STATE, (uint64_t)rank * cw, cw, 0,
           (uint32_t)(nranks - 1), 0});
    for (uint64_t k = 0; k < pieces; ++k, ++group) {
        const uint64_t off = k * piece, len = cw - off < piece ? cw - off : piece;
        for (int d = 1; d < nranks; ++d) {
            const int to = (rank + d) % nranks, from = (rank - d + nranks) % nranks;
            P.put({group, LASPJ_AE_SEND, to, LASPJ_AE_BUF_STATE, (uint64_t)rank * cw + off, len,
                   0, 0, (uint32_t)k});
            P.put({group, LASPJ_AE_RECV, from, LASPJ_AE_BUF_STATE, (uint64_t)from * cw + off,
                   len, 0, 0, (uint32_t)k});
        }
    }
}

// the words a SEND / RECV step reads / writes
uint64_t* step_words(const laspj_ae_step& s, laspj_batch* state, laspj_batch* recv) {
    uint64_t* bufs[2] = {state->dev, recv ? recv->dev : nullptr};
    return bufs[s.buf] + s.offset;
}

// a REDUCE step: the rank's own chunk joined in place with the received copies
int reduce_step(laspj_ctx* ctx, const laspj_ae_step& s, laspj_batch* state, laspj_batch* recv) {
    uint64_t* own = state->dev + s.offset;
    const uint64_t* srcs[8];
    srcs[0] = own;
    for (uint32_t j = 0; j < s.nsrc; ++j) srcs[1 + j] = recv->dev + s.src + j * s.words;
    LJ_HIP(ctx, laspj::launch_reduce_ptrs(ctx, own, srcs, s.nsrc + 1, s.words,
                                          state->kind == LASPJ_KIND_GCOUNTER));
    return LASPJ_OK;
}

// one step of a plan on the context's stream
int run_step(const Rccl* R, laspj_comm* c, const laspj_ae_step& s, laspj_batch* state,
             laspj_batch* recv) {
    laspj_ctx* ctx = c->ctx;
    switch (s.op) {
    case LASPJ_AE_SEND:
        LJ_NCCL(ctx, R, R->Send(step_words(s, state, recv), s.words, ncclUint64, s.peer, c->comm,
                                ctx->stream));
        return LASPJ_OK;
    case LASPJ_AE_RECV:
        LJ_NCCL(ctx, R, R->Recv(step_words(s, state, recv), s.words, ncclUint64, s.peer, c->comm,
                                ctx->stream));
        return LASPJ_OK;
    case LASPJ_AE_REDUCE:
        return reduce_step(ctx, s, state, recv);
    case LASPJ_AE_ALLREDUCE_MAX:
        LJ_NCCL(ctx, R, R->AllReduce(state->dev + s.offset, state->dev + s.offset, s.words,
                                     ncclUint64, ncclMax, c->comm, ctx->stream));
        return LASPJ_OK;
    }
    return fail(ctx, LASPJ_E_INVAL, "antientropy: bad plan step");
}

}  // namespace

extern "C" {

int laspj_comm_unique_id(uint8_t* id) {
    if (!id) return LASPJ_E_INVAL;
    const Rccl* R = rccl();
    if (!R) return LASPJ_E_UNSUPPORTED;
    ncclUniqueId u;
    if (R->GetUniqueId(&u) != ncclSuccess) return LASPJ_E_COMM;
    memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
    return LASPJ_OK;
}

int laspj_comm_init_rank(laspj_ctx* ctx, int nranks, const uint8_t* id, int rank,
                         laspj_comm** out) {
    if (!ctx || !id || !out || nranks < 1 || rank < 0 || rank >= nranks)
        return fail(ctx, LASPJ_E_INVAL, "comm_init_rank: bad argument");
    *out = nullptr;
    const Rccl* R = rccl();
    if (!R) return fail(ctx, LASPJ_E_UNSUPPORTED, "comm_init_rank: RCCL not loadable: %s",
                        g_rccl.why.c_str());
    auto* c = new (std::nothrow) laspj_comm;
    if (!c) return fail(ctx, LASPJ_E_NOMEM, "comm_init_rank: host allocation");
    c->ctx = ctx;
    c->rank = rank;
    c->nranks = nranks;
    ncclUniqueId u;
    memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
    ncclResult_t e;
    {
        CGuard g(ctx);
        e = R->CommInitRank(&c->comm, nranks, u, rank);
    }
    if (e != ncclSuccess) {
        delete c;
        return fail(ctx, LASPJ_E_COMM, "ncclCommInitRank: %s", R->GetErrorString(e));
    }
    *out = c;
    return LASPJ_OK;
}

int laspj_comm_init_all(laspj_ctx* const* ctxs, int n, laspj_comm** out) {
    if (!ctxs || !out || n < 1) return LASPJ_E_INVAL;
    for (int i = 0; i < n; ++i) {
        if (!ctxs[i]) return LASPJ_E_INVAL;
        out[i] = nullptr;
    }
    const Rccl* R = rccl();
    if (!R) return fail(ctxs[0], LASPJ_E_UNSUPPORTED, "comm_init_all: RCCL not loadable: %s",
                        g_rccl.why.c_str());
    std::vector<int> devs(n);
    for (int i = 0; i < n; ++i) devs[i] = ctxs[i]->device;
    std::vector<ncclComm_t> comms(n);
    ncclResult_t e = R->CommInitAll(comms.data(), n, devs.data());
    if (e != ncclSuccess)
        return fail(ctxs[0], LASPJ_E_COMM, "ncclCommInitAll: %s", R->GetErrorString(e));
    for (int i = 0; i < n; ++i) {
        auto* c = new (std::nothrow) laspj_comm;
        if (!c) {
            for (int j = 0; j < n; ++j) {
                if (j < i) delete out[j];
                R->CommDestroy(comms[j]);
                out[j] = nullptr;
            }
            return fail(ctxs[0], LASPJ_E_NOMEM, "comm_init_all: host allocation");
        }
        c->ctx = ctxs[i];
        c->comm = comms[i];
        c->rank = i;
        c->nranks = n;
        out[i] = c;
    }
    return LASPJ_OK;
}

int laspj_comm_destroy(laspj_comm* c) {
    if (!c) return LASPJ_E_INVAL;
    const Rccl* R = rccl();
    {
        CGuard g(c->ctx);
        hipStreamSynchronize(c->ctx->stream);
        if (R && c->comm) R->CommDestroy(c->comm);
    }
    delete c;
    return LASPJ_OK;
}

int laspj_comm_info(const laspj_comm* c, int* rank, int* nranks) {
    if (!c) return LASPJ_E_INVAL;
    if (rank) *rank = c->rank;
    if (nranks) *nranks = c->nranks;
    return LASPJ_OK;
}

int laspj_antientropy(laspj_comm* c, laspj_batch* state, laspj_batch* recv, laspj_batch* chunk) {
    return laspj_antientropy_group(&c, &state, &recv, &chunk, 1);
}

int laspj_antientropy_group(laspj_comm* const* cs, laspj_batch* const* state,
                            laspj_batch* const* recv, laspj_batch* const* chunk, int n) {
    if (!cs || !state || n < 1) return LASPJ_E_INVAL;
    for (int i = 0; i < n; ++i)
        if (!cs[i] || !cs[i]->ctx) return LASPJ_E_INVAL;
    const Rccl* R = rccl();
    if (!R) return fail(cs[0]->ctx, LASPJ_E_UNSUPPORTED, "antientropy: RCCL not loadable");
    for (int i = 0; i < n; ++i)
        if (int s = round_checks(cs[i], state[i], recv ? recv[i] : nullptr,
                                 chunk ? chunk[i] : nullptr, "antientropy"))
            return s;
    const bool max_join = state[0]->kind == LASPJ_KIND_GCOUNTER;
    for (int i = 1; i < n; ++i)
        if ((state[i]->kind == LASPJ_KIND_GCOUNTER) != max_join ||
            cs[i]->nranks != cs[0]->nranks || laspj::bytes_of(state[i]) != laspj::bytes_of(state[0]))
            return fail(cs[0]->ctx, LASPJ_E_KIND, "antientropy: one group needs one kind, "
                        "world and state size");
    // one process may drive several GPUs: group g of every communicator's plan is one RCCL
    // group over all of them (the device is set per call; the contexts' mutexes serialise
    // other callers)
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < i; ++j)
            if (cs[j]->ctx == cs[i]->ctx)
                return fail(cs[0]->ctx, LASPJ_E_INVAL, "antientropy: one context twice");
    std::vector<std::vector<laspj_ae_step>> plans(n);
    for (int i = 0; i < n; ++i) {
        const uint64_t words = state[i]->replicas * state[i]->words_per_replica;
        Plan P{nullptr, 0};
        plan_steps(P, state[i]->kind, cs[i]->rank, cs[i]->nranks, words, kPiece);
        plans[i].resize(P.n);
        Plan Q{plans[i].data(), P.n};
        plan_steps(Q, state[i]->kind, cs[i]->rank, cs[i]->nranks, words, kPiece);
    }
    std::vector<std::unique_ptr<CGuard>> guards;
    for (int i = 0; i < n; ++i) guards.emplace_back(new CGuard(cs[i]->ctx));
    std::vector<size_t> at(n, 0);
    for (uint32_t g = 0;; ++g) {
        bool any = false, comm = false;
        for (int i = 0; i < n; ++i)
            if (at[i] < plans[i].size() && plans[i][at[i]].group == g) {
                any = true;
                const int32_t op = plans[i][at[i]].op;
                comm |= op == LASPJ_AE_SEND || op == LASPJ_AE_RECV || op == LASPJ_AE_ALLREDUCE_MAX;
            }
        if (!any) break;
        if (comm) LJ_NCCL(cs[0]->ctx, R, R->GroupStart());
        for (int i = 0; i < n; ++i) {
            hipSetDevice(cs[i]->ctx->device);
            for (; at[i] < plans[i].size() && plans[i][at[i]].group == g; ++at[i])
                if (int s = run_step(R, cs[i], plans[i][at[i]], state[i], recv ? recv[i] : nullptr)) {
                    if (comm) R->GroupEnd();
                    return s;
                }
        }
        if (comm) LJ_NCCL(cs[0]->ctx, R, R->GroupEnd());
    }
    return LASPJ_OK;
}

int laspj_antientropy_loopback(laspj_ctx* ctx, int nranks, laspj_batch* const* state,
                               laspj_batch* const* recv, uint64_t piece_words) {
    if (!ctx || !state || nranks < 1 || nranks > 8)
        return fail(ctx, LASPJ_E_INVAL, "antientropy_loopback: bad argument");
    std::vector<laspj_comm> cs(nranks);
    for (int i = 0; i < nranks; ++i) {
        cs[i].ctx = ctx;
        cs[i].rank = i;
        cs[i].nranks = nranks;
        if (!state[i]) return fail(ctx, LASPJ_E_INVAL, "antientropy_loopback: null state");
        if (int s = round_checks(&cs[i], state[i], recv ? recv[i] : nullptr, nullptr,
                                 "antientropy_loopback"))
            return s;
        if (state[i]->kind != state[0]->kind || laspj::bytes_of(state[i]) != laspj::bytes_of(state[0]))
            return fail(ctx, LASPJ_E_KIND, "antientropy_loopback: one kind and size");
        for (int j = 0; j < i; ++j)
            if (state[j] == state[i] || (recv && recv[i] && recv[j] == recv[i]))
                return fail(ctx, LASPJ_E_INVAL, "antientropy_loopback: a buffer twice");
    }
    const uint64_t words = state[0]->replicas * state[0]->words_per_replica;
    const uint64_t piece = piece_words ? piece_words : kPiece;
    std::vector<std::vector<laspj_ae_step>> plans(nranks);
    for (int i = 0; i < nranks; ++i) {
        Plan P{nullptr, 0};
        plan_steps(P, state[0]->kind, i, nranks, words, piece);
        plans[i].resize(P.n);
        Plan Q{plans[i].data(), P.n};
        plan_steps(Q, state[0]->kind, i, nranks, words, piece);
    }
    CGuard g(ctx);
    std::vector<size_t> at(nranks, 0);
    for (uint32_t grp = 0;; ++grp) {
        // this group's steps of every rank (SENDs first: a RECV takes its peer's SEND)
        std::vector<std::pair<int, const laspj_ae_step*>> steps;
        for (int i = 0; i < nranks; ++i)
            for (; at[i] < plans[i].size() && plans[i][at[i]].group == grp; ++at[i])
                steps.push_back({i, &plans[i][at[i]]});
        if (steps.empty()) break;
        for (auto& [i, s] : steps) {
            laspj_batch* rv = recv ? recv[i] : nullptr;
            if (s->op == LASPJ_AE_RECV) {
                const laspj_ae_step* snd = nullptr;
                for (auto& [k, t] : steps)
                    if (k == s->peer && t->op == LASPJ_AE_SEND && t->peer == i && t->tag == s->tag)
                        snd = t;
                if (!snd || snd->words != s->words)
                    return fail(ctx, LASPJ_E_INVAL, "antientropy_loopback: unmatched RECV");
                LJ_HIP(ctx, hipMemcpyAsync(step_words(*s, state[i], rv),
                                           step_words(*snd, state[s->peer], recv ? recv[s->peer] : nullptr),
                                           8ull * s->words, hipMemcpyDeviceToDevice, ctx->stream));
            } else if (s->op == LASPJ_AE_REDUCE) {
                if (int st = reduce_step(ctx, *s, state[i], rv)) return st;
            } else if (s->op == LASPJ_AE_ALLREDUCE_MAX && i == 0) {
                // every rank's piece -> their unsigned max in rank 0's, then copied out
                const uint64_t* srcs[8];
                for (int k = 0; k < nranks; ++k) srcs[k] = state[k]->dev + s->offset;
                LJ_HIP(ctx, laspj::launch_reduce_ptrs(ctx, state[0]->dev + s->offset, srcs,
                                                      (uint32_t)nranks, s->words, true));
                for (int k = 1; k < nranks; ++k)
                    LJ_HIP(ctx, hipMemcpyAsync(state[k]->dev + s->offset, state[0]->dev + s->offset,
                                               8ull * s->words, hipMemcpyDeviceToDevice,
                                               ctx->stream));
            }
        }
    }
    return LASPJ_OK;
}

int laspj_antientropy_plan(int32_t kind, int rank, int nranks, uint64_t state_words,
                           uint64_t piece_words, laspj_ae_step* steps, uint64_t cap,
                           uint64_t* nsteps) {
    if (!nsteps || !set_kind(kind) || nranks < 1 || nranks > 8 || rank < 0 || rank >= nranks ||
        (kind != LASPJ_KIND_GCOUNTER && state_words % (uint64_t)nranks))
        return LASPJ_E_INVAL;
    Plan P{steps, steps ? cap : 0};
    plan_steps(P, kind, rank, nranks, state_words, piece_words ? piece_words : kPiece);
    *nsteps = P.n;
    return steps && P.n > cap ? LASPJ_E_RANGE : LASPJ_OK;
}

}  // extern "C"
