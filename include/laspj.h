/*
 * laspj.h — C ABI of the MI355X lattice-join engine (liblaspj.so).
 *
 * This is the drop-in boundary for Lasp's CRDT hot path.  In the reference every
 * CRDT is an Erlang module dispatched as `Type:Fun(...)` (the riak_dt behaviour,
 * SURVEY.md §8b); an Erlang NIF module that keeps those signatures binds exactly the
 * entry points below (INTEGRATION.md shows the binding).  Each entry point cites the
 * reference function it replaces (paths relative to the reference checkout).
 *
 * Conventions
 *   - every function returns an int status: LASPJ_OK (0) or a negative LASPJ_E_*;
 *     the message of the last failure on a context is laspj_ctx_last_error(ctx).
 *     No C++ exception crosses this ABI.
 *   - handles are opaque; sizes are explicit; no torch / HIP types in signatures.
 *   - device work is enqueued on the context's own HIP stream and is asynchronous,
 *     except *_download / *_upload and laspj_ctx_synchronize, which return after the
 *     copy (resp. all queued work) has completed.  Results written to a laspj_buf are
 *     valid after the next synchronising call on the same context.
 *   - a context serialises its own calls with a mutex (many BEAM schedulers may call
 *     one context); use one context per scheduler for concurrency.
 *
 * Data layout in HBM
 *   OR-Set batch: R replicas x E element slots; per (replica, slot) one 16-byte cell
 *     { uint64 p; uint64 r; } — bit k of p: token slot k of that element is present
 *     in the replica's orddict; bit k of r: that token's removed flag is `true`.
 *     r ⊆ p.  The element is present in the replica's orddict iff p != 0.
 *     Replica-major: cell (i, e) at byte offset (i*E + e)*16.
 *   G-Set batch: R replicas x W = ceil(E/64) uint64 words; bit e%64 of word e/64.
 *   Element slots and token slots are dictionary positions owned by the host (the NIF
 *   keeps the terms); every batch that meets in one call shares those dictionaries.
 */
#ifndef LASPJ_H
#define LASPJ_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LASPJ_ABI_VERSION 2

/* status codes */
#define LASPJ_OK               0
#define LASPJ_E_INVAL         -1   /* bad argument / null handle (NIF: badarg)          */
#define LASPJ_E_NOMEM         -2   /* device or host allocation failed                  */
#define LASPJ_E_DEVICE        -3   /* HIP runtime / kernel error                         */
#define LASPJ_E_SHAPE         -4   /* operand shapes do not agree (NIF: badarg)          */
#define LASPJ_E_KIND          -5   /* OR-Set batch where a G-Set batch was expected ...  */
#define LASPJ_E_RANGE         -6   /* replica / offset / byte range out of bounds        */
#define LASPJ_E_COMM          -7   /* RCCL communicator error                            */
#define LASPJ_E_UNSUPPORTED   -8   /* built without the feature                          */
#define LASPJ_E_FUN           -9   /* a host-evaluated fun failed on a key that is in the
                                      list (the reference's combinator body crashes)     */

#define LASPJ_KIND_ORSET         1
#define LASPJ_KIND_GSET          2
/* combinator outputs whose reference list is not an orddict of the input shape:     */
#define LASPJ_KIND_ORSET_CONCAT  3  /* intersection: 32 B/cell {pL, rL, pR, rR}; the
                                       element's token list decodes as Cx ++ Cy       */
#define LASPJ_KIND_ORSET_PRODUCT 4  /* product: EL x ER cells of uint32
                                       {pX:8, rX:8, pY:8, rY:8}, cell (x,y) at x*ER+y  */
#define LASPJ_KIND_GSET_PRODUCT  5  /* product: EL rows x ceil(ER/64) words           */
#define LASPJ_KIND_ORSET_PRODUCT_WIDE 7  /* product with any token slots: EL x ER cells
                                            of 32 B {pX, rX, pY, rY}                  */
#define LASPJ_KIND_GCOUNTER      6  /* riak_dt_gcounter: R x E actor slots, uint64 count
                                       per slot (0 = actor absent from the orddict)   */
#define LASPJ_KIND_ORSET_WIDE   10  /* OR-Set with T = 64 k token slots per element: per
                                       (replica, slot) k {p, r} pairs (16 k bytes), token
                                       slot t in pair t / 64, bit t % 64              */

typedef struct laspj_ctx   laspj_ctx;
typedef struct laspj_buf   laspj_buf;
typedef struct laspj_batch laspj_batch;
typedef struct laspj_event laspj_event;
typedef struct laspj_comm  laspj_comm;

typedef struct laspj_batch_info {
    int32_t  kind;               /* LASPJ_KIND_*                                       */
    uint32_t elements;           /* E: element slots per replica (EL for products)     */
    uint64_t replicas;           /* R                                                  */
    uint64_t bytes_per_replica;  /* 16*E (OR-Set) or 8*ceil(E/64) (G-Set) ...          */
    uint64_t bytes;              /* R * bytes_per_replica                              */
    uint32_t elements_r;         /* ER for product batches, else 0                     */
    uint32_t token_words;        /* k {p, r} pairs per cell (LASPJ_KIND_ORSET_WIDE), else 1 */
    uint64_t cells_per_replica;  /* E, or EL*ER for products                           */
} laspj_batch_info;

/* One update operation (lasp_orset:update/3, lasp_orset.erl:99-117;
 * lasp_gset:update/3, lasp_gset.erl:84-88), applied by laspj_*_apply_ops. */
#define LASPJ_OP_ADD     1  /* add / add_by_token: token slot `slot` of `element` := false */
#define LASPJ_OP_REMOVE  2  /* remove: every token of `element` := true, or
                               {error,{precondition,{not_present,E}}} if absent       */
#define LASPJ_OP_INSERT  3  /* lasp_orset_gbtree add (lasp_orset_gbtree.erl:232-240): like ADD,
                               but gb_trees:insert of a token already present raises
                               {key_exists, Token}: status KEY_EXISTS, call not applied */
#define LASPJ_OP_FLAG_NEW_CALL 1  /* this op starts a new update/3 call; ops of one call
                                     are all-or-nothing ({update, Ops}, remove_all)   */
typedef struct laspj_op {
    uint64_t replica;
    uint32_t element;
    uint8_t  kind;
    uint8_t  slot;               /* token slot 0..63 (ADD on an OR-Set)                */
    uint8_t  flags;
    uint8_t  pad;                /* LASPJ_KIND_ORSET_WIDE: token slot bits 8..15 (0 else) */
} laspj_op;
/* per-op status written by apply_ops */
#define LASPJ_OPST_APPLIED   0
#define LASPJ_OPST_NOT_PRESENT 1   /* this op's precondition failed; call rolled back */
#define LASPJ_OPST_ROLLED_BACK 2   /* another op of the same call failed              */
#define LASPJ_OPST_KEY_EXISTS  3   /* INSERT of a present token; call not applied      */

/* ------------------------------------------------------------------ library / context */
int         laspj_abi_version(void);
const char* laspj_strerror(int status);
int         laspj_device_count(int* n);
int         laspj_ctx_create(int device, laspj_ctx** out);
int         laspj_ctx_destroy(laspj_ctx* ctx);
const char* laspj_ctx_last_error(const laspj_ctx* ctx);
int         laspj_ctx_synchronize(laspj_ctx* ctx);
/* (A/B knobs for benchmarks and tests: include/laspj_tune.h — not part of the NIF's
 * contract; every default is the measured best) */

/* ------------------------------------------------------------------ device buffers */
int      laspj_buf_create(laspj_ctx* ctx, uint64_t bytes, laspj_buf** out);
int      laspj_buf_destroy(laspj_buf* buf);
uint64_t laspj_buf_bytes(const laspj_buf* buf);
/* the bytes are taken (src may be reused) on return; a small upload (<= 64 KiB) to a
 * buffer whose device address was never handed out completes on the context's stream
 * (before any later call's work), a larger one or one to an exported buffer before return */
int      laspj_buf_upload(laspj_ctx* ctx, laspj_buf* buf, uint64_t offset,
                          const void* src, uint64_t bytes);
int      laspj_buf_download(laspj_ctx* ctx, const laspj_buf* buf, uint64_t offset,
                            void* dst, uint64_t bytes);
/* device address of a buffer (to wrap sub-ranges as batches, or hand to a collective).
 * Destroying a buffer or batch is ordered with its context's stream only, and released
 * blocks are reused by later allocations of the context; a buffer / batch whose address
 * was handed out here therefore synchronises the whole device when it is destroyed, so
 * work another stream still runs on it finishes first. */
int      laspj_buf_device_ptr(const laspj_buf* buf, void** out);

/* ------------------------------------------------------------------ batches */
/* lasp_orset:new/0 (lasp_orset.erl:63-65) for R replicas over E element slots */
int laspj_orset_batch_create(laspj_ctx* ctx, uint64_t replicas, uint32_t elements,
                             laspj_batch** out);
/* lasp_orset:new/0 (lasp_orset.erl:63-65) with T = 64 * token_words token slots per
 * element (token_words 1..16): an element re-added many times keeps its tokens
 * (add_elem mints one per add and never collects them, lasp_orset.erl:222-241, 261-262).
 * The OR-Set entry points join / reduce / equal / value / removed / stats / inflation /
 * apply_ops / fragment / precondition_context and bind_many / inflation_many take these
 * batches (both operands wide with the same token_words); the combinator bodies and the
 * codec take narrow batches only. */
int laspj_orset_wide_batch_create(laspj_ctx* ctx, uint64_t replicas, uint32_t elements,
                                  uint32_t token_words, laspj_batch** out);
/* dst := src re-laid with dst's token_words (the same value: src's pairs first, the rest
 * {0, 0}); src narrow or wide with at most dst's token_words, same replicas and element
 * slots.  A variable whose value gains an element's 65th token moves to wide cells so. */
int laspj_orset_widen(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src);
/* lasp_gset:new/0 (lasp_gset.erl:70-72) */
int laspj_gset_batch_create(laspj_ctx* ctx, uint64_t replicas, uint32_t elements,
                            laspj_batch** out);
int laspj_batch_destroy(laspj_batch* batch);
/* A non-owning OR-Set / G-Set / G-Counter batch over caller device memory (e.g. a
 * buffer another allocator or a collective library owns; the bytes must stay valid
 * until destroy).  `kind` is LASPJ_KIND_ORSET, LASPJ_KIND_GSET or LASPJ_KIND_GCOUNTER;
 * `bytes` must equal the batch size. */
int laspj_batch_wrap(laspj_ctx* ctx, int32_t kind, void* device_ptr, uint64_t bytes,
                     uint64_t replicas, uint32_t elements, laspj_batch** out);
int laspj_batch_info_get(const laspj_batch* batch, laspj_batch_info* out);
/* device address of a batch's first word (to wrap replica ranges with laspj_batch_wrap
 * or hand them to a collective; its destroy then synchronises the device, as for
 * laspj_buf_device_ptr); list batches have no flat layout (LASPJ_E_KIND) */
int laspj_batch_device_ptr(const laspj_batch* batch, void** out);
/* bytes [offset, offset + bytes) of a batch's device image (synchronous), e.g. one row
 * window of a product batch */
int laspj_batch_download_range(laspj_ctx* ctx, const laspj_batch* batch, uint64_t offset,
                               uint64_t bytes, void* host);
/* host <-> device, replicas [first, first+count), host layout = device layout */
int laspj_batch_upload(laspj_ctx* ctx, laspj_batch* batch, uint64_t first, uint64_t count,
                       const void* host);
int laspj_batch_download(laspj_ctx* ctx, const laspj_batch* batch, uint64_t first,
                         uint64_t count, void* host);
/* every replica := new() */
int laspj_batch_clear(laspj_ctx* ctx, laspj_batch* batch);
/* deterministic synthetic replicas (oracle/laspj_oracle.c restates the
 * OR-Set and G-Set streams): replica i of the batch is synthetic replica
 * (replica_base + i) of stream `seed`; G-Counter batches get 20-bit counts (bench data) */
int laspj_batch_fill_synthetic(laspj_ctx* ctx, laspj_batch* batch, uint64_t seed,
                               uint64_t replica_base);
/* the OR-Set stream restricted to token_slots token slots: p and r masked to the low
 * token_slots bits, and every element present (p = 1 when the mask leaves none, and no
 * 5 % of absent elements) — BASELINE configs 4 / 5: sets of exactly E elements, T = 3 */
int laspj_batch_fill_synthetic_tokens(laspj_ctx* ctx, laspj_batch* batch, uint64_t seed,
                                      uint64_t replica_base, uint32_t token_slots);

/* Slot-wise join of two batches of the same kind and shape (any kind): dst = a | b
 * word by word.  For OR-Set / G-Set batches this is merge/2; for combinator outputs
 * it ORs both halves of CONCAT cells and the packed masks of PRODUCT cells; for
 * G-Counter batches it is the per-actor max (riak_dt_gcounter merge, as
 * laspj_gcounter_join). */
int laspj_batch_join(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* a,
                     const laspj_batch* b);

/* Many variables per launch (the bind path and the process loop over a store of
 * one-replica batches, lasp_core.erl:291-312, lasp_process.erl:61-95): n triples /
 * pairs of one-replica OR-Set, G-Set or G-Counter batches (a triple's batches share
 * kind and shape; triples may differ), one kernel over all of them.
 * bind_many: status[i] = 0 when cur[i] =:= val[i] (bind is a no-op, :294-296); else
 *   dst[i] := merge(cur[i], val[i]) and status[i] = 1 (a canonical merge always
 *   inflates cur, and the reference writes whenever it does, :301-303).  dst[i] may be
 *   cur[i] exactly; otherwise no dst may overlap any cur / val or another dst
 *   (LASPJ_E_INVAL).  inflation_many: out[i] = is_inflation (strict = 0) / is_strict_inflation
 *   (strict = 1) of prev[i] -> cur[i] per kind (lasp_lattice.erl:137-161, 169-179,
 *   212-253, 273-275).  inflation_many returns after the work has completed; bind_many
 *   once it is enqueued on the context's stream (every later call of the context sees
 *   its results; it waits for the work itself when a batch's or the status buffer's
 *   device address was handed out, or when there are many items). */
int laspj_batch_bind_many(laspj_ctx* ctx, uint32_t n, laspj_batch* const* dst,
                          const laspj_batch* const* cur, const laspj_batch* const* val,
                          laspj_buf* status);
/* bind_many with the statuses in host memory (n bytes): returns after the work has
 * completed, with one synchronisation (the kernel writes them into the context's pinned
 * memory) — what a bind/3 caller needs before it can answer */
int laspj_batch_bind_many_host(laspj_ctx* ctx, uint32_t n, laspj_batch* const* dst,
                               const laspj_batch* const* cur, const laspj_batch* const* val,
                               uint8_t* status);
int laspj_batch_inflation_many(laspj_ctx* ctx, uint32_t n, const laspj_batch* const* prev,
                               const laspj_batch* const* cur, int strict, laspj_buf* out);

/* Anti-entropy reduce step: src holds nchunks copies of dst's replica
 * range laid out chunk-major (what an all-to-all delivers); dst[i] = ⊔_j src[j*R + i].
 * Any kind; src.replicas = nchunks * dst.replicas.  ⊔ is the kind's join: OR of the
 * words for bitmap kinds, per-actor max for G-Counters. */
int laspj_batch_reduce_chunks(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                              uint32_t nchunks);

/* foldl(Type:merge, new(), Replies) over n separately held batches — the coordinator's
 * N-way merge of the replies it received (lasp_update_fsm.erl:189-192,
 * lasp_bind_fsm.erl:185-188) and the anti-entropy round's reduce, which reads the
 * rank's own copy in place: dst = srcs[0] ⊔ ... ⊔ srcs[n-1], 1 <= n <= 8, batches of one
 * kind and shape (any non-list kind; ⊔ as laspj_batch_join).  dst may alias any
 * source. */
int laspj_batch_join_n(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* const* srcs,
                       uint32_t n);

/* ------------------------------------------------------------------ lasp_orset */
/* merge/2 — lasp_orset.erl:128-134: dst[i] = a[i] ⊔ b[i]  (p|p', r|r').
 * dst may alias a or b (the bind path merges in place, lasp_core.erl:300-303). */
int laspj_orset_join(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* a,
                     const laspj_batch* b);
/* foldl(merge, new(), Replies) over groups of `group` consecutive replicas —
 * lasp_update_fsm.erl:189-192 / lasp_bind_fsm.erl:185-188: dst[g] = ⊔ src[g*group+j] */
int laspj_orset_reduce(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                       uint32_t group);
/* value/1 — lasp_orset.erl:67-73: bit e of replica i set iff element e has a token
 * with flag false.  out: R * ceil(C/64) uint64 words, C = cells per replica.
 * Also accepts combinator outputs: a CONCAT cell is visible if Cx ++ Cy has a false
 * flag, a PRODUCT cell (x, y) iff both x and y have one. */
int laspj_orset_value(laspj_ctx* ctx, const laspj_batch* batch, laspj_buf* out_bits);
/* value({tokens, E}, S) / value({fragment, E}, S) — lasp_orset.erl:76-89: out receives
 * the 16-byte cell of element slot `element` of every replica (R cells; a wide batch's
 * k pairs per replica, 16 k bytes): its tokens are E's token orddict ([] when p = 0), the
 * fragment is [{E, Tokens}] or [] */
int laspj_orset_fragment(laspj_ctx* ctx, const laspj_batch* batch, uint32_t element,
                         laspj_buf* out);
/* precondition_context/1 — lasp_orset.erl:147-154 with minimum_tokens (:264-267): every
 * element keeps the tokens flagged false (p & ~r, r = 0) and drops out when none is
 * left; dst may alias src; wide batches pair by pair */
int laspj_orset_precondition_context(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src);
/* value(removed, S) — lasp_orset.erl:90-95: elements with a token flagged true */
int laspj_orset_removed(laspj_ctx* ctx, const laspj_batch* batch, laspj_buf* out_bits);
/* stats/1 — lasp_orset.erl:156-192: per replica {element_count, adds_count,
 * removes_count} as 3 uint64 (waste_pct = round(removes/(adds+removes)*100) host-side) */
int laspj_orset_stats(laspj_ctx* ctx, const laspj_batch* batch, laspj_buf* out_counts);
/* equal/2 — lasp_orset.erl:136-138: out[i] = (a[i] == b[i]) as one byte */
int laspj_orset_equal(laspj_ctx* ctx, const laspj_batch* a, const laspj_batch* b,
                      laspj_buf* out);
/* is_inflation/3 (strict = 0) — lasp_lattice.erl:97-98,153-161,277-285 — and
 * is_strict_inflation/3 (strict = 1) — lasp_lattice.erl:105-106,235-253.
 * prev has R replicas or 1 (broadcast); out[i] = one byte per cur replica.
 * threshold_met(lasp_orset, V, T) (lasp_lattice.erl:72-75) is inflation(T, V). */
int laspj_orset_inflation(laspj_ctx* ctx, const laspj_batch* prev, const laspj_batch* cur,
                          int strict, laspj_buf* out);
/* update/3 — lasp_orset.erl:99-117 (add_elem :222-230, remove_elem :232-241).
 * ops: host array sorted by replica (stable within a replica); status: nops int32, or
 * null when every op is an ADD (no precondition can fail: nothing is read back, the call
 * returns without waiting for the device) */
int laspj_orset_apply_ops(laspj_ctx* ctx, laspj_batch* batch, const laspj_op* ops,
                          uint64_t nops, int32_t* status);
/* union body for lasp_orset — lasp_core.erl:616-618: orddict:merge keep-left:
 * dst[i][e] = (l[i][e].p != 0) ? l[i][e] : r[i][e] */
int laspj_orset_union(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                      const laspj_batch* r);
/* filter body — lasp_core.erl:681-712: keep element e iff bit e of `keep` (the
 * predicate F(X) evaluated once per element slot, ceil(E/64) words); tombstoned
 * elements are kept like live ones. */
int laspj_orset_filter(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                       const laspj_buf* keep);

/* intersection body for lasp_orset — lasp_core.erl:546-589 with
 * lasp_lattice:orset_causal_union/2 (:311-312): element e of L that keyfind-s in R
 * becomes {e, Cx ++ Cy}.  l, r: OR-Set batches over the same element slots;
 * dst: LASPJ_KIND_ORSET_CONCAT batch of the same shape. */
int laspj_orset_concat_batch_create(laspj_ctx* ctx, uint64_t replicas, uint32_t elements,
                                    laspj_batch** out);
int laspj_orset_intersection(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                             const laspj_batch* r);
/* product body for lasp_orset — lasp_core.erl:499-533 with
 * lasp_lattice:orset_causal_product/2 (:303-308): cell (x, y) holds the 8-bit token
 * masks of x and y (the token set is Tx x Ty, flag = Dx orelse Dy).  Token slots must
 * be < 8 for a PRODUCT dst (else LASPJ_E_RANGE, checked on the device); a
 * PRODUCT_WIDE dst takes any slots.  l has EL slots, r ER slots. */
int laspj_orset_product_batch_create(laspj_ctx* ctx, uint64_t replicas, uint32_t el,
                                     uint32_t er, laspj_batch** out);
/* the same with 32-byte cells, for inputs that use token slots >= 8 */
int laspj_orset_product_wide_batch_create(laspj_ctx* ctx, uint64_t replicas, uint32_t el,
                                          uint32_t er, laspj_batch** out);
int laspj_orset_product(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                        const laspj_batch* r);
/* product followed by filter(fun({X, Y}) -> X =:= Y) (lasp_core.erl:499-533 then
 * :681-712; BASELINE config 5's fused variant), over ONE element dictionary shared by l
 * and r (slot e is the same term on both sides, so X =:= Y iff the slots agree): dst is
 * a PRODUCT batch with EL = E and ER = 1 whose cell (e, 0) is the product cell of l[e]
 * and r[e] ({{X, X}, orset_causal_product(Cx, Cy)}, kept tombstoned like any filter
 * output), 0 when e is absent on either side.  Token slots must be < 8 (LASPJ_E_RANGE). */
int laspj_orset_product_diag(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                             const laspj_batch* r);
/* map / fold bodies — lasp_core.erl:641-667, :460-486: output slot o takes the cell of
 * input slot index[o] (uint32 per dst slot; 0xFFFFFFFF = empty).  The host builds the
 * index from F over the element dictionary (a map is one slot per input slot, a fold
 * one slot per F(X) entry, in list order). */
int laspj_orset_gather(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                       const laspj_buf* index);

/* A combinator stage whose output is threshold-read in the same pass (BASELINE config 4:
 * map -> filter -> fold -> read {strict, Prev}, lasp_core.erl:641-712, 460-486, and
 * lasp_process.erl:61-95): dst = src gathered through index (as laspj_orset_gather; the
 * host composes the stages' indexes: fold slot o <- filtered slot f[o] <- mapped slot
 * <- src slot m[f[o]], or empty when the filter drops it) and out[i] = one byte,
 * is_inflation (strict = 0) / is_strict_inflation (strict = 1) of prev[i] -> dst[i]
 * (lasp_lattice.erl:153-161, 235-253).  prev has dst's shape or 1 replica. */
int laspj_orset_gather_inflation(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                                 const laspj_buf* index, const laspj_batch* prev, int strict,
                                 laspj_buf* out);
/* laspj_orset_gather_inflation compares prev and dst slot by slot, which is the
 * reference's lists:keyfind when the output keys are distinct, or when every slot
 * sharing a key takes the same src slot (fold X -> [X, X, X]).  When keys repeat across
 * src slots (a collapsing map such as X div 3, a fold whose F(X) lists overlap), keyfind
 * pairs each Prev entry with the FIRST Cur entry of its key: the keyed form takes, per
 * dst slot o (uint32 each), head[o] = the first dst slot with o's key and next[o] = the
 * next one in list order (0xFFFFFFFF after the last), and compares every present prev
 * slot with the first present dst slot of its key chain.  Tokens of different src slots
 * are taken to be different terms (Lasp mints a fresh token per add, lasp_orset.erl:
 * 261-262); a host whose dictionary shares a token term between elements of one key
 * uses list values instead. */
int laspj_orset_gather_inflation_keyed(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                                       const laspj_buf* index, const laspj_buf* head,
                                       const laspj_buf* next, const laspj_batch* prev,
                                       int strict, laspj_buf* out);

/* ------------------------------------------------------------------ lasp_gset */
/* merge/2 — lasp_gset.erl:99-101 (ordsets:union on canonical sets = OR) */
int laspj_gset_join(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* a,
                    const laspj_batch* b);
/* foldl(merge, new(), Replies) over groups of `group` consecutive replicas —
 * lasp_update_fsm.erl:189-192 / lasp_bind_fsm.erl:185-188, as laspj_orset_reduce */
int laspj_gset_reduce(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                      uint32_t group);
/* stat(element_count) — lasp_gset.erl:135-136: one uint64 per replica */
int laspj_gset_stats(laspj_ctx* ctx, const laspj_batch* batch, laspj_buf* out_counts);
/* equal/2 — lasp_gset.erl:103-105 (GSet1 == GSet2): out[i] = (a[i] == b[i]) as one byte */
int laspj_gset_equal(laspj_ctx* ctx, const laspj_batch* a, const laspj_batch* b,
                     laspj_buf* out);
/* is_inflation — lasp_lattice.erl:137-140; strict — :212-215 */
int laspj_gset_inflation(laspj_ctx* ctx, const laspj_batch* prev, const laspj_batch* cur,
                         int strict, laspj_buf* out);
/* update/3 add / add_all — lasp_gset.erl:84-88 (LASPJ_OP_ADD only; status may be null:
 * nothing read back, no wait) */
int laspj_gset_apply_ops(laspj_ctx* ctx, laspj_batch* batch, const laspj_op* ops,
                         uint64_t nops, int32_t* status);

/* union body for lasp_gset — lasp_core.erl:620 binds `L ++ R`; on ordsets that are
 * disjoint and ordered this is their union, which is what this computes (bitwise OR);
 * an overlapping L ++ R is not a set and is not produced. */
int laspj_gset_union(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                     const laspj_batch* r);
/* intersection body for lasp_gset — lasp_core.erl:569-576 (lists:member) */
int laspj_gset_intersection(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                            const laspj_batch* r);
/* filter body for lasp_gset — lasp_core.erl:681-712 */
int laspj_gset_filter(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                      const laspj_buf* keep);
/* product body for lasp_gset — lasp_core.erl:518-520: bit (x, y) = x in L and y in R */
int laspj_gset_product_batch_create(laspj_ctx* ctx, uint64_t replicas, uint32_t el,
                                    uint32_t er, laspj_batch** out);
int laspj_gset_product(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                       const laspj_batch* r);
/* map / fold bodies for lasp_gset: dst bit o = src bit index[o] */
int laspj_gset_gather(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                      const laspj_buf* index);

/* ------------------------------------------------------------------ riak_dt_gcounter */
/* The G-Counter the ad counter's threshold reads use.  State is
 * the orddict Actor -> Count of riak_dt_gcounter (third-party riak_dt, not vendored;
 * its merge is the per-actor max, its value the sum).  Actor slots are host
 * dictionary positions, like element slots. */
typedef struct laspj_incr {
    uint64_t replica;
    uint32_t actor;              /* actor slot */
    uint32_t reserved;
    uint64_t amount;             /* increment = 1 / {increment, N}: N > 0 (riak_dt_gcounter
                                    rejects other N with function_clause; the NIF checks
                                    it before the call).  Counts are uint64: riak_dt's are
                                    bignums, so counts and sums wrap at 2^64 here.       */
} laspj_incr;
int laspj_gcounter_batch_create(laspj_ctx* ctx, uint64_t replicas, uint32_t actors,
                                laspj_batch** out);
/* merge/2: per-actor max */
int laspj_gcounter_join(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* a,
                        const laspj_batch* b);
/* value/1: one uint64 sum per replica */
int laspj_gcounter_value(laspj_ctx* ctx, const laspj_batch* batch, laspj_buf* out_sums);
/* threshold_met(riak_dt_gcounter, V, T) — lasp_lattice.erl:87-90:
 * T =< value(V) (strict = 0) or T < value(V) (strict = 1); one byte per replica */
int laspj_gcounter_threshold(laspj_ctx* ctx, const laspj_batch* batch, uint64_t threshold,
                             int strict, laspj_buf* out);
/* is_inflation — lasp_lattice.erl:169-179 (every Prev actor in Cur with Count =< Count1);
 * strict — :273-275 (value(Prev) < value(Cur)); prev may be one broadcast replica */
int laspj_gcounter_inflation(laspj_ctx* ctx, const laspj_batch* prev, const laspj_batch* cur,
                             int strict, laspj_buf* out);
int laspj_gcounter_equal(laspj_ctx* ctx, const laspj_batch* a, const laspj_batch* b,
                         laspj_buf* out);
/* update(increment | {increment, N}, Actor, C): counts are commutative, any order */
int laspj_gcounter_apply_increments(laspj_ctx* ctx, laspj_batch* batch,
                                    const laspj_incr* incs, uint64_t n);
/* FSM N-way merge over groups of `group` replicas (per-actor max) */
int laspj_gcounter_reduce(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                          uint32_t group);

/* ------------------------------------------------------------------ wire codec */
/* to_binary/1 — lasp_orset.erl:198-200, lasp_gset.erl:111-113:
 *   <<?TAG:8, ?V1_VERS:8, (riak_dt:to_binary(S))/binary>>, riak_dt:to_binary = term_to_binary
 * written on the device for every replica of a batch.  The
 * payload of replica i is the external term format image (version byte 131, then the
 * orddict [{Elem, [{Token, Bool}]}] as LIST_EXT / SMALL_TUPLE_EXT / ATOM_EXT, or the
 * G-Set ordset as LIST_EXT or, for all-byte integers, STRING_EXT), prefixed by the two
 * bytes (tag, vers) when tag >= 0 (tag < 0: the bare term_to_binary/1 image).  The
 * compressed form ({compressed, N}) is not produced here.
 *
 * The dictionary holds each dictionary term's own external image (no version byte),
 * which the host encodes once per distinct term:
 *   elem_blob[elem_off[e] .. elem_off[e+1])         element slot e   (empty: unused)
 *   elem_order[0 .. E)                              element slots in Erlang term order
 *                                                   (a permutation of 0 .. E-1, else
 *                                                   LASPJ_E_RANGE)
 *   tok_blob[tok_off[64e+k] .. tok_off[64e+k+1])    token slot k of element e (empty: unused)
 *   tok_order[64e + j], j < 64                      token slots of e in term order,
 *                                                   0xFF after the last used one
 * tok_* may be NULL for a G-Set-only dictionary.  Encoding a cell whose slots are not
 * in the dictionary fails with LASPJ_E_RANGE and writes nothing meaningful. */
typedef struct laspj_etf_dict laspj_etf_dict;
int laspj_etf_dict_create(laspj_ctx* ctx, uint32_t elements, const uint8_t* elem_blob,
                          const uint32_t* elem_off, const uint32_t* elem_order,
                          const uint8_t* tok_blob, const uint32_t* tok_off,
                          const uint8_t* tok_order, laspj_etf_dict** out);
int laspj_etf_dict_destroy(laspj_etf_dict* d);
/* sizes: offsets (a buffer of R+1 uint64) receives the exclusive prefix sum of the
 * per-replica payload sizes; *total = offsets[R] (synchronous). */
int laspj_orset_etf_size(laspj_ctx* ctx, const laspj_batch* batch, const laspj_etf_dict* d,
                         int tag, laspj_buf* offsets, uint64_t* total);
/* payloads: replica i at out[offsets[i] .. offsets[i+1]); offsets from *_etf_size
 * with the same batch, dictionary and tag presence; out holds >= total bytes */
int laspj_orset_etf_write(laspj_ctx* ctx, const laspj_batch* batch, const laspj_etf_dict* d,
                          int tag, int vers, const laspj_buf* offsets, laspj_buf* out);
int laspj_gset_etf_size(laspj_ctx* ctx, const laspj_batch* batch, const laspj_etf_dict* d,
                        int tag, laspj_buf* offsets, uint64_t* total);
int laspj_gset_etf_write(laspj_ctx* ctx, const laspj_batch* batch, const laspj_etf_dict* d,
                         int tag, int vers, const laspj_buf* offsets, laspj_buf* out);
/* from_binary/1 — lasp_orset.erl:202-214 (riak_dt:from_binary/1 = binary_to_term/1) for
 * a batch: payload bytes [offsets[i], offsets[i+1]) are decoded into replica i of
 * `batch` (cleared first; replicas with a non-zero status are undefined).  A payload
 * is <<Tag, Vers>> (when tag >= 0) ++ the external term format image of an orddict
 * whose element and token terms are in the dictionary, in term order, with flags
 * `true` / `false` (ATOM_EXT, ATOM_UTF8_EXT or SMALL_ATOM_UTF8_EXT).  Needs a dictionary
 * whose token images all have one length (else LASPJ_E_UNSUPPORTED); element images up
 * to ~2 KiB.  status: R int32 of LASPJ_DEC_*. */
#define LASPJ_DEC_OK                  0
#define LASPJ_DEC_INVALID_BINARY      1  /* not <<Tag, _, ...>>: ?INVALID_BINARY            */
#define LASPJ_DEC_UNSUPPORTED_VERSION 2  /* tag matches, version does not: ?UNSUPPORTED_VERSION(V) */
#define LASPJ_DEC_MALFORMED           3  /* binary_to_term would fail (no 131, truncated,
                                            trailing bytes) or the term is not an orddict
                                            of {Elem, [{Token, Flag}]}                    */
#define LASPJ_DEC_UNKNOWN_TERM        4  /* an element or token outside the dictionary, or
                                            out of term order (not an orddict)           */
#define LASPJ_DEC_UNREPRESENTABLE     5  /* an element with no tokens or more than 64     */
#define LASPJ_DEC_EQUAL_TERMS         6  /* host dictionary only: a term `==` to one that
                                            already holds a slot under another image (1 vs
                                            1.0, {a, 1} vs {a, 1.0}, an atom in another
                                            encoding) — orddict:merge / ordsets:union treat
                                            them as one key, separate slots would not; the
                                            NIF hands such operands to the reference's
                                            clause (lasp_orset.erl:128-138, SURVEY.md
                                            Appendix A)                                   */
int laspj_orset_etf_read(laspj_ctx* ctx, laspj_batch* batch, const laspj_etf_dict* d,
                         int tag, int vers, const laspj_buf* payload,
                         const laspj_buf* offsets, laspj_buf* status);
/* from_binary/1 — lasp_gset.erl:122-128 — for a G-Set batch: the payload is <<Tag, Vers>>
 * (tag >= 0) ++ the external term image of an ordset whose elements are in the dictionary:
 * [] (NIL_EXT), a LIST_EXT of element images with a [] tail, or STRING_EXT (every element
 * an integer 0..255, as term_to_binary/1 writes it).  Statuses as for OR-Sets: MALFORMED
 * when binary_to_term/1 would fail or the term is not a proper list, UNKNOWN_TERM for an
 * element outside the dictionary or out of strict term order (not an ordset) or a term
 * kind no dictionary holds (pids, refs, funs, maps, bit strings: the NIF hands such
 * payloads to binary_to_term/1). */
int laspj_gset_etf_read(laspj_ctx* ctx, laspj_batch* batch, const laspj_etf_dict* d,
                        int tag, int vers, const laspj_buf* payload,
                        const laspj_buf* offsets, laspj_buf* status);

/* ------------------------------------------------------------------ anti-entropy */
/* Gossip anti-entropy across GPUs over RCCL (xGMI) — the reference's N-way merge and
 * read-repair (lasp_update_fsm.erl:174-216, lasp_bind_fsm.erl:170-212) and coverage
 * reduce (lasp_execute_coverage_fsm.erl:59-62) as one all-reduce with the lattice's
 * join.  Every rank holds one replica of each of R objects (a batch with R replicas);
 * after a round every rank holds the join of all ranks' replicas of every object.
 *   OR-Set / G-Set: grouped ncclSend/ncclRecv all-to-all (rank j receives every rank's
 *     copy of object chunk j, objects chunk-major: rank j owns objects
 *     [j*R/n, (j+1)*R/n)), the reduce kernel (OR over the n copies, in place), then an
 *     all-gather of the joined chunks made of grouped ncclSend/ncclRecv pieces — RCCL
 *     has no bitwise-OR reduction;
 *   G-Counter: one ncclAllReduce(ncclMax) over the uint64 counts (in place).
 * Everything is enqueued on the contexts' streams (no host synchronisation); results
 * are valid after the next synchronising call.  LASPJ_E_UNSUPPORTED when RCCL cannot be
 * loaded, LASPJ_E_COMM for RCCL failures. */
#define LASPJ_COMM_ID_BYTES 128
/* a fresh communicator id (ncclGetUniqueId); rank 0 makes it, the caller hands it to
 * every rank (the NIF: over Erlang distribution) */
int laspj_comm_unique_id(uint8_t* id);
/* one process per GPU: this context joins communicator `id` as `rank` of `nranks` */
int laspj_comm_init_rank(laspj_ctx* ctx, int nranks, const uint8_t* id, int rank,
                         laspj_comm** out);
/* one process owning n GPUs (one BEAM node driving all 8): a communicator per context,
 * out[i] for ctxs[i] (ncclCommInitAll over the contexts' devices) */
int laspj_comm_init_all(laspj_ctx* const* ctxs, int n, laspj_comm** out);
int laspj_comm_destroy(laspj_comm* comm);
int laspj_comm_info(const laspj_comm* comm, int* rank, int* nranks);
/* one round on this rank: state (R objects, R % nranks == 0, nranks <= 8) and recv (at
 * least (nranks-1) * R / nranks objects of state's kind: the peers' copies of this
 * rank's chunk land there, peer p's in slot p - (p > rank)).  The rank's own chunk is
 * joined in place in state and sent from there; `chunk` is not needed (may be NULL; when
 * given it must hold R / nranks objects and is left untouched).  recv may be NULL for
 * G-Counters and when nranks == 1.  The round runs laspj_antientropy_plan's steps. */
int laspj_antientropy(laspj_comm* comm, laspj_batch* state, laspj_batch* recv,
                      laspj_batch* chunk);
/* the same for n communicators of one process (laspj_comm_init_all): step g of every
 * communicator's plan goes into one RCCL group */
int laspj_antientropy_group(laspj_comm* const* comms, laspj_batch* const* state,
                            laspj_batch* const* recv, laspj_batch* const* chunk, int n);

/* The schedule of one rank's round — pure host code, no GPU or RCCL needed — which
 * laspj_antientropy executes step for step (and a test can execute over any transport).
 * Word offsets into two buffers: STATE (state_words = R objects, chunk-major: rank j owns
 * words [j*cw, (j+1)*cw), cw = state_words / nranks) and RECV ((nranks-1) slots of cw).
 * Steps carry a group number: groups run in order; the SEND / RECV steps of one group are
 * one RCCL group (at most 2 (nranks-1) point-to-point calls, each of at most piece_words
 * words; 0 = 2^27 = 1 GiB, as one RCCL p2p call moves at most 4 GiB); a REDUCE or
 * ALLREDUCE_MAX group holds that one step.  A SEND and the peer's matching RECV carry the
 * same tag (the piece number within the phase).  kind: LASPJ_KIND_ORSET / GSET (all-to-all
 * -> reduce -> all-gather) or LASPJ_KIND_GCOUNTER (all-reduce(max) in pieces).  *nsteps
 * receives the step count; steps may be NULL (count only); LASPJ_E_RANGE when cap is
 * smaller than the count. */
#define LASPJ_AE_SEND          1  /* send words [offset, +words) of buf to peer          */
#define LASPJ_AE_RECV          2  /* receive words from peer into [offset, +words) of buf */
#define LASPJ_AE_REDUCE        3  /* STATE[offset, +words) := itself ⊔ RECV[src + j*words,
                                     +words) for j < nsrc (the kind's join)              */
#define LASPJ_AE_ALLREDUCE_MAX 4  /* STATE[offset, +words) := the unsigned max of every
                                     rank's words (G-Counters)                           */
#define LASPJ_AE_BUF_STATE 0
#define LASPJ_AE_BUF_RECV  1
typedef struct laspj_ae_step {
    uint32_t group;
    int32_t  op;                 /* LASPJ_AE_*                                          */
    int32_t  peer;               /* SEND / RECV: the peer rank; else -1                 */
    int32_t  buf;                /* SEND: the buffer read; RECV: the buffer written     */
    uint64_t offset;             /* words                                               */
    uint64_t words;
    uint64_t src;                /* REDUCE: first source word in RECV                   */
    uint32_t nsrc;               /* REDUCE: source runs                                 */
    uint32_t tag;                /* SEND / RECV: piece number                           */
} laspj_ae_step;
int laspj_antientropy_plan(int32_t kind, int rank, int nranks, uint64_t state_words,
                           uint64_t piece_words, laspj_ae_step* steps, uint64_t cap,
                           uint64_t* nsteps);
/* Every rank's plan of one round executed on ONE context, rank i's buffers being state[i]
 * / recv[i]: a SEND / RECV pair becomes a device copy between the two ranks' buffers,
 * REDUCE is the round's reduce step (the same word arithmetic and kernel as
 * laspj_antientropy), ALLREDUCE_MAX the unsigned max of every rank's piece.  The same
 * argument checks as a round.  For testing the round's step arithmetic at nranks > 1 where
 * one process has one GPU (RCCL refuses one device twice in a communicator). */
int laspj_antientropy_loopback(laspj_ctx* ctx, int nranks, laspj_batch* const* state,
                               laspj_batch* const* recv, uint64_t piece_words);

/* ------------------------------------------------------------------ list values */
/* List-faithful values.  The combinator bodies of lasp_core bind lists that are not
 * orddicts: intersection entries carry `Cx ++ Cy` (lasp_core.erl:546-589,
 * lasp_lattice.erl:311-312), product entries the fully reversed token pairs of
 * orset_causal_product (lasp_core.erl:499-533, lasp_lattice.erl:303-308), a map or fold
 * may reorder or repeat keys (:641-667, :460-486), and the G-Set union binds `L ++ R`
 * (:620).  Every later re-run binds its new output with Type:merge (lasp_core.erl:300),
 * i.e. orddict:merge / ordsets:union run as written over those lists: a two-finger
 * merge that can interleave and duplicate keys and tokens.  A LIST batch holds such
 * values exactly, in list order, and the entry points below restate every list
 * operation of the path over them on the device.
 *
 * Layout: R replicas, each a list of up to cap_entries entries and cap_tokens tokens:
 *   entry i of replica r: key item key[r][i]; its token run tok[r][toff[r][i] ..
 *   toff[r][i+1]) (OR-Set lists; a G-Set list has keys only).
 * Key item (uint64):  bit 62 clear: element slot e (bits 0-30);
 *                     bit 62 set:   the pair {X, Y} of element slots x (bits 31-61), y
 *                                   (bits 0-30) — product keys.
 * Token item (uint64): bit 63: the {Token, Bool} flag (1 = true);
 *                     bit 62 clear: token g = 64*e + k, token slot k of element slot e;
 *                     bit 62 set:   the 2-list [Tx, Ty] of tokens gx (bits 31-61) and
 *                                   gy (bits 0-30) — product tokens.
 * Order: term order is given by rank tables the host derives from its dictionaries
 * (laspj_list_order): krank[e] = rank of element slot e's term, grank[g] = rank of
 * token g's term (equal terms share a rank); pairs and 2-lists compare element-wise;
 * a 2-list token sorts below every simple token (lists < binaries).  Comparisons and
 * equality are by rank, so `==`-equal terms held in different slots are equal.
 * Entry points that produce a list size their dst themselves: dst (a LIST batch of the
 * right kind and replica count) is re-allocated when its capacity is too small.  They
 * synchronise (they read back sizes and argument checks).  LASPJ_E_UNSUPPORTED: a
 * product of product outputs (nested pairs), which this layout does not express. */
#define LASPJ_KIND_ORSET_LIST 8
#define LASPJ_KIND_GSET_LIST  9
#define LASPJ_LIST_PAIR      (1ull << 62)
#define LASPJ_LIST_COMPOUND  (1ull << 62)
#define LASPJ_LIST_REMOVED   (1ull << 63)
typedef struct laspj_list_order {
    const laspj_buf* krank;      /* uint32 per element slot                          */
    uint32_t         nkeys;      /* element slots covered by krank                   */
    uint32_t         ntokens;    /* tokens covered by grank (64 * element slots)     */
    const laspj_buf* grank;      /* uint32 per token g; may be NULL for G-Set lists  */
} laspj_list_order;
int laspj_list_batch_create(laspj_ctx* ctx, int32_t kind, uint64_t replicas,
                            uint32_t cap_entries, uint32_t cap_tokens, laspj_batch** out);
/* per replica {entries, tokens} as 2 uint32 (synchronous) */
int laspj_list_counts(laspj_ctx* ctx, const laspj_batch* list, uint32_t* out);
/* replica `replica` := the list (keys[n], toff[n+1] with toff[0] = 0, toks[toff[n]]) */
int laspj_list_upload(laspj_ctx* ctx, laspj_batch* list, uint64_t replica, uint32_t n,
                      const uint64_t* keys, const uint32_t* toff, const uint64_t* toks);
/* the list of replica `replica` (sizes from laspj_list_counts; toff gets n+1 words) */
int laspj_list_download(laspj_ctx* ctx, const laspj_batch* list, uint64_t replica,
                        uint64_t* keys, uint32_t* toff, uint64_t* toks);
/* a canonical OR-Set / G-Set batch as lists: elements in term order (elem_order: the
 * nslots element slots in term order, uint32), tokens of element e in term order
 * (tok_order: 64 uint8 per element slot, token slots ascending in term order, 0xFF
 * after the last; NULL for G-Sets) */
int laspj_list_from_set(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                        const laspj_buf* elem_order, uint32_t nslots,
                        const laspj_buf* tok_order);
/* dst := Type:merge(a, b) — lasp_orset:merge/2 (lasp_orset.erl:128-134: nested
 * orddict:merge, inner BoolA or BoolB) on OR-Set lists, lasp_gset:merge/2
 * (lasp_gset.erl:99-101: ordsets:union, OTP 17 clauses incl. the argument switch) on
 * G-Set lists; run as written on any list */
int laspj_list_merge(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* a,
                     const laspj_batch* b, const laspj_list_order* ord);
/* out[i] = (a[i] =:= b[i]) as one byte — the `case Value0 of Value` match of bind/3
 * (lasp_core.erl:294-296) */
int laspj_list_equal(laspj_ctx* ctx, const laspj_batch* a, const laspj_batch* b,
                     const laspj_list_order* ord, laspj_buf* out);
/* is_inflation / is_strict_inflation of prev -> cur (lasp_lattice.erl:137-161, 212-253,
 * 277-285: lists:keyfind first match, ids_inflated, order-sensitive =/=, length/1;
 * G-Sets: sets:is_subset, usort =/=); prev has R replicas or 1 (broadcast) */
int laspj_list_inflation(laspj_ctx* ctx, const laspj_batch* prev, const laspj_batch* cur,
                         int strict, const laspj_list_order* ord, laspj_buf* out);
/* lasp_core:bind/3 on list values (lasp_core.erl:291-312) in one call, per replica:
 * status[i] = 0 when cur[i] =:= val[i] (the no-op of :294-296); else dst[i] :=
 * Type:merge(cur[i], val[i]) (as laspj_list_merge) and status[i] = 1 when
 * is_inflation(cur[i], dst[i]) (:301, the bind writes dst[i]) or 2 when not (no write).
 * status is host memory, R bytes.  One synchronisation (the equalities, the merge sized
 * from the inputs' counts, the inflations, then sizes, bytes and the error flag read
 * together) instead of the separate calls' six; dst holds the merge for every replica
 * (what the bind writes where status is 1).  On an error status, status[] and dst hold
 * no result. */
int laspj_list_bind(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* cur,
                    const laspj_batch* val, const laspj_list_order* ord, uint8_t* status);
/* value/1 of OR-Set lists (lasp_orset.erl:67-73): the keys of entries with a {_, false}
 * token, in list order, as a G-Set list dst */
int laspj_list_value(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src);
/* union body (lasp_core.erl:616-620): OR-Set lists orddict:merge keeping the left
 * tokens; G-Set lists `L ++ R` */
int laspj_list_union(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                     const laspj_batch* r, const laspj_list_order* ord);
/* intersection body (lasp_core.erl:546-589): per entry of l in order, lists:keyfind in r
 * (first match) -> {X, Cx ++ Cy}; G-Set lists: lists:member -> X */
int laspj_list_intersection(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                            const laspj_batch* r, const laspj_list_order* ord);
/* the intersection body with a canonical right side (lasp_core.erl:546-589): r is an
 * OR-Set (G-Set) batch of l's replicas; keyfind / member of X in r's list form is r's cell
 * of X's slot, whose tokens follow Cx in term order (tok_order: laspj_list_from_set's
 * 64-byte rows) — what laspj_list_from_set(r) then laspj_list_intersection gives, without
 * the conversion or its hash.  Distinct slots must be distinct terms (== apart), as the
 * host dictionaries guarantee. */
int laspj_list_intersection_set(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                                const laspj_batch* r, const laspj_buf* tok_order);
/* product body (lasp_core.erl:499-533): l-major pairs {X, Y}; OR-Set tokens
 * orset_causal_product(Cx, Cy) (both runs reversed, [Tx, Ty], Dx orelse Dy) */
int laspj_list_product(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* l,
                       const laspj_batch* r);
/* map / filter / fold bodies (lasp_core.erl:641-667, 681-712, 460-486) over a list in
 * list order.  The fun runs on the host once per key (an Erlang fun); its results come
 * as tables indexed by the entry's element slot (per_entry = 0; simple keys only) or by
 * entry position (per_entry = 1):
 *   map:    keys[idx] = the output key item;
 *   filter: keep[idx] = 1 to keep the entry (tombstoned entries are kept like others);
 *   fold:   the output key items of entry idx are keys[off[idx] .. off[idx+1]), each
 *           with a copy of the entry's tokens.
 * A fun that raised on a key is marked in its table entry (map / fold key item
 * ~0; filter keep = 2): if that key is in the list, the call fails with LASPJ_E_FUN
 * (the reference's body would crash there); entries for keys not in the list are never
 * looked at. */
int laspj_list_map(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                   const laspj_buf* keys, uint32_t nidx, int per_entry);
int laspj_list_filter(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                      const laspj_buf* keep, uint32_t nidx, int per_entry);
int laspj_list_fold(laspj_ctx* ctx, laspj_batch* dst, const laspj_batch* src,
                    const laspj_buf* off, const laspj_buf* keys, uint32_t nidx,
                    int per_entry);

/* ------------------------------------------------------------------ list bodies from images */
/* The combinator bodies (lasp_core.erl:460-712) and bind/3 (:291-312) on list values as a
 * NIF holds them: term_to_binary/1 images in (131 + a list: OR-Set lists of
 * {Key, [{Token, true|false}]}, G-Set lists of terms, in any order, keys / elements and
 * tokens repeated or not), the answer's image out (*out valid until the context's next
 * call), run on the device's list kernels above over a dictionary of the call's own terms
 * (calls are self-contained).  kind: LASPJ_KIND_ORSET or LASPJ_KIND_GSET (the type of
 * #dv).  verdict LASPJ_NIF_FALLBACK: a value this path does not take (not such a list, a
 * key with more than 64 distinct tokens, two `==`-equal terms under different images, a
 * G-Set intersection / product over 2-tuple elements) — the NIF runs the reference's
 * body.  A fun is the caller's to evaluate: laspj_list_etf_args gives the distinct values
 * the body passes it (the keys; a G-Set element, or the first component of a 2-tuple
 * element, lasp_core.erl:648-655, 688-695) in first-appearance order as a list image, and
 * the map / filter / fold entry points take the image of the list of its results in that
 * order (LASPJ_E_INVAL when the counts differ; fold: each result a list).  The fun is
 * taken to be pure: it is called once per distinct argument, where the reference's bodies
 * call it once per entry (lasp_core.erl:466-476, 641-709) — the same results for a pure fun,
 * fewer calls (and side effects) when keys repeat. */
/* the fun's distinct arguments (map/6, filter/6, fold/6 bodies) */
int laspj_list_etf_args(laspj_ctx* ctx, int32_t kind, const uint8_t* v, uint64_t nv,
                        const uint8_t** out, uint64_t* out_len, int32_t* verdict);
/* map/6 body — lasp_core.erl:641-667: {F(X), Causality} / F(X) in list order */
int laspj_list_etf_map(laspj_ctx* ctx, int32_t kind, const uint8_t* v, uint64_t nv,
                       const uint8_t* results, uint64_t nr, const uint8_t** out,
                       uint64_t* out_len, int32_t* verdict);
/* filter/6 body — lasp_core.erl:681-712: entries whose F(X) =:= true, tombstones kept */
int laspj_list_etf_filter(laspj_ctx* ctx, int32_t kind, const uint8_t* v, uint64_t nv,
                          const uint8_t* results, uint64_t nr, const uint8_t** out,
                          uint64_t* out_len, int32_t* verdict);
/* fold/6 body — lasp_core.erl:460-486: [{V, Causality} || V <- F(X)] / F(X), appended */
int laspj_list_etf_fold(laspj_ctx* ctx, int32_t kind, const uint8_t* v, uint64_t nv,
                        const uint8_t* results, uint64_t nr, const uint8_t** out,
                        uint64_t* out_len, int32_t* verdict);
/* union/7 body — lasp_core.erl:602-627: OR-Set orddict:merge keeping the left tokens,
 * G-Set L ++ R */
int laspj_list_etf_union(laspj_ctx* ctx, int32_t kind, const uint8_t* l, uint64_t nl,
                         const uint8_t* r, uint64_t nr, const uint8_t** out, uint64_t* out_len,
                         int32_t* verdict);
/* intersection/7 body — lasp_core.erl:546-589: {X, Cx ++ Cy} for lists:keyfind hits /
 * lists:member */
int laspj_list_etf_intersection(laspj_ctx* ctx, int32_t kind, const uint8_t* l, uint64_t nl,
                                const uint8_t* r, uint64_t nr, const uint8_t** out,
                                uint64_t* out_len, int32_t* verdict);
/* product/7 body — lasp_core.erl:499-533: X-major {{X, Y}, orset_causal_product(Cx, Cy)}
 * (lasp_lattice.erl:303-308, descending token pairs) / {X, Y} */
int laspj_list_etf_product(laspj_ctx* ctx, int32_t kind, const uint8_t* l, uint64_t nl,
                           const uint8_t* r, uint64_t nr, const uint8_t** out, uint64_t* out_len,
                           int32_t* verdict);
/* Type:value/1 of a list value — lasp_orset.erl:67-73 (keys with a {_, false} token, list
 * order) / lasp_gset.erl:74-76 (the identity) */
int laspj_list_etf_value(laspj_ctx* ctx, int32_t kind, const uint8_t* v, uint64_t nv,
                         const uint8_t** out, uint64_t* out_len, int32_t* verdict);
/* bind/3 on list values — lasp_core.erl:291-312: *status 0 when value0 =:= value (no-op),
 * 1 when merge(value0, value) (orddict:merge / ordsets:union run as written) inflates
 * value0 (lasp_lattice.erl:137-161, lists:keyfind first match: the bind writes *out), 2
 * when it does not (no write, *out null) */
int laspj_list_etf_bind(laspj_ctx* ctx, int32_t kind, const uint8_t* value0, uint64_t n0,
                        const uint8_t* value, uint64_t n, const uint8_t** out, uint64_t* out_len,
                        int32_t* status, int32_t* verdict);

/* ------------------------------------------------------------------ host dictionary */
/* The NIF side of the boundary, native (no GPU involved): element / token dictionaries
 * over external-term-format images (term_to_binary/1 of each term, no version byte),
 * ordered by Erlang term order, plus the encoder of whole values into cells.  Values
 * arrive as payloads: optional <<Tag, Vers>> (tag >= 0) + 131 + the ETF of the orddict
 * [{Elem, [{Token, true|false}]}] (OR-Set) or the ordset list (G-Set), back to back in
 * `blob` with n + 1 offsets.  Per-payload statuses are the LASPJ_DEC_* codes above. */
typedef struct laspj_dict laspj_dict;
/* Erlang term order of two ETF images (-1, 0, 1 in *out); LASPJ_E_UNSUPPORTED for terms
 * outside this path (pids, refs, funs, maps, bit strings, improper lists) */
int laspj_term_compare(const uint8_t* a, size_t na, const uint8_t* b, size_t nb, int* out);
int laspj_dict_create(laspj_dict** out);
int laspj_dict_destroy(laspj_dict* dict);
/* register every element and token term the payloads hold (append-only slots; an
 * element keeps at most 64 token slots: LASPJ_DEC_UNREPRESENTABLE past that).  A payload
 * whose status is not LASPJ_DEC_OK registers nothing (binary_to_term/1 rejects it whole). */
int laspj_dict_add(laspj_dict* dict, int32_t kind, const uint8_t* blob, const uint64_t* offsets,
                   uint64_t n, int tag, int32_t* status);
int laspj_dict_info(const laspj_dict* dict, uint32_t* elements, uint64_t* elem_bytes,
                    uint64_t* tok_bytes);
/* the arrays laspj_etf_dict_create takes, for E >= elements slots: elem_blob (elem_bytes)
 * / elem_off (E + 1) / elem_order (E: slots in term order, unused slots last); tok_blob
 * (tok_bytes) / tok_off (64 E + 1) / tok_order (64 E, 0xFF after the last) may be NULL */
int laspj_dict_export(const laspj_dict* dict, uint32_t E, uint8_t* elem_blob, uint32_t* elem_off,
                      uint32_t* elem_order, uint8_t* tok_blob, uint32_t* tok_off,
                      uint8_t* tok_order);
/* payloads -> cells over the dictionary (offsets must not descend: LASPJ_E_INVAL): out
 * holds n replicas of the batch layout
 * (OR-Set 2E words, G-Set ceil(E/64) words).  A value that is not an orddict / ordset
 * (keys or tokens not strictly ascending in term order) or holds a term outside the
 * dictionary gets LASPJ_DEC_UNKNOWN_TERM and an empty replica — such lists take the
 * list path (laspj_list_upload) */
int laspj_dict_encode(const laspj_dict* dict, int32_t kind, const uint8_t* blob,
                      const uint64_t* offsets, uint64_t n, int tag, uint32_t E, uint64_t* out,
                      int32_t* status);

/* ------------------------------------------------------------------ NIF entry points */
/* What a NIF function does between enif_term_to_binary/3 and enif_binary_to_term/4, as
 * one call: the operands arrive as term_to_binary/1 images (131 + the orddict
 * [{Elem, [{Token, true|false}]}], no tag bytes), are decoded on the device against the
 * context's own dictionary, answered there and encoded back — one copy each way and one
 * host synchronisation when every term is already in the dictionary; terms it has not
 * seen are registered (laspj_dict_add) and the device pass runs again.  Each context keeps
 * its own dictionary, device images, pinned staging and scratch (one context per BEAM
 * scheduler; no process globals); a context serialises its calls.
 *
 * verdict LASPJ_NIF_OK: the answer is valid.  LASPJ_NIF_FALLBACK: an operand this path
 * does not take — not a list of {Elem, [{Token, true|false}]} with keys and tokens
 * strictly ascending in term order, an element with no tokens or more than 64, a term
 * kind no dictionary holds — and the NIF runs the reference's own Erlang clause on the
 * terms (so the caller gets the reference's answer, or its exception).  A non-zero return
 * status is a library failure (E_NOMEM / E_DEVICE: raise).
 *
 * *out points into the context's pinned memory and stays valid until the next call on the
 * same context: the NIF hands it to enif_binary_to_term at once. */
#define LASPJ_NIF_OK       0
#define LASPJ_NIF_FALLBACK 1
/* merge/2 — lasp_orset.erl:128-134 (as lasp_core:bind/3 calls it, lasp_core.erl:298-311):
 * *out = term_to_binary(merge(A, B)) */
int laspj_orset_etf_merge(laspj_ctx* ctx, const uint8_t* a, uint64_t na, const uint8_t* b,
                          uint64_t nb, const uint8_t** out, uint64_t* out_len, int32_t* verdict);
/* n merges in one pass (a vnode's queued binds, lasp_vnode.erl:213-237): out[i], out_len[i],
 * verdict[i] per pair */
int laspj_orset_etf_merge_many(laspj_ctx* ctx, uint32_t n, const uint8_t* const* a,
                               const uint64_t* na, const uint8_t* const* b, const uint64_t* nb,
                               const uint8_t** out, uint64_t* out_len, int32_t* verdict);
/* value/1 — lasp_orset.erl:67-73: *out = term_to_binary(value(S)) (the keys with a
 * {_, false} token, in term order) */
int laspj_orset_etf_value(laspj_ctx* ctx, const uint8_t* s, uint64_t ns, const uint8_t** out,
                          uint64_t* out_len, int32_t* verdict);
/* equal/2 — lasp_orset.erl:136-138 (ORDictA == ORDictB): *result 1 / 0 */
int laspj_orset_etf_equal(laspj_ctx* ctx, const uint8_t* a, uint64_t na, const uint8_t* b,
                          uint64_t nb, int32_t* result, int32_t* verdict);
/* is_inflation (strict = 0) / is_strict_inflation (strict = 1) of prev -> cur —
 * lasp_lattice.erl:97-98,153-161 / 105-106,235-253: *result 1 / 0 */
int laspj_orset_etf_inflation(laspj_ctx* ctx, const uint8_t* prev, uint64_t np,
                              const uint8_t* cur, uint64_t nc, int strict, int32_t* result,
                              int32_t* verdict);
/* lasp_gset (lasp_gset.erl:39-43) at the same boundary, over the context's G-Set
 * dictionary (payloads: 131 + an ordset, LIST_EXT / STRING_EXT / NIL_EXT; verdicts as
 * above, FALLBACK for a list that is not an ordset in term order):
 * merge/2 — lasp_gset.erl:99-101 (ordsets:union): *out = term_to_binary(merge(A, B)) */
int laspj_gset_etf_merge(laspj_ctx* ctx, const uint8_t* a, uint64_t na, const uint8_t* b,
                         uint64_t nb, const uint8_t** out, uint64_t* out_len, int32_t* verdict);
int laspj_gset_etf_merge_many(laspj_ctx* ctx, uint32_t n, const uint8_t* const* a,
                              const uint64_t* na, const uint8_t* const* b, const uint64_t* nb,
                              const uint8_t** out, uint64_t* out_len, int32_t* verdict);
/* value/1 — lasp_gset.erl:74-76 (ordsets:to_list/1, the identity): *out = s itself */
int laspj_gset_etf_value(laspj_ctx* ctx, const uint8_t* s, uint64_t ns, const uint8_t** out,
                         uint64_t* out_len, int32_t* verdict);
/* equal/2 — lasp_gset.erl:103-105 (GSet1 == GSet2): *result 1 / 0 */
int laspj_gset_etf_equal(laspj_ctx* ctx, const uint8_t* a, uint64_t na, const uint8_t* b,
                         uint64_t nb, int32_t* result, int32_t* verdict);
/* is_inflation (strict = 0) / is_strict_inflation (strict = 1) — lasp_lattice.erl:137-140
 * (sets:is_subset) / 212-215 (and lists:usort =/=); threshold_met(lasp_gset, V, T) of
 * lasp_lattice.erl:62-65 is inflation(T, V) */
int laspj_gset_etf_inflation(laspj_ctx* ctx, const uint8_t* prev, uint64_t np,
                             const uint8_t* cur, uint64_t nc, int strict, int32_t* result,
                             int32_t* verdict);

/* ------------------------------------------------------------------ resident variables */
/* `#dv.value` (include/lasp.hrl:60-63) kept on the device between calls.  A variable is
 * one OR-Set or G-Set value over the dictionary of its own token namespace;
 * lasp_core:bind/3 (lasp_core.erl:291-312) then ships only the incoming `Value` — its
 * image is decoded on the device, `Value0 =:= Value` and merge/2 decided against the
 * resident cells by one kernel, and only the status comes back; update/4 (:283-287) runs on
 * the cells without shipping anything but the operation; the value is encoded when it is
 * read.
 *
 * Namespaces: each variable's dictionary holds the terms of its own value (as each
 * #dv.value is independent), so variables never share an element's token slots — a
 * vnode's many variables holding the same element do not crowd one another out.  Replicas
 * of one variable held in one context (laspj_var_create_replica) share a namespace: the
 * tokens one mints are known to the others, so binding a replica's state decodes with
 * every token known; so may the variables of one dataflow (laspj_var_union takes its
 * operands in one namespace).  An element past 64 tokens (add_elem never collects one)
 * widens its namespace: cells of k {p, r} pairs, up to 1024 tokens of one image length.
 * Tokens a namespace has not seen — binaries of its token length on known elements, as
 * another node's unique/1 mints them — are taken by the decoder in the same device pass
 * (laspj_nif_stats [18]).
 *
 * Ownership: the NIF wraps a laspj_var in an enif_alloc_resource
 * whose destructor calls laspj_var_destroy; the resource keeps its context's resource
 * alive (enif_keep_resource), since a variable belongs to one context (its device memory)
 * and every call on it is serialised by that context, from any scheduler.
 *
 * A value the columnar form does not hold (verdict FALLBACK of laspj_var_etf_write: an
 * element past 64 tokens whose token images differ in length, `==`-equal terms under two
 * images) is kept as its image on the host: laspj_var_etf_read answers that image, and
 * bind / update / threshold / value answer FALLBACK — the NIF runs the reference's clause
 * over the read term and stores the outcome with laspj_var_etf_write.  A namespace whose
 * dictionary grows past 2^20 elements starts a fresh one on write/4 and writes its
 * resident variables out to their images first; each is decoded again on its next call. */
typedef struct laspj_var laspj_var;
/* declare/3 (lasp_core.erl:208-218): a variable holding Type:new() = [] (kind
 * LASPJ_KIND_ORSET or LASPJ_KIND_GSET), in a namespace of its own */
int laspj_var_create(laspj_ctx* ctx, int32_t kind, laspj_var** out);
/* another replica of `peer`'s variable (its kind, context and namespace), holding new() */
int laspj_var_create_replica(laspj_var* peer, laspj_var** out);
int laspj_var_destroy(laspj_var* var);
#define LASPJ_BIND_NOOP    0
#define LASPJ_BIND_WRITTEN 1
/* bind/3 (lasp_core.erl:291-312): status LASPJ_BIND_NOOP when `Value0 =:= Value`
 * (:294-296), LASPJ_BIND_WRITTEN when Value0 := merge(Value0, Value) was written (a
 * canonical merge always inflates Value0, :300-304).  verdict FALLBACK: the variable is
 * unchanged and the NIF binds in Erlang (as above).  Calls arriving on one context while a
 * device pass runs are served together by the next pass (group commit, as bind_many);
 * while it waits, a caller copies its own image (64 KiB or more) into a pinned block the
 * pass gathers from, so `value` must stay valid until the call returns, as always. */
int laspj_var_etf_bind(laspj_var* var, const uint8_t* value, uint64_t n, int32_t* status,
                       int32_t* verdict);
/* n binds (lasp_core.erl:291-312) of distinct variables of one kind and context in one
 * device pass (a vnode's queued binds, lasp_vnode.erl:213-237) */
int laspj_var_etf_bind_many(laspj_ctx* ctx, uint32_t n, laspj_var* const* vars,
                            const uint8_t* const* values, const uint64_t* lens, int32_t* status,
                            int32_t* verdict);
/* write/4 (lasp_core.erl:839-844): the variable := value (verdict FALLBACK: held as the
 * image on the host) */
int laspj_var_etf_write(laspj_var* var, const uint8_t* value, uint64_t n, int32_t* verdict);
/* #dv.value as term_to_binary/1 (*out valid until the context's next call) */
int laspj_var_etf_read(laspj_var* var, const uint8_t** out, uint64_t* out_len, int32_t* verdict);
/* Type:value(#dv.value) — lasp_orset.erl:67-73 / lasp_gset.erl:74-76 */
int laspj_var_etf_value(laspj_var* var, const uint8_t** out, uint64_t* out_len,
                        int32_t* verdict);
/* threshold_met(Type, #dv.value, Threshold) — lasp_lattice.erl:62-75, as read/6 asks it
 * (lasp_core.erl:331-364): is_inflation (strict = 0, Threshold) or is_strict_inflation
 * (strict = 1, {strict, Threshold}) of Threshold -> the variable's value */
int laspj_var_etf_threshold(laspj_var* var, const uint8_t* threshold, uint64_t n, int strict,
                            int32_t* result, int32_t* verdict);
/* 1 when the value (#dv.value, include/lasp.hrl:60-63) is on the device, 0 when it is
 * held as an image */
int laspj_var_resident(const laspj_var* var, int32_t* resident);
/* lasp_core:union/7 (lasp_core.erl:602-627) re-run over resident variables: AccValue =
 * orddict:merge(fun(_, L, _) -> L end, l, r) — per element l's tokens where l holds it,
 * else r's — then bind/3 of AccValue into out (:291-312): status LASPJ_BIND_WRITTEN when
 * out changed, LASPJ_BIND_NOOP when not.  Nothing crosses PCIe but the status.  OR-Sets
 * of one namespace (laspj_var_create_replica); verdict FALLBACK otherwise (G-Sets — the
 * body's `LValue ++ RValue` is a list value —, variables of different namespaces,
 * host-held values): the NIF reads l and r and runs the body on their images
 * (laspj_list_etf_union) as before.  out may be l or r. */
int laspj_var_union(laspj_var* out, laspj_var* l, laspj_var* r, int32_t* status,
                    int32_t* verdict);
/* lasp_core:update/4 (lasp_core.erl:283-287) on the variable: {ok, Value} =
 * Type:update(Op, Actor, Value0) (lasp_orset.erl:99-117, 222-262; lasp_gset.erl:84-88)
 * applied to the resident cells, then bind/3 of Value, which a successful update always
 * inflates — the variable := Value.  op: term_to_binary/1 of Op — OR-Sets {add, E},
 * {add_by_token, T, E}, {add_all, Es}, {remove, E}, {remove_all, Es}, {update, Ops};
 * G-Sets {add, E}, {add_all, Es}.  Actor is not an argument: neither type's update reads it
 * (unique/1 ignores it, lasp_orset.erl:261-262).  {add, E} / {add_all, Es} mint each
 * token as unique/1 does (20 random bytes, crypto:strong_rand_bytes(20)) from the kernel's
 * CSPRNG; *minted (optional) points at the nminted tokens' bytes, 20 each, in op order
 * (valid until the context's next call).  The new terms join the variable's namespace and
 * its device images at once (a token on a known element is patched in place).
 * *result: LASPJ_UPDATE_OK, or LASPJ_UPDATE_NOT_PRESENT — the reference's
 * {error, {precondition, {not_present, E}}} (:232-241: a remove of an absent element; the
 * whole call is void, as remove_elems / apply_ops return the error and not a state), which
 * lasp_core:update/4's `{ok, Value} =` turns into a badmatch — with *err_elem / *err_len
 * (optional) the image of E (valid until the context's next call).  An update that only
 * adds returns once its kernel is enqueued; one that removes waits for the statuses.
 * verdict FALLBACK: an Op no clause of the reference's update/3 takes as written (it
 * raises), a term `==` to one the namespace holds under another image, a token of another
 * image length in a wide namespace, a host-held variable — the NIF runs the reference's
 * update on the read value and writes the result (an element's 65th token widens the
 * namespace instead). */
#define LASPJ_UPDATE_OK          0
#define LASPJ_UPDATE_NOT_PRESENT 1
int laspj_var_etf_update(laspj_var* var, const uint8_t* op, uint64_t nop, int32_t* result,
                         const uint8_t** err_elem, uint64_t* err_len, const uint8_t** minted,
                         uint32_t* nminted, int32_t* verdict);

/* counters of this context's NIF path: [0] calls, [1] device passes, [2] dictionary
 * registrations, [3] dictionary resets, [4] device image rebuilds, [5] host-encoded passes
 * (token images of mixed lengths), [6] FALLBACK verdicts, [7] dictionary elements (both
 * kinds); host nanoseconds summed over device passes: [8] staging + enqueueing, [9] waiting
 * for the device, [10] reading the answers after it, [11] the part of [8] spent copying
 * operands into pinned memory, [12] registering operands' terms in the host dictionary,
 * [13] rebuilding or patching the device images; [14] device image patches (registrations
 * that only added tokens to known elements, rewritten in place instead of rebuilt); [15]
 * merge passes run again because a segment chain checked beside the join broke before
 * any failing segment (a false element-header match: only a serial decode can judge);
 * [16] resident variables written out to their images by a dictionary reset; [17]
 * variables decoded back onto the device after one; [18] tokens a single bind's decoder
 * took that its namespace had not seen (registered after the pass: no second pass); [19]
 * namespaces widened (an element past 64 tokens: cells of k {p, r} pairs) */
#define LASPJ_NIF_STATS 20
int laspj_nif_stats(laspj_ctx* ctx, uint64_t* out, uint32_t n);
/* drop the context's dictionaries (their memory; the next call registers afresh;
 * resident variables are written out to their images and decoded again when used) */
int laspj_nif_reset(laspj_ctx* ctx);

/* ------------------------------------------------------------------ timing */
int laspj_event_create(laspj_ctx* ctx, laspj_event** out);
int laspj_event_destroy(laspj_event* ev);
int laspj_event_record(laspj_ctx* ctx, laspj_event* ev);
int laspj_event_elapsed_ms(laspj_event* start, laspj_event* stop, float* ms);

#ifdef __cplusplus
}
#endif
#endif /* LASPJ_H */
