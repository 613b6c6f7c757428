"""lasp_orset mirror over the MI355X engine (the NIF module's behaviour, in Python).

Same names, argument meaning and error behaviour as src/lasp_orset.erl; states are
Erlang-shaped orddicts (see lasp_amd.terms).  Each call encodes its operands into a
batch of a per-call Domain, runs the HIP kernel through the C ABI and decodes the
result — the single-object path of the drop-in.  Throughput callers batch many
objects per call (`merge_many`, or lasp_amd.engine directly).
"""

from __future__ import annotations

import os
from typing import List, Sequence, Tuple

import numpy as np

from . import _lib, engine
from .codec import Domain, NonCanonical  # noqa: F401  (re-exported error type)
from .terms import Atom

_CTX = None


def context() -> engine.Context:
    """The process-wide engine context (device $LASPJ_DEVICE, default 0)."""
    global _CTX
    if _CTX is None:
        _CTX = engine.Context(int(os.environ.get("LASPJ_DEVICE", "0")))
    return _CTX


# an element keeps up to 64 * TOKEN_WORDS tokens: values naming a token slot >= 64 go to
# wide cells (LASPJ_KIND_ORSET_WIDE, k {p, r} pairs per element)
TOKEN_WORDS = 16


def _domain() -> Domain:
    return Domain(token_capacity=64 * TOKEN_WORDS)


def _new(R: int, E: int, k: int):
    return context().orset_batch(R, E) if k == 1 else context().orset_wide_batch(R, E, k)


def _batch(dom: Domain, states: Sequence, k: int = 1) -> Tuple[engine.ORSetBatch, int]:
    k = max(k, dom.orset_words(states))
    E = max(1, dom.size)
    b = _new(len(states), E, k)
    b.upload(dom.encode_orset(states, E) if k == 1 else dom.encode_orset_wide(states, E, k))
    return b, E


def _decode(dom: Domain, cells: np.ndarray) -> list:
    return dom.decode_orset_wide(cells) if cells.ndim == 3 else dom.decode_orset(cells)


# --------------------------------------------------------------------------- API

def new():
    """new/0 — lasp_orset.erl:63-65."""
    return []


def merge(a, b):
    """merge/2 — lasp_orset.erl:128-134 (device join)."""
    return merge_many([(a, b)])[0]


def merge_many(pairs: Sequence[Tuple[list, list]]) -> List[list]:
    """merge/2 over many independent pairs in one launch."""
    if not pairs:
        return []
    dom = _domain()
    k = dom.orset_words([p[0] for p in pairs] + [p[1] for p in pairs])
    A, E = _batch(dom, [p[0] for p in pairs], k)
    B, _ = _batch(dom, [p[1] for p in pairs], k)
    C = _new(len(pairs), E, k)
    C.join(A, B)
    out = C.download()
    return [_decode(dom, out[i]) for i in range(len(pairs))]


def value(s):
    """value/1 — lasp_orset.erl:67-73 (device value bitmap)."""
    dom = _domain()
    b, _ = _batch(dom, [s])
    return dom.decode_value_bits(b.value_bits()[0])


def value2(query, s):
    """value/2 — lasp_orset.erl:75-97."""
    if isinstance(query, tuple) and len(query) == 2 and query[0] == "fragment":
        toks = value2(("tokens", query[1]), s)
        return [] if toks == [] else [(query[1], toks)]
    if isinstance(query, tuple) and len(query) == 2 and query[0] == "tokens":
        # orddict:find(Elem, ORSet): the element's cell, read on the device
        dom = _domain()
        b, _ = _batch(dom, [s])
        es = dom.element_slot(query[1], create=False)
        if es < 0:
            return []
        pairs = b.fragment(es)[0].reshape(-1, 2)
        p = sum(int(pairs[j, 0]) << (64 * j) for j in range(len(pairs)))
        r = sum(int(pairs[j, 1]) << (64 * j) for j in range(len(pairs)))
        td = dom.tokens[es]
        return [(td.terms[k], bool((r >> int(k)) & 1)) for k in td.order() if (p >> int(k)) & 1]
    if query == "removed":
        dom = _domain()
        b, _ = _batch(dom, [s])
        return dom.decode_value_bits(b.value_bits(removed=True)[0])
    return value(s)


def precondition_context(s):
    """precondition_context/1 — lasp_orset.erl:147-154: the adds observed (tokens
    flagged false), computed on the device."""
    dom = _domain()
    b, E = _batch(dom, [s])
    out = _new(1, E, getattr(b, "token_words", 1)).precondition_context(b)
    return _decode(dom, out.download()[0])


def update(op, actor, s):
    """update/3 — lasp_orset.erl:99-117.  Returns ("ok", S1) or
    ("error", ("precondition", ("not_present", Elem)))."""
    dom = _domain()
    k = dom.orset_words([s])
    ops = []
    _compile(op, dom, ops, new_call=True)
    k = max([k] + [(o[3] >> 6) + 1 for o in ops if o[2] != _lib.OP_REMOVE])
    b, _E = _batch(dom, [s], k)
    st = b.apply_ops(ops)
    bad = np.nonzero(st == _lib.OPST_NOT_PRESENT)[0]
    if len(bad):
        return ("error", ("precondition", ("not_present", dom.elements.terms[ops[bad[0]][1]])))
    return ("ok", _decode(dom, b.download()[0]))


def update4(op, actor, s, _ctx=None):
    """update/4 — lasp_orset.erl:119-122 (context ignored)."""
    return update(op, actor, s)


def parent_clock(_clock, s):
    """parent_clock/2 — lasp_orset.erl:124-126 (identity)."""
    return s


def to_version(_version, s):
    """to_version/2 — lasp_orset.erl:216-218 (identity)."""
    return s


def _unique(_actor) -> bytes:
    """unique/1 — lasp_orset.erl:261-262: 20 random bytes."""
    return os.urandom(20)


def _compile(op, dom: Domain, ops: list, new_call: bool) -> None:
    kind = op[0]
    flag = _lib.OP_FLAG_NEW_CALL if new_call else 0
    if kind in ("add", "add_by_token"):
        elem = op[1] if kind == "add" else op[2]
        tok = _unique(None) if kind == "add" else op[1]
        es = dom.element_slot(elem)
        ops.append((0, es, _lib.OP_ADD, dom.token_slot(es, tok), flag))
    elif kind == "add_all":
        # foldl of update({add, E}) (:106-111): every add is its own call
        for e in op[1]:
            es = dom.element_slot(e)
            ops.append((0, es, _lib.OP_ADD, dom.token_slot(es, _unique(None)),
                        _lib.OP_FLAG_NEW_CALL))
    elif kind == "remove":
        ops.append((0, dom.element_slot(op[1]), _lib.OP_REMOVE, 0, flag))
    elif kind == "remove_all":
        # remove_elems/2 (:244-250): one all-or-nothing call
        for k, e in enumerate(op[1]):
            ops.append((0, dom.element_slot(e), _lib.OP_REMOVE, 0, flag if k == 0 else 0))
    elif kind == "update":
        # apply_ops/3 (:253-259): the whole list is one all-or-nothing call
        first = len(ops)
        for sub in op[1]:
            _compile(sub, dom, ops, new_call=False)
        if len(ops) > first:
            r, e, k, sl, _f = ops[first]
            ops[first] = (r, e, k, sl, flag)
        for j in range(first + 1, len(ops)):
            r, e, k, sl, _f = ops[j]
            ops[j] = (r, e, k, sl, 0)
    else:
        raise ValueError(f"function_clause: {op!r}")


def equal(a, b) -> bool:
    """equal/2 — lasp_orset.erl:136-138."""
    dom = _domain()
    k = dom.orset_words([a, b])
    A, _E = _batch(dom, [a], k)
    B, _E = _batch(dom, [b], k)
    return bool(A.equal(B)[0])


def stats(s):
    """stats/1 — lasp_orset.erl:156-161."""
    dom = _domain()
    b, _ = _batch(dom, [s])
    elems, adds, rems = (int(x) for x in b.stats()[0])
    return [("element_count", elems), ("adds_count", adds), ("removes_count", rems),
            ("waste_pct", _waste_pct(adds, rems))]


def stat(name, s):
    """stat/2 — lasp_orset.erl:163-192 (unknown stat -> undefined)."""
    for k, v in stats(s):
        if k == name:
            return v
    return Atom("undefined")


def _waste_pct(adds: int, rems: int) -> int:
    # case Tags of 0 -> 0; _ -> round(Tombs / AllTags * 100) end  (erlang:round: half away)
    if adds == 0:
        return 0
    import math
    return int(math.floor(rems / (adds + rems) * 100 + 0.5))


# --------------------------------------------------------------------------- wire codec

def to_binary(s, tag: int = None) -> bytes:
    """to_binary/1 — lasp_orset.erl:198: <<?TAG, ?V1_VERS, term_to_binary(S)>>,
    assembled on the device from the cells (laspj_orset_etf_write)."""
    from . import etf
    from .engine import ETFDict
    dom = Domain()
    b, _ = _batch(dom, [s])
    E = b.elements
    d = ETFDict(context(), E, *dom.etf_arrays(E, tokens=True))
    return b.to_binaries(d, etf.DT_ORSET_TAG if tag is None else tag, etf.V1_VERS)[0]


def to_binary2(vers, s):
    """to_binary/2: version 1 -> {ok, Bin}; else {error, unsupported_version, Vers}."""
    if vers == 1:
        return ("ok", to_binary(s))
    return ("error", "unsupported_version", vers)


def from_binary(b: bytes, tag: int = None):
    """from_binary/1 — lasp_orset.erl:198-214: binary_to_term of the payload after
    <<?TAG, 1>> (returned bare, as riak_dt:from_binary/1 returns it);
    {error, unsupported_version, V} or {error, invalid_binary} otherwise."""
    from . import etf
    tag = etf.DT_ORSET_TAG if tag is None else tag
    b = bytes(b)
    if len(b) >= 2 and b[0] == tag:
        if b[1] != etf.V1_VERS:
            return ("error", "unsupported_version", b[1])
        state = etf.binary_to_term(b[2:])
        return state
    return ("error", "invalid_binary")
