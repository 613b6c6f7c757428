"""lasp_orset restatement — oracle (TEST INFRASTRUCTURE).

Follows src/lasp_orset.erl line by line.  State is an orddict Elem -> orddict
Token -> Removed (bool).  Tokens are 20-byte binaries; the reference draws them from
`crypto:strong_rand_bytes(20)` (lasp_orset.erl:261-262), which is not reproducible, so
the oracle takes an injectable token source (`TokenSource`) and the golden vectors use
`add_by_token` (lasp_orset.erl:101-102).
"""

from __future__ import annotations

import hashlib

from . import otp


class PreconditionError(Exception):
    """{error, {precondition, {not_present, Elem}}} (lasp_orset.erl:240)."""

    def __init__(self, elem):
        super().__init__(("precondition", ("not_present", elem)))
        self.elem = elem


class TokenSource:
    """Deterministic stand-in for `unique/1` (lasp_orset.erl:261-262): 20-byte tokens
    derived from a seed and a counter."""

    def __init__(self, seed: int = 0):
        self.seed = seed
        self.n = 0

    def __call__(self, actor=None) -> bytes:
        self.n += 1
        return hashlib.sha1(f"lasp-token:{self.seed}:{self.n}".encode()).digest()


_default_tokens = TokenSource(0)


def new():
    """new/0 — lasp_orset.erl:63-65."""
    return otp.orddict_new()


def value(s):
    """value/1 — lasp_orset.erl:67-73: elements with at least one {Token, false}."""
    kept = otp.orddict_filter(
        lambda _e, toks: len([t for t, rm in otp.orddict_to_list(toks) if rm is False]) > 0, s)
    return otp.orddict_fetch_keys(kept)


def value2(query, s):
    """value/2 — lasp_orset.erl:75-97."""
    if isinstance(query, tuple) and len(query) == 2 and query[0] == "fragment":
        toks = value2(("tokens", query[1]), s)
        if toks == []:
            return otp.orddict_new()
        return otp.orddict_store(query[1], toks, otp.orddict_new())
    if isinstance(query, tuple) and len(query) == 2 and query[0] == "tokens":
        found = otp.orddict_find(query[1], s)
        return otp.orddict_new() if found is None else found[1]
    if query == "removed":
        kept = otp.orddict_filter(
            lambda _e, toks: len([t for t, rm in otp.orddict_to_list(toks) if rm is True]) > 0, s)
        return otp.orddict_fetch_keys(kept)
    return value(s)


def _add_elem(elem, token, s):
    """add_elem/3 — lasp_orset.erl:222-230."""
    found = otp.orddict_find(elem, s)
    if found is not None:
        toks1 = otp.orddict_store(token, False, found[1])
        return otp.orddict_store(elem, toks1, s)
    toks = otp.orddict_store(token, False, otp.orddict_new())
    return otp.orddict_store(elem, toks, s)


def _remove_elem(elem, s):
    """remove_elem/2 — lasp_orset.erl:232-241: every token of Elem becomes true."""
    found = otp.orddict_find(elem, s)
    if found is None:
        raise PreconditionError(elem)
    toks1 = otp.orddict_fold(lambda tok, _v, acc: otp.orddict_store(tok, True, acc),
                             otp.orddict_new(), found[1])
    return otp.orddict_store(elem, toks1, s)


def update(op, actor, s, tokens=None):
    """update/3 — lasp_orset.erl:99-117.  Returns ("ok", S1) or
    ("error", ("precondition", ("not_present", E)))."""
    tokens = tokens or _default_tokens
    try:
        return ("ok", _update(op, actor, s, tokens))
    except PreconditionError as e:
        return ("error", ("precondition", ("not_present", e.elem)))


def _update(op, actor, s, tokens):
    kind = op[0]
    if kind == "add_by_token":
        return _add_elem(op[2], op[1], s)
    if kind == "add":
        return _add_elem(op[1], tokens(actor), s)
    if kind == "add_all":
        for e in op[1]:
            s = _add_elem(e, tokens(actor), s)
        return s
    if kind == "remove":
        return _remove_elem(op[1], s)
    if kind == "remove_all":
        # remove_elems/2 (:244-250) stops at the first error; the caller keeps the
        # original state because Erlang terms are immutable.
        for e in op[1]:
            s = _remove_elem(e, s)
        return s
    if kind == "update":
        # apply_ops/3 (:253-259)
        for sub in op[1]:
            s = _update(sub, actor, s, tokens)
        return s
    raise ValueError(f"function_clause: unknown op {op!r}")


def merge(a, b):
    """merge/2 — lasp_orset.erl:128-134: nested orddict:merge with `or`."""
    return otp.orddict_merge(
        lambda _e, ta, tb: otp.orddict_merge(lambda _t, ba, bb: ba or bb, ta, tb), a, b)


def equal(a, b) -> bool:
    """equal/2 — lasp_orset.erl:136-138 (structural ==)."""
    from .terms import eq
    return eq(_as_term(a), _as_term(b))


def _as_term(s):
    return [(e, [(t, r) for t, r in toks]) for e, toks in s]


def precondition_context(s):
    """precondition_context/1 — lasp_orset.erl:147-154 (+ minimum_tokens :264-267)."""
    def step(elem, toks, acc):
        live = otp.orddict_filter(lambda _t, removed: not removed, toks)
        if live == []:
            return acc
        return otp.orddict_store(elem, live, acc)
    return otp.orddict_fold(step, otp.orddict_new(), s)


def stat(name, s):
    """stat/2 — lasp_orset.erl:163-192."""
    if name == "element_count":
        return otp.orddict_size(s)
    if name == "adds_count":
        return sum(1 for _e, toks in s for _t, rm in toks if rm is False)
    if name == "removes_count":
        return sum(1 for _e, toks in s for _t, rm in toks if rm is True)
    if name == "waste_pct":
        tags = sum(1 for _e, toks in s for _t, rm in toks if rm is False)
        tombs = sum(1 for _e, toks in s for _t, rm in toks if rm is True)
        if tags == 0:
            return 0
        return erlang_round(tombs / (tags + tombs) * 100)
    return None


def stats(s):
    """stats/1 — lasp_orset.erl:156-161."""
    return [(n, stat(n, s)) for n in ("element_count", "adds_count", "removes_count", "waste_pct")]


def erlang_round(x: float) -> int:
    """erlang:round/1 rounds half away from zero."""
    import math
    return int(math.floor(x + 0.5)) if x >= 0 else -int(math.floor(-x + 0.5))
