"""lasp_orset_gbtree restatement — oracle (TEST INFRASTRUCTURE).

Follows src/lasp_orset_gbtree.erl line by line on top of the gb_trees restatement
(oracle/gbtrees.py).  State: gb_tree Elem -> gb_tree Token -> Removed (bool).
Differences from lasp_orset that the restatement keeps:
  * add_elem uses gb_trees:insert for the token (:232-240), so adding a token that is
    already present raises {key_exists, Token} instead of resetting its flag;
  * the outer tree is updated with gb_trees:enter (insert on a new element);
  * equal/2 is gb_trees_ext:equal (:142-144): inner trees are compared by shape.
"""

from __future__ import annotations

from . import gbtrees as gb
from .orset import PreconditionError, TokenSource, erlang_round

_default_tokens = TokenSource(7)


def new():
    """new/0 — :63-65."""
    return gb.empty()


def _valid_tokens(toks):
    return [t for t, rm in gb.to_list(toks) if rm is False]


def _removed_tokens(toks):
    return [t for t, rm in gb.to_list(toks) if rm is True]


def value(s):
    """value/1 — :67-76: in-order fold, `Acc0 ++ [Elem]` when a token is live."""
    return gb.ext_fold(lambda e, toks, acc: acc + [e] if len(_valid_tokens(toks)) > 0 else acc,
                       [], s)


def value2(query, s):
    """value/2 — :78-104 (a `{tokens, E}` result is a tree, never `[]`, so
    `{fragment, E}` of an absent E is `{E, empty()}` in a one-entry tree)."""
    if isinstance(query, tuple) and len(query) == 2 and query[0] == "fragment":
        toks = value2(("tokens", query[1]), s)
        if toks == []:              # `[] -> gb_trees:empty()` only matches the list []
            return gb.empty()
        return gb.enter(query[1], toks, gb.empty())
    if isinstance(query, tuple) and len(query) == 2 and query[0] == "tokens":
        if gb.is_defined(query[1], s):
            return gb.get(query[1], s)
        return gb.empty()
    if query == "removed":
        return gb.ext_fold(
            lambda e, toks, acc: acc + [e] if len(_removed_tokens(toks)) > 0 else acc, [], s)
    return value(s)


def _add_elem(elem, token, s):
    """add_elem/3 — :232-240."""
    found = gb.lookup(elem, s)
    if found is not None:
        toks1 = gb.insert(token, False, found[1])
        return gb.enter(elem, toks1, s)
    toks = gb.insert(token, False, gb.empty())
    return gb.enter(elem, toks, s)


def _remove_elem(elem, s):
    """remove_elem/2 — :242-253: rebuild the token tree with every flag true."""
    found = gb.lookup(elem, s)
    if found is None:
        raise PreconditionError(elem)
    toks1 = gb.ext_fold(lambda k, _v, acc: gb.enter(k, True, acc), gb.empty(), found[1])
    return gb.enter(elem, toks1, s)


def update(op, actor, s, tokens=None):
    """update/3 — :106-124.  ("ok", S1) or ("error", ("precondition", ("not_present",
    E))); a duplicate add_by_token token raises gbtrees.KeyExists (a crash in the
    reference)."""
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
        for e in op[1]:              # remove_elems/2 (:255-263)
            s = _remove_elem(e, s)
        return s
    if kind == "update":
        for sub in op[1]:            # apply_ops/3 (:266-274)
            s = _update(sub, actor, s, tokens)
        return s
    raise ValueError(f"function_clause: unknown op {op!r}")


def merge(a, b):
    """merge/2 — :134-140: gb_trees_ext:merge of gb_trees_ext:merge with `or`."""
    return gb.ext_merge(a, b, lambda ta, tb: gb.ext_merge(ta, tb, lambda x, y: x or y))


def equal(a, b) -> bool:
    """equal/2 — :142-144."""
    return gb.ext_equal(a, b)


def precondition_context(s):
    """precondition_context/1 — :153-162 (+ minimum_tokens :279-287).  Note the
    reference stores the `[{Key, false}]` LIST that minimum_tokens returns."""
    def step(elem, toks, acc):
        live = gb.ext_fold(lambda k, rm, a: a if rm is True else a + [(k, rm)], [], toks)
        if live == []:
            return acc
        return gb.enter(elem, live, acc)
    return gb.ext_fold(step, gb.empty(), s)


def stat(name, s):
    """stat/2 — :171-200."""
    pairs = [(rm) for _e, toks in gb.to_list(s) for _t, rm in gb.to_list(toks)]
    if name == "element_count":
        return gb.size(s)
    if name == "adds_count":
        return sum(1 for rm in pairs if rm is False)
    if name == "removes_count":
        return sum(1 for rm in pairs if rm is True)
    if name == "waste_pct":
        tags = sum(1 for rm in pairs if rm is False)
        tombs = sum(1 for rm in pairs if rm is True)
        if tags == 0:
            return 0
        return erlang_round(tombs / (tags + tombs) * 100)
    return None


def stats(s):
    """stats/1 — :164-169."""
    return [(n, stat(n, s)) for n in ("element_count", "adds_count", "removes_count", "waste_pct")]


def to_orddict(s):
    """The orddict-shaped content of a gbtree OR-Set (in-order walk of both levels)."""
    return [(e, gb.to_list(toks)) for e, toks in gb.to_list(s)]
