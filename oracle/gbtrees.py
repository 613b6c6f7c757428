"""OTP `gb_trees` and the reference's `gb_trees_ext` — oracle restatement
(TEST INFRASTRUCTURE; only tests/, smoke() and bench.py's cpu_baseline use it).

`lasp_orset_gbtree` (src/lasp_orset_gbtree.erl) keeps its state in OTP's general
balanced trees, a third-party stdlib module not vendored in the reference (OTP
R16/17 era).  The clauses below restate OTP 17's published
`gb_trees.erl` (Andersson's general balanced trees, p = 2) exactly as written,
because the TREE SHAPE is observable on this path: `gb_trees_ext:equal/2`
(src/gb_trees_ext.erl:59-71) and `is_lattice_strict_inflation`'s `Ids =/= Ids1`
(src/lasp_lattice.erl:224-231) compare inner trees structurally.

Term encoding: a tree is `(Size, Node)`; `Node` is `NIL` or `(Key, Value, Smaller,
Bigger)` — the same tuples `term_to_binary` would see.  Comparisons are Erlang term
order (terms.compare): `<` / `>` in the guards, so `1` and `1.0` address the same key.
"""

from __future__ import annotations

from .terms import Atom, compare, exact_eq

NIL = Atom("nil")


class KeyExists(Exception):
    """erlang:error({key_exists, Key}) from gb_trees:insert/3."""

    def __init__(self, key):
        super().__init__(("key_exists", key))
        self.key = key


class _Triple:
    """insert_1/4's `{T, H, S}` return while the path below is being measured."""

    __slots__ = ("t", "h", "s")

    def __init__(self, t, h, s):
        self.t, self.h, self.s = t, h, s


def empty():
    """empty() -> {0, nil}."""
    return (0, NIL)


def size(t) -> int:
    return t[0]


def _lookup_node(key, node):
    while node != NIL:
        k1, _v, sm, bi = node
        c = compare(key, k1)
        if c < 0:
            node = sm
        elif c > 0:
            node = bi
        else:
            return node
    return None


def lookup(key, t):
    """lookup/2 -> {value, V} | none."""
    n = _lookup_node(key, t[1])
    return None if n is None else ("value", n[1])


def is_defined(key, t) -> bool:
    return _lookup_node(key, t[1]) is not None


def get(key, t):
    n = _lookup_node(key, t[1])
    if n is None:
        raise KeyError(key)         # function_clause in get_1/2
    return n[1]


def _update_1(key, val, node):
    k1, v, sm, bi = node
    c = compare(key, k1)
    if c < 0:
        return (k1, v, _update_1(key, val, sm), bi)
    if c > 0:
        return (k1, v, sm, _update_1(key, val, bi))
    # update_1(Key, Value, {_, _, Smaller, Bigger}) -> {Key, Value, Smaller, Bigger}
    return (key, val, sm, bi)


def update(key, val, t):
    return (t[0], _update_1(key, val, t[1]))


def _count(node):
    """count({_,_,nil,nil}) -> {1,1}; count({_,_,Sm,Bi}) -> {2*max(H1,H2), S1+S2+1};
    count(nil) -> {1,0}."""
    if node == NIL:
        return (1, 0)
    _k, _v, sm, bi = node
    if sm == NIL and bi == NIL:
        return (1, 1)
    h1, s1 = _count(sm)
    h2, s2 = _count(bi)
    return (2 * max(h1, h2), s1 + s2 + 1)


def _to_list_node(node, acc):
    # to_list({Key, Value, Small, Big}, L) -> to_list(Small, [{Key, Value} | to_list(Big, L)])
    if node == NIL:
        return acc
    k, v, sm, bi = node
    return _to_list_node(sm, [(k, v)] + _to_list_node(bi, acc))


def _balance_list_1(lst, i, s):
    """balance_list_1(L, S) over lst[i:]; returns (Tree, next index)."""
    if s > 1:
        sm = s - 1
        s2 = sm // 2
        s1 = sm - s2
        t1, i = _balance_list_1(lst, i, s1)
        k, v = lst[i]
        t2, i = _balance_list_1(lst, i + 1, s2)
        return (k, v, t1, t2), i
    if s == 1:
        k, v = lst[i]
        return (k, v, NIL, NIL), i + 1
    return NIL, i


def _balance(node, s):
    t, _ = _balance_list_1(_to_list_node(node, []), 0, s)
    return t


def _insert_1(key, val, node, s):
    """insert_1/4 with p = 2 (?pow(A, _) = A * A, ?div2(X) = X bsr 1)."""
    if node == NIL:
        if s == 0:
            return _Triple((key, val, NIL, NIL), 1, 1)
        return (key, val, NIL, NIL)
    k1, v, sm, bi = node
    c = compare(key, k1)
    if c == 0:
        raise KeyExists(key)
    if c < 0:
        r = _insert_1(key, val, sm, s >> 1)
        if not isinstance(r, _Triple):
            return (k1, v, r, bi)
        t = (k1, v, r.t, bi)
        h2, s2 = _count(bi)
    else:
        r = _insert_1(key, val, bi, s >> 1)
        if not isinstance(r, _Triple):
            return (k1, v, sm, r)
        t = (k1, v, sm, r.t)
        h2, s2 = _count(sm)
    h = 2 * max(r.h, h2)
    ss = r.s + s2 + 1
    if h > ss * ss:
        return _balance(t, ss)
    return _Triple(t, h, ss)


def insert(key, val, t):
    """insert(Key, Val, {S, T}) -> S1 = S+1, {S1, insert_1(Key, Val, T, ?pow(S1, ?p))}."""
    s1 = t[0] + 1
    r = _insert_1(key, val, t[1], s1 * s1)
    if isinstance(r, _Triple):
        r = r.t
    return (s1, r)


def enter(key, val, t):
    """enter/3: update if defined, else insert."""
    return update(key, val, t) if is_defined(key, t) else insert(key, val, t)


def to_list(t):
    return _to_list_node(t[1], [])


def from_pairs_by_insert(pairs):
    """The tree a left fold of gb_trees:insert/3 over `pairs` builds from empty()
    (what gb_trees_ext:merge's do_merge does, in walk order)."""
    t = empty()
    for k, v in pairs:
        t = insert(k, v, t)
    return t


def structurally_equal(a, b) -> bool:
    """Erlang `=:=` on two gb_trees terms (shape, keys and values)."""
    return exact_eq(a, b)


# ----------------------------------------------------------------------- gb_trees_ext

def ext_merge(t1, t2, fun):
    """gb_trees_ext:merge/3 — src/gb_trees_ext.erl:28-57: a two-finger walk of both
    in-order iterators, inserting every key into a fresh tree in walk order;
    Fun(V1, V2) on `==` keys (keeping Key1)."""
    l1, l2 = to_list(t1), to_list(t2)
    i = j = 0
    out = empty()
    while i < len(l1) or j < len(l2):
        if i < len(l1) and j < len(l2):
            (k1, v1), (k2, v2) = l1[i], l2[j]
            c = compare(k1, k2)
            if c == 0:
                out = insert(k1, fun(v1, v2), out)
                i += 1
                j += 1
            elif c < 0:
                out = insert(k1, v1, out)
                i += 1
            else:
                out = insert(k2, v2, out)
                j += 1
        elif i < len(l1):
            out = insert(l1[i][0], l1[i][1], out)
            i += 1
        else:
            out = insert(l2[j][0], l2[j][1], out)
            j += 1
    return out


def ext_equal(t1, t2) -> bool:
    """gb_trees_ext:equal/2 — src/gb_trees_ext.erl:59-71: both iterators yield the same
    `{Key, Value}` (a pattern match: exact `=:=`, inner trees compared by shape) and
    end together."""
    l1, l2 = to_list(t1), to_list(t2)
    if len(l1) != len(l2):
        return False
    return all(exact_eq(k1, k2) and exact_eq(v1, v2) for (k1, v1), (k2, v2) in zip(l1, l2))


def ext_fold(fun, acc, t):
    """gb_trees_ext:fold/3 — src/gb_trees_ext.erl:73-81: in-order left fold."""
    for k, v in to_list(t):
        acc = fun(k, v, acc)
    return acc
