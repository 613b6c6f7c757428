"""gb_trees terms on the host side of the engine (what the NIF receives and returns
for `lasp_orset_gbtree` states).

A tree is `(Size, Node)`, `Node` = `nil` | `(Key, Value, Smaller, Bigger)`.  The
device holds only contents (the columnar cells); shapes are produced here:

* `walk(tree)` — in-order `(Key, Value)` pairs (gb_trees:to_list/1), to encode.
* `build_sorted(pairs)` — the exact tree OTP's `gb_trees:insert/3` builds when the
  keys arrive in ascending order starting from `empty()`.  That is how
  `gb_trees_ext:merge/3` (src/gb_trees_ext.erl:28-57) builds every merged tree, and
  how `remove_elem` rebuilds a token tree (src/lasp_orset_gbtree.erl:242-253), so it
  is the shape of every value `lasp_core:bind/3` stores.

Ascending inserts always descend the right spine, so `build_sorted` keeps the spine
as an explicit path instead of recursing: at depth d the insert budget is
`S1^2 >> d`; a leaf placed where the budget is 0 starts the height/size measurement
(`{T, H, S}` in insert_1/4), which climbs the spine and rebalances the first ancestor
whose measured height exceeds its size squared (p = 2).
"""

from __future__ import annotations

from .terms import Atom

NIL = Atom("nil")


def empty():
    return (0, NIL)


def is_tree(t) -> bool:
    return isinstance(t, tuple) and len(t) == 2 and isinstance(t[0], int) \
        and not isinstance(t[0], bool) and (t[1] == NIL or (isinstance(t[1], tuple)
                                                           and len(t[1]) == 4))


def walk(t) -> list:
    """gb_trees:to_list/1 (in-order), iteratively."""
    if not is_tree(t):
        raise ValueError(f"badarg: not a gb_tree: {t!r}")
    out, stack, node = [], [], t[1]
    while stack or node != NIL:
        while node != NIL:
            stack.append(node)
            node = node[2]
        node = stack.pop()
        out.append((node[0], node[1]))
        node = node[3]
    return out


def _freeze(n):
    if n is None:
        return NIL
    return (n[0], n[1], _freeze(n[2]), _freeze(n[3]))


def _measure(n):
    """count/1 of a mutable subtree: (H, S)."""
    if n is None:
        return 1, 0
    if n[2] is None and n[3] is None:
        return 1, 1
    h1, s1 = _measure(n[2])
    h2, s2 = _measure(n[3])
    return 2 * max(h1, h2), s1 + s2 + 1


def _inorder(n, out):
    stack = []
    while stack or n is not None:
        while n is not None:
            stack.append(n)
            n = n[2]
        n = stack.pop()
        out.append(n)
        n = n[3]


def _perfect(nodes, lo, s):
    """balance_list_1/2: S nodes from nodes[lo:] -> (subtree, next)."""
    if s == 0:
        return None, lo
    if s == 1:
        n = nodes[lo]
        n[2] = n[3] = None
        return n, lo + 1
    s2 = (s - 1) // 2
    left, i = _perfect(nodes, lo, s - 1 - s2)
    root = nodes[i]
    right, i = _perfect(nodes, i + 1, s2)
    root[2], root[3] = left, right
    return root, i


def build_sorted(pairs) -> tuple:
    """The gb_tree of `pairs` (ascending, distinct keys) inserted in order."""
    root = None
    n = 0
    for k, v in pairs:
        n += 1
        budget = n * n
        leaf = [k, v, None, None]
        spine = []
        node = root
        while node is not None:
            spine.append(node)
            node = node[3]
            budget >>= 1
        if not spine:
            root = leaf
            continue
        spine[-1][3] = leaf
        if budget != 0:
            continue
        h, s = 1, 1                     # measuring from the new leaf upwards
        for depth in range(len(spine) - 1, -1, -1):
            anc = spine[depth]
            h2, s2 = _measure(anc[2])
            h = 2 * max(h, h2)
            s = s + s2 + 1
            if h > s * s:
                nodes = []
                _inorder(anc, nodes)
                sub, _ = _perfect(nodes, 0, s)
                if depth == 0:
                    root = sub
                else:
                    spine[depth - 1][3] = sub
                break
    return (n, _freeze(root))


# --------------------------------------------------------------------------- any order
# OTP 17 gb_trees:insert/3, update/3, enter/3 and lookup/2 on the same terms, for the
# shapes the reference's update path builds: add_elem inserts a token into the element's
# existing token tree and enters the element into the set (src/lasp_orset_gbtree.erl:
# 231-240), so a tree built by updates keeps the shape of its insertion history.  The
# engine computes contents on the device; these functions only place keys (values are
# filled in afterwards, in order, from the device's result).

def _cmp(a, b) -> int:
    from .terms import term_cmp
    return term_cmp(a, b)


def _count(n):
    """count/1: (H, S) of an immutable subtree."""
    if n == NIL:
        return 1, 0
    if n[2] == NIL and n[3] == NIL:
        return 1, 1
    h1, s1 = _count(n[2])
    h2, s2 = _count(n[3])
    return 2 * max(h1, h2), s1 + s2 + 1


def _balance(n, s):
    """balance/2: the perfectly balanced tree of n's S nodes."""
    nodes = []
    _inorder_t(n, nodes)
    lst = [[k, v, None, None] for k, v in nodes]
    sub, _ = _perfect(lst, 0, s)
    return _freeze(sub)


def _inorder_t(n, out):
    stack = []
    while stack or n != NIL:
        while n != NIL:
            stack.append(n)
            n = n[2]
        n = stack.pop()
        out.append((n[0], n[1]))
        n = n[3]


class KeyExists(Exception):
    """erlang:error({key_exists, Key}) from gb_trees:insert/3."""


class _Measured:
    """{T, H, S}: a subtree whose height is being measured on the way up."""
    __slots__ = ("t", "h", "s")

    def __init__(self, t, h, s):
        self.t, self.h, self.s = t, h, s


def _insert_1(key, val, n, s):
    """insert_1/4: a node, or _Measured while the height is being measured."""
    if n == NIL:
        return _Measured((key, val, NIL, NIL), 1, 1) if s == 0 else (key, val, NIL, NIL)
    c = _cmp(key, n[0])
    if c == 0:
        raise KeyExists(key)
    r = _insert_1(key, val, n[2] if c < 0 else n[3], s >> 1)
    if isinstance(r, _Measured):
        t = (n[0], n[1], r.t, n[3]) if c < 0 else (n[0], n[1], n[2], r.t)
        h2, s2 = _count(n[3] if c < 0 else n[2])
        h = 2 * max(r.h, h2)
        ss = r.s + s2 + 1
        if h > ss * ss:
            return _balance(t, ss)
        return _Measured(t, h, ss)
    return (n[0], n[1], r, n[3]) if c < 0 else (n[0], n[1], n[2], r)


def insert(key, val, t):
    s1 = t[0] + 1
    r = _insert_1(key, val, t[1], s1 * s1)
    return (s1, r.t if isinstance(r, _Measured) else r)


def lookup(key, t):
    n = t[1]
    while n != NIL:
        c = _cmp(key, n[0])
        if c == 0:
            return n[1]
        n = n[2] if c < 0 else n[3]
    return None


def _update_1(key, val, n):
    c = _cmp(key, n[0])
    if c < 0:
        return (n[0], n[1], _update_1(key, val, n[2]), n[3])
    if c > 0:
        return (n[0], n[1], n[2], _update_1(key, val, n[3]))
    return (n[0], val, n[2], n[3])


def update(key, val, t):
    return (t[0], _update_1(key, val, t[1]))


def enter(key, val, t):
    return update(key, val, t) if lookup(key, t) is not None else insert(key, val, t)


def keys(t) -> list:
    return [k for k, _v in walk(t)]


def shape(t):
    """The tree with its values dropped: two trees of equal contents are the same term
    exactly when their shapes are equal."""
    def strip(n):
        return NIL if n == NIL else (n[0], strip(n[2]), strip(n[3]))
    return (t[0], strip(t[1]))


def fill(t, values) -> tuple:
    """t with its in-order values replaced by `values` (same length, in order)."""
    it = iter(values)

    def go(n):
        if n == NIL:
            return NIL
        left = go(n[2])
        v = next(it)
        return (n[0], v, left, go(n[3]))
    out = (t[0], go(t[1]))
    if next(it, None) is not None:
        raise ValueError("more values than keys")
    return out
