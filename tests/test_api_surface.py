"""The host mirrors export every function the reference modules export (the riak_dt
behaviour callers dispatch to as Type:Fun(...)), with Erlang arity
overloads named value2 / update4 / to_binary2.  The identity callbacks are checked
here; everything else that computes is a device call covered by the GPU tests.

Reference export lists: src/lasp_orset.erl:32-36, src/lasp_gset.erl:39-43,
src/lasp_orset_gbtree.erl:32-36.
"""

from lasp_amd import gset, orset, orset_gbtree

ORSET = ["new", "value", "value2", "update", "update4", "merge", "equal", "to_binary",
         "to_binary2", "from_binary", "precondition_context", "stats", "stat",
         "parent_clock", "to_version"]
GSET = ["new", "value", "value2", "update", "update4", "merge", "equal", "to_binary",
        "to_binary2", "from_binary", "stats", "stat", "parent_clock", "to_version"]


def test_orset_exports():
    for name in ORSET:
        assert callable(getattr(orset, name)), name


def test_gset_exports():
    for name in GSET:
        assert callable(getattr(gset, name)), name


def test_gbtree_exports():
    for name in ["new", "value", "value2", "update", "update4", "merge", "equal", "stats",
                 "stat", "parent_clock", "to_version"]:
        assert callable(getattr(orset_gbtree, name)), name


def test_identity_callbacks():
    s = [(1, [(b"t" * 20, False)])]
    assert orset.parent_clock([], s) is s
    assert orset.to_version(2, s) is s
    g = [1, 2, 3]
    assert gset.parent_clock([], g) is g
    assert gset.to_version(1, g) is g
    # lasp_gset:value/2 is "not implemented yet, same as value/1" (lasp_gset.erl:78-81)
    assert gset.value2(("tokens", 1), g) == [1, 2, 3]
    assert gset.new() == [] and orset.new() == []
