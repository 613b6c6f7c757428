"""The pin chain's missing link: the C restatement (oracle/laspj_oracle.c), which the
full-size GPU parity tests use as their checker, against the KAT-pinned Python oracle
(oracle/orset.py, lattice.py, core.py — pinned by tests/test_oracle_kats.py and
test_oracle_eqc.py) on the same random canonical orddicts.

Covered: merge/2 (lasp_orset.erl:128-134), value/1 (:67-73), stats (:156-192),
is_inflation (lasp_lattice.erl:153-161, 277-285), is_strict_inflation (:235-253), the
union body (lasp_core.erl:616-618) and the filter body (:681-712).  The same comparison
runs once more on an AddressSanitizer + UBSan build of the C source in a child process
(host code only; libasan preloaded), so out-of-bounds reads in the checker cannot hide.
"""

import os
import subprocess
import sys

import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

SOAK = int(__import__("os").environ.get("LASPJ_SOAK", "1"))   # x examples for a soak run

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
E = 12          # element ids 0..11 (the C restatement keys are the element ints)
T = 8           # token pool per test: 20-byte binaries


def _tokens(seed):
    rng = np.random.default_rng(seed)
    pool = [bytes(rng.integers(0, 256, 20, dtype=np.uint8)) for _ in range(T - 2)]
    # two tokens sharing a long prefix: memcmp order = Erlang binary order
    base = bytes(rng.integers(0, 256, 19, dtype=np.uint8))
    return pool + [base + b"\x00", base + b"\xff"]


def build(ops, pool):
    """A canonical orddict from add_by_token / remove ops (oracle orset.update)."""
    from oracle import orset
    s = orset.new()
    for kind, e, t in ops:
        op = ("add_by_token", pool[t], e) if kind == "add" else ("remove", e)
        r = orset.update(op, None, s)
        if r[0] == "ok":
            s = r[1]
    return s


def _dictionary(states):
    """Per element, the distinct tokens in byte order: slot k = k-th smallest (the C
    restatement's from_cells lists slots in order, so they must be sorted)."""
    toks = np.zeros((E, 64, 20), dtype=np.uint8)
    slot = {}
    for e in range(E):
        seen = sorted({t for s in states for x, ts in s if x == e for t, _ in ts})
        for k, t in enumerate(seen):
            toks[e, k] = np.frombuffer(t, dtype=np.uint8)
            slot[(e, t)] = k
    return toks, slot


def _cells(s, slot):
    c = np.zeros((E, 2), dtype=np.uint64)
    for x, ts in s:
        for t, rm in ts:
            c[x, 0] |= np.uint64(1 << slot[(x, t)])
            if rm:
                c[x, 1] |= np.uint64(1 << slot[(x, t)])
    return c


def _decode(c, toks):
    out = []
    for x in range(E):
        p, r = int(c[x, 0]), int(c[x, 1])
        if p:
            out.append((x, [(bytes(toks[x, k]), bool((r >> k) & 1))
                            for k in range(64) if (p >> k) & 1]))
    return out


def compare_one(a, b):
    """Every restated function on (a, b) through the C restatement vs the Python oracle."""
    from oracle import columnar as orc, core, lattice, orset
    from oracle.terms import exact_eq
    m = orset.merge(a, b)
    toks, slot = _dictionary([a, b])
    A = orc.ORDict.from_cells(_cells(a, slot), toks)
    B = orc.ORDict.from_cells(_cells(b, slot), toks)
    M = A.merge(B)
    assert exact_eq(_decode(M.to_cells(toks), toks), m), "merge/2"
    assert M.equal(orc.ORDict.from_cells(_cells(m, slot), toks))
    assert exact_eq(_decode(A.union(B).to_cells(toks), toks),
                    core.union_body("lasp_orset", a, b)), "union body"
    assert exact_eq(_decode(A.filter_even().to_cells(toks), toks),
                    core.filter_body("lasp_orset", lambda x: x % 2 == 0, a)), "filter body"
    for s, S in ((a, A), (b, B), (m, M)):
        assert list(S.value()) == orset.value(s), "value/1"
        st_ = dict(orset.stats(s))
        assert S.stats() == (st_["element_count"], st_["adds_count"], st_["removes_count"])
    for p, c, P, Cc in ((a, m, A, M), (b, m, B, M), (a, b, A, B), (b, a, B, A),
                        (m, a, M, A), (a, a, A, A)):
        assert Cc.is_inflation_of(P) == lattice.is_inflation("lasp_orset", p, c), "inflation"
        assert Cc.is_strict_inflation_of(P) == \
            lattice.is_strict_inflation("lasp_orset", p, c), "strict inflation"


OP = st.tuples(st.sampled_from(["add", "add", "remove"]), st.integers(0, E - 1),
               st.integers(0, T - 1))


@settings(max_examples=300 * SOAK, deadline=None)
@given(st.lists(OP, max_size=24), st.lists(OP, max_size=24), st.integers(0, 3))
def test_c_restatement_matches_python_oracle(aops, bops, seed):
    pool = _tokens(seed)
    compare_one(build(aops, pool), build(bops, pool))


def test_c_restatement_edges():
    from oracle import orset
    pool = _tokens(7)
    full = build([("add", e, t) for e in range(E) for t in range(T)], pool)
    dead = build([("add", e, 0) for e in range(E)] + [("remove", e, 0) for e in range(E)], pool)
    for a, b in ((orset.new(), orset.new()), (orset.new(), full), (full, orset.new()),
                 (full, full), (dead, full), (full, dead), (dead, dead)):
        compare_one(a, b)


ASAN_DRIVER = r"""
import sys
sys.path.insert(0, sys.argv[1])
import numpy as np
sys.path.insert(0, sys.argv[1] + "/tests")
import test_oracle_pin as t
rng = np.random.default_rng(1234)
for i in range(int(sys.argv[2])):
    pool = t._tokens(i % 4)
    mk = lambda: [(("add", "add", "remove")[rng.integers(3)], int(rng.integers(t.E)),
                   int(rng.integers(t.T))) for _ in range(int(rng.integers(0, 30)))]
    t.compare_one(t.build(mk(), pool), t.build(mk(), pool))
print("asan ok")
"""


def _libasan():
    try:
        out = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True,
                             text=True, check=True).stdout.strip()
    except (OSError, subprocess.CalledProcessError):
        return None
    return out if os.path.isabs(out) and os.path.exists(out) else None


def test_c_restatement_under_asan_ubsan(tmp_path):
    asan = _libasan()
    if asan is None:
        pytest.skip("gcc has no libasan here")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True)
    so = os.path.join(ROOT, "oracle", "build", "liblaspj_oracle_asan.so")
    drv = tmp_path / "drv.py"
    drv.write_text(ASAN_DRIVER)
    env = dict(os.environ, LD_PRELOAD=asan, LASPJ_ORACLE_SO=so,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    res = subprocess.run([sys.executable, str(drv), ROOT, "400"], capture_output=True,
                         text=True, timeout=300, env=env)
    assert res.returncode == 0 and "asan ok" in res.stdout, res.stderr[-4000:]
