#!/usr/bin/env python3
"""Generate tests/golden/*.json with the oracle (oracle/), from seeded inputs.

Inputs are built with lasp_orset:update({add_by_token, Token, E}) / {remove, E}
(lasp_orset.erl:101-102,112-113) and deterministic 20-byte tokens, so every vector is
reproducible; expected outputs are the oracle's restatement of the reference
(merge/2, value/1, value(removed), stats/1, is_inflation/3, is_strict_inflation/3,
the union / intersection / product / filter / map / fold bodies).  The reference's
own known answers are re-checked by tests/test_oracle_kats.py.

    python tests/golden/make_golden.py        # rewrites the fixtures
"""
import hashlib
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import core, gset, lattice, orset  # noqa: E402
from oracle.terms import Atom  # noqa: E402
from tests.golden.termjson import enc  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def tok(seed, i):
    return hashlib.sha1(f"golden:{seed}:{i}".encode()).digest()


def rand_orset(rng, seed, n_ops, universe):
    s = orset.new()
    k = 0
    for _ in range(n_ops):
        e = rng.choice(universe)
        if rng.random() < 0.75:
            k += 1
            s = orset.update(("add_by_token", tok(seed, k), e), None, s)[1]
        else:
            r = orset.update(("remove", e), None, s)
            if r[0] == "ok":
                s = r[1]
    return s


def main():
    rng = random.Random(0x4C415350)
    ints = list(range(40))
    mixed = [0, 1, 7, -3, Atom("a"), Atom("zz"), b"bin", b"", (1, 2), (Atom("x"),), [1], [1, 2]]
    cases = []
    for n in range(60):
        universe = mixed if n % 5 == 4 else ints
        # shared ancestry: b starts from a so some tokens coincide
        a = rand_orset(rng, 2 * n, rng.randint(0, 18), universe)
        b = a if n % 7 == 3 else rand_orset(rng, 2 * n + 1, rng.randint(0, 18), universe)
        if n % 3 == 0:
            b = orset.merge(a, b)
            b = orset.update(("add_by_token", tok(999, n), rng.choice(universe)), None, b)[1]
        m = orset.merge(a, b)
        cases.append({
            "a": enc(a), "b": enc(b), "merge": enc(m),
            "value_a": enc(orset.value(a)), "removed_a": enc(orset.value2("removed", a)),
            "stats_a": [list(x) for x in orset.stats(a)],
            "equal_ab": orset.equal(a, b),
            "infl_a_m": lattice.is_inflation("lasp_orset", a, m),
            "infl_b_a": lattice.is_inflation("lasp_orset", b, a),
            "strict_a_m": lattice.is_strict_inflation("lasp_orset", a, m),
            "strict_a_a": lattice.is_strict_inflation("lasp_orset", a, a),
            "strict_b_a": lattice.is_strict_inflation("lasp_orset", b, a),
            "union": enc(core.union_body("lasp_orset", a, b)),
            "filter_even": enc(core.filter_body(
                "lasp_orset", lambda x: isinstance(x, int) and x % 2 == 0, a)),
            "intersection": enc(core.intersection_body("lasp_orset", a, b)),
            "product": enc(core.product_body("lasp_orset", a[:4], b[:4])),
            "map_x2": enc(core.map_body("lasp_orset", lambda x: x * 2, a)) if universe is ints else None,
            "fold_x3": enc(core.fold_body("lasp_orset", lambda x: [x, x, x], a)),
        })
    with open(os.path.join(HERE, "orset_cases.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "cases": cases}, f)

    gcases = []
    for n in range(40):
        universe = mixed if n % 4 == 3 else ints
        a = gset.new()
        b = gset.new()
        for _ in range(rng.randint(0, 25)):
            a = gset.update(("add", rng.choice(universe)), None, a)[1]
        for _ in range(rng.randint(0, 25)):
            b = gset.update(("add", rng.choice(universe)), None, b)[1]
        m = gset.merge(a, b)
        gcases.append({
            "a": enc(a), "b": enc(b), "merge": enc(m),
            "equal_ab": gset.equal(a, b),
            "infl_a_m": lattice.is_inflation("lasp_gset", a, m),
            "infl_b_a": lattice.is_inflation("lasp_gset", b, a),
            "strict_a_m": lattice.is_strict_inflation("lasp_gset", a, m),
            "strict_m_m": lattice.is_strict_inflation("lasp_gset", m, m),
            "stats_a": [list(x) for x in gset.stats(a)],
        })
    with open(os.path.join(HERE, "gset_cases.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "cases": gcases}, f)
    print(len(cases), len(gcases))


if __name__ == "__main__":
    main()
