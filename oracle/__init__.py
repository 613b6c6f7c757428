"""CPU oracle for the lattice-join hot path — TEST INFRASTRUCTURE ONLY.

This package restates, on the CPU, the reference algorithms of Applied-Duality/lasp
for the OR-Set / G-Set lattice join, the value / threshold / inflation predicates and
the monotonic set combinators, together with the OTP stdlib clauses they rely on
(`orddict`, `ordsets`, `lists`).  Every function cites the
reference file:line it follows (paths relative to the reference checkout).

Who may use it: only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s
`cpu_baseline` leg, and there only as the *checker* (or as the timed CPU baseline),
never as the product path.  The product (`lasp_amd`) never imports this package.

Parity pinning: the reference is Erlang and no Erlang toolchain exists in this
image, so the reference cannot be run here.  The restatement is
pinned by the reference's own known-answer tests (eunit `stat_test`s, the
`lasp_lattice` inflation tests, the riak_test combinator results) and by the
`crdt_statem_eqc` convergence model re-run with `hypothesis` (tests/test_oracle_*.py).
Behaviour on non-canonical lists (unsorted / duplicated keys) follows the OTP 17
clauses restated in `otp.py` and is *parity unpinned* beyond those tests.

Modules:
  terms      Erlang term model and term order (Appendix A).
  otp        orddict / ordsets / lists / sets clauses.
  orset      lasp_orset (src/lasp_orset.erl).
  gset       lasp_gset  (src/lasp_gset.erl).
  lattice    lasp_lattice orset / gset / gcounter clauses (src/lasp_lattice.erl).
  core       lasp_core bind / update / read / combinators (src/lasp_core.erl).
  columnar   ctypes wrapper over the C restatement (oracle/laspj_oracle.c):
             synthetic generator, faithful orddict merge, columnar join & predicates.
"""
