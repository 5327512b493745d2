"""CPU oracle for the MI355X PH hot path -- TEST INFRASTRUCTURE ONLY.

This package restates, on the CPU with numpy/scipy, the algorithm of the
reference's progressive-hedging hot path (mpi-sppy @ /root/reference):

* the scenario instance generators of the reference examples
  (``examples/farmer/farmer.py``, ``doc/src/examples.rst`` textbook farmer,
  ``examples/hydro/hydro.py``),
* the PH control flow of ``mpisppy/phbase.py`` (Iter0, iterk_loop,
  Compute_Xbar, Update_W, convergence_diff, Eobjective, Ebound,
  post_solve_bound) and the Lagrangian spoke's bound
  (``mpisppy/cylinders/lagrangian_bounder.py``),
* the per-scenario subproblem solve, which the reference delegates to a
  commercial solver through Pyomo.  Here HiGHS (bundled with scipy 1.15.3,
  HiGHS 1.8.0) solves the LPs exactly (simplex) and the PH prox-QPs are
  polished to machine precision by an active-set KKT solve (``solve.py``).

Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import this package, and only as the checker / CPU
baseline.  The product path (``mpi-sppy_amd/mpisppy_amd``) never imports it.

Pinning: ``tests/test_oracle.py`` checks this oracle against every golden
value the reference itself publishes for this path (doc farmer LP/EF/PH
values, ``doc/src/examples.rst:113,241-245,323-334``; hydro PH trivial bound
and unweighted Eobjective, ``mpisppy/tests/test_ef_ph.py:541-559``).
"""
