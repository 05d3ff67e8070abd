"""CPU oracle for the scenario-batched PH iterate — TEST INFRASTRUCTURE ONLY.

This package is a plain-numpy restatement of the reference's PH path
(garg02/mpi-sppy ``mpisppy/phbase.py``, ``mpisppy/spopt.py``,
``mpisppy/spbase.py``) with scipy's bundled HiGHS 1.8.0 standing in for the
external LP/QP solver the reference reaches through Pyomo
(``spopt.py:166-168``), followed by an active-set KKT polish.

Rules (see DESIGN.md "Oracle"):
  * Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
    ``cpu_baseline`` leg may import it, and only as the checker / the CPU
    baseline — never as the thing measured or shipped.  The product package
    (``mpi-sppy_amd/``) never imports it and fails loudly if its HIP library
    is missing.
  * Parity is PINNED: ``tests/test_oracle_golden.py`` checks this oracle against
    the reference's own committed golden vectors (w/xbar CSV fixture,
    docs-farmer PH trajectory, farmer-30 trivial bound, converged farmer
    nonants, aircond EF objective).
"""
