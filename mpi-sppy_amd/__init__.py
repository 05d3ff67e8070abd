"""mpisppy_amd — MI355X-native batched Progressive Hedging engine.

Drop-in for the scenario-batched PH iterate of garg02/mpi-sppy: the same
PHBase / PH API (options dict, scenario_creator callbacks, extension and
converger hooks, hub ``spcomm`` contract), with the per-scenario external
solver loop and the per-node MPI reductions replaced by hand-written gfx950
HIP kernels (``csrc/``, C ABI in ``include/phx.h``) and RCCL collectives.

Import path: the package directory is ``mpi-sppy_amd/``; it is importable as
``mpisppy_amd`` via the loader shim ``mpisppy_amd.py`` at the repository root.
"""
__version__ = "0.1.0"
