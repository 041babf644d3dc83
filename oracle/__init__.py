"""CPU oracle for the headland-turn hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product package
(`headland_trajectory_planning_amd`) imports, links or executes this
directory.  Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s
`cpu_baseline` leg use it, and only as the checker / timed CPU baseline.

Contents
--------
nlp.py        numpy restatement of the OBCA NLP built by
              R/obca_py/optimizer.py:228-473 (x0, bounds, f, g, J, Hessian).
halfspace.py  restatement of pypoman.compute_polytope_halfspaces (cddlib)
              as called at R/obca_py/optimizer.py:184-186,198-200.
ipm.py        restatement of the published IPOPT algorithm (Waechter &
              Biegler 2006, IPOPT 3.14 defaults) that R/obca_py/optimizer.py:489
              calls through CasADi.  Dense LDL^T (Bunch-Kaufman) KKT solves.
reeds_shepp.py  restatement of R/path_planner/utils/reeds_shepp.py.

Parity status: the NLP restatement is pinned by the notebook's structural
counts (R/test/obca.ipynb:401-403).  The IPOPT restatement has no reference
output to pin against in this container (casadi is absent), so state-trajectory
parity *versus CasADi* is "parity unpinned"; the HIP solver is checked against
this restatement and by KKT residuals of the NLP restatement.
"""
