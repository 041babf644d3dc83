"""Oracle NLP restatement: structural pins + derivative checks.

Pins: R/test/obca.ipynb:396,401-403 -- N=66, 8 quads, body+pruner, time-opt on
-> 8978 variables / 2447 equality / 2112 inequality constraints.
"""
import numpy as np
import pytest

from headland_trajectory_planning_amd import synth
from oracle.nlp import ObcaNLP


def _inst(N, M, imp, pid=3, **kw):
    return synth.make_instance(pid, N=N, M=M, implement=imp, **kw)


def test_notebook_structure_pin():
    nlp = ObcaNLP(_inst(66, 8, "pruner"))
    assert nlp.counts() == {"n_var": 8978, "n_eq": 2447, "n_ineq": 2112}


@pytest.mark.parametrize("cfg,expect", [("A", 962), ("B", 4482), ("C", 8322), ("E", 32002)])
def test_config_sizes(cfg, expect):
    _, N, M, imp = synth.CONFIGS[cfg]
    assert ObcaNLP(_inst(N, M, imp)).n == expect


def _perturbed(nlp, seed):
    rng = np.random.default_rng(seed)
    x = nlp.x0 + 0.05 * rng.standard_normal(nlp.n)
    x[nlp.oU:nlp.oMU] = 0.3 * rng.standard_normal(nlp.oMU - nlp.oU)
    if nlp.topt:
        x[nlp.oTAU:nlp.oS] = rng.uniform(0.5, 1.0, nlp.oS - nlp.oTAU)
    x[nlp.oS:] = 0.1 * rng.standard_normal(5)
    return x


@pytest.mark.parametrize("topt", [True, False])
def test_derivatives_fd(topt):
    W = np.diag([10.0, 0.1 if topt else 0.0])
    nlp = ObcaNLP(_inst(6, 2, "mower", W=W))
    x = _perturbed(nlp, 1)
    y = np.random.default_rng(2).standard_normal(nlp.m)
    eps = 1e-6
    g0 = nlp.grad_f(x)
    J = nlp.jac(x).toarray()
    H = nlp.hess(x, y, 0.7).toarray()
    assert np.allclose(H, H.T, atol=1e-12)
    for j in range(nlp.n):
        e = np.zeros(nlp.n)
        e[j] = eps
        fd = (nlp.f(x + e) - nlp.f(x - e)) / (2 * eps)
        assert abs(fd - g0[j]) < 1e-6 * max(1, abs(g0[j])), j
        col = (nlp.cons(x + e) - nlp.cons(x - e)) / (2 * eps)
        assert np.allclose(col, J[:, j], atol=1e-6), j
        hcol = (0.7 * (nlp.grad_f(x + e) - nlp.grad_f(x - e)) + (nlp.jac(x + e) - nlp.jac(x - e)).T @ y) / (2 * eps)
        assert np.allclose(hcol, H[:, j], atol=2e-5), j
