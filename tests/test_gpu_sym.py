"""Symmetric-pair phi pass (k_phi_sym, SVGD_PHI_SYM=1) against the oracle.  GPU only.

Each unordered pair of particle blocks is visited once and its kernel values
feed both the row sums and the column sums; the result must match the oracle
within the same tolerance as the row-stream path (max-abs <= 1e-10).  Sizes
cover one block (n <= 768), ragged last blocks, odd and even block counts and
the full-matrix scale.
"""
import numpy as np
import pytest

import svgdcpp_amd as S
from svgdcpp_amd import _capi as C

pytestmark = pytest.mark.gpu

PHI_TOL = 1e-10


@pytest.fixture(autouse=True)
def _sym_on(monkeypatch):
    monkeypatch.setenv("SVGD_PHI_SYM", "1")


@pytest.mark.parametrize("n,d", [(10, 2), (700, 3), (769, 2), (1536, 8), (1600, 1), (2400, 5),
                                 (4096, 2), (5000, 8), (3000, 16)])
def test_sym_phi_matches_oracle(oracle, n, d):
    X = oracle.splitmix((n, d), 2.0, 300 + n + d)
    G = oracle.splitmix((n, d), 1.0, 400 + n + d)
    a = 0.37 / d
    c = S.Context(d, n)
    c.set_particles(X)
    ph = c.phi(G, a)
    assert np.all(np.isfinite(ph))
    ref = oracle.phi(X, G, a)
    assert np.max(np.abs(ph - ref)) <= PHI_TOL


def test_sym_phi_matrix_scale(oracle):
    n, d = 2000, 4
    X = oracle.splitmix((n, d), 2.0, 77)
    G = oracle.splitmix((n, d), 1.0, 78)
    B = oracle.splitmix((d, d), 0.3, 79)
    M = B @ B.T + 0.2 * np.eye(d)
    c = S.Context(d, n)
    c.set_particles(X)
    c.set_scale_matrix(M)
    ph = c.phi(G, 0.0)
    ref = oracle.phi_matrix(X, G, M)
    assert np.max(np.abs(ph - ref)) <= PHI_TOL


def test_sym_steps_match_row_path(oracle, monkeypatch):
    n, d = 4096, 2
    X0 = oracle.splitmix((n, d), 3.0, 5)
    mus = oracle.splitmix((2, d), 3.0, 6)
    model = S.GaussianSum(mus, np.stack([np.eye(d)] * 2))
    out = {}
    for sym in ("1", "0"):
        monkeypatch.setenv("SVGD_PHI_SYM", sym)
        c = S.Context(d, n)
        c.set_particles(X0)
        c.set_optimizer(C.SVGD_OPT_ADAM, 0.1, 0.9, 0.999)
        for _ in range(5):
            c.step_with_model(model)
        out[sym] = c.get_particles()
    assert np.all(np.isfinite(out["1"]))
    assert np.max(np.abs(out["1"] - out["0"])) <= 1e-9
