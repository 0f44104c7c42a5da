"""Parity with ``heat/graph/tests/test_laplacian.py``: every Laplacian variant (weighted / simple /
eNeighbour with both threshold keys) against a NumPy construction, and the errors."""
import numpy as np
from scipy.spatial.distance import cdist as sp_cdist

import heat_amd as ht

from ._util import close, raises


def _np_laplacian(S, definition="norm_sym", weighted=True, mode="fully_connected", key="upper", value=1.0):
    A = S.copy()
    if mode == "eNeighbour":
        keep = (A < value) if key == "upper" else (A > value)
        A = np.where(keep, A if weighted else 1.0, 0.0)
    np.fill_diagonal(A, 0.0)
    d = A.sum(1)
    if definition == "simple":
        return np.diag(d) - A
    inv = np.where(d > 0, 1.0 / np.sqrt(np.where(d > 0, d, 1.0)), 0.0)
    return np.eye(len(d)) - inv[:, None] * A * inv[None, :]


def test_laplacian():
    size, rank = ht.MPI_WORLD.size, ht.MPI_WORLD.rank
    X = ht.ones((size * 2, 4), split=0)
    X.larray[0, :] *= rank
    X.larray[1, :] *= rank + 0.5
    xn = X.numpy().astype(np.float64)
    D = sp_cdist(xn, xn)
    cd = lambda x: ht.spatial.cdist(x, quadratic_expansion=True)  # noqa: E731
    cases = [({}, dict()), ({"weighted": False}, dict(weighted=False)), ({"definition": "simple"}, dict(definition="simple")),
             ({"mode": "eNeighbour"}, dict(mode="eNeighbour")),
             ({"mode": "eNeighbour", "threshold_key": "lower", "threshold_value": 3.0},
              dict(mode="eNeighbour", key="lower", value=3.0))]
    for kw, npkw in cases:
        res = ht.graph.Laplacian(cd, **kw).construct(X)
        assert isinstance(res, ht.DNDarray) and res.shape == (size * 2, size * 2) and res.split == 0
        close(res, _np_laplacian(D, **npkw), atol=2e-3)
    res = ht.graph.Laplacian(lambda x: ht.spatial.rbf(x, sigma=1.0, quadratic_expansion=True)).construct(X)
    assert res.shape == (size * 2, size * 2) and res.split == 0
    close(res, _np_laplacian(np.exp(-D ** 2 / 2.0)), atol=2e-3)
    raises(ValueError, ht.graph.Laplacian, cd, threshold_key="both")
    raises(NotImplementedError, ht.graph.Laplacian, cd, mode="kNN")
    raises(NotImplementedError, ht.graph.Laplacian, cd, definition="norm_rw")
