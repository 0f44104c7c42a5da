"""Parity with ``heat/core/linalg/tests/test_qr.py``: QR of wide, square and tall matrices on both
splits and both tile counts (A = QR, Q orthogonal), R-only mode, and the errors."""
import numpy as np
import torch

import heat_amd as ht

from ._util import close, raises, rng


def _check(st, tol):
    m = st.shape[0]
    for t in (1, 2):
        for sp in (0, 1):
            a = ht.array(st, split=sp)
            qr = a.qr(tiles_per_proc=t)
            close(qr.Q @ qr.R, st, rtol=tol, atol=tol)
            close(qr.Q.T @ qr.Q, np.eye(qr.Q.shape[1]), rtol=tol, atol=tol)
            if qr.Q.shape[1] == m:
                close(qr.Q @ qr.Q.T, np.eye(m), rtol=tol, atol=tol)
            r = qr.R.numpy()
            assert np.allclose(np.tril(r, -1), 0, atol=tol)


def test_qr():
    _check(rng(1).standard_normal((20, 40)).astype(np.float32), 1e-4)
    _check(rng(2).standard_normal((40, 40)).astype(np.float32), 1e-4)
    _check(rng(3).standard_normal((40, 20)), 1e-9)
    st2 = rng(3).standard_normal((40, 20))
    for sp in (0, 1):
        r0 = ht.qr(ht.array(st2, split=sp), calc_q=False, overwrite_a=True)
        assert r0.Q is None
        # R (complete, m x n for small m like the reference) is unique up to row signs
        close(np.abs(r0.R.numpy()), np.abs(np.linalg.qr(st2, mode="complete")[1]), rtol=1e-8, atol=1e-8)
    raises(TypeError, ht.qr, "asdf")
    raises(TypeError, ht.qr, ht.array(st2), tiles_per_proc="ls")
    raises(TypeError, ht.qr, ht.array(st2), tiles_per_proc=1, calc_q=30)
    raises(TypeError, ht.qr, ht.array(st2), tiles_per_proc=1, overwrite_a=30)
    raises(ValueError, ht.qr, ht.array(st2), tiles_per_proc=torch.tensor([1, 2, 3]))
    raises(ValueError, ht.qr, ht.zeros((3, 4, 5)))


def test_qr_sp0_ext():
    m, n = 203, 17
    a = rng(4).standard_normal((m, n))
    for t in (1, 2, 3):
        qr = ht.qr(ht.array(a, split=0), tiles_per_proc=t)
        close(qr.Q @ qr.R, a, rtol=1e-9, atol=1e-9)
        close(qr.Q.T @ qr.Q, np.eye(qr.Q.shape[1]), atol=1e-9)


def test_qr_sp1_ext():
    m, n = 17, 203
    a = rng(5).standard_normal((m, n))
    for t in (1, 2, 3):
        qr = ht.qr(ht.array(a, split=1), tiles_per_proc=t)
        close(qr.Q @ qr.R, a, rtol=1e-9, atol=1e-9)
        close(qr.Q.T @ qr.Q, np.eye(qr.Q.shape[1]), atol=1e-9)
