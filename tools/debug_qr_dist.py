"""Per-split report of check_linalg's QR cases (run through tools/run_check_gpu.py)."""
import numpy as np

import heat_amd as ht


def check_qr_report():
    rng = np.random.default_rng(6)
    rng.standard_normal((9, 7)), rng.standard_normal((7, 5)), rng.standard_normal(7)
    tall = rng.standard_normal((40, 6))
    for mode in (None, "reduced", "complete"):
        for s in (None, 0, 1):
            q, r = ht.linalg.qr(ht.array(tall, split=s), mode=mode)
            qn, rn = q.numpy(), r.numpy()
            err = np.abs(qn @ rn - tall).max()
            orth = np.abs(qn.T @ qn - np.eye(qn.shape[1])).max()
            if ht.MPI_WORLD.rank == 0:
                print("mode", mode, "split", s, "q", qn.shape, "r", rn.shape, "rec", err, "orth", orth,
                      "r00", rn[0, :3], "rtail", np.abs(rn[6:]).max() if rn.shape[0] > 6 else None, flush=True)
