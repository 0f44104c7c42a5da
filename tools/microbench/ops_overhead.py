"""Framework overhead on one GPU: common DNDarray operations against the plain torch op on the same
local tensor (world of one, so the difference is the framework's own work: sanitation, result
wrapping, extra copies, host syncs). One JSON line per op: ht_ms, torch_ms, ratio."""
import json
import time

import torch

import heat_amd as ht


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    ht.use_device("gpu")
    ht.random.seed(3)
    n = 1 << 26
    a = ht.random.rand(n, split=0)
    b = ht.random.rand(n, split=0)
    M = ht.random.rand(8192, 8192, split=0)
    ta, tb, tM = a.larray, b.larray, M.larray
    idx = ht.array(torch.randint(0, n, (1 << 20,), device="cuda"), split=0)
    mask = a > 0.5
    cases = {
        "add": (lambda: a + b, lambda: ta + tb),
        "mul_scalar": (lambda: a * 2.0, lambda: ta * 2.0),
        "exp": (lambda: ht.exp(a), lambda: torch.exp(ta)),
        "sum": (lambda: ht.sum(a), lambda: torch.sum(ta)),
        "mean": (lambda: ht.mean(a), lambda: torch.mean(ta)),
        "max": (lambda: ht.max(a), lambda: torch.max(ta)),
        "argmax": (lambda: ht.argmax(a), lambda: torch.argmax(ta)),
        "sum_axis0_2d": (lambda: ht.sum(M, axis=0), lambda: torch.sum(tM, 0)),
        "sum_axis1_2d": (lambda: ht.sum(M, axis=1), lambda: torch.sum(tM, 1)),
        "where": (lambda: ht.where(mask, a, b), lambda: torch.where(mask.larray, ta, tb)),
        "getitem_slice": (lambda: a[1000:n - 1000], lambda: ta[1000:n - 1000]),
        "getitem_bool": (lambda: a[mask], lambda: ta[mask.larray]),
        "getitem_int": (lambda: a[idx], lambda: ta[idx.larray]),
        "sort": (lambda: ht.sort(a), lambda: torch.sort(ta)),
        "cumsum": (lambda: ht.cumsum(a, 0), lambda: torch.cumsum(ta, 0)),
        "transpose_copy": (lambda: M.T.copy(), lambda: tM.T.contiguous()),
        "reshape": (lambda: ht.reshape(M, (4096, 16384)), lambda: tM.reshape(4096, 16384)),
        "concatenate": (lambda: ht.concatenate([a, b]), lambda: torch.cat([ta, tb])),
        "astype_f64": (lambda: a.astype(ht.float64), lambda: ta.double()),
        "matmul_2k": (lambda: ht.matmul(M[:2048, :2048], M[:2048, :2048]),
                      lambda: tM[:2048, :2048] @ tM[:2048, :2048]),
        "abs": (lambda: ht.abs(a - 0.5), lambda: torch.abs(ta - 0.5)),
        "clip": (lambda: ht.clip(a, 0.2, 0.8), lambda: torch.clamp(ta, 0.2, 0.8)),
        "percentile": (lambda: ht.percentile(a, 50.0), lambda: torch.quantile(ta[: 1 << 24], 0.5)),
    }
    for name, (fh, ft) in cases.items():
        try:
            th = timed(fh)
            tt = timed(ft)
            print(json.dumps({"op": name, "ht_ms": round(th, 4), "torch_ms": round(tt, 4),
                              "ratio": round(th / tt, 2)}), flush=True)
        except Exception as e:  # noqa: BLE001 - report and continue
            print(json.dumps({"op": name, "error": repr(e)[:200]}), flush=True)


if __name__ == "__main__":
    main()
