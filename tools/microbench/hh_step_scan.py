"""Per-step time of the Householder panel (hh_colsums + 32 hh_step launches on a compact m x 32
fp32 panel) over m: the intercept is the fixed cost per launch (start-up S gather, fixed-order
block-sum tail, launch gap), the slope the streaming cost. One JSON line per m."""
import ctypes
import json
import time

import torch

from heat_amd import ops
from heat_amd.ops import kernels as K


def main():
    L = ops.lib()
    nb, slen = L.ha_hh_nb(), L.ha_hh_slen()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    tau = torch.empty(nb, device="cuda")
    for m in (2048, 65536, 250_000, 625_000, 1_250_000, 2_500_000):
        P = torch.randn(m, nb, device="cuda")
        hpart = torch.empty(max(1, L.ha_hh_part_len(m)), dtype=torch.float64, device="cuda")
        hcnt = torch.zeros(L.ha_hh_counters(), dtype=torch.int32, device="cuda")
        S = torch.zeros((nb + 1, slen), dtype=torch.float64, device="cuda")

        def panel():
            S.zero_()
            K.check(L.ha_hh_colsums(K._ptr(P), 0, m, nb, 0, 0, nb, 0, K._ptr(S[0]), K._ptr(hpart), K._ptr(hcnt), st),
                    "colsums")
            for j in range(nb):
                last = j + 1 == nb
                K.check(L.ha_hh_step(K._ptr(P), 0, m, nb, 0, 0, 0, nb, j, K._ptr(S[j]),
                                     K._ptr(None) if last else K._ptr(S[j + 1]), K._ptr(tau), K._ptr(None),
                                     K._ptr(hpart), K._ptr(hcnt), st), "step")

        panel()
        torch.cuda.synchronize()
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            panel()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / reps * 1e3
        print(json.dumps({"m": m, "panel_ms": ms, "us_per_launch": ms * 1e3 / (nb + 1),
                          "panel_bytes_GB": m * nb * 4 / 1e9}), flush=True)


if __name__ == "__main__":
    main()
