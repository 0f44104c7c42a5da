"""torch.quantile on the GPU vs NumPy for a short fp64 vector and several q (probe for the
percentile oracle check)."""
import numpy as np
import torch

rng = np.random.default_rng(12)
a = rng.standard_normal(31)
qs = [0.05, 0.5, 0.95]
t = torch.tensor(a, device="cuda")
for dt in (torch.float64, torch.float32):
    for meth in ("linear", "lower", "higher", "midpoint", "nearest"):
        g = torch.quantile(t.to(dt), torch.tensor(qs, dtype=dt, device="cuda"), interpolation=meth).cpu().numpy()
        c = torch.quantile(t.cpu().to(dt), torch.tensor(qs, dtype=dt), interpolation=meth).numpy()
        print(dt, meth, "gpu", g, "cpu", c, "numpy", np.percentile(a, [100 * q for q in qs], method=meth))
s = torch.sort(t).values.cpu().numpy()
print("sort ok", np.array_equal(s, np.sort(a)))
for q in qs:
    print(q, torch.quantile(t, q).item(), np.quantile(a, q))
