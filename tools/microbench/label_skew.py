import torch, heat_amd as ht
from heat_amd import ops
ht.use_device("gpu")
ht.random.seed(1234)
x = ht.random.randn(12_500_000, 64, split=0)
km = ht.cluster.KMeans(n_clusters=1024, init="random", max_iter=1, tol=None, random_state=42)
km.step(x)
for it in range(3):
    lab, _ = ops.kmeans_assign(x.larray, km.cluster_centers_.larray)
    bc = torch.bincount(lab.long(), minlength=1024)
    print("iter", it, "max", bc.max().item(), "nonzero", (bc > 0).sum().item(), "top8 share", bc.sort(descending=True).values[:8].sum().item() / 12.5e6)
    km.step(x)
