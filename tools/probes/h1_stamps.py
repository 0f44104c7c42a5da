"""Phase timing of the kNN screening kernel (h1_topk) from a measurement build with s_memtime
stamps (tools/probes/knn_h1_stamps.so, built with -DHEAT_H1_STAMPS): for the 32 waves of
workgroups 0..7 and 64 steady-state chunks, cycles spent per phase of a chunk iteration:
  0->1 waiting for this wave's DMA (vmcnt), 1->2 the chunk barrier, 2->3 tile 0 (MFMAs +
  epilogue of the previous tile), 3->4 its selection, 4->5 tile 1, 5->6 its selection,
  6->next 0 loop overhead."""
import ctypes
import json
import os
import sys

import torch

from heat_amd import ops
from heat_amd.ops import kernels as K

so = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "knn_h1_stamps.so"))
P, I32, I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
so.ha_h1_topk.argtypes = [P, P, I64, I32, P, I32, I64, P, I32, I32, P, P, P, P]
so.ha_h1_topk.restype = I32
L = ops.lib()
g = torch.Generator(device="cuda").manual_seed(0)
n, f, k, kp = int(os.environ.get("H1_N", "1000000")), 128, 8, 32
x = torch.randn(n, f, device="cuda", generator=g)
pk = K.kmeans_pack_points(x)
ws = torch.empty(L.ha_h1_workspace_bytes(n, f), dtype=torch.uint8, device="cuda")
dist = torch.empty((n, kp), device="cuda")
idx = torch.zeros((n, kp), dtype=torch.int32, device="cuda")
cert = torch.empty(n, dtype=torch.uint8, device="cuda")
st = ctypes.c_void_p(ops.stream_ptr(x.device))
for rep in range(2):
    rc = so.ha_h1_topk(K._ptr(pk.planes), K._ptr(pk.sx), n, f, K._ptr(x), n, x.stride(0), K._ptr(ws), k, kp,
                       K._ptr(dist), K._ptr(idx), K._ptr(cert), st)
    assert rc == 0, rc
    torch.cuda.synchronize()
t = idx.reshape(-1)[: 32 * 64 * 8].view(torch.int32).cpu().numpy().astype("int64") & 0xFFFFFFFF
t = t.reshape(32, 64, 8)
import numpy as np

d = np.diff(t[:, :, :7], axis=2) % (1 << 32)           # phases 0->1 .. 5->6
loop = (t[:, 1:, 0] - t[:, :-1, 6]) % (1 << 32)        # 6 -> next chunk's 0
names = ["dma_wait", "barrier", "tile0", "select0", "tile1", "select1"]
res = {nm: float(np.median(d[:, :, i])) for i, nm in enumerate(names)}
res.update({nm + "_mean": float(d[:, :, i].mean()) for i, nm in enumerate(names)})
res["loop"] = float(np.median(loop))
res["chunk_total_mean"] = float(((t[:, 1:, 0] - t[:, :-1, 0]) % (1 << 32)).mean())
print(json.dumps(res), flush=True)
