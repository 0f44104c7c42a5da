"""Can RCCL run a world of 2 ranks that share ONE GPU (torch ProcessGroupNCCL and the native
communicator)? Launch with `python -m torch.distributed.run --nproc-per-node 2 --master-addr
127.0.0.1 ...`. Prints one JSON line per rank and step; a rank that RCCL refuses prints the error."""
import json
import os
import sys
import time

import torch
import torch.distributed as dist


def main():
    rank = int(os.environ["RANK"])
    ws = int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    out = {"rank": rank, "ws": ws}
    try:
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
        x = torch.full((1 << 20,), float(rank + 1), device="cuda")
        dist.all_reduce(x)
        torch.cuda.synchronize()
        out["torch_allreduce_ok"] = bool((x == ws * (ws + 1) / 2).all())
        g = [torch.empty(4, device="cuda") for _ in range(ws)]
        dist.all_gather(g, torch.full((4,), float(rank), device="cuda"))
        out["torch_allgather_ok"] = all(bool((t == i).all()) for i, t in enumerate(g))
    except Exception as e:  # noqa: BLE001 - the probe reports whatever RCCL says
        out["torch_error"] = repr(e)[:400]
        print(json.dumps(out), flush=True)
        return 1
    try:
        import heat_amd as ht
        from heat_amd.parallel import native_comm

        nc = native_comm.NativeComm(ht.MPI_WORLD)
        y = torch.full((1000,), float(rank + 1), device="cuda")
        nc.allreduce_(y, "sum")
        torch.cuda.synchronize()
        out["native_allreduce_ok"] = bool((y == ws * (ws + 1) / 2).all())
        t0 = time.perf_counter()
        for _ in range(100):
            nc.allreduce_(y, "sum")
        torch.cuda.synchronize()
        out["native_allreduce_us"] = (time.perf_counter() - t0) * 1e4
        nc.close()
    except Exception as e:  # noqa: BLE001
        out["native_error"] = repr(e)[:400]
    print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
