"""
Shared pieces of the ImageNet-style examples (reference ``examples/nn/imagenet.py`` and
``imagenet-DASO.py``): a ResNet built from torch.nn (torchvision is not installed here), a
synthetic ImageNet-shaped dataset (no network for the real one), top-k accuracy, averaged
metrics and checkpointing.

The synthetic images are class prototypes plus noise, so the loss and accuracy actually move and
the training loop can be checked end to end; ``--image-size 224 --classes 1000`` gives the real
ImageNet tensor shapes.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import time

import torch
import torch.nn as nn
import torch.nn.functional as F

import heat_amd as ht


class BasicBlock(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.c1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.b1 = nn.BatchNorm2d(cout)
        self.c2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.b2 = nn.BatchNorm2d(cout)
        self.short = None
        if stride != 1 or cin != cout:
            self.short = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        y = F.relu(self.b1(self.c1(x)))
        y = self.b2(self.c2(y))
        return F.relu(y + (x if self.short is None else self.short(x)))


class ResNet(nn.Module):
    """ResNet-18/34 layout (``layers`` blocks per stage) with a configurable base width."""

    def __init__(self, layers=(2, 2, 2, 2), width=64, classes=1000):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, width, 7, 2, 3, bias=False), nn.BatchNorm2d(width), nn.ReLU(),
                                  nn.MaxPool2d(3, 2, 1))
        blocks, cin = [], width
        for i, n in enumerate(layers):
            cout = width * (2 ** i)
            for j in range(n):
                blocks.append(BasicBlock(cin, cout, 2 if (j == 0 and i > 0) else 1))
                cin = cout
        self.body = nn.Sequential(*blocks)
        self.fc = nn.Linear(cin, classes)

    def forward(self, x):
        x = self.body(self.stem(x))
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))


class SyntheticImageNet:
    """Per-rank shard of a class-prototype image set, generated batch by batch on the device
    (deterministic per (rank, epoch, batch))."""

    def __init__(self, samples, image_size, classes, batch_size, comm, device, seed=0):
        self.n = samples // comm.size
        self.bs = batch_size
        self.size = image_size
        self.classes = classes
        self.rank = comm.rank
        self.dev = device
        g = torch.Generator().manual_seed(seed)
        self.protos = (torch.randn(classes, 3, 8, 8, generator=g) * 1.5).to(device)
        self.epoch = 0

    def __len__(self):
        return max(1, self.n // self.bs)

    def __iter__(self):
        for b in range(len(self)):
            g = torch.Generator(device="cpu").manual_seed(hash((self.rank, self.epoch, b)) & 0x7FFFFFFF)
            y = torch.randint(0, self.classes, (self.bs,), generator=g).to(self.dev)
            base = F.interpolate(self.protos[y], size=self.size, mode="bilinear", align_corners=False)
            noise = torch.randn(self.bs, 3, self.size, self.size, generator=g).to(self.dev)
            yield base + noise, y
        self.epoch += 1


def accuracy(output, target, topk=(1, 5)):
    k = min(max(topk), output.shape[1])
    _, pred = output.topk(k, 1, True, True)
    correct = pred.t().eq(target.view(1, -1))
    return [correct[: min(t, k)].reshape(-1).float().sum() * (100.0 / target.shape[0]) for t in topk]


def reduce_mean(value: float, comm) -> float:
    return comm.allreduce(float(value), ht.MPI.SUM) / comm.size


def lr_warmup(optimizer, base_lr, epoch, batch, batches, warmup_epochs=2):
    """Linear warm-up over the first epochs (reference ``lr_warmup``)."""
    if epoch < warmup_epochs:
        frac = (epoch * batches + batch + 1) / (warmup_epochs * batches)
        for g in optimizer.param_groups:
            g["lr"] = base_lr * frac


def save_checkpoint(path, model, optimizer, epoch, comm):
    if comm.rank == 0:
        torch.save({"epoch": epoch, "state_dict": model.state_dict(), "optimizer": optimizer.state_dict()}, path)
    comm.Barrier()


def load_checkpoint(path, model, optimizer, device):
    ck = torch.load(path, map_location=device, weights_only=True)
    model.load_state_dict(ck["state_dict"])
    optimizer.load_state_dict(ck["optimizer"])
    return int(ck["epoch"]) + 1


def parser(desc):
    p = argparse.ArgumentParser(description=desc)
    p.add_argument("--epochs", type=int, default=4)
    p.add_argument("--batch-size", type=int, default=64, help="per-rank batch")
    p.add_argument("--samples", type=int, default=8192, help="images per epoch over all ranks")
    p.add_argument("--image-size", type=int, default=64)
    p.add_argument("--classes", type=int, default=100)
    p.add_argument("--width", type=int, default=32, help="ResNet base width (64 = ResNet-18)")
    p.add_argument("--layers", type=str, default="2,2,2,2")
    p.add_argument("--lr", type=float, default=0.05)
    p.add_argument("--momentum", type=float, default=0.9)
    p.add_argument("--weight-decay", type=float, default=1e-4)
    p.add_argument("--bf16", action="store_true", help="bf16 autocast on the device")
    p.add_argument("--checkpoint", type=str, default="")
    p.add_argument("--resume", action="store_true")
    p.add_argument("--print-freq", type=int, default=10)
    return p


def device():
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


def report(comm, name, args, t_train, images):
    if comm.rank == 0:
        print(json.dumps({"example": name, "ranks": comm.size, "epochs": args.epochs,
                          "images_per_s": round(images / max(t_train, 1e-9), 1)}), flush=True)


def print0(comm, *a):
    if comm.rank == 0:
        print(*a, flush=True)


def autocast(args, dev):
    if args.bf16 and dev.type == "cuda":
        return torch.autocast("cuda", dtype=torch.bfloat16)
    return torch.autocast("cpu", enabled=False)


__all__ = ["ResNet", "SyntheticImageNet", "accuracy", "reduce_mean", "lr_warmup", "save_checkpoint",
           "load_checkpoint", "parser", "device", "report", "print0", "autocast", "math", "os", "time"]
