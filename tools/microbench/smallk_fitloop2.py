"""Bisect the 580 / 710 us alternation of the fused small-k pass inside the Lloyd loop."""
import json

import torch

from heat_amd import ops

g = torch.Generator(device="cuda").manual_seed(0)
X = torch.randn(12_500_000, 64, device="cuda", generator=g)
C0 = X[:8].clone()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(41)]


def run(name, body):
    C = C0.clone()
    for _ in range(3):
        C = body(C)
    torch.cuda.synchronize()
    ev[0].record()
    for i in range(40):
        C = body(C)
        ev[i + 1].record()
    torch.cuda.synchronize()
    ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(40)]
    print(json.dumps({name: [round(x, 3) for x in ms[-12:]], "mean": round(sum(ms[-20:]) / 20, 4)}), flush=True)


def step_finalize(C):
    lab, s, c = ops.kmeans_step_small(X, C)
    newC, _ = ops.kmeans_finalize(None, C, sums=s, counts=c)
    return newC


def step_finalize_fixed(C):
    lab, s, c = ops.kmeans_step_small(X, C)
    ops.kmeans_finalize(None, C, sums=s, counts=c)
    return C


def step_torch_update(C):
    lab, s, c = ops.kmeans_step_small(X, C)
    return torch.where(c.unsqueeze(1) > 0, s / c.clamp(min=1).unsqueeze(1), C)


def step_copy_back(C):
    lab, s, c = ops.kmeans_step_small(X, C)
    newC, _ = ops.kmeans_finalize(None, C, sums=s, counts=c)
    C.copy_(newC)
    return C


tiny = torch.zeros(64, device="cuda")


def step_tiny(C):
    ops.kmeans_step_small(X, C)
    tiny.fill_(1.0)
    return C


def step_tiny2(C):
    ops.kmeans_step_small(X, C)
    tiny.fill_(1.0)
    tiny.fill_(2.0)
    return C


run("lloyd_fused_newC", lambda C: ops.kmeans_lloyd_small(X, C)[1])
run("step_only_fixedC", lambda C: (ops.kmeans_step_small(X, C), C)[1])
run("step_plus_1_fill", step_tiny)
run("step_plus_2_fills", step_tiny2)
run("step_finalize_newC", step_finalize)
run("step_finalize_fixedC", step_finalize_fixed)
run("step_torch_update_newC", step_torch_update)
run("step_finalize_copy_into_C", step_copy_back)
run("lloyd_fused_newC_last", lambda C: ops.kmeans_lloyd_small(X, C)[1])   # again, clocks warm
