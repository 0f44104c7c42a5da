"""
ImageNet-style training with DASO (reference ``examples/nn/imagenet-DASO.py``): the model is
wrapped in ``ht.nn.DataParallelMultiGPU`` (node-local DDP over RCCL/xGMI) and optimised by
``ht.optim.DASO`` - node-local gradient averaging every step, global parameter averaging across
nodes only every few batches with bf16 payloads, the skip rate adapted from the epoch loss
(warm-up, cycling, cool-down). Synthetic ImageNet-shaped data (no network here); checkpoint /
resume; ReduceLROnPlateau on the globally averaged loss.

    python -m heat_amd.run -n 8 examples/nn/imagenet-DASO.py --epochs 8 --image-size 224 \\
        --classes 1000 --width 64 --bf16
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

import heat_amd as ht  # noqa: E402
from imagenet_common import (ResNet, SyntheticImageNet, accuracy, autocast, device, load_checkpoint,  # noqa: E402
                             lr_warmup, parser, print0, reduce_mean, report, save_checkpoint)


def main():
    p = parser("ImageNet-style training with DASO")
    p.add_argument("--max-global-skips", type=int, default=4)
    p.add_argument("--warmup-epochs", type=int, default=1)
    p.add_argument("--cooldown-epochs", type=int, default=1)
    args = p.parse_args()
    comm = ht.MPI_WORLD
    dev = device()
    torch.manual_seed(0)
    layers = tuple(int(v) for v in args.layers.split(","))
    model = ResNet(layers, args.width, args.classes).to(dev)
    optimizer = torch.optim.SGD(model.parameters(), args.lr, momentum=args.momentum, weight_decay=args.weight_decay)
    daso = ht.optim.DASO(local_optimizer=optimizer, total_epochs=args.epochs, comm=comm,
                         warmup_epochs=args.warmup_epochs, cooldown_epochs=args.cooldown_epochs,
                         max_global_skips=args.max_global_skips, stability_level=0.05)
    scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(optimizer, factor=0.5, patience=5, threshold=0.05,
                                                           min_lr=1e-4)
    htmodel = ht.nn.DataParallelMultiGPU(model, daso, comm)
    criterion = torch.nn.CrossEntropyLoss()
    start = 0
    if args.resume and args.checkpoint and os.path.isfile(args.checkpoint):
        start = load_checkpoint(args.checkpoint, model, optimizer, dev)
        print0(comm, "=> resumed from '{}' at epoch {}".format(args.checkpoint, start))
    data = SyntheticImageNet(args.samples, args.image_size, args.classes, args.batch_size, comm, dev)
    daso.last_batch = len(data) - 1
    t_train, images = 0.0, 0
    for epoch in range(start, args.epochs):
        htmodel.train()
        t0 = time.perf_counter()
        tot, top1 = 0.0, 0.0
        for i, (x, y) in enumerate(data):
            lr_warmup(optimizer, args.lr, epoch, i, len(data))
            with autocast(args, dev):
                out = htmodel(x)
                loss = criterion(out.float(), y)
            daso.zero_grad()
            loss.backward()
            daso.step()
            tot += float(loss.detach())
            if i % args.print_freq == 0 or i == len(data) - 1:
                a1, _ = accuracy(out.detach().float(), y)
                top1 = float(a1)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        t_train += dt
        images += len(data) * args.batch_size * comm.size
        avg = reduce_mean(tot / len(data), comm)
        daso.epoch_loss_logic(avg, loss_globally_averaged=True)
        scheduler.step(avg)
        print0(comm, "epoch {} loss {:.4f} top1(last batch) {:.1f} global_skip {} local_skip {} {:.1f} img/s".format(
            epoch, avg, reduce_mean(top1, comm), daso.global_skip, daso.local_skip,
            len(data) * args.batch_size * comm.size / dt))
        if args.checkpoint:
            save_checkpoint(args.checkpoint, model, optimizer, epoch, comm)
    report(comm, "imagenet-DASO", args, t_train, images)


if __name__ == "__main__":
    main()
