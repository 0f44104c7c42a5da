"""
ImageNet-style data-parallel training (reference ``examples/nn/imagenet.py``): the model is
wrapped in ``ht.nn.DataParallel`` (bucketed gradient all-reduces overlapped with backward, RCCL
over xGMI on MI355X) and stepped by ``ht.optim.DataParallelOptimizer``. Synthetic ImageNet-shaped
data (no network here); top-1/top-5 accuracy averaged over the ranks; checkpoint / resume.

    python -m heat_amd.run -n 8 examples/nn/imagenet.py --image-size 224 --classes 1000 --width 64 --bf16
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
    args = parser("ImageNet-style data-parallel training").parse_args()
    comm = ht.MPI_WORLD
    dev = device()
    torch.manual_seed(0)
    layers = tuple(int(v) for v in args.layers.split(","))
    model = ResNet(layers, args.width, args.classes).to(dev)
    sgd = torch.optim.SGD(model.parameters(), args.lr, momentum=args.momentum, weight_decay=args.weight_decay)
    opt = ht.optim.DataParallelOptimizer(sgd, blocking=False)
    dp = ht.nn.DataParallel(model, comm, opt)
    criterion = torch.nn.CrossEntropyLoss()
    start = 0
    if args.resume and args.checkpoint and os.path.isfile(args.checkpoint):
        start = load_checkpoint(args.checkpoint, model, sgd, dev)
        print0(comm, "=> resumed from '{}' at epoch {}".format(args.checkpoint, start))
    data = SyntheticImageNet(args.samples, args.image_size, args.classes, args.batch_size, comm, dev)
    t_train, images = 0.0, 0
    for epoch in range(start, args.epochs):
        dp.train()
        t0 = time.perf_counter()
        tot, a1s, a5s = 0.0, 0.0, 0.0
        for i, (x, y) in enumerate(data):
            lr_warmup(sgd, args.lr, epoch, i, len(data))
            opt.zero_grad()
            with autocast(args, dev):
                out = dp(x)
                loss = criterion(out.float(), y)
            loss.backward()
            opt.step()
            tot += float(loss.detach())
            a1, a5 = accuracy(out.detach().float(), y)
            a1s, a5s = a1s + float(a1), a5s + float(a5)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        t_train += dt
        images += len(data) * args.batch_size * comm.size
        n = len(data)
        print0(comm, "epoch {} loss {:.4f} top1 {:.1f} top5 {:.1f} {:.1f} img/s".format(
            epoch, reduce_mean(tot / n, comm), reduce_mean(a1s / n, comm), reduce_mean(a5s / n, comm),
            n * args.batch_size * comm.size / dt))
        if args.checkpoint:
            save_checkpoint(args.checkpoint, model, sgd, epoch, comm)
    report(comm, "imagenet", args, t_train, images)


if __name__ == "__main__":
    main()
