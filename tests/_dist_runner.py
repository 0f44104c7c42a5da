import importlib
import sys
import traceback


def main():
    target = sys.argv[1]
    mod, fn = target.split(":")
    try:
        import heat_amd  # noqa: F401  (initialises the process group)

        getattr(importlib.import_module(mod), fn)()
    except BaseException:
        traceback.print_exc()
        sys.stdout.flush()
        import os

        os._exit(1)
    import torch.distributed as dist

    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
