"""Run many check functions in ONE set of ranks (one interpreter start per rank instead of one
per check). Each check's outcome is agreed on by all ranks and written by rank 0 as a JSON line
``{"name": ..., "ok": bool, "error": str}``; a check that raised on any rank counts as failed.
A deadlocked check is bounded by the short collective timeout the harness sets."""
import importlib
import json
import sys
import traceback


def main():
    out_path, mod_name = sys.argv[1], sys.argv[2]
    names = sys.argv[3:]
    import heat_amd as ht  # noqa: F401  (initialises the process group)

    mod = importlib.import_module(mod_name)
    comm = ht.MPI_WORLD
    results = []
    for name in names:
        err = None
        try:
            getattr(mod, name)()
        except BaseException:  # noqa: B902 - reported
            err = traceback.format_exc()[-4000:]
        errs = comm.allgather(err)
        bad = [(r, e) for r, e in enumerate(errs) if e is not None]
        results.append({"name": name, "ok": not bad,
                        "error": "" if not bad else "rank {}:\n{}".format(bad[0][0], bad[0][1])})
        if comm.rank == 0:
            with open(out_path, "a") as f:
                f.write(json.dumps(results[-1]) + "\n")
    import torch.distributed as dist

    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
