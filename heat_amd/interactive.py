"""
SPMD interactive interpreter (reference ``scripts/interactive.py``): start with
``python -m heat_amd.run -n 4 --no-prefix -m heat_amd.interactive``. Rank 0 reads each line and
broadcasts it; every rank executes it; a barrier follows each statement so output stays ordered.
"""
from __future__ import annotations

import code
import sys

import heat_amd as ht


class HeatInterpreter(code.InteractiveConsole):
    def __init__(self, comm=ht.MPI_WORLD, locals=None):
        super().__init__(locals=locals if locals is not None else {"ht": ht, "heat_amd": ht})
        self.comm = comm

    def raw_input(self, prompt: str = "") -> str:
        line = None
        if self.comm.rank == 0:
            try:
                line = input(prompt)
            except EOFError:
                line = "\x04"
        line = self.comm.bcast(line, root=0)
        if line == "\x04":
            raise EOFError
        return line

    def runcode(self, codeobj):
        super().runcode(codeobj)
        sys.stdout.flush()
        self.comm.Barrier()


def main():
    HeatInterpreter().interact(banner="heat_amd {} on {} rank(s)".format(ht.__version__, ht.MPI_WORLD.size)
                               if ht.MPI_WORLD.rank == 0 else "", exitmsg="")


if __name__ == "__main__":
    main()
