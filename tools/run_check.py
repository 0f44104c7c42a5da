"""Run one check (``module:function``) in N gloo ranks and print each failing rank's last error
lines: ``python tools/run_check.py tests.parity.statistics_checks:test_mean 8``."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tests._dist import run_distributed  # noqa: E402


def main():
    target, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2
    try:
        run_distributed(target, n)
        print("{} ok at {} ranks".format(target, n))
    except AssertionError as e:
        for blk in str(e).split("----- rank")[1:]:
            lines = [ln for ln in blk.splitlines() if ln.strip() and "socket.cpp" not in ln and "[Gloo]" not in ln]
            if any("Connection" in ln for ln in lines[-2:]):
                continue
            print("rank" + "\n".join(lines[:1] + lines[-8:]))
        sys.exit(1)


if __name__ == "__main__":
    main()
