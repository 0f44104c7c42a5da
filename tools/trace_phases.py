"""Per-phase summary of a rocprofv3 kernel-trace CSV whose workload separates its loops by idle
gaps (> 20 ms), e.g. tools/microbench/smallk_trace.py: kernel counts, the mean / min / max duration
of the kernels whose name contains KEY (default ks_wave64), the mean start-to-start interval of
those kernels, and the kernels of one step with their start offsets and durations (us).
usage: python tools/trace_phases.py <kernel_trace.csv> [KEY]"""
import csv
import sys
from collections import Counter


def short(n):
    for k in ("ks_wave64", "ks_reduce_fin", "ks_fin", "ks_reduce", "ks_step", "ks_pad", "km_finalize"):
        if k in n:
            return k
    return n[:30]


def main(path, key="ks_wave64"):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    phases, prev = [[]], None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if prev is not None and s - prev > 20e6:
            phases.append([])
        phases[-1].append((s, e, r["Kernel_Name"]))
        prev = e
    for i, p in enumerate(phases):
        passes = [(s, e) for s, e, n in p if key in n]
        if len(passes) < 12:
            continue
        d = [(e - s) / 1e3 for s, e in passes[5:]]
        per = [(passes[j + 1][0] - passes[j][0]) / 1e3 for j in range(5, len(passes) - 1)]
        print(i, len(p), Counter(short(n) for _, _, n in p).most_common(8))
        print("  %s us mean %.1f min %.1f max %.1f | start-to-start mean %.1f" % (key, sum(d) / len(d), min(d), max(d),
                                                                                 sum(per) / len(per)))
        s0, s1 = passes[10][0], passes[11][0]
        print("  step:", [(short(n), round((s - s0) / 1e3, 1), round((e - s) / 1e3, 1)) for s, e, n in p if s0 <= s < s1])


if __name__ == "__main__":
    main(*sys.argv[1:])
