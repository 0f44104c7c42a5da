#!/usr/bin/env python
"""Per-kernel statistics (calls, total/avg/min/max ns, share) from a rocprofv3 ``*_results.db``
(rocpd SQLite output) as CSV, the same columns as rocprofv3's ``kernel_stats.csv``.

usage: python tools/rocpd_stats.py <results.db> [out.csv] [--top N]
"""
import csv
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    rows = c.execute(
        "select s.string, d.end - d.start from rocpd_kernel_dispatch d "
        "join rocpd_info_kernel_symbol k on d.kernel_id = k.id "
        "join rocpd_string s on k.kernel_name_id = s.id").fetchall() if _has(c, "kernel_name_id") else c.execute(
        "select k.kernel_name, d.end - d.start from rocpd_kernel_dispatch d "
        "join rocpd_info_kernel_symbol k on d.kernel_id = k.id").fetchall()
    agg = {}
    for name, dur in rows:
        a = agg.setdefault(name, [0, 0, None, None])
        a[0] += 1
        a[1] += dur
        a[2] = dur if a[2] is None else min(a[2], dur)
        a[3] = dur if a[3] is None else max(a[3], dur)
    total = sum(a[1] for a in agg.values()) or 1
    out = [(n, a[0], a[1], a[1] / a[0], a[2], a[3], 100.0 * a[1] / total) for n, a in agg.items()]
    out.sort(key=lambda r: -r[2])
    return out


def _has(c, col):
    cols = [r[1] for r in c.execute("pragma table_info(rocpd_info_kernel_symbol)")]
    return col in cols


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else None
    if "--top" in sys.argv:
        args.remove(str(top))
    rows = stats(args[0])
    if top:
        rows = rows[:top]
    f = open(args[1], "w", newline="") if len(args) > 1 else sys.stdout
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
    for r in rows:
        w.writerow([r[0][:200], r[1], r[2], "%.1f" % r[3], r[4], r[5], "%.2f" % r[6]])


if __name__ == "__main__":
    main()
