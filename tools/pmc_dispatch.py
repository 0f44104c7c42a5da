"""Per-dispatch rows of rocprofv3 --pmc passes (one pass per counter group, same workload): for each
dispatch of the kernels whose name contains FILTER, duration, effective clock, MFMA-busy share,
VALU / MFMA, wave-cycle breakdown, HBM bytes (FETCH_SIZE: 2 x 64 B per 128-B request on gfx950,
WRITE_SIZE as is) and LDS bank-conflict share, as markdown table rows. Dispatches of the passes
are paired in order (the workload is deterministic).

    python tools/pmc_dispatch.py FILTER pass_A_dir [pass_F_dir [pass_W_dir]] [--label TEXT]

Normalisation as tools/pmc_summary.py (8 XCDs, 1024 SIMDs)."""
import collections
import csv
import glob
import os
import sys


def load(d):
    if not d:
        return [], {}
    f = glob.glob(os.path.join(d, "*counter_collection.csv"))
    if not f:
        return [], {}
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for r in csv.DictReader(open(f[0])):
        k = int(r["Dispatch_Id"])
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        meta[k] = (r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    return sorted(per), (per, meta)


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:48]


def main(argv):
    label = ""
    if "--label" in argv:
        i = argv.index("--label")
        label = argv[i + 1]
        argv = argv[:i] + argv[i + 2:]
    filt, dirs = argv[0], argv[1:] + [None, None]
    passes = [load(d) for d in dirs[:3]]
    ids = [[k for k in ks if filt in (pm[1][k][0] if pm else "")] for ks, pm in passes]
    rows = []
    for n, ka in enumerate(ids[0]):
        per, meta = passes[0][1]
        m = per[ka]
        name, d = meta[ka]
        grbm = m.get("GRBM_GUI_ACTIVE", 0.0)
        clk = grbm / 8 / d / 1e9 if d > 0 else 0.0
        busy = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / 1024 / (grbm / 8) if grbm else 0.0
        mf = m.get("SQ_INSTS_MFMA", 0.0)
        vpm = m.get("SQ_INSTS_VALU", 0.0) / mf if mf else float("nan")
        wc = m.get("SQ_WAVE_CYCLES", 0.0)
        wi = m.get("SQ_WAIT_INST_ANY", 0.0) / wc if wc else 0.0
        wa = m.get("SQ_WAIT_ANY", 0.0) / wc if wc else 0.0
        rd = wr = lds = float("nan")
        if len(ids[1]) > n:
            f = passes[1][1][0][ids[1][n]]
            if "FETCH_SIZE" in f:
                rd = 2 * 1024 * f["FETCH_SIZE"] / 1e9
            if f.get("SQ_LDS_IDX_ACTIVE"):
                lds = f.get("SQ_LDS_BANK_CONFLICT", 0.0) / f["SQ_LDS_IDX_ACTIVE"]
        if len(ids[2]) > n:
            w = passes[2][1][0][ids[2][n]]
            if "WRITE_SIZE" in w:
                wr = 1024 * w["WRITE_SIZE"] / 1e9
        rows.append("| {}`{}` | {:.1f} | {:.2f} | {:.0%} | {:.2f} | {:.0%} / {:.0%} | {:.2f} | {:.2f} | {:.1%} |".format(
            label, short(name), d * 1e6, clk, busy, vpm, wi, wa, rd, wr, lds))
    print("| kernel | us | clock GHz | MFMA busy | VALU/MFMA | wait-inst / wait-any | read GB | write GB | LDS conflict |")
    print("|---|---|---|---|---|---|---|---|---|")
    print("\n".join(rows))


if __name__ == "__main__":
    main(sys.argv[1:])
