"""Summary of tools/pmc_ab_r05.sh: per variant, the C2-size k_verify launches' shader cycles
(GRBM_GUI_ACTIVE / 8 XCDs, millions), their median, and VALU instructions per wave.

    python3 tools/pmc_ab_summary.py gpurun_out/OUTTAG
"""
import collections
import csv
import glob
import os
import sys


def main():
    root = sys.argv[1]
    for d in sorted(glob.glob(os.path.join(root, "*/"))):
        fs = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not fs:
            continue
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(fs[0])):
            agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        big = [(v["GRBM_GUI_ACTIVE"] / 8e6, v["SQ_INSTS_VALU"] / v["SQ_WAVES"]) for v in agg.values()
               if v["SQ_WAVES"] > 15000]
        if not big:
            continue
        cyc = sorted(c for c, _ in big)
        print("%-12s median %.3f M cycles  [%s]  VALU/wave %.0f" % (
            os.path.basename(d.rstrip("/")), cyc[len(cyc) // 2], " ".join("%.3f" % c for c, _ in big), big[0][1]))


if __name__ == "__main__":
    main()
