"""Summarize a tools/gpu_pmc.sh run: per-kernel counter values (largest dispatch = the full-size
launch) and the HBM-traffic estimate used by bench.py's roofline.traffic.

    python tools/pmc_summary.py gpurun_out/<tag>_pmc profiles/<round>/pmc_k_verify.json

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KiB) reports 1/2 of the bytes of wide
(16 B/lane) reads -> x2 (k_verify's table gathers are 16-B-per-lane global_load_dwordx4);
WRITE_SIZE (KiB) is exact for 16-B stores and uncalibrated for the 4-B SoA stores used here.
"""
import collections
import csv
import glob
import json
import os
import sys


def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "pmc_pass*.csv"))):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return agg, dur


def main():
    src, dst = sys.argv[1], sys.argv[2]
    agg, dur = load(src)
    out = {"source": src, "kernels": {}}
    for k, d in agg.items():
        row = {c: max(v) for c, v in d.items()}
        if "FETCH_SIZE" in row:
            row["hbm_read_bytes_corrected"] = row["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in row:
            row["hbm_write_bytes"] = row["WRITE_SIZE"] * 1024
        if "SQ_WAVE_CYCLES" in row and "SQ_WAIT_ANY" in row and "SQ_WAIT_INST_ANY" in row:
            wc = row["SQ_WAVE_CYCLES"]
            row["frac_wait_mem"] = row["SQ_WAIT_ANY"] / wc
            row["frac_wait_issue"] = row["SQ_WAIT_INST_ANY"] / wc
            row["frac_active"] = row.get("SQ_ACTIVE_INST_ANY", 0) / wc
        if "SQ_INSTS_VALU" in row and "SQ_WAVES" in row:
            row["valu_insts_per_wave"] = row["SQ_INSTS_VALU"] / row["SQ_WAVES"]
        if "GRBM_GUI_ACTIVE" in row:
            row["max_dispatch_us"] = max(dur[k])
            row["effective_clock_ghz"] = row["GRBM_GUI_ACTIVE"] / 8 / (max(dur[k]) * 1e3)
            if "SQ_THREAD_CYCLES_VALU" in row:
                # VALU busy cycles per SIMD (thread-cycles / 64 lanes) over the kernel's cycles x 1024 SIMDs
                row["valu_utilization"] = (row["SQ_THREAD_CYCLES_VALU"] / 64.0) / (row["GRBM_GUI_ACTIVE"] / 8 * 1024)
        out["kernels"][k] = row
    kv = [k for k in out["kernels"] if k.startswith("nw::k_verify")]
    if kv:
        r = out["kernels"][kv[0]]
        out["k_verify"] = kv[0]
        out["hbm_bytes_per_launch"] = r.get("hbm_read_bytes_corrected", 0) + r.get("hbm_write_bytes", 0)
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in out if k != "kernels"}))


if __name__ == "__main__":
    main()
