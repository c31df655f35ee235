"""Clock-normalised roofline fraction of k_verify.

Both the v_mad_u64_u32 peak (tools/valu_peak) and k_verify ran under one rocprofv3 PMC pass with
GRBM_GUI_ACTIVE (one PMC pass each, tools/gpu_pmc.sh), so each is known in shader cycles, not only in wall time:
  peak_per_cycle = v_mad_u64_u32 lane-ops of the microbenchmark / its GPU cycles
  kverify        = algorithmic MADs per launch (162 FM x 100 per signature at C2) / its GPU cycles
  frac_per_cycle = kverify / peak_per_cycle     (independent of the clock either kernel ran at)
GRBM_GUI_ACTIVE is summed over the 8 XCDs: cycles = GRBM_GUI_ACTIVE / 8.
Usage: python tools/clock_frac.py PEAK_COUNTERS.csv KV_COUNTERS.csv SIGS_PER_LAUNCH FM_PER_SIG > out.json
"""
import collections
import csv
import json
import sys

LANES_PER_WAVE = 64


def load(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    dur, name = {}, {}
    for r in csv.DictReader(open(path)):
        k = r["Dispatch_Id"]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[k] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        name[k] = r["Kernel_Name"]
    return agg, dur, name


def main():
    peak_csv, kv_csv, sigs, fm = sys.argv[1], sys.argv[2], float(sys.argv[3]), float(sys.argv[4])
    agg, dur, name = load(peak_csv)
    peaks = []
    for k, d in agg.items():
        if "k_mad_u64_u32" not in name[k]:
            continue
        cycles = d["GRBM_GUI_ACTIVE"] / 8
        lane_ops = d["SQ_INSTS_VALU_INT64"] * LANES_PER_WAVE   # every INT64 op of this kernel is the MAD
        peaks.append({"dispatch": k, "cycles": cycles, "us": dur[k] / 1e3, "clock_ghz": cycles / dur[k],
                      "mad_per_cycle": lane_ops / cycles, "mad_per_s": lane_ops / (dur[k] * 1e-9)})
    agg, dur, name = load(kv_csv)
    kvs = []
    work = sigs * fm * 100
    for k, d in agg.items():
        if "k_verify" not in name[k]:
            continue
        cycles = d["GRBM_GUI_ACTIVE"] / 8
        kvs.append({"dispatch": k, "cycles": cycles, "us": dur[k] / 1e3, "clock_ghz": cycles / dur[k],
                    "valu_per_wave": d["SQ_INSTS_VALU"] / d["SQ_WAVES"],
                    "int64_per_wave": d["SQ_INSTS_VALU_INT64"] / d["SQ_WAVES"],
                    "alg_mad_per_cycle": work / cycles, "alg_mad_per_s": work / (dur[k] * 1e-9)})
    ppc = sorted(p["mad_per_cycle"] for p in peaks)[len(peaks) // 2]
    kpc = sorted(x["alg_mad_per_cycle"] for x in kvs)[len(kvs) // 2]
    out = {"peak_mad_per_cycle": ppc, "kverify_alg_mad_per_cycle": kpc, "frac_per_cycle": kpc / ppc,
           "work_model": "%d sigs x %d FM x 100 MADs per launch" % (sigs, fm),
           "peak_runs": peaks, "kverify_runs": kvs,
           "note": "cycles from GRBM_GUI_ACTIVE / 8 XCDs; the wall-time frac of bench.py divides by the "
                   "peak's wall-time rate, measured at the ~2.2 GHz the microbenchmark holds, while k_verify "
                   "runs at 1.6-2.1 GHz"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
