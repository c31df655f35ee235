"""k_verify roofline fraction recomputed from a rocprofv3 kernel trace (per-launch durations), for
comparison with the live HIP-event figure in bench.py's JSON line.

Usage: python tools/roofline_rocprof.py TRACE.csv [--bench BENCH.json] [--skip N]

Takes the k_verify<...> launches of the trace, drops the first N (warm-up; default: the launches
before the first one of full size is repeated), and applies bench.py's work model
(kverify_fm_per_sig x 100 u32 MADs per signature) to the signatures per launch and the mean duration.
Prints one JSON object."""
import argparse
import csv
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--bench", help="bench.py JSON line of the same build (key window, sigs/launch, live frac)")
    ap.add_argument("--skip", type=int, default=2, help="warm-up launches to drop")
    ap.add_argument("--take", type=int, default=0, help="launches to use after the skipped ones (0: all; bench.py's "
                                                          "timed region is followed by 3 isolated launches)")
    ap.add_argument("--sigs", type=float, default=1000042.0, help="signatures per k_verify launch")
    ap.add_argument("--key-window", type=int, default=20)
    ap.add_argument("--base-window", type=int, default=24)
    a = ap.parse_args()
    import bench
    durs = []
    with open(a.trace) as f:
        for row in csv.DictReader(f):
            if re.match(r"void nw::k_verify<0, \d+(, (true|false))?>", row["Kernel_Name"]):
                durs.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    live = None
    kw, bw, sigs = a.key_window, a.base_window, a.sigs
    if a.bench:
        with open(a.bench) as f:
            b = json.loads([ln for ln in f if ln.startswith("{")][-1])
        live = b["roofline"]
        kw = b["config"]["key_window"]
    kept = durs[a.skip:a.skip + a.take] if a.take else durs[a.skip:]
    mean = sum(kept) / len(kept)
    fm = bench.kverify_fm_per_sig(kw, bw)
    peak = bench.valu_peak_mad_per_s()
    achieved = sigs * fm * bench.MADS_PER_FM / mean
    out = {"kernel": "k_verify", "launches_in_trace": len(durs), "launches_used": len(kept),
           "mean_ms": mean * 1e3, "min_ms": min(kept) * 1e3, "max_ms": max(kept) * 1e3,
           "fm_per_sig": fm, "sigs_per_launch": sigs, "achieved_TMADps": achieved / 1e12,
           "peak_TMADps": peak / 1e12, "frac_rocprof": achieved / peak}
    if live:
        out["frac_live_events"] = live["frac"]
        out["avg_launch_ms_live"] = live["avg_launch_ms"]
        if live.get("isolated"):
            out["isolated_live"] = live["isolated"]
        out["rocprof_vs_live"] = out["frac_rocprof"] / live["frac"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
