"""Timeline of the worker_digest leg's last window size (tools/worker_trace.sh): digest kernels and
host-to-device copies of the final submissions, times in ms from the first of them."""
import csv
import glob
import json
import os
import sys


def rows(d, suffix):
    out = []
    for p in glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True):
        with open(p) as f:
            out.extend(csv.DictReader(f))
    return out


def main():
    d, js = sys.argv[1], sys.argv[2]
    leg = json.loads(open(js).read().strip().splitlines()[-1])
    w = leg["windows"]["1250"]
    print("WINDOW 1250: %.0f batches/s, p50 %.1f ms" % (w["batches_per_s"], w["p50_latency_ms"]))
    ks = [r for r in rows(d, "kernel_trace.csv") if "sha512" in r["Kernel_Name"]]
    ks.sort(key=lambda r: int(r["Start_Timestamp"]))
    cs = rows(d, "memory_copy_trace.csv")
    cs.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the last window-1250 run: its submissions are the last digest kernels before the one-batch calls
    big = [r for r in ks if int(r.get("Grid_Size", r.get("Grid_Size_X", "0")) or 0) >= 192 * 8]
    tail = big[-6:]
    if not tail:
        print("no multi-workgroup digest kernels found")
        return
    t0 = int(tail[0]["Start_Timestamp"]) - 60_000_000
    keys = [k for k in ("Queue_Id", "Stream_Id", "Grid_Size", "Workgroup_Size", "LDS_Block_Size") if k in tail[0]]
    print("kernels (start, end, dur ms) " + " ".join(keys))
    for r in tail:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print("  %9.3f %9.3f %7.3f  %s" % ((s - t0) / 1e6, (e - t0) / 1e6, (e - s) / 1e6, " ".join(r[k] for k in keys)))
    t_end = int(tail[-1]["End_Timestamp"])
    ckeys = [k for k in ("Direction", "Size", "Queue_Id", "Stream_Id") if k in (cs[0] if cs else {})]
    print("copies in the window (start, end, dur ms, GB/s) " + " ".join(ckeys))
    n = 0
    for r in cs:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s < t0 or s > t_end:
            continue
        n += 1
        if n % 8 == 1:   # every 8th copy (4 MiB pieces)
            sz = float(r.get("Size", 0) or 0)
            print("  %9.3f %9.3f %7.3f %6.1f  %s" % ((s - t0) / 1e6, (e - t0) / 1e6, (e - s) / 1e6,
                                                    sz / max(1, e - s), " ".join(r[k] for k in ckeys)))
    print("copies in window:", n)


if __name__ == "__main__":
    main()
