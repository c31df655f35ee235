"""Timeline (kernels, copies, HIP API calls) of one call from a rocprofv3 trace database:
python tools/trace_timeline.py DB KERNEL_SUBSTR OCCURRENCE [N_EVENTS]"""
import glob, sqlite3, sys
db, key, occ = sys.argv[1], sys.argv[2], int(sys.argv[3])
n_ev = int(sys.argv[4]) if len(sys.argv) > 4 else 40
c = sqlite3.connect(glob.glob(db)[0])
ev = [(s, e, "K " + n.split("(")[0][-30:]) for n, s, e in c.execute("select name,start,end from kernels")]
cols = [r[1] for r in c.execute("pragma table_info(memory_copies)")]
for r in c.execute("select * from memory_copies"):
    d = dict(zip(cols, r))
    ev.append((d["start"], d["end"], "M %s %s stream %s" % (d.get("name"), d.get("size"), d.get("stream_id"))))
cols = [r[1] for r in c.execute("pragma table_info(regions)")]
for r in c.execute("select * from regions"):
    d = dict(zip(cols, r))
    ev.append((d["start"], d["end"], "A " + str(d["name"])[:40]))
ev.sort()
hits = [i for i, x in enumerate(ev) if key in x[2]]
i = hits[occ]
t0 = ev[i][0]
for s, e, n in ev[max(0, i - n_ev // 2):i + n_ev // 2]:
    print("%9.1f %8.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, n))
