"""Per-phase summary of a k_msm_bucket NW_MSM_TIMING run: python tools/msm_timing_summary.py LOG"""
import sys, collections
rows=[l.split() for l in open(sys.argv[1]) if l.startswith("MSMT")]
# keep the last call's launch: rt0 clusters; split by big gaps
rows=[(int(b),int(w),int(m),int(rt),int(a),int(c),int(d),int(e),int(h)) for _,b,w,m,rt,a,c,d,e,h in rows]
rows.sort(key=lambda r:r[3])
groups=[[rows[0]]]
for r in rows[1:]:
    if r[3]-groups[-1][-1][3] > 20000: groups.append([r])   # >200 us gap: next launch
    else: groups[-1].append(r)
g=groups[-1]
t0=min(r[3] for r in g)
print("launches seen", len(groups), "rows in last", len(g))
for heavy in (True, False):
    sel=[r for r in g if (r[1]<16)==heavy]
    if not sel: continue
    n=len(sel)
    avg=lambda i: sum(r[i] for r in sel)/n
    print("%s windows: n=%d entries~%d  start skew us max %.1f  sort %.0fk  scan+scatter %.0fk  accum %.0fk  merge+reduce %.0fk cycles"
          % ("R+A" if heavy else "A  ", n, avg(2), max((r[3]-t0)/100 for r in sel), avg(4)/1e3, avg(5)/1e3, avg(6)/1e3, avg(7)/1e3))
    print("   accum min/max %.0fk/%.0fk" % (min(r[6] for r in sel)/1e3, max(r[6] for r in sel)/1e3))
