"""Per-kernel time in the timed windows of tools/c5_probe.py under
rocprofv3 --kernel-trace: each window starts at a flip marker kernel.

    python tools/trace_windows.py run_kernel_trace.csv
"""
import csv, sys, collections
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r["Start_Timestamp"]))
marks=[i for i,r in enumerate(rows) if "flip" in r["Kernel_Name"].lower()]
print("markers", len(marks))
# windows: after the last two markers
segs=[]
for m in marks[-2:]:
    segs.append(m)
for wi,(a) in enumerate(segs):
    b = segs[wi+1] if wi+1<len(segs) else len(rows)
    # restrict to first 2000 kernels after the marker (the timed window)
    win=rows[a+1:b]
    agg=collections.defaultdict(lambda:[0,0])
    for r in win:
        n=r["Kernel_Name"].split("(")[0][-40:]
        d=int(r["End_Timestamp"])-int(r["Start_Timestamp"])
        agg[n][0]+=1; agg[n][1]+=d
    t0=int(win[0]["Start_Timestamp"]); t1=max(int(r["End_Timestamp"]) for r in win)
    print("window",wi,"span us",(t1-t0)/1e3,"kernels",len(win))
    for n,(c,d) in sorted(agg.items(), key=lambda x:-x[1][1])[:14]:
        print(f"   {n:42s} {c:6d} {d/c/1e3:8.2f} us avg {d/1e3:10.1f} total")
