#!/usr/bin/env python3
"""Event sequence (kernels + copies, per stream/queue) of the steady state of a
pipelined run, from a rocprofv3 --kernel-trace --memory-copy-trace directory:
python tools/r03/trace_sequence.py DIR [N]  (CPU only)."""
import csv
import sys
d=sys.argv[1]; n=int(sys.argv[2]) if len(sys.argv)>2 else 70
ks=list(csv.DictReader(open(d+"/run_kernel_trace.csv")))
cs=list(csv.DictReader(open(d+"/run_memory_copy_trace.csv")))
ev=[(int(k["Start_Timestamp"]),int(k["End_Timestamp"]),k["Kernel_Name"].split("(")[0][-26:],k["Stream_Id"],k["Queue_Id"],k["Grid_Size_X"]) for k in ks]
ev+=[(int(c["Start_Timestamp"]),int(c["End_Timestamp"]),"COPY "+c["Direction"][12:],c["Stream_Id"],"-","") for c in cs]
ev.sort()
segs=[];cur=[ev[0]]
for x in ev[1:]:
    if x[0]-cur[-1][0]>2_000_000: segs.append(cur); cur=[]
    cur.append(x)
segs.append(cur)
seg=max(segs,key=lambda g: sum(1 for x in g if x[2].startswith("COPY")))
w=seg[len(seg)//2:]
t0=w[0][0]
for x in w[:n]:
    print(f"{(x[0]-t0)/1e3:8.2f} {(x[1]-t0)/1e3:8.2f} {(x[1]-x[0])/1e3:6.2f} s{x[3]} q{x[4]} {x[2]} g{x[5]}")
