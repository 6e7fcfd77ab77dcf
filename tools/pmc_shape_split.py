#!/usr/bin/env python3
"""Per-shape means of the headline kernel's counters from the tools/pmc_limits.sh
`shape*` passes (tools/shape_probe.py pmc runs 5 shapes x 24 launches in that
order; the first 8 launches of each are skipped), normalised to 64 Mpx where a
counter scales with pixels; also the TCC fabric-side read / write latency
(LEVEL / REQ).  usage: tools/pmc_shape_split.py shape_sq1 shape_sq2 shape_tcc1 ...
(directories under gpurun_out/pmc_limits/)"""
import csv,glob,sys
from collections import defaultdict
dirs=sys.argv[1:]
shapes=[("8192x8192",8192*8192),("16384x4096",16384*4096),("4096x16384",4096*16384),("2048x16384",2048*16384),("16384x16384",16384**2)]
for d in dirs:
    rows=defaultdict(dict)
    for f in glob.glob(f"gpurun_out/pmc_limits/{d}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "8217" not in r["Kernel_Name"]: continue
            rows[int(r["Dispatch_Id"])][r["Counter_Name"]]=float(r["Counter_Value"])
    ids=sorted(rows)
    for k,(s,px) in enumerate(shapes):
        blk=ids[k*24+8:(k+1)*24]
        m=defaultdict(float)
        for i in blk:
            for c,v in rows[i].items(): m[c]+=v/len(blk)
        sc=(1<<26)/px
        out=f"{d} {s:12s}"
        for c in sorted(m):
            out+=f" {c}={m[c]*sc:.4g}"
        if "TCC_EA0_WRREQ_LEVEL" in m: out+=f" WRlat={m['TCC_EA0_WRREQ_LEVEL']/m['TCC_EA0_WRREQ']:.0f}"
        if "TCC_EA0_RDREQ_LEVEL" in m: out+=f" RDlat={m['TCC_EA0_RDREQ_LEVEL']/m['TCC_EA0_RDREQ']:.0f}"
        print(out)
