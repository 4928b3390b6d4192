#!/usr/bin/env python3
"""Summarise tools/exp_r03i.sh counter passes: EA read / write latency and
requests in flight per shape (SHAPE_DIR: gpurun_out or profiles/r03/shape
with the per-pass CSVs renamed). Not product code."""
import csv,collections,os
shapes=["rs 10 4 1M enc_split","rs 10 4 1M dec_inplace","rs 8 2 4K enc_split","rs 12 2 4K enc_inplace","cauchy 12 2 4K enc_inplace"]
for i,sh in enumerate(shapes,1):
    out={}
    for p in 'abc':
        f=os.path.join(os.environ.get('SHAPE_DIR', 'gpurun_out'), 'shape_%s_%d/run_counter_collection.csv' % (p, i))
        if not os.path.exists(f): continue
        agg=collections.defaultdict(float); disp=set()
        for r in csv.DictReader(open(f)):
            if 'gf8_kernel' not in r['Kernel_Name'] and 'bm_kernel' not in r['Kernel_Name']: continue
            agg[r['Counter_Name']]+=float(r['Counter_Value']); disp.add(r['Dispatch_Id'])
        for c,v in agg.items(): out[c]=v/len(disp)
    g=out.get('GRBM_GUI_ACTIVE',1)
    rdl=out.get('TCC_EA0_RDREQ_LEVEL_sum',0)/max(out.get('TCC_EA0_RDREQ_sum',1),1)
    wrl=out.get('TCC_EA0_WRREQ_LEVEL_sum',0)/max(out.get('TCC_EA0_WRREQ_sum',1),1)
    tcpl=out.get('TCP_TCC_READ_REQ_LATENCY_sum',0)/max(out.get('TCP_TCC_READ_REQ_sum',1),1)
    print(sh, "| EA rd lat %.0f wr lat %.0f | TCP rd lat %.0f | rd-in-flight %.0f wr-in-flight %.0f" % (rdl, wrl, tcpl, out.get('TCC_EA0_RDREQ_LEVEL_sum',0)/g, out.get('TCC_EA0_WRREQ_LEVEL_sum',0)/g))
    print("   ", {k: "%.3g"%v for k,v in out.items()})
