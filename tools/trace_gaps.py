#!/usr/bin/env python3
"""Idle gaps of one solve in a rocprofv3 kernel trace (tools/trace_c4.py under --kernel-trace): the
last solve's wall, busy and idle time, a histogram of the gaps between consecutive kernels, and the
gaps summed by (previous kernel, next kernel) pair.

usage: python tools/trace_gaps.py RUN_kernel_trace.csv [nocut]   (nocut: the last segment is one solve)
"""
import csv, collections, re, sys
import numpy as np
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
def nm(k):
    k=k.replace('(anonymous namespace)::','').replace('void ','')
    m=re.match(r'([\w:]+(<[^()]*>)?)',k)
    return m.group(1)[:44] if m else k[:44]
ts=[(int(r['Start_Timestamp']),int(r['End_Timestamp']),nm(r['Kernel_Name'])) for r in rows]
segs=[[ts[0]]]
for a,b in zip(ts,ts[1:]):
    if b[0]-a[1]>3e6: segs.append([])
    segs[-1].append(b)
s=segs[-1]
# split into solves: the largest gap
g=[b[0]-a[1] for a,b in zip(s,s[1:])]
cut=int(np.argmax(g))+1 if len(sys.argv)<3 else 0
print('segments',[len(x) for x in segs],'cut at',cut,'gap',g[cut-1]/1e3,'us')
s=s[cut:]
busy=sum(e-b for b,e,_ in s); wall=s[-1][1]-s[0][0]
print('solve: kernels',len(s),'wall ms',wall/1e6,'busy',busy/1e6,'idle',(wall-busy)/1e6)
gaps=collections.defaultdict(lambda:[0,0.0])
allg=[]
for a,b in zip(s,s[1:]):
    g=b[0]-a[1]
    allg.append(g)
    if g>1500:
        k=(a[2], b[2]); gaps[k][0]+=1; gaps[k][1]+=g/1e3
allg=np.array(allg)
print('gaps >1.5us:', (allg>1500).sum(), 'sum us', allg[allg>1500].sum()/1e3, ' <=1.5us sum', allg[allg<=1500].sum()/1e3)
print('gap histogram (us):', np.histogram(allg/1e3,[0,1.5,3,5,8,12,20,40,100,1000,10000])[0])
for k,v in sorted(gaps.items(), key=lambda kv:-kv[1][1])[:30]:
    print(f"{v[0]:3d} {v[1]:8.1f}us  {k[0]:44s} -> {k[1]}")
