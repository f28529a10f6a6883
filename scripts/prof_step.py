#!/usr/bin/env python3
"""One steady training step of a rocprofv3 kernel trace (between the last two
softmax forwards, i.e. one whole-step hipGraph replay), per kernel family.

    python scripts/prof_step.py gpurun_out/prof_train_fused
"""
import csv,glob,collections,re,sys
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
from prof_summary import family
f=glob.glob(sys.argv[1]+'/*/run_kernel_trace.csv')[0]
rows=list(csv.DictReader(open(f)))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
idx=[i for i,r in enumerate(rows) if 'softmax_warp_forward' in r['Kernel_Name']]
a,b=idx[-3],idx[-2]
step=rows[a:b]
t0=int(step[0]['Start_Timestamp']); t1=int(rows[b]['Start_Timestamp'])
print("one steady step (between the last softmax forwards): dispatches",len(step),"span us %.1f"%((t1-t0)/1e3))
agg=collections.defaultdict(lambda:[0,0])
for r in step:
    d=(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3
    n=r['Kernel_Name']
    k=family(n)
    if k.startswith('void (anonymous namespace)::'): k=k[len('void (anonymous namespace)::'):]
    if 'FillFunctor' in n: k='torch fill '+('fp32' if 'FillFunctor<float>' in n else 'bf16')
    if 'wgrad_reduce' in n: k='vgpu wgrad split-K reduce'
    agg[k][0]+=1; agg[k][1]+=d
tot=sum(v[1] for v in agg.values())
print("busy us %.1f"%tot)
print("| us/step | % | dispatches | avg us | family |\n|---|---|---|---|---|")
for k,(c,d) in sorted(agg.items(),key=lambda kv:-kv[1][1]):
    print(f"| {d:.1f} | {100*d/tot:.1f} | {c} | {d/c:.1f} | {k} |")
