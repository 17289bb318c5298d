import csv,glob,sys
d='gpurun_out/tl'
mk=list(csv.DictReader(open(glob.glob(d+'/*marker_api_trace.csv')[0])))
kt=list(csv.DictReader(open(glob.glob(d+'/*kernel_trace.csv')[0])))
mc=list(csv.DictReader(open(glob.glob(d+'/*memory_copy_trace.csv')[0])))
steps=sorted([(int(r['Start_Timestamp']),int(r['End_Timestamp'])) for r in mk if r['Function']=='bench.step'])
for want in map(int,sys.argv[1:]):
    s0,s1=steps[want]
    f=lambda x:(x-s0)/1e3
    loads=sorted((int(r['Start_Timestamp']),int(r['End_Timestamp'])) for r in mk if r['Function']=='nm03.load' and s0<=int(r['Start_Timestamp'])<=s1)
    exps=sorted((int(r['Start_Timestamp']),int(r['End_Timestamp'])) for r in mk if r['Function']=='nm03.export' and s0<=int(r['Start_Timestamp'])<=s1)
    gb=sorted((int(r['Start_Timestamp']),int(r['End_Timestamp'])) for r in mk if r['Function']=='nm03.gpu_batch' and s0<=int(r['Start_Timestamp'])<=s1)
    ks={}
    for r in kt:
        a=int(r['Start_Timestamp'])
        if s0<=a<=s1: ks.setdefault(r['Stream_Id'],[]).append((a,int(r['End_Timestamp']),r['Kernel_Name'][:20]))
    cs={}
    for r in mc:
        a=int(r['Start_Timestamp'])
        if s0<=a<=s1: cs.setdefault(r['Stream_Id'],[]).append((a,int(r['End_Timestamp'])))
    print(f"step {want} wall {f(s1):.0f}  loads {f(loads[0][0]):.0f}..{f(max(b for a,b in loads)):.0f} (n={len(loads)})  exports {f(exps[0][0]):.0f}..{f(max(b for a,b in exps)):.0f}")
    for g in gb: print(f"   gpu_batch {f(g[0]):.0f}..{f(g[1]):.0f}")
    for sid in sorted(ks):
        k=sorted(ks[sid]); c=sorted(cs.get(sid,[]))
        print(f"   stream {sid}: h2d {[(round(f(a)),round((b-a)/1e3)) for a,b in c]}  kernels {f(k[0][0]):.0f}..{f(k[-1][1]):.0f}")
