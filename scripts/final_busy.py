"""Final-hop stream occupancy of a pipelined batch from a rocprofv3 kernel trace: per 25-launch group (5 warm-up + 20 timed), the span of the timed final hops, the time any final hop runs and the time two run at once.
Usage: python scripts/final_busy.py gpurun_out/<trace dir>"""
import csv,sys,glob
f=glob.glob(sys.argv[1]+"/**/*kernel_trace.csv",recursive=True)[0]
rows=sorted(csv.DictReader(open(f)),key=lambda r:int(r["Start_Timestamp"]))
fin=[r for r in rows if "ngx_jit_final" in r["Kernel_Name"]]
# timed batch of the last round: finals after the last warmup... take the last 20 finals of each 25-group
n=int(sys.argv[2]) if len(sys.argv)>2 else 25
groups=[fin[i:i+n] for i in range(0,len(fin),n)]
for g in groups:
    t=g[5:]  # timed 20
    if len(t)<2: continue
    t0=int(t[0]["Start_Timestamp"]); t1=max(int(r["End_Timestamp"]) for r in t)
    iv=sorted((int(r["Start_Timestamp"]),int(r["End_Timestamp"])) for r in t)
    busy=0; cur=None
    for s,e in iv:
        if cur is None or s>cur[1]:
            if cur: busy+=cur[1]-cur[0]
            cur=[s,e]
        else: cur[1]=max(cur[1],e)
    busy+=cur[1]-cur[0]
    two=0
    # time with 2 finals concurrently
    ev=[]
    for s,e in iv: ev+= [(s,1),(e,-1)]
    ev.sort(); c=0; last=None
    for x,d in ev:
        if last is not None and c>=2: two+=x-last
        c+=d; last=x
    print("span %.1f us, any-final busy %.1f us (%.0f%%), two-finals %.1f us, per step %.1f"%((t1-t0)/1e3,busy/1e3,100*busy/(t1-t0),two/1e3,(t1-t0)/1e3/len(t)))
