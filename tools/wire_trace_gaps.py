"""Copy gaps of each host nwc_sanitize_messages call in a tools/trace_wire_host.sh trace:
per H2D copy "gap-before/duration" in us, and the kernel that ended just before a gap > 100 us.
  python tools/wire_trace_gaps.py TRACE_DIR"""
import csv, sys
d=sys.argv[1]
K=list(csv.DictReader(open(d+'/run_kernel_trace.csv')))
M=list(csv.DictReader(open(d+'/run_memory_copy_trace.csv')))
ks=sorted((int(k['Start_Timestamp']),int(k['End_Timestamp']),k['Queue_Id'],k['Kernel_Name'][:30]) for k in K)
h=sorted((int(m['Start_Timestamp']),int(m['End_Timestamp'])) for m in M if m['Direction'].endswith('HOST_TO_DEVICE'))
# split into calls: a gap > 0.8ms between copies; print per call copy durations and gaps
calls=[];cur=[h[0]]
for e in h[1:]:
    if e[0]-cur[-1][1]>1.0e6: calls.append(cur);cur=[e]
    else: cur.append(e)
calls.append(cur)
for c in calls:
    if len(c)<8: continue
    t0=c[0][0]
    s=[]
    for i,e in enumerate(c):
        gap=(e[0]-c[i-1][1])/1e3 if i else 0
        # kernel ending just before copy start
        prev=[k for k in ks if k[1]<=e[0] and k[1]>e[0]-80000]
        tag=('<'+prev[-1][3][5:18]+'@q'+prev[-1][2]) if gap>100 and prev else ''
        s.append('%.0f/%.0f%s'%(gap,(e[1]-e[0])/1e3,tag))
    tot=(c[-1][1]-t0)/1e6
    busy=sum(e[1]-e[0] for e in c)/1e6
    print('span %.3f busy %.3f :'%(tot,busy),' '.join(s))
