"""Leaf-stream (hardware queue 2) utilisation of each host nwc_sanitize_messages call in a
tools/trace_wire_host.sh trace: when the copies end, when k_finalize_messages ends, and the
queue's busy time (and how much of it is kernels under 20 us).
  python tools/wire_trace_queues.py TRACE_DIR"""
import csv, sys
d=sys.argv[1]
K=list(csv.DictReader(open(d+'/run_kernel_trace.csv')))
M=list(csv.DictReader(open(d+'/run_memory_copy_trace.csv')))
h=sorted((int(m['Start_Timestamp']),int(m['End_Timestamp'])) for m in M if m['Direction'].endswith('HOST_TO_DEVICE'))
calls=[];cur=[h[0]]
for e in h[1:]:
    if e[0]-cur[-1][1]>1.0e6: calls.append(cur);cur=[e]
    else: cur.append(e)
calls.append(cur)
calls=[c for c in calls if len(c)>=8]
ks=sorted((int(k['Start_Timestamp']),int(k['End_Timestamp']),k['Queue_Id'],k['Kernel_Name']) for k in K)
for c in calls:
    t0=c[0][0]; tl=c[-1][1]
    fin=[k for k in ks if 'finalize' in k[3] and k[0]>t0][0]
    q2=[k for k in ks if k[2]=='2' and t0<=k[0]<=fin[0]]
    busy=sum(k[1]-k[0] for k in q2)/1e3
    small=sum(k[1]-k[0] for k in q2 if k[1]-k[0]<20000)/1e3
    nsmall=sum(1 for k in q2 if k[1]-k[0]<20000)
    span=(fin[1]-q2[0][0])/1e3
    print('copies end %.0f, final end %.0f us; q2 span %.0f busy %.0f (small %d kernels %.0f us)'%((tl-t0)/1e3,(fin[1]-t0)/1e3,span,busy,nsmall,small))
