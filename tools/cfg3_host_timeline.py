"""Per-call timeline of nwc_verify_batch_many in a tools/trace_cfg3_host.sh trace: t = 0 at the
call's first H2D copy; H2D copies summarised (count, bytes, last end), every kernel listed.
  python tools/cfg3_host_timeline.py TRACE_DIR"""
import csv
import sys

d = sys.argv[1]
K = list(csv.DictReader(open(d + "/run_kernel_trace.csv")))
M = list(csv.DictReader(open(d + "/run_memory_copy_trace.csv")))
h = sorted((int(m["Start_Timestamp"]), int(m["End_Timestamp"]), int(m.get("Size", 0) or 0)) for m in M
           if m["Direction"].endswith("HOST_TO_DEVICE"))
calls, cur = [], [h[0]]
for e in h[1:]:
    if e[0] - cur[-1][1] > 2.0e6:
        calls.append(cur)
        cur = [e]
    else:
        cur.append(e)
calls.append(cur)
calls = [c for c in calls if sum(x[1] - x[0] for x in c) > 5e6]   # > 5 ms of copies (no byte counts in the trace)
ks = sorted((int(k["Start_Timestamp"]), int(k["End_Timestamp"]), k["Queue_Id"], k["Kernel_Name"]) for k in K)
for ci, c in enumerate(calls):
    t0, tl = c[0][0], c[-1][1]
    nxt = calls[ci + 1][0][0] if ci + 1 < len(calls) else float("inf")
    kk = [k for k in ks if t0 - 1e5 <= k[0] < nxt and k[0] < tl + 30e6]
    end = max(k[1] for k in kk) if kk else tl
    print("call: %d H2D copies, last lands %.0f us, last kernel ends %.0f us" % (len(c), (tl - t0) / 1e3, (end - t0) / 1e3))
    for k in kk:
        if k[1] - k[0] >= 20000 or "verify" in k[3]:
            print("  q%-3s %8.0f .. %8.0f (%6.0f)  %s" % (k[2], (k[0] - t0) / 1e3, (k[1] - t0) / 1e3, (k[1] - k[0]) / 1e3,
                                                     k[3].split("(")[0].replace("void ", "")[:60]))
