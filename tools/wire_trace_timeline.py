"""Per-call kernel timeline of nwc_sanitize_messages in a tools/trace_wire_host.sh trace: t = 0 at
the call's first H2D copy of message bytes; every kernel's queue, start, end (us) and name, and
when the last copy landed.
  python tools/wire_trace_timeline.py TRACE_DIR [CALL_INDEX]"""
import csv
import sys

d = sys.argv[1]
want = int(sys.argv[2]) if len(sys.argv) > 2 else -1
K = list(csv.DictReader(open(d + "/run_kernel_trace.csv")))
M = list(csv.DictReader(open(d + "/run_memory_copy_trace.csv")))
h = sorted((int(m["Start_Timestamp"]), int(m["End_Timestamp"]), int(m.get("Size", 0) or 0)) for m in M
           if m["Direction"].endswith("HOST_TO_DEVICE"))
calls, cur = [], [h[0]]
for e in h[1:]:
    if e[0] - cur[-1][1] > 1.0e6:
        calls.append(cur)
        cur = [e]
    else:
        cur.append(e)
calls.append(cur)
calls = [c for c in calls if len(c) >= 8]
ks = sorted((int(k["Start_Timestamp"]), int(k["End_Timestamp"]), k["Queue_Id"], k["Kernel_Name"]) for k in K)
sel = [calls[want]] if want >= 0 else calls
for ci, c in enumerate(sel):
    t0, tl = c[0][0], c[-1][1]
    nxt = calls[calls.index(c) + 1][0][0] if calls.index(c) + 1 < len(calls) else float("inf")
    fin = [k for k in ks if "finalize" in k[3] and t0 < k[0] < nxt]
    tend = fin[0][1] if fin else tl
    print("call: %d copies, last copy lands %.0f us, k_finalize_messages ends %.0f us" % (len(c), (tl - t0) / 1e3, (tend - t0) / 1e3))
    for k in ks:
        if t0 - 2e5 <= k[0] <= tend:
            print("  q%-3s %8.0f .. %8.0f (%6.0f)  %s" % (k[2], (k[0] - t0) / 1e3, (k[1] - t0) / 1e3, (k[1] - k[0]) / 1e3,
                                                     k[3].split("(")[0].replace("void ", "")[:56]))
