"""Per-call timeline of nwc_verify_strict_many in a tools/trace_strict_host.sh trace: the call's
first H2D copy is t = 0; every verification kernel's queue, start and end (us), the copies' end,
and the D2H verdict copy's end.
  python tools/strict_trace_timeline.py TRACE_DIR"""
import csv
import sys

d = sys.argv[1]
K = list(csv.DictReader(open(d + "/run_kernel_trace.csv")))
M = list(csv.DictReader(open(d + "/run_memory_copy_trace.csv")))
h2d = sorted((int(m["Start_Timestamp"]), int(m["End_Timestamp"])) for m in M if m["Direction"].endswith("HOST_TO_DEVICE"))
d2h = sorted((int(m["Start_Timestamp"]), int(m["End_Timestamp"])) for m in M if m["Direction"].endswith("DEVICE_TO_HOST"))
calls, cur = [], [h2d[0]]
for e in h2d[1:]:
    if e[0] - cur[-1][1] > 1.5e6:
        calls.append(cur)
        cur = [e]
    else:
        cur.append(e)
calls.append(cur)
calls = [c for c in calls if sum(b - a for a, b in c) > 1e6]   # the large calls (> 1 ms of copies)
ks = sorted((int(k["Start_Timestamp"]), int(k["End_Timestamp"]), k["Queue_Id"], k["Kernel_Name"]) for k in K)
for ci, c in enumerate(calls):
    t0, tc = c[0][0], c[-1][1]
    t_next = calls[ci + 1][0][0] if ci + 1 < len(calls) else float("inf")
    vk = [k for k in ks if t0 <= k[0] < min(tc + 20e6, t_next) and "k_verify" in k[3]]
    end = max(k[1] for k in vk)
    dh = [x for x in d2h if x[0] >= end - 1000][:1]
    print("call: %d H2D copies over %.0f us; last kernel ends %.0f us, D2H ends %.0f us" % (
        len(c), (tc - t0) / 1e3, (end - t0) / 1e3, ((dh[0][1] if dh else end) - t0) / 1e3))
    for k in vk:
        print("  q%-3s %8.0f .. %8.0f  (%6.0f us)  %s" % (k[2], (k[0] - t0) / 1e3, (k[1] - t0) / 1e3, (k[1] - k[0]) / 1e3,
                                                       k[3].split("(")[0][:60]))
