"""Per-call device timeline from a rocprofv3 kernel (+ memory-copy) trace: each
k_match_fused launch opens a call; prints every op of the last calls with its
start relative to the call's first op, and the idle time before each call."""
import csv
import glob
import sys

d = sys.argv[1]
ops = []
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
for f in glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "")))
ops.sort()
starts = [i for i, o in enumerate(ops) if "k_match_fused" in o[2]]
# a call begins with the ops just before its k_match_fused that follow the previous call's end
for c, i in enumerate(starts[-4:]):
    j = i
    while j > 0 and ops[j - 1][0] > ops[i][0] - 2_000_000 and "k_assemble" not in ops[j - 1][2] and "copy" not in ops[j - 1][2]:
        j -= 1
    k = i
    nxt = starts[starts.index(i) + 1] if starts.index(i) + 1 < len(starts) else len(ops)
    t0 = ops[j][0]
    prev_end = ops[j - 1][1] if j > 0 else t0
    print("call: idle before %.1f us" % ((t0 - prev_end) / 1e3))
    for o in ops[j:nxt]:
        if "k_match_fused" in o[2] or o is ops[j] or True:
            print("  %9.1f %9.1f  %s" % ((o[0] - t0) / 1e3, (o[1] - o[0]) / 1e3, o[2]))
        if o[2].startswith("copy") and o[1] - t0 > 5e6:
            break
