"""HIP API calls of the last match calls in a rocprofv3 --hip-runtime-trace: each call
is delimited by the k_match_fused launch; prints API name, start offset and duration (us)."""
import csv
import glob
import sys

d = sys.argv[1]
api = []
for f in glob.glob(d + "/**/*hip_api_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        api.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"], r.get("Thread_Id", "")))
api.sort()
kern = []
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_match_fused" in r["Kernel_Name"]:
            kern.append(int(r["Start_Timestamp"]))
kern.sort()
# the launch API call of each k_match_fused: the last hipLaunchKernel / hipModuleLaunchKernel before it starts
launches = [i for i, a in enumerate(api) if "Launch" in a[2]]
if len(kern) < 3:
    sys.exit("too few calls")
for c in range(len(kern) - 3, len(kern) - 1):
    t0 = kern[c] - 400_000  # 400 us before this call's walk starts
    t1 = kern[c + 1]
    print("=== call %d" % c)
    for a in api:
        if t0 <= a[0] < t1 and (a[1] - a[0]) >= 500:
            print("  %9.1f %8.1f  %s" % ((a[0] - kern[c]) / 1e3, (a[1] - a[0]) / 1e3, a[2]))
    tot = {}
    for a in api:
        if kern[c] <= a[0] < t1:
            tot[a[2]] = tot.get(a[2], 0) + (a[1] - a[0])
    print("  totals between walk starts:", {k: round(v / 1e3, 1) for k, v in sorted(tot.items(), key=lambda x: -x[1])[:12]})
