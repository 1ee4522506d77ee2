"""Host HIP API calls of one bench step from a rocprofv3 --runtime-trace run
(scripts/gpu_r04r.sh): per call name, count and total host time inside the
last timed step, beside the step's kernels.  Usage: api_step.py DIR"""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
kt = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
at = glob.glob(d + "/**/*hip_api_trace.csv", recursive=True)[0]
ks = sorted(csv.DictReader(open(kt)), key=lambda r: int(r["Start_Timestamp"]))
resets = [i for i, r in enumerate(ks) if r["Kernel_Name"].startswith("k_reset")]
t0, t1 = int(ks[resets[-2]]["Start_Timestamp"]), int(ks[resets[-1]]["Start_Timestamp"])
print("step: %.1f us (k_reset to k_reset)" % ((t1 - t0) / 1e3))
api = [r for r in csv.DictReader(open(at))]
# the host calls that enqueued this step: those ending between the previous
# step's enqueue and this one's -- approximate with a window of one step
# ending at the first kernel of the step
agg = defaultdict(lambda: [0, 0.0])
sel = [r for r in api if t0 - (t1 - t0) <= int(r["Start_Timestamp"]) < t0]
for r in sel:
    a = agg[r["Function"]]
    a[0] += 1
    a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
tot = sum(v[1] for v in agg.values())
print("host HIP API in the step window: %d calls, %.1f us" % (len(sel), tot))
for k, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
    print("  %-40s %4d  %8.1f us" % (k, n, us))
