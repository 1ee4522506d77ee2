"""One bench step's kernel timeline from a rocprofv3 --kernel-trace CSV: every
dispatch between two k_reset launches (start offset, duration, gap to the
previous end, queue, name) and the step's non-ingest kernel time.
Usage: step_timeline.py <run_kernel_trace.csv>"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
resets=[i for i,r in enumerate(rows) if 'k_reset' in r['Kernel_Name']]
a,b=resets[-3],resets[-2]
t0=int(rows[a]['Start_Timestamp']); prev_end=t0
tot=0
for r in rows[a:b+1]:
    s=int(r['Start_Timestamp']); e=int(r['End_Timestamp'])
    print("%8.1f %8.1f  gap %6.1f  q%s %s"%((s-t0)/1e3,(e-s)/1e3,(s-prev_end)/1e3, r['Queue_Id'], r['Kernel_Name'][:60]))
    if 'k_ingest_small' not in r['Kernel_Name'] and r is not rows[b]: tot+=(e-s)
    prev_end=max(prev_end,e)
print("non-ingest kernel time %.1f us"%(tot/1e3))
