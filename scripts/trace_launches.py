"""Per-launch durations, in order, of one kernel in a rocprofv3 --kernel-trace
CSV (the clock/power transients across a bench run).
usage: python scripts/trace_launches.py run_kernel_trace.csv [kernel_substring]"""
import csv
import sys

path = sys.argv[1]
name = sys.argv[2] if len(sys.argv) > 2 else "chroma_kernel"
rows = [r for r in csv.DictReader(open(path)) if name in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
prev = None
print(f"{len(rows)} launches of {name}")
print(f"{'t (ms)':>9} {'dur (us)':>9} {'gap (us)':>9}")
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e6:9.3f} {(e - s) / 1e3:9.1f} {((s - prev) / 1e3 if prev else 0):9.1f}")
    prev = e
