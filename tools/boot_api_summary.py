"""Kernel-activity gaps and slow HIP API calls over tools/boot_prof.py's run (three bootstrap
calls; the first pays the first-call costs): every idle gap > 1 ms between kernels and every API
call > 0.5 ms, in time order, relative to the first kernel."""
import csv, glob, sys

d = sys.argv[1]
kt = [r for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True) for r in csv.DictReader(open(f))]
at = [r for f in glob.glob(d + "/**/*hip_api_trace.csv", recursive=True) for r in csv.DictReader(open(f))]
kt.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(kt[0]["Start_Timestamp"])
ev = []
mx = t0
for r in kt:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s > mx + 1e6:
        ev.append((mx, f"GAP {(s - mx) / 1e6:8.2f} ms before {r['Kernel_Name'][:60]}"))
    mx = max(mx, e)
by_corr = {r.get("Correlation_Id"): r["Kernel_Name"] for r in kt}
for r in at:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if e - s > 5e5 and s >= t0 - 1e9:
        k = by_corr.get(r.get("Correlation_Id"), "")
        ev.append((s, f"API {r['Function']:28s} {(e - s) / 1e6:8.2f} ms {k[:70]}"))
ev.sort()
for t, m in ev:
    print(f"{(t - t0) / 1e6:10.1f} ms  {m}")
print(f"kernels {len(kt)}, end {(mx - t0) / 1e6:.1f} ms")
