"""Idle time between kernels in a rocprofv3 kernel trace (one GPU, one queue of work): total gap, a histogram of gap
sizes, and the largest gaps with the kernels on either side (where the host, not the GPU, set the pace).
  python tools/trace_gaps.py <dir with *_kernel_trace.csv> [top=25]"""
import csv
import glob
import sys

d = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
path = sorted(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True))[0]
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]) for r in rows]
busy_end = ev[0][1]
gaps = []
for i in range(1, len(ev)):
    s, e, n = ev[i]
    if s > busy_end:
        gaps.append((s - busy_end, i))
    busy_end = max(busy_end, e)
span = busy_end - ev[0][0]
tot = sum(g for g, _ in gaps)
print(f"{path}: {len(ev)} kernels over {span / 1e6:.1f} ms; idle {tot / 1e6:.1f} ms ({100 * tot / span:.2f} %) in "
      f"{len(gaps)} gaps")
for lo, hi in ((0, 2e3), (2e3, 10e3), (10e3, 100e3), (100e3, 1e6), (1e6, 1e12)):
    sel = [g for g, _ in gaps if lo <= g < hi]
    print(f"  gaps {lo / 1e3:>7.0f}-{hi / 1e3:<9.0f} us: {len(sel):6d}  total {sum(sel) / 1e6:8.2f} ms")
for g, i in sorted(gaps, reverse=True)[:top]:
    print(f"  {g / 1e3:9.1f} us  after {ev[i - 1][2]}  before {ev[i][2]}  (t = {(ev[i][0] - ev[0][0]) / 1e6:.1f} ms)")
