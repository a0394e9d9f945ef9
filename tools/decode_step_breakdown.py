"""Per-step kernel breakdown of the graph-replayed decode steps from a rocprofv3 kernel trace of one batched
generate (tools/prof_generate.py): every dispatch from the first decode attention kernel on belongs to the steps;
prints, per kernel name, dispatches per step and microseconds per step, and the steps' total.
  python tools/decode_step_breakdown.py <dir with *_kernel_trace.csv> [num_layers]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
L = int(sys.argv[2]) if len(sys.argv) > 2 else 32
path = sorted(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True))[0]
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
is_att = lambda name: "decode_mfma_kernel" in name or "decode_kernel<" in name or "decode_kernelI" in name
# the packed prefill's last layer also runs the decode attention (one call per chunk); its projections run on
# gemm_w4_kernel's RoPE / residual epilogues (Li102 / Li101), which the steps never use (at >= 512 rows a step does run
# the 4-wave kernel, for gate/up + SiLU-mul and lm_head): the steps start at the first decode attention after the last
# of those dispatches
last_w4 = max([i for i, r in enumerate(rows) if "gemm_w4_kernel" in r["Kernel_Name"]
               and ("Li101" in r["Kernel_Name"] or "Li102" in r["Kernel_Name"])], default=-1)
first = next(i for i, r in enumerate(rows) if i > last_w4 and is_att(r["Kernel_Name"]))
steps_rows = rows[first:]
n_att = sum(1 for r in steps_rows if is_att(r["Kernel_Name"]))
n_steps = max(1, n_att // L)
tot = collections.defaultdict(float)
cnt = collections.Counter()
for r in steps_rows:
    name = r["Kernel_Name"]
    short = (name.split("(")[1] if name.startswith("void (") else name.split("(")[0])[:90]
    tot[short] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    cnt[short] += 1
span = (int(steps_rows[-1]["End_Timestamp"]) - int(steps_rows[0]["Start_Timestamp"])) / 1e3 / n_steps
busy = sum(tot.values()) / n_steps
print(f"{path}: {n_steps} steps; per step: wall span {span:.0f} us, kernel time {busy:.0f} us "
      f"(gaps {span - busy:.0f} us)")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"  {v / n_steps:9.1f} us  {cnt[k] / n_steps:6.1f}/step  {k}")
