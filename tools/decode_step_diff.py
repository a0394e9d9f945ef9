"""Per-step kernel breakdown of the graph-replayed decode step from two rocprofv3 --stats runs of
tools/prof_generate.py that differ only in --new: everything else (session setup, packed prefill, graph capture) is the
same work in both, so (kernel time of run B - run A) / (reps x (new_B - new_A)) is that kernel's time per step.

  python tools/decode_step_diff.py <dir A> <new A> <dir B> <new B> [reps]
"""
import csv
import glob
import sys


def stats(d):
    path = sorted(glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True))[0]
    out = {}
    for r in csv.DictReader(open(path)):
        n = r["Name"]
        t, c = out.get(n, (0.0, 0))
        out[n] = (t + float(r["TotalDurationNs"]), c + int(r["Calls"]))
    return out


def short(name):
    for key in ("gemm_w4_kernel", "gemm_sm_kernel", "gemm_combine_kernel", "gemm_tn_kernel", "gemm_splitk", "decode_mfma",
                "decode_kernel", "decode_combine", "rmsnorm", "rope", "silu_mul", "answer", "Cijk", "argmax", "elementwise",
                "reduce", "index", "copy", "fill"):
        if key in name:
            return key + ("" if key != "gemm_w4_kernel" else name[name.find("Li"):name.find("EEEv")])
    return name[:60]


def main():
    a, na, b, nb = sys.argv[1], int(sys.argv[2]), sys.argv[3], int(sys.argv[4])
    reps = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    sa, sb = stats(a), stats(b)
    steps = reps * (nb - na)
    rows = []
    for n in set(sa) | set(sb):
        dt = sb.get(n, (0.0, 0))[0] - sa.get(n, (0.0, 0))[0]
        dc = sb.get(n, (0.0, 0))[1] - sa.get(n, (0.0, 0))[1]
        if dc > 0 or abs(dt) > 1e3 * steps:
            rows.append((dt / steps / 1e3, dc / steps, short(n)))
    rows.sort(reverse=True)
    tot = sum(r[0] for r in rows)
    print(f"per decode step ({steps} steps differenced): {tot / 1e3:.3f} ms of kernel time")
    for us, calls, n in rows:
        print(f"  {us:9.1f} us  {calls:6.1f} launches  {100 * us / tot:5.1f} %  {n}")


if __name__ == "__main__":
    main()
