"""rocprofv3 PMC passes of the IE-sweep attention launch -> profiles/attn_pmc.json, or (--gemm) of the sweep's
dominant GEMM launch (gemm_w4_kernel, gate/up + SiLU-mul at M = 29,184; tools/pmc_gemm.sh) -> profiles/gemm_pmc.json.

Input: the directory tools/pmc_attn.sh wrote (p1..p5/p*_counter_collection.csv, one --pmc pass each, kernel-trace
only), or a directory holding them further down.  Output: what the north star asks rocprof to report for the
attention kernel — achieved HBM GB/s and MFMA utilisation against the gfx950 peak — plus the issue statistics,
tied to the kernel source hash of the build the passes ran on (bench.py copies them into its `roofline` only
when the running build hashes the same).

Corrections and units (MI355X_MICROARCH.md, HBM / rocprofv3 and the PMC-units row):
  * FETCH_SIZE / WRITE_SIZE are KiB; on gfx950 FETCH_SIZE counts half the bytes of 16 B/lane streaming reads
    (doubled here); WRITE_SIZE is exact for 16 B/lane stores;
  * GRBM_GUI_ACTIVE is summed over the 8 XCDs: kernel clock cycles = GRBM_GUI_ACTIVE / 8, effective clock =
    that / the dispatch's wall time (its Start/End timestamps in the same CSV);
  * SQ_VALU_MFMA_BUSY_CYCLES counts matrix-pipe cycles summed over the SIMDs (32 per v_mfma_f32_32x32x16_bf16), so
    mfma_busy = MFMA_BUSY / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs) = the fraction of SIMD-cycles the matrix pipe works;
  * MFMA issues x 32768 FLOP against the launch's algorithmic FLOPs counts the masked work that is still issued
    (half-masked diagonal blocks, the 32-key rounding of each block's last key).
"""
import collections
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from cram_amd.build import gemm_source_hash, kernel_source_hash  # noqa: E402
from cram_amd.ops import prefill_work  # noqa: E402

GEMM = "--gemm" in sys.argv or "--lt" in sys.argv
LT = "--lt" in sys.argv          # hipBLASLt's kernel for the same [gate; up] product (MODE=lt tools/pmc_gemm.sh)
ARGS = [a for a in sys.argv[1:] if a not in ("--gemm", "--lt")]
B, T, Hq, Hkv, d = 33, 962, 32, 8, 128          # tools/prof_attn.py's default: the IE sweep's attention launch
GM, GN, GK = 29184, 28672, 4096                  # tools/gemm_pmc.py: gate/up (+ SiLU-mul, output N / 2 wide)
SIMDS = 1024                                     # 256 CUs x 4 SIMDs
XCDS = 8
# FLOP per MFMA instruction: v_mfma_f32_32x32x16_bf16 (attention) / v_mfma_f32_16x16x32_bf16 (GEMM)
MFMA_FLOP = 16 * 16 * 32 * 2 if GEMM else 32 * 32 * 16 * 2
PEAK_TFLOPS, PEAK_GBS = 2500.0, 8000.0           # dense bf16 MFMA, HBM3E (MI355X_MICROARCH.md chip table)


def load(src):
    """{counter: [(value, duration_ns), ...]} over every dispatch of the attention kernel in every pass."""
    files = sorted(glob.glob(os.path.join(src, "**", "p*_counter_collection.csv"), recursive=True))
    if not files:
        raise SystemExit(f"no p*_counter_collection.csv under {src}")
    out = collections.defaultdict(list)
    kernels = set()
    for fn in files:
        for r in csv.DictReader(open(fn)):
            kernels.add(r.get("Kernel_Name", "?"))
            dur = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
            out[r["Counter_Name"]].append((float(r["Counter_Value"]), dur))
    return out, kernels


def mean(rows, what=0):
    return sum(x[what] for x in rows) / len(rows)


def main():
    src = ARGS[0] if ARGS else ("gpurun_out/gemm_pmc" if GEMM else "gpurun_out/pmc")
    dst = ARGS[1] if len(ARGS) > 1 else os.path.join(REPO, "profiles", "gemm_pmc.json" if GEMM else "attn_pmc.json")
    c, kernels = load(src)
    if GEMM:
        flops, alg_bytes = 2.0 * GM * GN * GK, 2.0 * (GM * GK + GN * GK + GM * (GN if LT else GN // 2))
    else:
        flops, alg_bytes = prefill_work(B, Hq, Hkv, T, T, d, 0)
    read_b = mean(c["FETCH_SIZE"]) * 1024 * 2
    write_b = mean(c["WRITE_SIZE"]) * 1024
    traffic = read_b + write_b
    # wall time per dispatch under the traffic passes (counters of those passes do not slow the kernel measurably)
    t_traffic = (mean(c["FETCH_SIZE"], 1) + mean(c["WRITE_SIZE"], 1)) / 2 * 1e-9
    grbm = mean(c["GRBM_GUI_ACTIVE"])
    t_grbm = mean(c["GRBM_GUI_ACTIVE"], 1) * 1e-9
    cycles = grbm / XCDS
    clock_ghz = cycles / t_grbm / 1e9
    mfma_busy = mean(c["SQ_VALU_MFMA_BUSY_CYCLES"]) / (cycles * SIMDS)
    n_mfma = mean(c["SQ_INSTS_MFMA"])
    out = {
        "kernel": " / ".join(sorted(kernels)),
        "shape": ({"M": GM, "N": GN, "K": GK, "epilogue": "store (hipBLASLt F.linear)" if LT else "SiLU-mul"} if GEMM else
                  {"B": B, "T": T, "Hq": Hq, "Hkv": Hkv, "d": d}),
        "dispatches": len(c["FETCH_SIZE"]),
        "fetch_size_kib": mean(c["FETCH_SIZE"]), "write_size_kib": mean(c["WRITE_SIZE"]),
        "hbm_read_bytes": read_b, "hbm_write_bytes": write_b, "hbm_bytes_per_launch": traffic,
        "algorithmic_bytes_per_launch": alg_bytes, "traffic_over_algorithmic": traffic / alg_bytes,
        "avg_launch_ms_under_pmc": round(t_traffic * 1e3, 4),
        "hbm_gbs": round(traffic / t_traffic / 1e9, 1),
        "hbm_frac": round(traffic / t_traffic / 1e9 / PEAK_GBS, 4),
        "tflops": round(flops / t_traffic / 1e12, 1),
        "mfma_frac_of_peak": round(flops / t_traffic / 1e12 / PEAK_TFLOPS, 4),
        "mfma_busy": round(mfma_busy, 4),
        "effective_clock_ghz": round(clock_ghz, 3),
        "valu_per_mfma": round(mean(c["SQ_INSTS_VALU"]) / n_mfma, 2),
        "mfma_issues_over_algorithmic": round(n_mfma * MFMA_FLOP / flops, 4),
        "wait_any_frac": round(mean(c["SQ_WAIT_ANY"]) / mean(c["SQ_WAVE_CYCLES"]), 4),
        "lds_bank_conflict_per_lds_inst": round(mean(c["SQ_LDS_BANK_CONFLICT"]) / mean(c["SQ_INSTS_LDS"]), 4),
        "source": os.path.relpath(os.path.abspath(src), REPO),
        "kernel_source_hash": None if LT else (gemm_source_hash() if GEMM else kernel_source_hash()),
        "note": (f"rocprofv3 --pmc in separate passes (tools/{'pmc_gemm' if GEMM else 'pmc_attn'}.sh). traffic: "
                 "FETCH_SIZE x2 (gfx950 16 B/lane "
                 "read undercount) + WRITE_SIZE, KiB -> B; hbm_gbs / tflops: over the dispatches' own wall time; "
                 "mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs); effective clock = "
                 f"GRBM_GUI_ACTIVE / 8 / wall; mfma issues x {MFMA_FLOP} FLOP / algorithmic FLOPs"),
    }
    if "TCC_EA0_RDREQ_128B_sum" in c:
        # request-size passes (EXTRA=1 tools/pmc_gemm.sh): beyond-L2 read bytes counted from the requests themselves
        n32, n64, n128 = (mean(c[f"TCC_EA0_RDREQ_{w}B_sum"]) for w in (32, 64, 128))
        req_b = 32 * n32 + 64 * n64 + 128 * n128
        out["rdreq_bytes"] = req_b
        out["rdreq_counts"] = {"all": mean(c["TCC_EA0_RDREQ_sum"]), "32B": n32, "64B": n64, "128B": n128}
        out["rdreq_bytes_over_fetch_size_x2"] = round(req_b / read_b, 4)
        out["traffic_by_request_sizes_over_algorithmic"] = round((req_b + write_b) / alg_bytes, 4)
        if "TCC_EA0_RDREQ_DRAM_32B_sum" in c:
            out["rdreq_dram_bytes"] = 32 * mean(c["TCC_EA0_RDREQ_DRAM_32B_sum"])
            out["rdreq_gmi_bytes"] = 32 * mean(c["TCC_EA0_RDREQ_GMI_32B_sum"])
            out["tcc_bubble_128B"] = mean(c["TCC_BUBBLE_sum"])
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
