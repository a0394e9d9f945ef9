"""profiles/<dir>/p{3,4}_counter_collection.csv -> profiles/attn_pmc.json (HBM bytes per prefill launch).

Corrections per MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE counts half the bytes of 16 B/lane streaming reads (double it), WRITE_SIZE is exact for
16 B/lane stores.  The PMC shape is tools/prof_attn.py's default (the IE-sweep attention launch).
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cram_amd.build import kernel_source_hash  # noqa: E402
from cram_amd.ops import prefill_work  # noqa: E402

src = sys.argv[1] if len(sys.argv) > 1 else "profiles/r01_pmc"
B, T, Hq, Hkv, d = 33, 962, 32, 8, 128


KERNELS = set()


def mean(name, f):
    import glob
    hits = [os.path.join(src, f)] if os.path.exists(os.path.join(src, f)) else \
        sorted(glob.glob(os.path.join(src, "**", f), recursive=True))
    rows = [r for r in csv.DictReader(open(hits[0])) if r["Counter_Name"] == name]
    KERNELS.update(r.get("Kernel_Name", "?") for r in rows)
    v = [float(r["Counter_Value"]) for r in rows]
    return sum(v) / len(v), len(v)


fetch_kib, n = mean("FETCH_SIZE", "p3_counter_collection.csv")
write_kib, _ = mean("WRITE_SIZE", "p4_counter_collection.csv")
read_b = fetch_kib * 1024 * 2
write_b = write_kib * 1024
_, alg = prefill_work(B, Hq, Hkv, T, T, d, 0)
out = {"kernel": " / ".join(sorted(KERNELS)), "shape": {"B": B, "T": T, "Hq": Hq, "Hkv": Hkv, "d": d}, "dispatches": n,
       "fetch_size_kib": fetch_kib, "write_size_kib": write_kib, "hbm_read_bytes": read_b, "hbm_write_bytes": write_b,
       "hbm_bytes_per_launch": read_b + write_b, "algorithmic_bytes_per_launch": alg,
       "traffic_over_algorithmic": (read_b + write_b) / alg,
       "source": os.path.relpath(os.path.abspath(src), os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
       "kernel_source_hash": kernel_source_hash(),
       "note": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes (tools/pmc_attn.sh); FETCH_SIZE x2 "
               "(gfx950 16B/lane read undercount), KiB -> B"}
json.dump(out, open("profiles/attn_pmc.json", "w"), indent=1)
print(json.dumps(out, indent=1))
