"""Instruction census of one kernel in a hipcc -S listing: MFMA / VALU / LDS / AGPR-move / scratch counts and the
register metadata (python3 tools/isa_stats.py file.s kernel_substring [--loop])."""
import re
import sys


def kernel_body(s, name):
    for m in re.finditer(r"^(_Z\w+):", s, re.M):
        if name in m.group(1):
            end = s.find(".Lfunc_end", m.end())
            return m.group(1), s[m.end():end]
    raise SystemExit(f"no kernel matching {name}")


def main():
    path, name = sys.argv[1], sys.argv[2]
    s = open(path).read()
    sym, body = kernel_body(s, name)
    lines = [ln.strip() for ln in body.splitlines() if ln.strip() and not ln.strip().startswith((";", "."))]
    cnt = lambda pat: sum(1 for ln in lines if re.match(pat, ln))
    print(sym)
    print(f"  instructions {len(lines)}  mfma {cnt(r'v_mfma')}  accvgpr {cnt(r'v_accvgpr')}  "
          f"valu {cnt(r'v_(?!mfma|accvgpr)')}  exp {cnt(r'v_exp')}  ds {cnt(r'ds_')}  "
          f"buffer/global {cnt(r'(buffer|global)_')}  scratch {cnt(r'scratch_')}  s_nop {cnt(r's_nop')}  "
          f"waitcnt {cnt(r's_waitcnt')}  barrier {cnt(r's_barrier')}  v_mov {cnt(r'v_mov')}")
    meta = s[s.find(f".amdhsa_kernel {sym}"):]
    for k in (".amdhsa_next_free_vgpr", ".amdhsa_accum_offset", ".amdhsa_next_free_sgpr",
              ".amdhsa_private_segment_fixed_size"):
        m = re.search(re.escape(k) + r"\s+(\d+)", meta)
        if m:
            print(f"  {k} {m.group(1)}")
    for k in (".vgpr_count", ".agpr_count", ".vgpr_spill_count", ".sgpr_spill_count"):
        i = s.find(f".name:           {sym}")
        blk = s[s.rfind("  - .agpr_count", 0, i) if i > 0 else 0: i]
        m = re.search(re.escape(k) + r":\s+(\d+)", blk)
        if m:
            print(f"  {k} {m.group(1)}")


if __name__ == "__main__":
    main()
