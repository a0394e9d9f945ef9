"""One line per bench JSON: value, decode questions/s, roofline fractions, CPU baselines.
   python tools/summ_bench.py gpurun_out/r04/cfg/*.json"""
import json
import sys

for fn in sys.argv[1:]:
    try:
        d = json.load(open(fn))
    except (OSError, ValueError) as e:
        print(f"{fn}: {e}")
        continue
    dec = d.get("decode") or {}
    lr = dec.get("leg_roofline") or {}
    ar = dec.get("attention_roofline") or {}
    cpu = d.get("cpu_baseline") or {}
    dcpu = dec.get("cpu_baseline") or {}
    roof = d.get("roofline") or {}
    print(f"{fn}: value {d.get('value')} {d.get('unit')} | roofline {roof.get('frac')} mfma_busy {roof.get('mfma_busy')} "
          f"| step {(d.get('step_roofline') or {}).get('frac')} | decode {round(dec.get('value', 0), 2)} q/s "
          f"B {dec.get('batch_per_gpu')} Q {dec.get('questions')} prefill {lr.get('prefill', {}).get('frac')} "
          f"steps {lr.get('steps', {}).get('frac')} ({lr.get('steps', {}).get('ms_per_step')} ms) attn {ar.get('frac')} "
          f"| cpu {cpu.get('value')} {cpu.get('unit')} | dec cpu {dcpu.get('value')} speedup {dec.get('speedup_vs_cpu')}")
