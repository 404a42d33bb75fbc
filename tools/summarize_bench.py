"""Print the headline numbers of a bench.py JSON line: python tools/summarize_bench.py bench.json"""
import json
import sys

d = json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
r = d["roofline"]
print(f"C2 {d['value']:.0f} img/s  {d['ms_per_step'] * 1e3:.2f} us/step  kernel {r['kernel_avg_launch_ms'] * 1e3:.2f} us"
      f"  frac {r['frac']:.3f}")
for k, v in d.get("extra", {}).items():
    if isinstance(v, dict) and "value" in v:
        print(f"{k} {v['value']:.0f} {v.get('unit', '')}  {v.get('ms_per_step', 0) * 1e3:.2f} us/step")
if "cpu_baseline" in d:
    print("cpu_baseline", round(d["cpu_baseline"]["value"]), d["cpu_baseline"]["sample"][:200])
