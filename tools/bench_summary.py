"""One line per bench.py result line: value, roofline frac, kernel ms (python tools/bench_summary.py f.json)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"headline {d['value']:.4g} {d['unit']} ms/step {d['ms_per_step']:.3f} frac {r['frac']:.3f} "
      f"exec {r.get('executed_frac', 0):.3f} kernel_ms {r['kernel_avg_ms']:.3f} ess/s {d['ess_per_s']:.3g}")
for k, v in d.get("secondary", {}).items():
    rr = v.get("roofline", {})
    cb = (v.get("cpu_baseline") or {}).get("value")
    print(f"{k}: {v['value']:.4g} {v.get('unit')} ms/step {v['ms_per_step']:.3f} frac {rr.get('frac')} "
          f"kernel {rr.get('kernel')} {rr.get('kernel_avg_ms')} cpu {cb}")
