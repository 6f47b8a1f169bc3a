"""Print the headline figures of a bench.py JSON line (the last line of a log)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"value {d['value']:.4g} img/s  {d['ms_per_step']:.4f} ms/step  {r['kernel']} frac {r['frac']:.3f} "
      f"avg {r['avg_launch_us']:.1f} us  traffic {r['traffic']}  serial {d.get('serial_images_per_s')}")
print("breakdown", json.dumps(d["breakdown"]))
for k, v in (d.get("other_configs") or {}).items():
    r = v["roofline"]
    print(f"{k}: {v['value']:.4g} img/s {v['ms_per_step']:.3f} ms/step {r['kernel']} frac {r['frac']:.3f} "
          f"avg {r['avg_launch_us']:.1f} us traffic {r['traffic']} cpu {(v.get('cpu_baseline') or {}).get('value')}")
    print("   ", json.dumps(v["breakdown"].get("factor_kernels")))
for n, e in (d.get("eig") or {}).items():
    if n != "cpu_baseline":
        print(f"eig {n}: {e['ms']:.2f} ms ({e['roofline']['achieved']} GB/s) cpu {e.get('cpu_baseline_ms')}")
print("cpu", (d.get("cpu_baseline") or {}).get("value"), (d.get("cpu_baseline") or {}).get("cores"))
