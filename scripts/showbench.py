import json, sys
d = json.loads(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/b.log").read().strip().splitlines()[-1])
r = d.get("roofline") or {}
print(f"value {d['value']:.4g} msgs/s  ms/step {d['ms_per_step']}  frac {r.get('frac')}  dev_ms {r.get('broadcast_device_ms')}")
print("  total_ms", r.get("kernels_total_ms"), "redos", r.get("exact_redos"))
