"""Summarise A/B bench lines (dev tool): value, ms/step, oracle agreement and class ms."""
import glob
import json
import sys

for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable", e)
        continue
    oc = d.get("oracle_check") or {}
    k = d.get("kernel_classes_ms_per_step") or {}
    keys = sys.argv[2].split(",") if len(sys.argv) > 2 else sorted(k)
    print("%-28s %9.1f %7.3f ms  oracle %-8s %s" % (
        f.split("/")[-1], d["value"], d["ms_per_step"], oc.get("chunks_identical_to_oracle"),
        " ".join("%s=%.3f" % (x, k.get(x, -1)) for x in keys)))
