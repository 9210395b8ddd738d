"""MFMA utilisation per kernel class from one rocprofv3 PMC pass
(--pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE):

    util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 4 * CUs)

SQ_VALU_MFMA_BUSY_CYCLES is summed over every SIMD (32 cycles per 32x32x16 bf16 MFMA);
GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md, PMC units / DVFS notes), so
GRBM_GUI_ACTIVE / 8 is the dispatch's length in clock cycles and 4 x 256 SIMDs could each be
busy for all of it.

    python tools/pmc_mfma.py counter_collection.csv [--classes enc_gemm,joiner,search_step]
"""
import argparse
import collections
import csv
import json

from pmc_traffic import in_class

CUS = 256


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--classes", default="enc_gemm,ffn_fused,attn,joiner,search_step,greedy_spec")
    a = ap.parse_args()
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), r["Kernel_Name"])
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
            names[key] = r["Kernel_Name"]
    out = {}
    for cls in a.classes.split(","):
        busy = active = 0.0
        n = 0
        for key, c in per.items():
            if in_class(names[key], cls) and "GRBM_GUI_ACTIVE" in c:
                busy += c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
                active += c["GRBM_GUI_ACTIVE"]
                n += 1
        if n:
            out[cls] = {"dispatches": n, "mfma_busy_cycles": busy,
                        "cycles_per_dispatch": round(active / 8 / n, 1),
                        "mfma_util": round(busy / (active / 8 * 4 * CUS), 4)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
