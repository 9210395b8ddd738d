"""Per-kernel SQ / LDS utilisation from rocprofv3 PMC passes (counter_collection.csv files of
separate --pmc runs of the same command), aggregated over every dispatch of each kernel
whose name contains one of the given substrings.

    python tools/pmc_kernels.py passA.csv passB.csv --kernels "attn_flash_kernel<0,..."

Normalisation (MI355X: 256 CUs x 4 SIMDs; GRBM_GUI_ACTIVE is summed over the 8 XCDs, so
GRBM_GUI_ACTIVE / 8 is a dispatch's length in clock cycles; the SQ_ACTIVE_* / SQ_WAIT_* /
SQ_WAVE_CYCLES counters are wave quad-cycles summed over the SIMDs):

  valu_busy   = 4 SQ_ACTIVE_INST_VALU / (cycles x 1024)   share of SIMD cycles in VALU work
  mfma_busy   = SQ_VALU_MFMA_BUSY_CYCLES / (cycles x 1024)
  lds_busy    = 4 SQ_ACTIVE_INST_LDS / (cycles x 1024)
  lds_bw      = 64 (SQ_INSTS_LDS_LOAD_BANDWIDTH + ..._STORE_BANDWIDTH) / (cycles x 256 x 128 B)
                (LDS bytes moved per CU cycle against 128 B / clk)
  lds_wait    = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES          share of wave time waiting to issue LDS
  bank_confl  = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  valu_per_wave, lds_per_wave, mfma_per_wave = instruction counts / SQ_WAVES
"""
import argparse
import collections
import csv
import json

CUS, SIMDS = 256, 1024


def load(paths):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for p in paths:
        with open(p) as f:
            for r in csv.DictReader(f):
                did = r.get("Dispatch_Id") or r.get("Correlation_Id")
                key = (p, did)
                per[key][r["Counter_Name"]] += float(r["Counter_Value"])
                names[key] = r["Kernel_Name"]
    return per, names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--kernels", required=True, help="comma-separated name substrings")
    a = ap.parse_args()
    per, names = load(a.csv)
    out = {}
    for pat in a.kernels.split(","):
        tot = collections.defaultdict(float)
        cyc = collections.defaultdict(float)  # GRBM cycles per pass file
        n = collections.Counter()
        for key, c in per.items():
            if pat not in names[key]:
                continue
            n[key[0]] += 1
            for k, v in c.items():
                tot[k] += v
            cyc[key[0]] += c.get("GRBM_GUI_ACTIVE", 0.0) / 8

        def cycles_for(counter):
            # the pass file a counter came from (each pass has its own dispatch lengths)
            for key, c in per.items():
                if pat in names[key] and counter in c:
                    return cyc[key[0]]
            return 0.0

        def ratio(num, den):
            return round(num / den, 4) if den else None

        r = {"dispatches_per_pass": dict(n)}
        if "SQ_ACTIVE_INST_VALU" in tot:
            r["valu_busy"] = ratio(4 * tot["SQ_ACTIVE_INST_VALU"], cycles_for("SQ_ACTIVE_INST_VALU") * SIMDS)
        if "SQ_ACTIVE_INST_LDS" in tot:
            r["lds_busy"] = ratio(4 * tot["SQ_ACTIVE_INST_LDS"], cycles_for("SQ_ACTIVE_INST_LDS") * SIMDS)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in tot:
            r["mfma_busy"] = ratio(tot["SQ_VALU_MFMA_BUSY_CYCLES"], cycles_for("SQ_VALU_MFMA_BUSY_CYCLES") * SIMDS)
        if "SQ_INSTS_LDS_LOAD_BANDWIDTH" in tot:
            b = 64 * (tot["SQ_INSTS_LDS_LOAD_BANDWIDTH"] + tot.get("SQ_INSTS_LDS_STORE_BANDWIDTH", 0.0))
            r["lds_bytes"] = b
            r["lds_bw"] = ratio(b, cycles_for("SQ_INSTS_LDS_LOAD_BANDWIDTH") * CUS * 128)
        if "SQ_WAIT_INST_LDS" in tot and "SQ_WAVE_CYCLES" in tot:
            r["lds_wait"] = ratio(tot["SQ_WAIT_INST_LDS"], tot["SQ_WAVE_CYCLES"])
        if "SQ_LDS_BANK_CONFLICT" in tot:
            r["bank_confl"] = ratio(tot["SQ_LDS_BANK_CONFLICT"], tot.get("SQ_LDS_IDX_ACTIVE", 0.0))
        if "SQ_WAIT_ANY" in tot and "SQ_ACTIVE_INST_ANY" in tot:
            r["wait_any_over_active_any"] = ratio(tot["SQ_WAIT_ANY"], tot["SQ_ACTIVE_INST_ANY"])
        waves = tot.get("SQ_WAVES", 0.0)
        for k, nm in (("SQ_INSTS_VALU", "valu_per_wave"), ("SQ_INSTS_LDS", "lds_per_wave"),
                      ("SQ_INSTS_MFMA", "mfma_per_wave")):
            if k in tot and waves:
                r[nm] = round(tot[k] / waves, 1)
        r["cycles_per_dispatch"] = {p: round(cyc[p] / n[p], 1) for p in n}
        r["raw"] = dict(tot)
        out[pat] = r
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
