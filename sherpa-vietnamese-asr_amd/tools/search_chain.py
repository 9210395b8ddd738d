"""Development tool (not part of libzasr): the per-frame critical chain of the search stream
from a rocprofv3 --kernel-trace CSV -- joiner and search-step kernel durations and the idle
gaps between consecutive dispatches of the chain (launch latency / waiting for CUs held by
the next batch's encoder).
Usage: python tools/search_chain.py gpurun_out/kt/run_kernel_trace.csv"""
import csv
import statistics
import sys

CHAIN = ("joiner", "search_step_kernel", "greedy_spec_kernel")


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    chain = [r for r in rows if any(c in r["Kernel_Name"] for c in CHAIN)]
    if not chain:
        print("no search-chain kernels")
        return
    by = {}
    gaps = []
    prev_end = None
    for r in chain:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = "joiner" if "joiner" in r["Kernel_Name"] else r["Kernel_Name"].split("<")[0].split("(")[0][-40:]
        by.setdefault(name, []).append((e - s) / 1e3)
        if prev_end is not None:
            g = (s - prev_end) / 1e3
            if 0 <= g < 200:  # same search chain (a larger gap is a batch boundary)
                gaps.append(g)
        prev_end = e
    for k, v in by.items():
        print(f"{k:40s} n={len(v):6d} mean={statistics.mean(v):8.2f} us  median={statistics.median(v):8.2f}"
              f"  p90={sorted(v)[int(0.9 * len(v))]:8.2f}  total={sum(v) / 1e3:8.2f} ms")
    if gaps:
        print(f"{'gap between chain dispatches':40s} n={len(gaps):6d} mean={statistics.mean(gaps):8.2f} us"
              f"  median={statistics.median(gaps):8.2f}  total={sum(gaps) / 1e3:8.2f} ms")


if __name__ == "__main__":
    main()
