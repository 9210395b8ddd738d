"""Development tool (not part of libzasr): summarise one decode step of a rocprofv3
--kernel-trace CSV.  A step starts at an fbank_kernel dispatch; the LAST complete step is
summarised per (kernel, grid) in dispatch order, with durations in microseconds.
Usage: python tools/trace_summary.py gpurun_out/kt/run_kernel_trace.csv [--by-name]"""
import csv
import re
import sys
from collections import OrderedDict


def short(name):
    name = name.replace("zasr::", "").replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name).replace("void ", "")
    return name[:80]


def main():
    path = sys.argv[1]
    by_name = "--by-name" in sys.argv
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "fbank_kernel" in r["Kernel_Name"]]
    if len(starts) < 2:
        print("need >= 2 steps")
        return
    a, b = starts[-2], starts[-1]
    step = rows[a:b]
    t0 = int(step[0]["Start_Timestamp"])
    t1 = int(step[-1]["End_Timestamp"])
    agg = OrderedDict()
    busy = 0.0
    for r in step:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        busy += d
        g = (r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
        key = short(r["Kernel_Name"]) if by_name else (short(r["Kernel_Name"]), g)
        e = agg.setdefault(key, [0, 0.0])
        e[0] += 1
        e[1] += d
    print(f"step wall {(t1 - t0) / 1e3:.1f} us, kernel busy {busy:.1f} us, {len(step)} dispatches")
    for k, (n, d) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{d:10.1f} us {n:6d}x {d / n:9.1f} us  {k}")


if __name__ == "__main__":
    main()
