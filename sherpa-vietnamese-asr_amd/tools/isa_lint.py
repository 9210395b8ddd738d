"""Development check (not part of libzasr): per kernel, count global loads that are waited for
immediately (`s_waitcnt vmcnt(0)` within the next few instructions) -- the signature of a
guarded load that hipcc turned into a branch, which serialises memory round trips -- and any
scratch use.  Usage: python tools/isa_lint.py csrc/gemm.hip [more.hip ...]"""
import os
import re
import subprocess
import sys
import tempfile


def lint(src):
    d = tempfile.mkdtemp()
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
                    "-c", os.path.abspath(src), "-o", os.path.join(d, "x.o"), "--save-temps"],
                   cwd=d, check=True, capture_output=True)
    asm = [f for f in os.listdir(d) if f.endswith("gfx950.s")][0]
    lines = open(os.path.join(d, asm)).read().splitlines()
    out = []
    cur, loads, serial, scratch = None, 0, 0, 0
    for i, l in enumerate(lines):
        m = re.match(r"^(_Z\S+):", l)
        if m:
            cur, loads, serial, scratch = m.group(1), 0, 0, 0
            continue
        if cur is None:
            continue
        if "global_load" in l or "buffer_load" in l:
            loads += 1
            nxt = [x for x in lines[i + 1:i + 4] if x.strip() and not x.strip().startswith(";")]
            if any("s_waitcnt vmcnt(0)" in x for x in nxt[:2]):
                serial += 1
        if "scratch_" in l:
            scratch += 1
        if l.startswith(".Lfunc_end"):
            out.append((cur, loads, serial, scratch))
            cur = None
    return out


if __name__ == "__main__":
    for src in sys.argv[1:]:
        for name, loads, serial, scratch in lint(src):
            flag = " <-- serial loads" if serial > 2 else ""
            flag += " <-- SCRATCH" if scratch else ""
            print("%-90s loads %4d serial %4d%s" % (name[:90], loads, serial, flag))
