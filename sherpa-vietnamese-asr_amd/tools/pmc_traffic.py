"""HBM traffic per launch of a kernel class from two rocprofv3 PMC passes (FETCH_SIZE and
WRITE_SIZE collected separately: together they exceed the gfx950 counter budget).

bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE / WRITE_SIZE are in KiB, and on
gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads (MI355X_MICROARCH.md, HBM).

  python tools/pmc_traffic.py FETCH.csv WRITE.csv --key "zipformer-68m|greedy_search|1|bf16|3600|enc_gemm"
          [--out profiles/pmc_traffic.json]

Kernel classes: enc_gemm = gemm_bf16_kernel / gemm_f32_kernel with the dense A loader
(template argument ALOAD = 0) and a [N][K] weight operand, the launches Engine::linear /
linear_h make (the NonlinAttention GEMM, EPI_MULAUX, is class attn_nonlin); any other class
name matches kernels whose name contains it; ffn_fused = the fused FeedforwardModule kernels
(bf16 ffn_fused / ffn_wide, f16x3 ffn_wide_h3 but its d = 128 ConvNeXt instance).
"""
import argparse
import csv
import json
import os
import re


def gemm_args(name: str):
    """(kind, template integer args) of a gemm kernel name, demangled or (for instantiations
    with __bf16 arguments, which rocprofv3 leaves mangled) mangled."""
    m = re.search(r"gemm_(bf16|f32)_kernel<([^>]*)>", name)
    if m:
        return m.group(1), [a.strip() for a in m.group(2).split(",")]
    m = re.search(r"gemm_(bf16|f32)_kernelI((?:Li\d+E|Lb[01]E)+)", name)
    if m:
        vals = re.findall(r"L(i|b)(\d+)E", m.group(2))
        return m.group(1), [("false" if v == "0" else "true") if t == "b" else v for t, v in vals]
    return None, None


def _int_args(name: str, kernel: str):
    m = re.search(kernel + r"<([^>]*)>", name)
    return [a.strip() for a in m.group(1).split(",")] if m else None


def in_class(name: str, cls: str) -> bool:
    if cls == "enc_gemm":
        # f16x3 projections: the row-resident kernel, and the dense-A instances of the LDS-DMA
        # and register-tile kernels (ALOAD 0; the others are the subsampling convolutions)
        if "gemm_h3r_kernel" in name:
            return True
        a = _int_args(name, "gemm_glds_h3_kernel")
        if a is not None:
            return a[5] == "0" and a[1] not in ("4", "5")
        a = _int_args(name, "gemm_x3_kernel")
        if a is not None:
            return a[4] == "0" and a[5] not in ("4", "5")
        if "gemm_glds_kernel" in name:  # multi-stage LDS-DMA variant: its EPI_MULAUX(16)
            # z-sliced instances are the NonlinAttention product (class attn_nonlin)
            m = re.search(r"gemm_glds_kernel(?:<\s*\d+,\s*(\d+)|ILi\d+ELi(\d+)E)", name)
            epi = (m.group(1) or m.group(2)) if m else "0"
            return epi not in ("4", "5")
        kind, args = gemm_args(name)
        if kind is None:
            return False
        m = re.match(r"(bf16|f32)", kind)
        if kind == "bf16":
            return args[5] == "0" and args[6] != "4"  # EPI_MULAUX = the NonlinAttention GEMM
        return args[4] == "0" and args[5] == "false"  # B n-contiguous = nonlin_attention

    if cls == "ffn_fused":  # the fused FeedforwardModule launches: bf16 ffn_fused / ffn_wide,
        # f16x3 ffn_wide_h3 except its d = 128 instance (the ConvNeXt MLP, class frontend_conv)
        if "ffn_wide_h3_kernel" in name:
            return "ffn_wide_h3_kernelILi128E" not in name and "ffn_wide_h3_kernel<128" not in name
        return "ffn_wide_kernel" in name or "ffn_fused_kernel" in name
    return cls in name


def total(path: str, counter: str, cls: str):
    s, n = 0.0, 0
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter and in_class(r["Kernel_Name"], cls):
                s += float(r["Counter_Value"])
                n += 1
    return s, n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--key", required=True)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    cls = a.key.split("|")[-1]
    f, nf = total(a.fetch_csv, "FETCH_SIZE", cls)
    w, nw = total(a.write_csv, "WRITE_SIZE", cls)
    if nf == 0 or nf != nw:
        raise SystemExit("dispatch counts differ or are zero: %d vs %d" % (nf, nw))
    per = (2.0 * f + w) * 1024.0 / nf
    rec = {"bytes_per_launch": round(per), "launches": nf,
           "fetch_kib_x2": round(2 * f), "write_kib": round(w),
           "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), "
                     "FETCH_SIZE x2 gfx950 correction; " + os.path.basename(os.path.dirname(a.fetch_csv))}
    print(json.dumps({a.key: rec}, indent=1))
    if a.out:
        tab = {}
        if os.path.exists(a.out):
            with open(a.out) as fh:
                tab = json.load(fh)
        tab[a.key] = rec
        with open(a.out, "w") as fh:
            json.dump(tab, fh, indent=1)


if __name__ == "__main__":
    main()
