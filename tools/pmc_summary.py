"""Summarise rocprofv3 PMC passes (tools/pmc_passes.sh) per kernel.

python tools/pmc_summary.py gpurun_out/TAG [--kernel REGEX] [--json out.json]
Per-dispatch means of every counter, plus derived metrics.  HBM traffic per
launch follows MI355X_MICROARCH.md section HBM: FETCH_SIZE (KiB) under-reports
16-B/lane streaming reads by exactly 2x on gfx950 -> x2; WRITE_SIZE is exact.
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def load(tag_dir, kregex):
    vals = defaultdict(list)  # (kernel, counter) -> per-dispatch values
    for f in glob.glob(os.path.join(tag_dir, "pmc*", "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        for r in csv.DictReader(open(f)):
            if not re.search(kregex, r["Kernel_Name"]):
                continue
            per[(r["Kernel_Name"], r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
        for (k, c, d), v in per.items():
            vals[(k, c)].append(v)
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag_dir")
    ap.add_argument("--kernel", default=".")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    vals = load(a.tag_dir, a.kernel)
    kernels = sorted({k for k, _ in vals})
    out = {}
    for k in kernels:
        m = {c: sum(v) / len(v) for (kk, c), v in vals.items() if kk == k}
        # drop the argument list only (names may hold "(anonymous namespace)")
        short = re.sub(r"\((?!anonymous namespace\))[^()]*\)\s*$", "", k).replace("(anonymous namespace)::", "")[:90]
        print("==", short)
        for c in sorted(m):
            print("  %-36s %16.1f" % (c, m[c]))
        d = {}
        g = lambda n: m.get(n)
        if g("SQ_WAVE_CYCLES") and g("SQ_BUSY_CYCLES"):
            wc = g("SQ_WAVE_CYCLES")
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if g(n) is not None:
                    d[n + "/WAVE_CYCLES"] = g(n) / wc
        if g("SQ_VALU_MFMA_BUSY_CYCLES") and g("GRBM_GUI_ACTIVE"):
            # busy cycles are per-SIMD cycles summed over SIMDs; 1024 SIMDs, GUI_ACTIVE summed over 8 XCDs
            d["mfma_busy_frac"] = g("SQ_VALU_MFMA_BUSY_CYCLES") / (1024 * g("GRBM_GUI_ACTIVE") / 8)
        if g("TCC_HIT_sum") is not None and g("TCC_MISS_sum"):
            d["L2_hit_rate"] = g("TCC_HIT_sum") / (g("TCC_HIT_sum") + g("TCC_MISS_sum"))
        if g("FETCH_SIZE") is not None:
            d["hbm_read_bytes_corrected"] = 2 * g("FETCH_SIZE") * 1024
        if g("WRITE_SIZE") is not None:
            d["hbm_write_bytes"] = g("WRITE_SIZE") * 1024
        if "hbm_read_bytes_corrected" in d and "hbm_write_bytes" in d:
            d["hbm_bytes_per_launch"] = d["hbm_read_bytes_corrected"] + d["hbm_write_bytes"]
        if g("SQ_INSTS_VALU") and g("SQ_INSTS_MFMA"):
            d["valu_per_mfma"] = g("SQ_INSTS_VALU") / g("SQ_INSTS_MFMA")
        for n, v in d.items():
            print("  %-36s %16.4g" % (n, v))
        out[short] = dict(counters=m, derived=d)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
