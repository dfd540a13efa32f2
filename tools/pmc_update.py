"""Fold a pmc_summary.py --json result into the committed roofline inputs.

python tools/pmc_update.py SUMMARY.json KERNEL_REGEX KEY --batch B --layers L \
    --source "..." [--alg-bytes N] [--insts] [--traffic]

--insts    profiles/pmc_insts.json[KEY] = instruction counts of the matched
           kernel (SQ_INSTS_VALU / _VALU_TRANS_F32 / _MFMA / _SALU / _LDS,
           SQ_WAVES, mfma_busy_frac, wait fraction) -- bench.py's VALU floor
--traffic  profiles/pmc_traffic.json[KEY] = HBM bytes per launch (FETCH_SIZE x2
           + WRITE_SIZE, MI355X_MICROARCH.md's gfx950 correction) -- the line's
           ``traffic``
The source string should name the commit the profiled build came from.
"""
import argparse
import json
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
PROF = os.path.join(os.path.dirname(HERE), "profiles")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("summary")
    ap.add_argument("kernel")
    ap.add_argument("key")
    ap.add_argument("--batch", type=int, required=True)
    ap.add_argument("--layers", type=int, default=1)
    ap.add_argument("--source", required=True)
    ap.add_argument("--alg-bytes", type=int, default=None)
    ap.add_argument("--insts", action="store_true")
    ap.add_argument("--traffic", action="store_true")
    ap.add_argument("--batch-exact", action="store_true",
                    help="bytes do not scale with the batch (bench.py uses the entry at this batch only)")
    a = ap.parse_args()
    summ = json.load(open(a.summary))
    hits = [k for k in summ if re.search(a.kernel, k)]
    if len(hits) != 1:
        raise SystemExit("kernel regex %r matches %s" % (a.kernel, hits))
    name = hits[0]
    c, d = summ[name]["counters"], summ[name]["derived"]
    if a.insts:
        p = os.path.join(PROF, "pmc_insts.json")
        tab = json.load(open(p)) if os.path.exists(p) else {}
        tab[a.key] = {
            "valu": int(c["SQ_INSTS_VALU"]), "valu_trans": int(c["SQ_INSTS_VALU_TRANS_F32"]),
            "mfma": int(c["SQ_INSTS_MFMA"]), "salu": int(c["SQ_INSTS_SALU"]), "lds": int(c["SQ_INSTS_LDS"]),
            "waves": int(c["SQ_WAVES"]), "batch": a.batch, "layers": a.layers,
            "mfma_busy_frac": round(d.get("mfma_busy_frac", 0.0), 4),
            "wait_any_frac": round(d.get("SQ_WAIT_ANY/WAVE_CYCLES", 0.0), 4),
            "kernel": name, "source": a.source}
        json.dump(tab, open(p, "w"), indent=1)
        print("pmc_insts.json[%s] <- %s" % (a.key, name))
    if a.traffic:
        p = os.path.join(PROF, "pmc_traffic.json")
        tab = json.load(open(p)) if os.path.exists(p) else {}
        rd, wr = d["hbm_read_bytes_corrected"], d["hbm_write_bytes"]
        ent = {"bytes_per_launch": int(rd + wr), "read_bytes_corrected": int(rd), "write_bytes": int(wr),
               "batch": a.batch, "kernel": name, "source": a.source}
        if a.alg_bytes:
            ent["algorithmic_bytes_per_launch"] = a.alg_bytes
        if a.batch_exact:
            ent["batch_exact"] = True
        tab[a.key] = ent
        json.dump(tab, open(p, "w"), indent=1)
        print("pmc_traffic.json[%s] <- %s: %d B/launch" % (a.key, name, int(rd + wr)))


if __name__ == "__main__":
    main()
