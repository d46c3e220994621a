"""Per-kernel means of rocprofv3 ``--pmc`` passes (``*_counter_collection.csv``).

    python scripts/pmc_summary.py gpurun_out/pmc_b4/p1 gpurun_out/pmc_b4/p2 [--match lenet] [--jsonl out.jsonl]

Every directory is searched recursively for counter-collection CSVs. Counter values are summed
per dispatch (rocprofv3 writes one row per counter per dispatch, or per dimension instance), then
averaged over the dispatches of each kernel. Derived ratios are printed when their inputs exist.
"""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> value
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r.get("Kernel_Name") or r.get("Kernel-Name") or r.get("kernel_name") or "?"
                disp = r.get("Dispatch_Id") or r.get("Correlation_Id") or r.get("dispatch_id") or "0"
                name = r.get("Counter_Name") or r.get("counter_name")
                val = float(r.get("Counter_Value") or r.get("counter_value") or 0.0)
                per[(k, disp)][name] += val
    out = defaultdict(lambda: defaultdict(list))
    for (k, _), cs in per.items():
        for n, v in cs.items():
            out[k][n].append(v)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default="")
    ap.add_argument("--jsonl", default=None)
    ap.add_argument("--short", type=int, default=70)
    a = ap.parse_args()
    merged = defaultdict(dict)
    ndisp = {}
    for d in a.dirs:
        for k, cs in load(d).items():
            if a.match and a.match not in k:
                continue
            for n, vals in cs.items():
                merged[k][n] = sum(vals) / len(vals)
                ndisp[k] = max(ndisp.get(k, 0), len(vals))
    rows = []
    for k, cs in sorted(merged.items()):
        r = {"kernel": k[:a.short], "dispatches": ndisp[k]}
        r.update({n: round(v, 1) for n, v in sorted(cs.items())})
        wc = cs.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
                if n in cs:
                    r["pct_" + n[3:].lower()] = round(100.0 * cs[n] / wc, 1)
        if cs.get("SQ_LDS_IDX_ACTIVE"):
            r["lds_conflict_pct"] = round(100.0 * cs.get("SQ_LDS_BANK_CONFLICT", 0.0) / cs["SQ_LDS_IDX_ACTIVE"], 1)
        if cs.get("SQ_WAVES") and cs.get("SQ_INSTS_VALU"):
            r["valu_insts_per_wave"] = round(cs["SQ_INSTS_VALU"] / cs["SQ_WAVES"], 1)
        rows.append(r)
    for r in rows:
        print(json.dumps(r))
    if a.jsonl:
        with open(a.jsonl, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
