#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/pmc.sh output): mean per dispatch per kernel."""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name):
    for key in ("tx_fast", "rx_fast", "tx_mfma", "rx_mfma", "tx_generic", "rx_generic", "fir_real", "prng_bits",
                "chain_small", "chain_mfma", "chain_flow"):
        if key in name:
            return name.split("(")[0].replace("void mk::", "")
    return None


def main(d):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "p*", "run_counter_collection.csv")):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Kernel_Name"])
                if k:
                    vals[k][(row["Dispatch_Id"], row["Counter_Name"])].append(float(row["Counter_Value"]))
    out = {}
    for k, dv in vals.items():
        agg = defaultdict(list)
        for (disp, cname), v in dv.items():
            agg[cname].append(sum(v))      # sum over dimension instances of one dispatch
        out[k] = {c: sum(v) / len(v) for c, v in agg.items()}
    return out


if __name__ == "__main__":
    res = main(sys.argv[1])
    for k, cs in sorted(res.items()):
        print(k)
        for c, v in sorted(cs.items()):
            print(f"   {c:24s} {v:16.1f}")
