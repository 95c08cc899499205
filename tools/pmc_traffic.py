#!/usr/bin/env python3
"""HBM traffic per launch from tools/pmc.sh output -> profiles/pmc_traffic.json (bench.py reads it).

Corrections per MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes read, so it is doubled. Calibrated for every load
width the kernels use by tools/ubench/fetch_cal.hip (profiles/r04_fetch_cal.txt): 64 MiB read
once with 4-, 8- and 16-B-per-lane loads (the TX's bit words at 4 and 8 bits per symbol, the
RX's sample quads) reports exactly 0.500 of the bytes in each case. WRITE_SIZE is taken as
reported (the floor kernels' writes match their byte counts exactly, profiles/r04_chain_floor.txt).

    python3 tools/pmc_traffic.py <pmc dir> <config> [profiles/pmc_traffic.json]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_summary  # noqa: E402


def main(d, config, path):
    res = pmc_summary.main(d)
    entry = {"unit": "bytes per launch", "source": d,
             "correction": "2 x FETCH_SIZE (KiB) + WRITE_SIZE (KiB), x1024; the x2 calibrated for 4/8/16-B "
                           "per-lane loads (profiles/r04_fetch_cal.txt)"}
    for k, cs in res.items():
        # names may come demangled ("tx_mfma<...>") or mangled ("_ZN2mk7tx_mfma...")
        kind = "tx" if ("tx_mfma" in k or "tx_fast" in k) else "rx" if ("rx_mfma" in k or "rx_fast" in k) \
            else "chain" if "chain_" in k else None
        if kind and "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            entry[kind] = int(round((2 * cs["FETCH_SIZE"] + cs["WRITE_SIZE"]) * 1024))
            entry[kind + "_kernel"] = k
            entry[kind + "_read"] = int(round(2 * cs["FETCH_SIZE"] * 1024))
            entry[kind + "_write"] = int(round(cs["WRITE_SIZE"] * 1024))
    try:
        with open(path) as f:
            allc = json.load(f)
    except (OSError, ValueError):
        allc = {}
    allc[config] = entry
    with open(path, "w") as f:
        json.dump(allc, f, indent=1, sort_keys=True)
    print(json.dumps(entry, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_traffic.json")
