#!/usr/bin/env python3
"""HBM traffic per launch from tools/pmc.sh output -> profiles/pmc_traffic.json (bench.py reads it).

Corrections per MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of a 16-B-per-lane streaming read, so it is
doubled (RX reads its samples 16 B per lane; TX's 4-B-per-lane bit loads are uncalibrated and
get the same factor, which matches their known byte count); WRITE_SIZE is taken as reported.

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
             "correction": "2 x FETCH_SIZE (KiB) + WRITE_SIZE (KiB), x1024"}
    for k, cs in res.items():
        # names may come demangled ("tx_mfma<...>") or mangled ("_ZN2mk7tx_mfma...")
        kind = "tx" if ("tx_mfma" in k or "tx_fast" in k) else "rx" if ("rx_mfma" in k or "rx_fast" in k) else None
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
