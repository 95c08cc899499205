#!/usr/bin/env python3
"""The bench's three timing legs read back from a rocprofv3 kernel trace of the bench command
(run_kernel_trace.csv): runs of back-to-back RX launches (the RX-only leg), of TX launches
(TX-only) and of alternating TX, RX (the chain). For each run, span / launches (first start to
last end, as the bench's two HIP events bracket it), median over runs — comparable with
`chain_roofline.{tx_ms,rx_ms,chain_ms}` of the bench line. The per-dispatch averages of the
--stats summary read ≈1 us high per launch (their TX + RX exceeds the chain's span).

    python3 tools/trace_legs.py <run_kernel_trace.csv> [rx-name-part] [tx-name-part] [min_run]

(name parts select one configuration's kernels, default the C3 ones: rx_mfmaILi4ELi6,
tx_mfmaILi4ELi2.)
"""
import csv
import json
import statistics
import sys


def main(path, rxn="rx_mfmaILi4ELi6", txn="tx_mfmaILi4ELi2", min_run=10):
    rows = []
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"]
        kind = "rx" if rxn in n else "tx" if txn in n else None
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, n))
    rows.sort()
    out = {}
    for leg in ("rx", "tx", "chain"):
        spans, i = [], 0
        while i < len(rows):
            j = i
            if leg == "chain":
                while j + 1 < len(rows) and rows[j][2] == "tx" and rows[j + 1][2] == "rx":
                    j += 2
                n = (j - i) // 2
                if n >= min_run:
                    spans.append((rows[j - 1][1] - rows[i][0]) / n)
                i = j + 1 if j == i else j
            else:
                while j < len(rows) and rows[j][2] == leg:
                    j += 1
                n = j - i
                if n >= min_run:
                    spans.append((rows[j - 1][1] - rows[i][0]) / n)
                i = j if j > i else i + 1
        out[leg] = {"runs": len(spans), "us_per_launch_median": round(statistics.median(spans) / 1e3, 3) if spans else None}
    for leg in ("rx", "tx"):
        d = [r[1] - r[0] for r in rows if r[2] == leg]
        out[leg]["dispatch_duration_mean_us"] = round(statistics.mean(d) / 1e3, 3) if d else None
    print(json.dumps(out, indent=1))
    return out


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], *(a[1:3]), *([int(a[3])] if len(a) > 3 else []))
