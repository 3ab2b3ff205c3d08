#!/usr/bin/env python3
"""Per-launch means of the PMC counters of one kernel in a rocprofv3 counter CSV,
plus the derived fractions this repo reports (LDS conflict share, wait share).

    python tools/pmc_brief.py <run_counter_collection.csv> <kernel substring>
"""
import collections
import csv
import json
import sys


def main(path, kern):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if kern in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {c: sum(v) / len(v) for c, v in agg.items()}
    out = {"kernel": kern, "launches": max((len(v) for v in agg.values()), default=0), "per_launch": m}
    if m.get("SQ_ACTIVE_INST_LDS"):
        out["lds_conflict_frac"] = m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_ACTIVE_INST_LDS"]
    if m.get("SQ_WAVE_CYCLES"):
        out["wait_frac"] = m.get("SQ_WAIT_ANY", 0) / m["SQ_WAVE_CYCLES"]
    print(json.dumps(out))


if __name__ == "__main__":
    main(*sys.argv[1:])
