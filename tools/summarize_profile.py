#!/usr/bin/env python3
"""Summarize a tools/rocprof_round.sh output directory into profiles/<tag>/.

Copies the kernel-trace stats CSV and writes pmc_summary.json: per-launch means
of every PMC counter for each kernel, with the gfx950 HBM-traffic estimate for
the pass kernel (MI355X_MICROARCH.md §HBM: FETCH_SIZE under-reports wide reads
by 1/2 — reported both raw and doubled; WRITE_SIZE exact for wide stores).
FETCH_SIZE / WRITE_SIZE are in KiB (rocprofv3 derived counters).

    python tools/summarize_profile.py gpurun_out/prof r01b profiles/r01

also writes profiles/latest_pmc.json, which bench.py reads for roofline.traffic.
"""
import collections
import csv
import json
import os
import shutil
import sys


def main(src, tag, dst):
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, f"{tag}_trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    out = {}
    for part in ("fetch", "write", "sq", "sq2"):
        path = os.path.join(src, f"{tag}_{part}", "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, cs in agg.items():
            for c, v in cs.items():
                out.setdefault(k, {})[c] = {"launches": len(v), "mean_per_launch": sum(v) / len(v)}
    pk = [k for k in out if "pass_kernel" in k]
    if pk:
        p = out[pk[0]]
        fetch = p.get("FETCH_SIZE", {}).get("mean_per_launch")
        write = p.get("WRITE_SIZE", {}).get("mean_per_launch")
        if fetch is not None and write is not None:
            out["pass_kernel_hbm_bytes_per_launch"] = {
                "fetch_bytes_raw": fetch * 1024, "fetch_bytes_x2_gfx950": 2 * fetch * 1024,
                "write_bytes": write * 1024,
                "traffic_bytes": (2 * fetch + write) * 1024,
                "note": "traffic = 2*FETCH_SIZE + WRITE_SIZE (KiB->B); FETCH counts Infinity-Cache hits too"}
    with open(os.path.join(dst, "pmc_summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    hb = out.get("pass_kernel_hbm_bytes_per_launch")
    if hb:
        # the record bench.py reads for roofline.traffic (same workload: bench.py defaults)
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        rel = os.path.relpath(os.path.join(dst, "pmc_summary.json"), root)
        with open(os.path.join(root, "profiles", "latest_pmc.json"), "w") as f:
            rec = {"workload": "bench.py default", "kernel": pk[0],
                   "traffic_bytes_per_launch": hb["traffic_bytes"], "source": rel}
            pc = out[pk[0]]
            m = lambda c: pc[c]["mean_per_launch"] if c in pc else None  # noqa: E731
            if m("SQ_WAVE_CYCLES"):
                rec["executed"] = {
                    "valu_insts_per_launch": m("SQ_INSTS_VALU"),
                    "fp64_fma_insts_per_launch": m("SQ_INSTS_VALU_FMA_F64"),
                    "valu_active_frac_of_wave_time": (m("SQ_ACTIVE_INST_VALU") or 0) / m("SQ_WAVE_CYCLES"),
                    "wait_frac_of_wave_time": (m("SQ_WAIT_ANY") or 0) / m("SQ_WAVE_CYCLES")}
            json.dump(rec, f, indent=1)
    print(json.dumps(hb, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
