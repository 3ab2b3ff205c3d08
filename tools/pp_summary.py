import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["order"], d["sort_points"], d["precision"], round(d["pass_ms_median"], 3), "slow/wave",
              round(d["slow_per_wave"], 3), "evals/wave", round(d["hull_evals_per_wave"], 3), "stageB",
              d["stageB_waves"], "scan", d["full_scan_lanes"])
