import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["order"], d["sort_points"], d["precision"], round(d["pass_ms_median"], 3), "slow/wave",
              round(d["slow_per_wave"], 3), "evals/wave", round(d["hull_evals_per_wave"], 3), "stageB",
              d["scan_waves"], "scan", d["full_scan_lanes"], "cand/wave", round(d.get("candidates_per_wave", -1), 2))
        if "cycle_frac" in d:
            print("   cycles/wave-iter", round(d["cycles_per_wave_iter"]), d["cycle_frac"])
