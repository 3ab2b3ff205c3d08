#!/usr/bin/env python3
"""A/B timing of pass-kernel builds (GPU box): runs bench.py once per library
(FLASHSDF_LIB override, see csrc/Makefile `make dev`), interleaved over
rounds, and prints the pass-kernel mean (HIP events), the step and the measured
prefetched frame (bench measured_frame, unless --no-full-iteration) per build.

    python tools/ab_bench.py ab/libA.so ab/libB.so [--rounds 3] [-- bench args]
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    argv = sys.argv[1:]
    extra = []
    if "--" in argv:
        i = argv.index("--")
        argv, extra = argv[:i], argv[i + 1:]
    rounds = 3
    if "--rounds" in argv:
        i = argv.index("--rounds")
        rounds = int(argv[i + 1])
        del argv[i:i + 2]
    libs = argv
    res = {lib: [] for lib in libs}
    for r in range(rounds):
        for lib in libs:
            env = dict(os.environ, FLASHSDF_LIB=os.path.abspath(lib))
            cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--inflight", "1", "--steps", "30",
                   "--warmup", "5"] + extra
            p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
            line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
            if p.returncode != 0 or not line:
                print(f"{lib}: FAILED rc={p.returncode}\n{p.stderr[-2000:]}", flush=True)
                return 1
            j = json.loads(line[-1])
            mf = (j.get("measured_frame") or j["config"].get("measured_frame") or {}).get("device_loop_prefetched", {})
            res[lib].append((j["roofline"]["kernel_ms"], j["ms_per_step"], mf.get("frame_ms", float("nan")),
                             mf.get("set_points_ms", float("nan"))))
            print(f"round {r} {os.path.basename(lib)}: pass {j['roofline']['kernel_ms']:.4f} ms, "
                  f"step {j['ms_per_step']:.4f} ms, prefetched frame {res[lib][-1][2]:.4f} ms "
                  f"(ingest {res[lib][-1][3]:.4f})", flush=True)
    print("summary (min over rounds):")
    for lib, v in res.items():
        print(f"  {os.path.basename(lib):32s} pass {min(x[0] for x in v):.4f} ms  step {min(x[1] for x in v):.4f} ms  "
              f"frame {min(x[2] for x in v):.4f} ms  ingest {min(x[3] for x in v):.4f} ms")
    return 0


if __name__ == "__main__":
    sys.exit(main())
