#!/usr/bin/env python3
"""The headline rollout's per-launch duration from a rocprofv3 --kernel-trace of bench.py,
next to the bench line the same command printed:

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o run --output-format csv -- \\
        python bench.py --steps 20 --warmup 5 > gpurun_out/prof_kt.log
    python tools/rocprof_headline.py gpurun_out/prof_kt/run_kernel_trace.csv gpurun_out/prof_kt.log \\
        --steps 20 --warmup 5 > profiles/r06_rocprof_headline.json

bench.py launches dpac::k_rollout_staged<float, ...> (f32, LQR d = 20, no cost / u outputs) in
this order: W warm-up + K timed launches over the 5 cold sets, then (only with --mall) 5
warm-up + k2 = max(20, K // 4) timed launches of the one-set (MALL-resident) variant.  Without
--mall every launch of that kernel is a cold one, so the rocprofv3 --stats summary of the
command (AverageNs of that kernel) is the mean over exactly the W + K headline launches.
"""
import argparse
import csv
import json
import statistics

# the last template argument is GEN: 0 = dw read from HBM (the headline); the in-kernel Philox
# variant runs the same kernel with generator wavefronts (GEN = 12) and is not counted here
KERNEL = "k_rollout_staged<float, dpac::EqLQR<float, 20, 16>, 20, 1, 0, 8, 0>"
B, N, D, HBM = 4096, 200, 20, 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench_log")
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--warmup", type=int, required=True)
    ap.add_argument("--mall", action="store_true", help="the bench ran with --mall")
    ap.add_argument("--stats", default=None, help="the run's kernel_stats.csv (its AverageNs is quoted)")
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if KERNEL in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]  # us
    W, K = a.warmup, a.steps
    k2 = max(20, K // 4) if a.mall else 0
    expect = W + K + (5 + k2 if a.mall else 0)
    assert len(dur) == expect, (len(dur), expect)
    cold_all, timed = dur[:W + K], dur[W:W + K]
    algo = B * N * (2 * D + 2) * 4
    frac = lambda us: algo / (us * 1e-6) / 1e9 / HBM
    line = [json.loads(l) for l in open(a.bench_log) if l.startswith("{")][-1]
    rf = line["roofline"]
    out = {"kernel": rows[0]["Kernel_Name"][:120], "dispatches": len(dur),
           "rocprof_all_cold_mean_us": statistics.mean(cold_all),
           "rocprof_timed_mean_us": statistics.mean(timed), "rocprof_timed_median_us": statistics.median(timed),
           "rocprof_per_launch_us": [round(x, 3) for x in cold_all],
           "frac_rocprof_all_cold": frac(statistics.mean(cold_all)), "frac_rocprof_timed": frac(statistics.mean(timed)),
           "bench_same_run": {"ms_per_step_us": line["ms_per_step"] * 1e3, "frac": rf["frac"],
                              "event_pair_us": rf.get("event_pair", {}).get("avg_launch_ms", float("nan")) * 1e3},
           "algorithmic_bytes_per_launch": algo}
    # first-to-last kernel span of the timed launches: the GPU-side time of the K steps,
    # gaps between back-to-back dispatches included
    span = (int(rows[W + K - 1]["End_Timestamp"]) - int(rows[W]["Start_Timestamp"])) / 1e3
    out["rocprof_timed_span_per_launch_us"] = span / K
    if a.mall:
        mall = dur[W + K + 5:W + K + 5 + k2]
        out["rocprof_mall_mean_us"] = statistics.mean(mall)
        out["frac_rocprof_mall"] = frac(statistics.mean(mall))
    if a.stats:
        for r in csv.DictReader(open(a.stats)):
            if KERNEL in r["Name"]:
                out["stats_average_us"] = float(r["AverageNs"]) / 1e3
                out["stats_calls"] = int(r["Calls"])
                out["frac_stats_average"] = frac(out["stats_average_us"])
    out["line_frac_over_stats_frac"] = rf["frac"] / out.get("frac_stats_average", out["frac_rocprof_all_cold"])
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
