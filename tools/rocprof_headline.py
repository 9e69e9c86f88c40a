#!/usr/bin/env python3
"""The headline rollout's per-launch duration from a rocprofv3 --kernel-trace of bench.py,
split into the HBM-cold launches (the 5 rotating buffer sets: warm-up, the timed region and
the bracketed pass) and the Infinity-Cache-resident ones (the one-set variant), next to the
bench line the same command printed:

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o run --output-format csv -- \\
        python bench.py --steps K --warmup W --no-cpu-baseline --no-train > gpurun_out/prof_kt.log
    python tools/rocprof_headline.py gpurun_out/prof_kt/run_kernel_trace.csv gpurun_out/prof_kt.log \\
        --steps K --warmup W > profiles/r03_rocprof_headline.json

bench.py launches dpac::k_rollout_staged<float, ...> (f32, LQR d = 20, no cost / u outputs) in
this order: W warm-up + K timed launches over the 5 cold sets, then 5 warm-up + k2 =
max(20, K // 4) timed launches of the one-set (MALL-resident) variant.
"""
import argparse
import csv
import json
import statistics

KERNEL = "k_rollout_staged<float, dpac::EqLQR<float, 20, 16>, 20, 1, 0,"
B, N, D, HBM = 4096, 200, 20, 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench_log")
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--warmup", type=int, required=True)
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if KERNEL in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]  # us
    W, K = a.warmup, a.steps
    k2 = max(20, K // 4)
    cold = dur[W:W + K]
    mall = dur[W + K + 5:W + K + 5 + k2]
    assert len(dur) == W + K + 5 + k2, (len(dur), W, K, k2)
    algo = B * N * (2 * D + 2) * 4
    frac = lambda us: algo / (us * 1e-6) / 1e9 / HBM
    line = [json.loads(l) for l in open(a.bench_log) if l.startswith("{")][-1]
    rf = line["roofline"]
    out = {"kernel": rows[0]["Kernel_Name"][:120], "dispatches": len(dur),
           "rocprof_cold_mean_us": statistics.mean(cold), "rocprof_cold_median_us": statistics.median(cold),
           "rocprof_mall_mean_us": statistics.mean(mall),
           "frac_rocprof_cold": frac(statistics.mean(cold)), "frac_rocprof_mall": frac(statistics.mean(mall)),
           "bench_same_run": {"avg_launch_us": rf["avg_launch_ms"] * 1e3, "frac": rf["frac"]},
           "algorithmic_bytes_per_launch": algo}
    out["bench_event_vs_rocprof_cold"] = out["bench_same_run"]["avg_launch_us"] / out["rocprof_cold_mean_us"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
