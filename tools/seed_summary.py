#!/usr/bin/env python3
"""Summarise full 50 000-iteration lqr_d20 runs (tools/seed_spread.sh -> tests/train_check.py
JSON) per precision: the converged err_value / err_control of each run as the mean of its last
`--tail` evaluations (solver.py:109-119 errors, logged every log_freq iterations), then the
mean and sample sd over the seeds, and |Δ mean| between precisions against the north-star bar
(1e-3) and the seed spread.

    python tools/seed_summary.py out.json gpurun_out/seed_gpu32_*.json gpurun_out/seed_gpu64_*.json
"""
import json
import statistics
import sys


def main():
    out, files = sys.argv[1], sys.argv[2:]
    tail = 20
    runs = {}
    for f in files:
        d = json.load(open(f))
        for name, r in d["runs"].items():
            h = r["history"]
            seed = f.rsplit("_", 1)[-1].split(".")[0]
            ent = {"file": f, "seed": seed, "iters": d["iters"], "log_freq": d["log_freq"], "batch": d["batch"],
                   "wall_s": r["wall_s"], "steps": [h["step"][0], h["step"][-1]],
                   "history": {k: h[k] for k in ("step", "err_value", "err_control") if k in h}}
            for k in ("err_value", "err_control"):
                if k in h:
                    last = h[k][-tail:]
                    ent[k + "_final_mean"] = statistics.mean(last)
                    ent[k + "_final_sd"] = statistics.stdev(last) if len(last) > 1 else 0.0
            runs.setdefault(name, []).append(ent)
    summary = {"tail_evaluations": tail, "runs": runs, "per_precision": {}}
    for name, rs in runs.items():
        p = {"seeds": [r["seed"] for r in rs]}
        for k in ("err_value", "err_control"):
            v = [r[k + "_final_mean"] for r in rs if k + "_final_mean" in r]
            if v:
                p[k + "_mean"] = statistics.mean(v)
                p[k + "_sd_over_seeds"] = statistics.stdev(v) if len(v) > 1 else None
        summary["per_precision"][name] = p
    pp = summary["per_precision"]
    if "gpu32" in pp and "gpu64" in pp:
        for k in ("err_value", "err_control"):
            if k + "_mean" in pp["gpu32"] and k + "_mean" in pp["gpu64"]:
                dm = abs(pp["gpu32"][k + "_mean"] - pp["gpu64"][k + "_mean"])
                sds = [s for s in (pp["gpu32"].get(k + "_sd_over_seeds"), pp["gpu64"].get(k + "_sd_over_seeds")) if s]
                summary[k + "_abs_diff_of_means"] = dm
                summary[k + "_within_1e-3"] = dm < 1e-3
                if sds:
                    summary[k + "_diff_over_max_seed_sd"] = dm / max(sds)
        # paired: the same seed (same initial weights, same Philox increments) in both precisions
        by = {n: {r["seed"]: r for r in runs[n]} for n in ("gpu32", "gpu64")}
        common = sorted(set(by["gpu32"]) & set(by["gpu64"]), key=int)
        for k in ("err_value", "err_control"):
            key = k + "_final_mean"
            v32 = [r[key] for r in runs["gpu32"]]
            v64 = [r[key] for r in runs["gpu64"]]
            if len(v32) > 1 and len(v64) > 1:  # unpaired: Welch's standard error of the difference of means
                se = (statistics.variance(v32) / len(v32) + statistics.variance(v64) / len(v64)) ** 0.5
                summary[k + "_unpaired"] = {"n32": len(v32), "n64": len(v64),
                                            "diff_of_means": statistics.mean(v32) - statistics.mean(v64),
                                            "se": se, "diff_of_medians": statistics.median(v32) - statistics.median(v64)}
            d = [by["gpu32"][s_][key] - by["gpu64"][s_][key] for s_ in common]
            if len(d) > 1:
                sd = statistics.stdev(d)
                summary[k + "_paired"] = {"seeds": common, "diffs": d, "mean": statistics.mean(d), "sd": sd,
                                          "se": sd / len(d) ** 0.5, "median": statistics.median(d),
                                          "max_abs": max(abs(x) for x in d),
                                          "mean_within_1e-3": abs(statistics.mean(d)) < 1e-3}
    json.dump(summary, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in summary.items() if k != "runs"}, indent=1))


if __name__ == "__main__":
    main()
