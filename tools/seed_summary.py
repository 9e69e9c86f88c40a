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
    json.dump(summary, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in summary.items() if k != "runs"}, indent=1))


if __name__ == "__main__":
    main()
