#!/usr/bin/env python3
"""Copy rocprofv3 summaries from gpurun_out/ into profiles/ and derive HBM traffic.

    python tools/collect_profiles.py r01

* profiles/<tag>_kernel_stats.csv  — rocprofv3 --kernel-trace --stats summary
* profiles/<tag>_pmc_rollout.json  — FETCH_SIZE / WRITE_SIZE per dpac::k_rollout_staged launch,
  corrected as MI355X_MICROARCH.md §HBM prescribes (separate passes; counters in KiB;
  gfx950 FETCH_SIZE reports half the bytes of a wide coalesced stream -> x2)
* profiles/pmc_traffic.json        — the per-launch HBM bytes bench.py reports as
  roofline.traffic for the matching workload key
* profiles/<tag>_rocprof_headline.json, <tag>_pmc_mlp.json, <tag>_train_timeline.txt
"""
import csv
import json
import os
import shutil
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")


def counter_mean(path, kernel_substr, counter):
    rows = [r for r in csv.DictReader(open(path))
            if kernel_substr in r["Kernel_Name"] and r["Counter_Name"] == counter]
    return statistics.mean(float(r["Counter_Value"]) for r in rows), len(rows), rows[0] if rows else None


def main(tag):
    os.makedirs(PROF, exist_ok=True)
    ks = os.path.join(OUT, "prof_kt", "run_kernel_stats.csv")
    if os.path.exists(ks):
        shutil.copy(ks, os.path.join(PROF, f"{tag}_kernel_stats.csv"))
    ts = os.path.join(OUT, "prof_train", "run_kernel_stats.csv")
    if os.path.exists(ts):  # lqr_d20 training iteration (tools/train_bench.py)
        shutil.copy(ts, os.path.join(PROF, f"{tag}_train_kernel_stats.csv"))
        tl = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "iter_timeline.py"),
                             os.path.join(OUT, "prof_train", "run_kernel_trace.csv")],
                            capture_output=True, text=True)
        if tl.returncode == 0:
            open(os.path.join(PROF, f"{tag}_train_timeline.txt"), "w").write(tl.stdout)
    hl = os.path.join(OUT, "headline.log")  # tools/rocprof_headline.py over prof_kt
    if os.path.exists(hl):
        txt = open(hl).read()
        if txt.lstrip().startswith("{"):
            open(os.path.join(PROF, f"{tag}_rocprof_headline.json"), "w").write(txt)
    hm = os.path.join(OUT, "headline_mall.log")  # the same over the --mall run
    if os.path.exists(hm):
        txt = open(hm).read()
        if txt.lstrip().startswith("{"):
            open(os.path.join(PROF, f"{tag}_rocprof_headline_mall.json"), "w").write(txt)
    pi = os.path.join(OUT, "pmc_iteration.log")  # tools/pmc_iteration.py over one training iteration
    if os.path.exists(pi):
        txt = open(pi).read()
        if txt.lstrip().startswith("{"):
            open(os.path.join(PROF, f"{tag}_pmc_iteration.json"), "w").write(txt)
    pm = os.path.join(OUT, "pmc_mlp", "summary.json")  # tools/pmc_mlp.sh
    if os.path.exists(pm):
        shutil.copy(pm, os.path.join(PROF, f"{tag}_pmc_mlp.json"))
    bl = os.path.join(OUT, "bench.log")
    if os.path.exists(bl):
        lines = [l for l in open(bl) if l.startswith("{")]
        if lines:
            with open(os.path.join(PROF, f"{tag}_bench.jsonl"), "a") as f:
                f.write(lines[-1])
    f = os.path.join(OUT, "pmc_fetch", "run_counter_collection.csv")
    w = os.path.join(OUT, "pmc_write", "run_counter_collection.csv")
    if not (os.path.exists(f) and os.path.exists(w)):
        print("no PMC passes found")
        return
    # canonical rollout: f32, LQR d=20 (16 lanes/trajectory), adaptive, dw from HBM, no cost/u outputs
    # (the LDS-staged kernel k_rollout_staged; k_rollout takes Philox / unstaged shapes)
    key_kernel = "k_rollout_staged<float, dpac::EqLQR<float, 20, 16>, 20, 1, 0, 8, 0>"  # GEN = 0: dw from HBM
    fetch_kib, nf, row = counter_mean(f, key_kernel, "FETCH_SIZE")
    write_kib, nw, _ = counter_mean(w, key_kernel, "WRITE_SIZE")
    fetch_b = fetch_kib * 1024 * 2  # gfx950: FETCH_SIZE counts 64 B per 128-B request
    write_b = write_kib * 1024
    B, N, d = 4096, 200, 20
    algo = B * N * (2 * d + 2) * 4 + B * d * 4  # + x0 read and x[0] write are per launch too
    summary = {
        "kernel": row["Kernel_Name"], "launches_fetch": nf, "launches_write": nw,
        "FETCH_SIZE_KiB": fetch_kib, "WRITE_SIZE_KiB": write_kib,
        "hbm_read_bytes_corrected": fetch_b, "hbm_write_bytes": write_b,
        "hbm_bytes_per_launch": fetch_b + write_b,
        "algorithmic_bytes_per_launch": algo,
        "traffic_over_algorithmic": (fetch_b + write_b) / algo,
        "vgpr": row["VGPR_Count"], "sgpr": row["SGPR_Count"], "grid": row["Grid_Size"],
        "workgroup": row["Workgroup_Size"],
        "correction": "FETCH_SIZE x2 (MI355X_MICROARCH.md §HBM), counters in KiB, separate --pmc passes",
    }
    json.dump(summary, open(os.path.join(PROF, f"{tag}_pmc_rollout.json"), "w"), indent=2)
    # bench.py's PMC passes time the launches rotating over its 5 buffer sets (cold cache)
    json.dump({"rollout_adaptive_f32_B4096_N200_d20_cold5": {"hbm_bytes_per_launch": fetch_b + write_b,
                                                              "source": f"profiles/{tag}_pmc_rollout.json"}},
              open(os.path.join(PROF, "pmc_traffic.json"), "w"), indent=2)
    print(json.dumps(summary, indent=2))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
