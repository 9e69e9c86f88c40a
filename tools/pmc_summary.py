#!/usr/bin/env python3
"""Per-kernel PMC summary from rocprofv3 --pmc passes (one counter set per pass directory).

    python tools/pmc_summary.py <dir with pmc_*/run_counter_collection.csv> <out.json> \
        [--kernels k_rollout_nn_bwd,k_rollout_nn<,k_param_grads<] [--bytes-per-kernel k=B ...]

Per kernel: the mean of every counter over its dispatches, the mean dispatch duration, and
derived figures (MI355X_MICROARCH.md §rocprofv3 PMC slots, §HBM):
  clock_GHz         = GRBM_GUI_ACTIVE / 8 XCDs / duration
  mfma_busy_chip    = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x duration cycles)
  mfma_busy_used    = the same over the SIMDs of the CUs the grid occupies
  wave_wait_frac    = SQ_WAIT_ANY / SQ_WAVE_CYCLES       (parked on s_waitcnt / barrier)
  wave_stall_frac   = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES  (issue stalls: MFMA dependency, pipe)
  wave_active_frac  = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  lds_conflict_frac = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  l2_hit            = TCC_HIT / (TCC_HIT + TCC_MISS)
  hbm_read_bytes    = FETCH_SIZE x 1024 x 2 (KiB; gfx950 counts half a wide read)
  hbm_write_bytes   = WRITE_SIZE x 1024
"""
import argparse
import collections
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("out")
    ap.add_argument("--kernels", default="k_rollout_nn_bwd,k_rollout_nn<,k_param_grads<,k_mlp_rows_fwd,"
                                         "k_mlp_rows_bwd,k_rollout<")
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    keys = a.kernels.split(",")
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(list)
    grid = {}
    for p in sorted(glob.glob(os.path.join(a.src, "pmc_*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(p)):
            for k in keys:
                if k in r["Kernel_Name"]:
                    vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                    durs[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                    grid[k] = (int(r["Grid_Size"]), int(r["Workgroup_Size"]), int(r["VGPR_Count"]),
                               int(r["Accum_VGPR_Count"]), int(r["LDS_Block_Size"]))
    out = {"source": a.src, "note": a.note, "kernels": {}}
    for k in keys:
        if k not in vals:
            continue
        c = {n: sum(v) / len(v) for n, v in vals[k].items()}
        dur_ns = sum(durs[k]) / len(durs[k])
        g = grid[k]
        wgs = g[0] // g[1]
        d = {"dispatch_us": dur_ns / 1e3, "grid": g[0], "workgroup": g[1], "workgroups": wgs,
             "vgpr": g[2], "agpr": g[3], "lds_bytes": g[4], "counters": c}
        ghz = c.get("GRBM_GUI_ACTIVE", 0) / 8 / dur_ns if "GRBM_GUI_ACTIVE" in c else 2.4
        d["clock_GHz"] = ghz
        cyc = dur_ns * ghz
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            d["mfma_busy_chip"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc)
            used_cus = min(256, wgs)
            d["mfma_busy_used"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (4 * used_cus * cyc)
        if "SQ_WAVE_CYCLES" in c:
            for n, key in (("wave_wait_frac", "SQ_WAIT_ANY"), ("wave_stall_frac", "SQ_WAIT_INST_ANY"),
                           ("wave_active_frac", "SQ_ACTIVE_INST_ANY")):
                if key in c:
                    d[n] = c[key] / c["SQ_WAVE_CYCLES"]
        if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_LDS_IDX_ACTIVE"):
            d["lds_conflict_frac"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]
        if "TCC_HIT_sum" in c:
            d["l2_hit"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
        if "FETCH_SIZE" in c:
            d["hbm_read_bytes"] = c["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in c:
            d["hbm_write_bytes"] = c["WRITE_SIZE"] * 1024
        if "SQ_WAVES" in c and "SQ_INSTS_MFMA" in c:
            for n in ("SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD",
                      "SQ_INSTS_VMEM_WR"):
                if n in c:
                    d.setdefault("insts_per_wave", {})[n] = c[n] / c["SQ_WAVES"]
        out["kernels"][k] = d
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    for k, d in out["kernels"].items():
        print(k, {n: round(v, 3) for n, v in d.items() if isinstance(v, float)})


if __name__ == "__main__":
    main()
