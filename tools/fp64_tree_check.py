#!/usr/bin/env python3
"""Whether the float64 production path of this tree computes exactly what round 4's did: a short
lqr_d20 run (tests/train_check.py --sampler device, same seed and data seed) compared entry by
entry with the first logged evaluations of a round-4 full run stored in
profiles/r04_seed_spread_lqr_d20.json (bitwise equality expected: round 5 changed only the
split-fp16 float32 kernels).

    python tools/fp64_tree_check.py gpurun_out/fp64_check_101.json 101
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    new_path, seed = sys.argv[1], sys.argv[2]
    new = json.load(open(new_path))["runs"]["gpu64"]["history"]
    old = [r for r in json.load(open(os.path.join(ROOT, "profiles", "r04_seed_spread_lqr_d20.json")))["runs"]["gpu64"]
           if r["seed"] == seed][0]["history"]
    n = len(new["step"])
    res = {"seed": seed, "steps_compared": new["step"], "r04_steps": old["step"][:n]}
    for k in ("err_value", "err_control"):
        a, b = new[k][:n], old[k][:n]
        res[k + "_new"], res[k + "_r04"] = a, b
        res[k + "_bitwise_equal"] = a == b
        res[k + "_max_abs_diff"] = max(abs(x - y) for x, y in zip(a, b))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
