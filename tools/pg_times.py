"""Average k_param_grads* durations per template instance in rocprofv3 kernel traces."""
import collections, csv, re, sys
for path in sys.argv[1:]:
    print("==", path)
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"]
        if "k_param_grads" in n:
            agg[re.sub(r"dpac::PgArgs<\w+>", "", n)[:80]].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in agg.items():
        print(f"{len(v):4d} {sum(v) / len(v):8.1f}  {k}")
