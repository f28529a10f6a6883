#!/usr/bin/env python3
"""Per-kernel breakdown of ONE training step from a rocprofv3 kernel trace:
the step is the span between the last two launches of a marker kernel (the
optimizer's), kernels aggregated by name.

    python scripts/step_breakdown.py gpurun_out/p32c/run_kernel_trace.csv [marker]
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
marker = sys.argv[2] if len(sys.argv) > 2 else "sgd_bf16"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
# consecutive marker launches (an optimizer split over several launches) form
# one boundary: the step runs from after one run of them to the end of the next
runs = [i for j, i in enumerate(idx) if j + 1 == len(idx) or idx[j + 1] != i + 1]
end, start = runs[-1], runs[-2] + 1
agg = {}
tot = 0.0
for r in rows[start:end + 1]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    a = agg.setdefault(r["Kernel_Name"][:70], [0, 0.0])
    a[0] += 1
    a[1] += d
span = (int(rows[end]["End_Timestamp"]) - int(rows[start]["Start_Timestamp"])) / 1e3
print(f"| kernel | launches | us |\n|---|---|---|")
for k, (n, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"| `{k}` | {n} | {t:.1f} |")
print(f"\n{end - start + 1} kernels, {tot:.1f} us of kernel time, {span:.1f} us span")
