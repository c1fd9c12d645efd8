"""Per workload: the bench line's per-step kernel time (hipExtLaunchKernel dispatch stamps, summed
over the step's kernels) beside rocprofv3's kernel stats of the same command (the sum of the
average durations of the library kernels that run every step), and their ratio.
    python3 scripts/rocprof_vs_bench.py gpurun_out/final [workloads...]"""
import csv
import json
import sys
from pathlib import Path

d = Path(sys.argv[1])
wls = sys.argv[2:] or "knn range c5 join ppoly ingest ppjoin ppknn knn_incr ppoly_incr".split()
out = {}
for w in wls:
    line = [x for x in open(d / f"bench_{w}.log") if x.startswith("{")][-1]
    b = json.loads(line)
    r = b.get("roofline") or {}
    steps = b["steps"]
    tot, names = 0.0, []
    for row in csv.DictReader(open(d / "prof" / f"{w}_kernel_stats.csv")):
        name = row["Name"]
        if not name.startswith(("geohip::", "void geohip::")) or "synth_uniform" in name:
            continue
        if int(row["Calls"]) < steps:  # set-up launches (count-only sizing, plans)
            continue
        tot += float(row["AverageNs"]) / 1e3
        names.append(name.split("(")[0])
    bench_us = r.get("avg_kernel_us")
    out[w] = {"bench_kernel_us": bench_us, "rocprof_kernel_us": tot,
              "ratio": (bench_us / tot) if bench_us and tot else None, "kernels": names}
    print(f"{w:11s} bench {bench_us or 0:9.1f} us  rocprof {tot:9.1f} us  ratio {out[w]['ratio'] or 0:.3f}  ({len(names)} kernels)")
json.dump(out, open(d / "rocprof_vs_bench.json", "w"), indent=1)
