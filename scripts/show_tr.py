"""Summarise gpurun_out/tr_c2.log (scripts/trace_pass.py output): median block phases, last block's final."""
import json
import sys

for l in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/tr_c2.log"):
    if not l.startswith("{"):
        continue
    d = json.loads(l)
    print("ablation", d["shape"]["ablation"])
    for r in ("rep0", "rep1", "rep2", "rep3"):
        x = d[r]
        print(" ", {k: x[k][2] for k in ("start", "stream_end", "flush")}, x["block_median"],
              {k: x[k][2] for k in ("drained", "arrived")}, "max_arrived", x["arrived"][4])
        print("    final", x["final"], x["stats"])
