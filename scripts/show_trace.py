"""Summarise gpurun_out/trace.log (scripts/trace_knn.py output): medians and maxima per phase."""
import json
import sys

t = open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/trace.log").read()
t = "\n".join(l for l in t.splitlines() if "amdgpu" not in l)
pos = 0
while True:
    i = t.find("shape", pos)
    if i < 0:
        break
    j = t.index("{", i)
    k = t.index("\n}\n", j) + 2
    print(t[i:j].strip())
    for r, v in json.loads(t[j:k]).items():
        print(" ", r, {kk: (x if kk == "final" else x[2::2]) for kk, x in v.items()})
    pos = k
print(t[pos:])
