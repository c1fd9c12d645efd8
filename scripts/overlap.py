"""Summarise a rocprofv3 kernel + memory-copy trace of scripts/e2e_trace.py: for the last
host-window kNN call, the H2D copies and the knn_pass kernels on a common clock (us), and how
many kernels ran while a later copy was still in flight (the staging overlap)."""
import csv
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40])
      for r in csv.DictReader(open(f"{d}/e2e_kernel_trace.csv")) if "knn" in r["Kernel_Name"]]
cs = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "H2D")
      for r in csv.DictReader(open(f"{d}/e2e_memory_copy_trace.csv")) if r["Direction"].endswith("HOST_TO_DEVICE")]
ks.sort()
cs.sort()
# the last call: its kernels are the last 10 knn_pass + rebase + merge; its copies the 20 before them
last_k = ks[-12:]
t0 = min(s for s, _, _ in last_k) - 6_000_000
ev = [e for e in ks + cs if e[0] >= t0]
ev.sort()
base = ev[0][0]
for s, e, n in ev:
    print(f"{(s - base) / 1e3:10.1f} {(e - base) / 1e3:10.1f}  {n}")
over = sum(1 for s, e, n in last_k if any(cs_ > s and cs_ < e or (cs_ <= s and ce_ >= s) for cs_, ce_, _ in cs
                                             if cs_ >= t0))
print("kernels of the last call overlapping an in-flight H2D copy:", over, "of", len(last_k))
