#!/bin/bash
# Runs tools/overlap_probe.hip (build line inside) plain and under rocprofv3 --kernel-trace: do kernels on two
# streams overlap on the GPU, and does the trace show it? → gpurun_out/ovl/
set -o pipefail
O=gpurun_out/ovl; mkdir -p $O
timeout -k 10 60 build/probes/overlap_probe > $O/plain.txt 2>&1 || exit 1
cat $O/plain.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o k -- build/probes/overlap_probe > $O/traced.txt 2>&1 || exit 2
cat $O/traced.txt | grep rep
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/ovl/tr/**/*kernel_trace.csv", recursive=True)[0]
rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Queue_Id"]) for r in csv.DictReader(open(f)) if "spin" in r["Kernel_Name"]]
rows.sort()
ov = sum(1 for i in range(1, len(rows)) if rows[i][0] < rows[i - 1][1])
print("spin kernels", len(rows), "starting before the previous one ended:", ov)
for a, b, s, q in rows[-6:]:
    print(f"  start {(a - rows[0][0]) / 1e6:9.3f} ms  dur {(b - a) / 1e6:7.3f} ms  stream {s} queue {q}")
PY
