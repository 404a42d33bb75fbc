#!/bin/bash
# Round 5: kernel timeline of the JPEG -> C2 decoder pipeline (tools/e2e_jpeg_only.py under rocprofv3
# --kernel-trace): GPU busy fraction and the gaps between windows (tools/trace_gaps.py).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r05"
mkdir -p "$O"
export TMPDIR=/tmp
rm -rf "$O/e2etrace"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/e2etrace" -o run --output-format csv -- python3 "$R/tools/e2e_jpeg_only.py" 30 > "$O/e2etrace.log" 2>&1) || { tail -5 "$O/e2etrace.log"; exit 1; }
grep "e2e" "$O/e2etrace.log"
f=$(find "$O/e2etrace" -name '*kernel_trace.csv' | head -n 1)
python3 - "$f" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "aeon" in r["Kernel_Name"]]
t0, t1 = int(rows[len(rows)//3]["Start_Timestamp"]), int(rows[-1]["End_Timestamp"])  # the last two thirds
busy, end, gaps = 0, t0, []
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if e < t0: continue
    s = max(s, t0)
    if s > end: gaps.append((s - end, r["Kernel_Name"][:40]))
    busy += max(0, e - max(s, end)); end = max(end, e)
print("span %.2f ms busy %.2f ms (%.0f %%)" % ((t1 - t0) / 1e6, busy / 1e6, 100 * busy / (t1 - t0)))
gaps.sort(reverse=True)
for g, n in gaps[:12]: print("gap %.1f us before %s" % (g / 1e3, n))
from collections import defaultdict
tot = defaultdict(float)
for r in rows:
    if int(r["Start_Timestamp"]) >= t0: tot[r["Kernel_Name"][:40]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
for k, v in sorted(tot.items(), key=lambda x: -x[1]): print("%-40s %.2f ms" % (k, v))
PY
