#!/bin/bash
# round 5: where the segment walk's time goes per segment size (kernel trace of the sweep, records in HBM)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05w; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 tools/wal_replay_big.py --steps 2 --compact 1 --device-recs 1 --seg-sweep 1048576,2097152,4194304 > $O/sweep.log 2>&1 || { echo "sweep failed"; tail -5 $O/sweep.log; exit 1; }
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r05w/kt/kt_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    n = r["Kernel_Name"]
    if "wal_seg" in n or "stream_kernel" in n or "compare" in n:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        print("%10.2f ms %9.1f us  %s" % ((int(r["Start_Timestamp"]) - t0) / 1e6, d, n.split("(")[0][:70]))
PY
