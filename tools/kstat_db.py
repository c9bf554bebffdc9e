"""Average kernel durations (us) of rocprofv3 --kernel-trace --stats databases, side by side:
python tools/kstat_db.py a/run_results.db b/run_results.db ..."""
import sqlite3
import sys

KEYS = ("pdsch_eq_rm", "pdsch_csimax_cols", "tdec_win_halfit", "ofdm_rx_n", "chest_estimate")

rows = {}
for path in sys.argv[1:]:
    db = sqlite3.connect(path)
    for name, calls, avg in db.execute("select name, total_calls, average from top_kernels"):
        for k in KEYS:
            if k in name:
                rows.setdefault(name.split("(")[0][:60], {})[path] = (calls, avg)
print("kernel".ljust(62) + "".join(p.split("/")[-2][:14].rjust(16) for p in sys.argv[1:]))
for name, d in sorted(rows.items()):
    print(name.ljust(62) + "".join((f"{d[p][1]:10.1f} x{d[p][0]:<4d}" if p in d else " " * 16) for p in sys.argv[1:]))
