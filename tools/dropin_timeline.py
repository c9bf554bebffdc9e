"""Per-TTI timeline of the drop-in loop from a rocprofv3 kernel + HIP runtime trace (tools/gpu/r06o.sh):
python tools/dropin_timeline.py <trace dir> [tti index from the end; default: the TTI of median span among the last 100]
Prints the HIP calls and kernels of one TTI (a TTI starts at the caller's host I/Q upload) with times relative to
its start, and per-TTI totals: API time by function, kernel time, and the idle GPU time inside the TTI."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
back = int(sys.argv[2]) if len(sys.argv) > 2 else -1
api = [r for r in csv.DictReader(open(glob.glob(d + "/*hip_api_trace.csv")[0]))]
ker = [r for r in csv.DictReader(open(glob.glob(d + "/*kernel_trace.csv")[0]))]
ev = [("api", r["Function"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Thread_Id"]) for r in api]
ev += [("ker", r["Kernel_Name"][:70], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"]) for r in ker]
ev.sort(key=lambda e: e[2])
# TTI boundaries: the OFDM kernel of the drop-in's fft_estimate (one per TTI)
starts = [e[2] for e in ev if e[0] == "ker" and "ofdm_rx" in e[1]]
print(f"{len(starts)} TTIs (ofdm_rx launches)")
if len(starts) < max(back, 100) + 2:
    sys.exit(0)
if back < 0:  # the TTI (ofdm launch to ofdm launch) of median length among the last 100
    spans = sorted((starts[-b] - starts[-b - 1], b) for b in range(1, 101))
    back = spans[50][1]
    print(f"TTI {back} from the end: ofdm-to-ofdm {spans[50][0] / 1e3:.1f} us (min {spans[0][0] / 1e3:.1f}, "
          f"max {spans[-1][0] / 1e3:.1f})")
t0, t1 = starts[-back - 1], starts[-back]
# the TTI begins at the first API call after the previous TTI's last kernel ended
prev_end = max(e[3] for e in ev if e[0] == "ker" and e[2] < t0)
first = min(e[2] for e in ev if e[0] == "api" and e[2] > prev_end)
nxt_end = max(e[3] for e in ev if e[0] == "ker" and e[2] < t1)
sel = [e for e in ev if first <= e[2] <= nxt_end]
apit = collections.Counter()
apin = collections.Counter()
kbusy = []
for kind, name, s, e, tid in sel:
    print(f"{(s - first) / 1e3:9.1f} {(e - s) / 1e3:8.1f} us  {kind} {name} [{tid}]")
    if kind == "api":
        apit[name] += e - s
        apin[name] += 1
    else:
        kbusy.append((s, e))
span = nxt_end - first
busy = 0
cur = None
for s, e in sorted(kbusy):
    if cur is None or s > cur[1]:
        if cur:
            busy += cur[1] - cur[0]
        cur = [s, e]
    else:
        cur[1] = max(cur[1], e)
if cur:
    busy += cur[1] - cur[0]
print(f"\nTTI span {span / 1e3:.1f} us, GPU busy {busy / 1e3:.1f} us, kernels {len(kbusy)}")
for k, v in apit.most_common(25):
    print(f"  {k:40s} {apin[k]:4d} calls {v / 1e3:8.1f} us")
