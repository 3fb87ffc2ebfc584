#!/usr/bin/env python3
"""Timeline of the timed region from a rocprofv3 --kernel-trace CSV (kernel_trace.csv).

Takes the last N launches of the anchor kernel (default ivf_screen_collect) and every
dispatch inside the window they span, then reports per kernel name the launches, mean
duration and busy share of the window, the union busy time of the anchor kernel and of all
kernels, the mean number of kernels running, and the window per anchor launch (the step).
usage: tools/timeline.py kernel_trace.csv [N=100] [anchor=ivf_screen_collect]
"""
import csv
import json
import sys
from collections import defaultdict


def union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    anchor = sys.argv[3] if len(sys.argv) > 3 else "ivf_screen_collect"
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name", "")
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            short = name.split("(")[0].replace("void ", "").replace("vdbk::", "")
            rows.append((s, e, short, r.get("Queue_Id", r.get("Stream_Id", ""))))
    rows.sort()
    anc = [x for x in rows if anchor in x[2]][-n:]
    if not anc:
        print(json.dumps({"error": f"no {anchor} launches"}))
        return
    t0, t1 = anc[0][0], anc[-1][1]
    win = [x for x in rows if x[0] >= t0 and x[1] <= t1]
    span = t1 - t0
    per = defaultdict(list)
    for s, e, k, _ in win:
        per[k].append(e - s)
    busy_all = union([(s, e) for s, e, _, _ in win])
    busy_anchor = union([(s, e) for s, e, k, _ in win if anchor in k])
    conc = sum(e - s for s, e, _, _ in win) / span
    out = {"window_us": round(span / 1e3, 1), "anchor_launches": len(anc),
           "step_us": round(span / 1e3 / max(len(anc) - 1, 1), 2),
           "anchor_busy_frac": round(busy_anchor / span, 4), "any_kernel_busy_frac": round(busy_all / span, 4),
           "mean_kernels_running": round(conc, 3), "queues": len({q for _, _, _, q in win}),
           "kernels": {k: {"n": len(v), "mean_us": round(sum(v) / len(v) / 1e3, 2),
                           "share_of_window": round(sum(v) / span, 4)}
                       for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1]))}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
