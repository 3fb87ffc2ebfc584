#!/usr/bin/env python3
"""Join queue_probe.py's launch plan with the kernel trace: stream tag -> Queue_Id."""
import csv
import json
import sys

plan = json.loads(next(l for l in open(sys.argv[2]) if l.startswith("PLAN "))[5:])
rows = sorted((int(r["Start_Timestamp"]), r.get("Queue_Id", "?"), r["Kernel_Name"][:40]) for r in csv.DictReader(open(sys.argv[1])))
rows = rows[-len(plan):]
for tag, (_, q, k) in zip(plan, rows):
    print(f"{tag:14s} queue {q}  {k}")
