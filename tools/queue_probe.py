#!/usr/bin/env python3
"""Which hardware queue does each stream get? Run under rocprofv3 --kernel-trace: one tiny
kernel per stream, in a known order, with a synchronize between launches; the trace's
Queue_Id per dispatch (in launch order) gives the stream -> queue mapping.
Phases: (a) 8 torch pool streams used in creation order; (b) 4 more pool streams used in
reverse order; (c) 4 streams from hipStreamCreateWithFlags used in order; (d) the null stream.
Prints the launch plan; tools/queue_probe_read.py joins it with the trace."""
import ctypes
import json
import torch

dev = torch.device("cuda", 0)
x = torch.zeros(1, device=dev)
plan = []


def hit(s, tag):
    with torch.cuda.stream(s):
        x.add_(1)
    torch.cuda.synchronize()
    plan.append(tag)


a = [torch.cuda.Stream(dev) for _ in range(8)]
for i, s in enumerate(a):
    hit(s, f"pool{i}")
b = [torch.cuda.Stream(dev) for _ in range(4)]
for i in reversed(range(4)):
    hit(b[i], f"pool{8 + i}(rev)")
path = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln)
hip = ctypes.CDLL(path)
raw = []
for i in range(4):
    h = ctypes.c_void_p()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(h), ctypes.c_uint(1)) == 0
    raw.append(h)
for i, h in enumerate(raw):
    hit(torch.cuda.ExternalStream(h.value, device=dev), f"raw{i}")
hit(torch.cuda.default_stream(dev), "default")
# (e) CU-masked streams, every CU enabled; (f) high-priority streams
ncu = torch.cuda.get_device_properties(dev).multi_processor_count
words = (ncu + 31) // 32
mask = (ctypes.c_uint32 * words)(*([0xFFFFFFFF] * words))
for i in range(3):
    h = ctypes.c_void_p()
    assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(words), mask) == 0
    hit(torch.cuda.ExternalStream(h.value, device=dev), f"cumask{i}")
for i in range(3):
    hit(torch.cuda.Stream(dev, priority=-1), f"prio{i}")
# (g) 3 more pool streams first used back to back (no sync between): the in-flight pattern
c = [torch.cuda.Stream(dev) for _ in range(3)]
for i, s in enumerate(c):
    with torch.cuda.stream(s):
        x.add_(1)
    plan.append(f"burst{i}")
torch.cuda.synchronize()
print("PLAN " + json.dumps(plan), flush=True)
