"""Probe (diagnostic, not a test): can RCCL put two ranks of one communicator on the same
GPU (single process, ncclCommInitAll with a repeated device)? Prints the result code."""
import ctypes

import torch  # noqa: F401  (loads the same librccl.so.1 the engine binds to)

L = ctypes.CDLL("librccl.so.1")
comms = (ctypes.c_void_p * 2)()
devs = (ctypes.c_int * 2)(0, 0)
rc = L.ncclCommInitAll(comms, 2, devs)
L.ncclGetErrorString.restype = ctypes.c_char_p
print("ncclCommInitAll([0, 0]) ->", rc, L.ncclGetErrorString(rc).decode())
for c in comms:
    if c:
        L.ncclCommDestroy(ctypes.c_void_p(c))
