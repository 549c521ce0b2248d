"""The synthetic capture probe (scripts/capture_probe.hip, built as libcapture_probe.so)
run inside a process that has initialised torch, with a torch stream as the capture origin
(the situation of tests/test_gpu_split.py), to tell a torch interaction from an engine one.

usage: python scripts/capture_probe_torch.py <nsplit> <nclass> <nsub> <piped> <shared> <features>
"""
import ctypes
import os
import sys

import torch

args = [int(a) for a in (sys.argv[1:] or ["2", "1", "3", "1", "0", "0"])]
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libcapture_probe.so"))
x = torch.ones(1024, device="cuda:0")
(x * 2).sum().item()  # torch's HIP context, allocator and default stream in use
s = torch.cuda.Stream()
print("torch-hosted probe", args, flush=True)
rc = lib.probe_run(*[ctypes.c_int(a) for a in args], ctypes.c_void_p(s.cuda_stream))
print("rc", rc, flush=True)
sys.exit(rc)
