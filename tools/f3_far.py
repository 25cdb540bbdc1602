#!/usr/bin/env python3
"""F3 diagnostic: how many walk steps leave the tiles' LDS copy of the
boundary chain (gt_lcpitv_far_reads) for one plan + one events pass.
usage: f3_far.py KIND BASES"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import genometools_smax_amd as G  # noqa: E402

kind, bases = sys.argv[1], int(float(sys.argv[2]))
text = G.synth_genome(kind, bases, 42, threads=16)
esa = G.DeviceEsa(text, device=0, keep_suftab=True)
L = G.lib()
L.gt_lcpitv_far_reads.restype = ctypes.c_longlong
L.gt_lcpitv_far_reads()
plan = esa.lcpitv_plan()
torch.cuda.synchronize()
a = L.gt_lcpitv_far_reads()
ev = torch.empty(7 * plan.num_events(), dtype=torch.int64, device="cuda")
plan.events(ev.data_ptr(), torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
b = L.gt_lcpitv_far_reads()
print("N=%d intervals=%d far reads: plan %d, events %d" % (esa.nonspecials, plan.intervals()[0], a, b))
plan.close()
esa.release()
