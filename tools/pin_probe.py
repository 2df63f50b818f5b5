#!/usr/bin/env python3
"""Diagnostics: what the HIP runtime reports for torch's pinned host tensors
(hipPointerGetAttributes type, hipHostGetDevicePointer) -- the caller-block
detection of dfmi_filter_project_host_batches_into depends on it."""
import ctypes as C
import os

import torch

lib = C.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))


class Attr(C.Structure):  # hipPointerAttribute_t (ROCm 6+): type, device, devicePointer, hostPointer, isManaged, allocationFlags
    _fields_ = [("type", C.c_int), ("device", C.c_int), ("devicePointer", C.c_void_p), ("hostPointer", C.c_void_p),
                ("isManaged", C.c_int), ("allocationFlags", C.c_uint)]


torch.cuda.init()
for n in (64, 1 << 16, 6488064, 64 << 20):
    t = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    a = Attr()
    rc = lib.hipPointerGetAttributes(C.byref(a), C.c_void_p(t.data_ptr()))
    dp = C.c_void_p()
    rc2 = lib.hipHostGetDevicePointer(C.byref(dp), C.c_void_p(t.data_ptr()), 0)
    flags = C.c_uint()
    rc3 = lib.hipHostGetFlags(C.byref(flags), C.c_void_p(t.data_ptr()))
    print("n=%d is_pinned=%s attr rc=%d type=%d dev=%d devptr=%s hostptr=%s | hostGetDevicePointer rc=%d %s | hostGetFlags rc=%d %d" % (
        n, t.is_pinned(), rc, a.type, a.device, a.devicePointer, a.hostPointer, rc2, dp.value, rc3, flags.value))
p = C.c_void_p()
lib.hipHostMalloc(C.byref(p), C.c_size_t(1 << 20), 0)
a = Attr()
rc = lib.hipPointerGetAttributes(C.byref(a), p)
print("hipHostMalloc: attr rc=%d type=%d" % (rc, a.type))
