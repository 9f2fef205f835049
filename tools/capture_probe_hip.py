#!/usr/bin/env python3
"""Which HIP calls made by one thread break a graph capture running in another
thread, under each capture mode of the capturing thread and of the calling
thread (HIP runtime only, through ctypes: no torch, no library).  One JSON
line per case: the call's status, and the capture's end status.

    python tools/capture_probe_hip.py
"""
from __future__ import annotations

import ctypes
import json
import mmap
import threading

H = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
vp = ctypes.c_void_p
GLOBAL, THREAD_LOCAL, RELAXED = 0, 1, 2


def ck(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: {rc}")


def stream():
    s = vp()
    ck(H.hipStreamCreateWithFlags(ctypes.byref(s), ctypes.c_uint(1)), "stream")
    return s


def main():
    ck(H.hipSetDevice(0), "setdevice")
    cap_stream = stream()
    dev = vp()
    ck(H.hipMalloc(ctypes.byref(dev), ctypes.c_size_t(1 << 20)), "malloc")
    own = stream()
    pinned = vp()
    ck(H.hipHostMalloc(ctypes.byref(pinned), ctypes.c_size_t(1 << 20), ctypes.c_uint(0)), "hostmalloc")
    pageable = ctypes.create_string_buffer(1 << 20)
    mm = mmap.mmap(-1, 1 << 20)                # page-aligned pageable range for registration
    reg = vp(ctypes.addressof(ctypes.c_char.from_buffer(mm)))

    def op_malloc_free():
        p = vp()
        rc = H.hipMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 20))
        rc2 = H.hipFree(p) if rc == 0 else -1
        return rc, rc2

    def op_malloc():
        p = vp()
        return H.hipMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 20)), None

    def op_ext_malloc():
        p = vp()
        return H.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(1 << 20), ctypes.c_uint(0x4)), None

    pre = []

    def op_free():
        p = pre.pop()
        return H.hipFree(p), None

    def op_host_malloc():
        p = vp()
        rc = H.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 20), ctypes.c_uint(3))
        return rc, None

    hpre = []

    def op_host_free():
        return H.hipHostFree(hpre.pop()), None

    def op_register():
        rc = H.hipHostRegister(reg, ctypes.c_size_t(1 << 20), ctypes.c_uint(3))
        rc2 = H.hipHostUnregister(reg) if rc == 0 else -1
        return rc, rc2

    def op_stream():
        s = vp()
        rc = H.hipStreamCreateWithFlags(ctypes.byref(s), ctypes.c_uint(1))
        rc2 = H.hipStreamDestroy(s) if rc == 0 else -1
        return rc, rc2

    def op_event():
        e = vp()
        rc = H.hipEventCreateWithFlags(ctypes.byref(e), ctypes.c_uint(2))
        rc2 = H.hipEventDestroy(e) if rc == 0 else -1
        return rc, rc2

    def op_copy_pinned():
        rc = H.hipMemcpyAsync(dev, pinned, ctypes.c_size_t(1 << 20), ctypes.c_int(1), own)
        return rc, H.hipStreamSynchronize(own)

    def op_copy_pageable():
        rc = H.hipMemcpyAsync(dev, pageable, ctypes.c_size_t(1 << 20), ctypes.c_int(1), own)
        return rc, H.hipStreamSynchronize(own)

    def op_stream_sync():
        return H.hipStreamSynchronize(own), None

    ops = {"malloc+free": op_malloc_free, "malloc": op_malloc, "ext_malloc_contig": op_ext_malloc,
           "free": op_free, "host_malloc": op_host_malloc, "host_free": op_host_free,
           "host_register+unregister": op_register, "stream_create+destroy": op_stream,
           "event_create+destroy": op_event, "memcpy_async_pinned+sync": op_copy_pinned,
           "memcpy_async_pageable+sync": op_copy_pageable, "stream_sync": op_stream_sync}
    for cap_mode in (GLOBAL, THREAD_LOCAL):
        for call_mode in (GLOBAL, RELAXED):
            for name, fn in ops.items():
                if name == "free":
                    p = vp()
                    ck(H.hipMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 20)), "malloc")
                    pre.append(p)
                if name == "host_free":
                    p = vp()
                    ck(H.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 20), ctypes.c_uint(3)), "hm")
                    hpre.append(p)
                out = {}

                def other():
                    if call_mode != GLOBAL:
                        m = ctypes.c_int(call_mode)
                        H.hipThreadExchangeStreamCaptureMode(ctypes.byref(m))
                    out["rc"] = fn()
                    H.hipGetLastError()

                ck(H.hipStreamBeginCapture(cap_stream, ctypes.c_int(cap_mode)), "begin")
                ck(H.hipMemsetAsync(dev, ctypes.c_int(0), ctypes.c_size_t(4096), cap_stream), "memset")
                th = threading.Thread(target=other)
                th.start()
                th.join(60)
                g = vp()
                end = H.hipStreamEndCapture(cap_stream, ctypes.byref(g))
                H.hipGetLastError()
                if end == 0 and g.value:
                    H.hipGraphDestroy(g)
                print(json.dumps({"capture_mode": ["global", "thread_local"][cap_mode],
                                  "caller_mode": ["global", "thread_local", "relaxed"][call_mode],
                                  "call": name, "call_rc": out.get("rc", "hung"), "end_capture_rc": end}),
                      flush=True)
    # Events recorded on a stream BEFORE that stream began capturing, used from another thread
    # while it captures: the event itself, and a mirror (a second stream waited on the event
    # before the capture, then recorded its own event).
    priv = stream()
    for cap_mode in (GLOBAL, THREAD_LOCAL):
        for name in ("query_event", "wait_event", "query_mirror", "wait_mirror"):
            cap_stream = stream()   # a fresh one per case: a stream whose capture was invalidated stays failed
            e, m = vp(), vp()
            ck(H.hipEventCreateWithFlags(ctypes.byref(e), ctypes.c_uint(2)), "event")
            ck(H.hipEventCreateWithFlags(ctypes.byref(m), ctypes.c_uint(2)), "event")
            ck(H.hipMemsetAsync(dev, ctypes.c_int(1), ctypes.c_size_t(4096), cap_stream), "memset")
            ck(H.hipEventRecord(e, cap_stream), "record")
            ck(H.hipStreamWaitEvent(priv, e, ctypes.c_uint(0)), "wait")
            ck(H.hipEventRecord(m, priv), "record m")
            ck(H.hipStreamSynchronize(cap_stream), "sync")
            ev = m if name.endswith("mirror") else e
            out = {}

            def other():
                m2 = ctypes.c_int(RELAXED)
                H.hipThreadExchangeStreamCaptureMode(ctypes.byref(m2))
                if name.startswith("query"):
                    out["rc"] = H.hipEventQuery(ev)
                else:
                    out["rc"] = H.hipStreamWaitEvent(own, ev, ctypes.c_uint(0))
                    out["rc2"] = H.hipStreamSynchronize(own)
                H.hipGetLastError()

            ck(H.hipStreamBeginCapture(cap_stream, ctypes.c_int(cap_mode)), "begin")
            ck(H.hipMemsetAsync(dev, ctypes.c_int(0), ctypes.c_size_t(4096), cap_stream), "memset")
            th = threading.Thread(target=other)
            th.start()
            th.join(60)
            g = vp()
            end = H.hipStreamEndCapture(cap_stream, ctypes.byref(g))
            H.hipGetLastError()
            if end == 0 and g.value:
                H.hipGraphDestroy(g)
            print(json.dumps({"capture_mode": ["global", "thread_local"][cap_mode], "caller_mode": "relaxed",
                              "call": name + " (recorded before the capture)", "call_rc": out.get("rc", "hung"),
                              "call_rc2": out.get("rc2"), "end_capture_rc": end}), flush=True)
            H.hipEventDestroy(e)
            H.hipEventDestroy(m)
    H.hipDeviceSynchronize()


if __name__ == "__main__":
    main()
