#!/usr/bin/env python3
"""Runs one of tests/test_gpu_capture.py's cross-thread capture cases against a
given product library (A/B of a fix: the same test on the library before and
after it), printing one JSON line per capture mode.

    python tools/capture_concurrency.py --lib tools/_pre/libshmr_ec.so
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "shmr_amd", "_lib", "libshmr_ec.so"))
    ap.add_argument("--test", default="test_library_allocations_while_another_thread_captures")
    a = ap.parse_args()
    import torch
    from shmr_amd import _native
    _native._PATHS["product"] = os.path.abspath(a.lib)
    spec = importlib.util.spec_from_file_location("tgc", os.path.join(ROOT, "tests", "test_gpu_capture.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    gpu = torch.device("cuda", 0)
    fn = getattr(mod, a.test)
    modes = ("global", "thread_local") if fn.__code__.co_argcount == 2 else (None,)
    for mode in modes:
        try:
            fn(gpu, mode) if mode else fn(gpu)
            out = "pass"
        except BaseException as e:   # noqa: BLE001 -- reported, next mode
            out = repr(e)[:600]
        print(json.dumps({"lib": a.lib, "test": a.test, "mode": mode, "result": out}), flush=True)


if __name__ == "__main__":
    main()
