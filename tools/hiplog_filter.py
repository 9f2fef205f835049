#!/usr/bin/env python3
"""Filters HIP's API log (AMD_LOG_LEVEL=3, AMD_LOG_MASK=1) on stdin down to its
failed calls: for every distinct (call, status) the count and the first few
occurrences with the same thread's preceding lines.  Used by tools/gpu/archive/r04l.sh
to find which runtime call a soak failure comes from.

    prog 2> >(python tools/hiplog_filter.py > errors.txt)
"""
import collections
import re
import sys

BENIGN = ("hipSuccess", "hipErrorNotReady")
tid_re = re.compile(r"tid:(0x[0-9a-f]+|\d+)")
ret_re = re.compile(r"(\w+): Returned (\w+)")
per_tid = collections.defaultdict(lambda: collections.deque(maxlen=12))
ev_re = re.compile(r"(\w+) \( event:(0x[0-9a-f]+)(?:, stream:(0x[0-9a-f]+|0))?")
cap_re = re.compile(r"(hipStreamBeginCapture|hipStreamEndCapture|hipStreamBeginCaptureToGraph) \( stream:(0x[0-9a-f]+)")
ev_hist = collections.defaultdict(lambda: collections.deque(maxlen=4))   # event -> its last calls
cap_hist = collections.defaultdict(lambda: collections.deque(maxlen=3))  # stream -> capture begin / end
last_ev = {}
counts = collections.Counter()
shown = collections.Counter()
n = 0
out = []
for line in sys.stdin:
    n += 1
    line = line.rstrip("\n")
    m = tid_re.search(line)
    tid = m.group(1) if m else "?"
    e = ev_re.search(line)
    if e:
        ev_hist[e.group(2)].append(f"line {n}: {line[-200:]}")
        if e.group(3):
            ev_hist[e.group(2)].append(f"   stream {e.group(3)} captures: {list(cap_hist[e.group(3)])}")
        last_ev[tid] = e.group(2)
    c = cap_re.search(line)
    if c:
        cap_hist[c.group(2)].append(f"line {n}: {c.group(1)}")
    r = ret_re.search(line)
    if r and r.group(2) not in BENIGN:
        key = (r.group(1), r.group(2))
        counts[key] += 1
        if shown[key] < 3:
            shown[key] += 1
            out.append(f"== {key[0]} -> {key[1]} (tid {tid}, line {n})")
            out.extend(per_tid[tid])
            out.append(line)
            if "Event" in r.group(2) and tid in last_ev:
                out.append(f"-- history of event {last_ev[tid]}:")
                out.extend(ev_hist[last_ev[tid]])
    per_tid[tid].append(line[-300:])
print(f"{n} log lines")
for (fn, st), c in counts.most_common():
    print(f"{c:8d}  {fn} -> {st}")
print()
print("\n".join(out))
