#!/usr/bin/env python3
"""Compare two stack_tx_bench --dump files (12-byte records: seq, ip_id, ip_sum, th_sum, len)."""
import sys

import numpy as np

dt = np.dtype([("seq", ">u4"), ("id", ">u2"), ("ip", ">u2"), ("th", ">u2"), ("len", ">u2")])
a, b = (np.fromfile(p, dtype=dt) for p in sys.argv[1:3])
print(f"records {len(a)} {len(b)}")
n = min(len(a), len(b))
bad = np.nonzero(a[:n] != b[:n])[0]
print(f"differing {len(bad)}")
for i in bad[:20]:
    print(i, a[i], b[i])
if len(bad):
    for f in ("seq", "id", "ip", "th", "len"):
        print(f, int((a[f][:n] != b[f][:n]).sum()))
